// Output-parity-class geometry shared by the implicit-GEMM convolution kernels.
//
// Forward form: one class; output o reads input o*s - p + t for every tap t.
// Transposed form: outputs o ≡ c (mod s) form class c; they read input (o + p - t)/s for the taps
// t ≡ (c + p) (mod s) only, so a class visits real taps exclusively (sub-pixel decomposition).
#pragma once
#include "common.h"

namespace mragan {

// per-dimension class geometry
struct DimGeo {
  int Q;       // number of output positions in the class along this dim
  int ntap;    // taps visited along this dim
  int t0, tstep;
  int a_mul;   // in = a_mul*q + base_add + sign*j
  int base_add;
  int sign;
  int o_mul, o_add;   // output coordinate = o_mul*q + o_add
};

__device__ __forceinline__ DimGeo dim_geo(int c, int O, int k, int s, int p, int trans) {
  DimGeo g;
  if (!trans) {
    g.Q = O; g.ntap = k; g.t0 = 0; g.tstep = 1;
    g.a_mul = s; g.base_add = -p; g.sign = 1;
    g.o_mul = 1; g.o_add = 0;
  } else {
    g.Q = (O - c + s - 1) / s;
    int t0 = (c + p) % s;
    g.t0 = t0; g.tstep = s;
    g.ntap = (t0 < k) ? (k - t0 + s - 1) / s : 0;
    g.a_mul = 1; g.base_add = (c + p - t0) / s; g.sign = -1;
    g.o_mul = s; g.o_add = c;
  }
  return g;
}

// Shell classes of a full transposed k×k×k stride-1 convolution (the data gradient of a valid
// conv on a replication-padded input: output extent O = input + k − 1 per dim, y[o] = Σ_t
// x[o − t]·Wp[t]).  The brick kernel computes the interior (every output with ≥ 1 real tap along
// each dim's full range, 1 … O−2 for k = 3); the shell — the outputs on the first / last plane of
// some dim — is split into 6 classes: class 2f + side has dim f on the low (side 0, o = 0, tap 0
// only) or high (side 1, o = O−1, tap k−1 only) plane, the dims before f interior, the dims after
// f over their full range.  Every shell output is in exactly one class (Σ = O³ − (O−2)³ for k = 3).
__device__ __forceinline__ DimGeo shell_geo(int cls, int dim, int O, int k) {
  const int f = cls >> 1, hi = cls & 1;
  DimGeo g;
  g.tstep = 1; g.a_mul = 1; g.sign = -1; g.o_mul = 1;
  if (dim == f) {
    g.Q = 1; g.ntap = 1; g.t0 = hi ? k - 1 : 0; g.base_add = hi ? O - k : 0; g.o_add = hi ? O - 1 : 0;
  } else if (dim < f) {
    g.Q = O - 2; g.ntap = k; g.t0 = 0; g.base_add = 1; g.o_add = 1;
  } else {
    g.Q = O; g.ntap = k; g.t0 = 0; g.base_add = 0; g.o_add = 0;
  }
  return g;
}

}  // namespace mragan
