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

}  // namespace mragan
