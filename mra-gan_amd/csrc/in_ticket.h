// In-launch InstanceNorm finalize ("last block done", ABI 15).
//
// A conv whose epilogue leaves InstanceNorm statistics partials [N][chunks][ny][2] (the K-split
// brick, conv_brick_ks.hip) can also finalize them: the blocks of one (instance, column tile) each
// store their partial row with write-through (sc1) stores, wait for them, and draw a ticket from a
// per-(instance, tile) counter; the block that draws the last ticket sums the tile's partial rows in
// a fixed order (deterministic whichever block is last) and writes μ / rstd — or the backward
// coefficients mean(g), mean(g·x̂) — for those columns.  The separate finalize launch and its
// dependency gap go (≈ 5 µs each under the two-lane schedule, r04v trace).
//
// Hand-off (MI355X_MICROARCH.md §inter-workgroup visibility, cdna_hip_programming.md §5 item 2):
// producer — sc1 stores of the partials, every wave `s_waitcnt vmcnt(0)`, a workgroup barrier, one
// lane's relaxed agent-scope fetch_add; reducer — lane 0's agent acquire fence + wait + barrier, then
// sc1 loads of every partial.  The counters live in a hipMalloc'd pool zeroed once by the host; the
// reducer resets its counter, so a slot is reusable as soon as its launch has finished (the host
// hands out slots round-robin: no two kernels that may run at once share one).
#pragma once

#include <hip/hip_runtime.h>

namespace mragan {

constexpr double kTicketInEps = (double)1e-5f;   // InstanceNorm3d eps, as instnorm.hip's (double)kInEps

__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// every thread of the block: true in the block that drew the last of `expected` tickets (then with
// the other blocks' partials visible to its sc1 loads); `flag` is one int of the block's LDS
__device__ __forceinline__ bool in_ticket_draw(unsigned* ticket, int expected, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = prev == (unsigned)(expected - 1) ? 1 : 0;
  }
  __syncthreads();
  const bool last = *flag != 0;
  if (last) {
    if (threadIdx.x == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return last;
}

// the reducer (256 threads): columns [c0, c0 + BN) of instance nb.  Stream (column, Σ | Σ²) is
// summed by TPS threads — thread j takes rows j, j + TPS, … — then a fixed xor butterfly over the
// TPS lanes.  mode 0: out0 = μ, out1 = rstd ([N][ny]); mode 1: out0 = (mean g, mean g·x̂) pairs
// ([N][ny][2]).  S = voxels per instance of the normalised tensor.
template <int BN>
__device__ __forceinline__ void in_ticket_reduce(const double* part, int chunks, int ny, int nb, int c0, int mode,
                                                 double S, float* out0, float* out1) {
  constexpr int NS = 2 * BN;
  static_assert(NS <= 256 && 256 % NS == 0, "one or more threads per stream");
  constexpr int TPS = 256 / NS;
  const int tid = threadIdx.x, st = tid / TPS, j = tid % TPS;
  const int col = st >> 1, q = st & 1;
  double* base = const_cast<double*>(part) + ((int64_t)nb * chunks * ny + c0 + col) * 2 + q;
  double acc = 0.0;
#pragma unroll 8
  for (int k = j; k < chunks; k += TPS)
    acc += __hip_atomic_load(base + (int64_t)k * ny * 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int off = TPS / 2; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
  const double sq = __shfl_down(acc, TPS);      // stream (col, Σ²) on the lanes of (col, Σ)
  if (j == 0 && q == 0) {
    const int i = nb * ny + c0 + col;
    if (mode == 0) {
      const double mu = acc / S;
      double var = sq / S - mu * mu;
      if (var < 0) var = 0;
      out0[i] = (float)mu;
      out1[i] = (float)(1.0 / sqrt(var + kTicketInEps));
    } else {
      out0[2 * i] = (float)(acc / S);
      out0[2 * i + 1] = (float)(sq / S);
    }
  }
}

}  // namespace mragan
