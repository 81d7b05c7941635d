// InstanceNorm3d(affine=False, track_running_stats=True), train mode, on NDHWC fp32
// (reference networks3D.py:15-24: get_norm_layer('instance'); used after every conv of G and
// the three middle convs of D).  Fusions:
//   forward : y = act((x − μ)·rstd) + residual, written straight into a replication-padded
//             output (the ReplicationPad3d that precedes the next conv, networks3D.py:185/211/
//             233/249) — so neither the pad nor the activation costs a separate pass.
//   backward: g = fold(dy_padded) (+ dy_add) (ReplicationPad3d backward), × act'(x̂),
//             dx = rstd·(g − mean(g) − x̂·mean(g·x̂)); optionally also writes the folded g
//             before act' (a ResnetBlock's input gradient, which its skip path needs again) —
//             the separate rpad_fold pass then disappears.
// Statistics are accumulated in fp64 from fp32 data (per-thread → block → chunk partials),
// so the single-pass Σx / Σx² form keeps full fp32 accuracy.
#include "kernels.h"

namespace mragan {

constexpr float kInEps = 1e-5f;


// partial bytes per instance the fused finalize + apply kernels reduce in every block (beyond it:
// a separate finalize launch).  Opt-in A/B switch MRAGAN_IN_FUSED=1, off by default: measured
// slower on MI355X (64³ b2 bf16 step 12.95 vs 12.32 ms, same box, r04j) — every apply block
// re-reads its instance's partials (up to 64 KB; 100 MB per launch for the 64³ norms), and the
// capped statistics chunks halve the parallelism of the statistics pass (C128 4×16³ backward
// 43.9 vs 23.1 µs)
constexpr int kFuseMaxBytes = 64 * 1024;
static const bool g_in_unfused = getenv("MRAGAN_IN_FUSED") == nullptr;
static bool in_fusable(int chunks, int C) { return (int64_t)chunks * C * 16 <= kFuseMaxBytes; }

// row chunks per instance: ≈2048 blocks per launch, but ≥ 4 float4 loads per thread, and few
// enough that the apply kernel can reduce them in-block (in_fusable)
static int in_chunks(const InShape& s) {
  const int rows = s.D * s.H;
  const int64_t rowq = (int64_t)s.W * (s.C / 4);
  int64_t want = (2048 + s.N - 1) / s.N;
  const int64_t fuse_cap = kFuseMaxBytes / ((int64_t)s.C * 16);
  if (!g_in_unfused && want > fuse_cap) want = fuse_cap;
  int64_t min_rows = (4 * 256 + rowq - 1) / rowq;            // rows per block for ≥ 4 loads/thread
  int64_t cap = (rows + min_rows - 1) / min_rows;
  if (want > cap) want = cap;
  if (want > rows) want = rows;
  if (want < 1) want = 1;
  return (int)want;
}

// all in-kernel offsets are 32-bit (element counts of every tensor < 2^31)
static bool in_fits(const InShape& s, int pad) {
  const int64_t e = (int64_t)s.N * (s.D + 2 * pad) * (s.H + 2 * pad) * (s.W + 2 * pad) * s.C;
  return e < (int64_t(1) << 31);
}

size_t instnorm_ws_bytes(int N, int D, int H, int W, int C) {
  InShape s{N, D, H, W, C};
  return (size_t)N * in_chunks(s) * C * 2 * sizeof(double) + 16;
}

// Σ over chunks of partials[n][chunk][C][2] in fixed order (deterministic).  Block = 4
// channels × 64 chunk rows, one wave per channel; grid (ceil(C/4), N): each lane sums ≤ chunks/64
// partials with its loads in flight together, then a fixed xor butterfly over the wave's 64 lanes
// (lane 0's result: the same association every launch).  The 64 row sums were combined by one
// thread per channel through LDS before: 64 dependent LDS round trips, most of a 4.8 µs launch
// (r04i trace, ≈ 250 of these per 64³ b2 step).
// mode 0: mean / rstd (out0, out1); mode 1: backward coefficients (out0 = coef[2C]).
__device__ void in_finalize_group_lds(const double* __restrict__ part, const InShape& s, int chunks, int n, int cgroup,
                                      int mode, float* __restrict__ out0, float* __restrict__ out1) {
  // A/B (MRAGAN_IN_FIN_LDS): the r04 form — channel fastest, 64 row sums combined by one thread
  __shared__ double fr[2][256];
  constexpr int CW = 4, ROWS = 64;
  const int tid = threadIdx.x, cl = tid % CW, row = tid / CW;
  const int c = cgroup * CW + cl;
  double sa = 0, sb = 0;
  if (c < s.C) {
#pragma unroll 8
    for (int k = row; k < chunks; k += ROWS) {
      const double2 p = *reinterpret_cast<const double2*>(part + (((int64_t)n * chunks + k) * s.C + c) * 2);
      sa += p.x; sb += p.y;
    }
  }
  fr[0][tid] = sa; fr[1][tid] = sb;
  __syncthreads();
  if (row == 0 && c < s.C) {
    double a = 0, b = 0;
    for (int r = 0; r < ROWS; ++r) { a += fr[0][r * CW + cl]; b += fr[1][r * CW + cl]; }
    const double S = (double)s.S();
    const int i = n * s.C + c;
    if (mode == 0) {
      const double mu = a / S;
      double var = b / S - mu * mu;
      if (var < 0) var = 0;
      out0[i] = (float)mu;
      out1[i] = (float)(1.0 / sqrt(var + (double)kInEps));
    } else {
      out0[2 * i] = (float)(a / S);
      out0[2 * i + 1] = (float)(b / S);
    }
  }
}

__device__ void in_finalize_group(const double* __restrict__ part, const InShape& s, int chunks, int n, int cgroup,
                                  int mode, float* __restrict__ out0, float* __restrict__ out1) {
  constexpr int CW = 4, ROWS = 64;
  const int tid = threadIdx.x, cl = tid / ROWS, row = tid % ROWS;
  const int c = cgroup * CW + cl;
  if (c >= s.C) return;                          // wave-uniform: the wave's channel
  double sa = 0, sb = 0;
#pragma unroll 8
  for (int k = row; k < chunks; k += ROWS) {
    const double2 p = *reinterpret_cast<const double2*>(part + (((int64_t)n * chunks + k) * s.C + c) * 2);
    sa += p.x; sb += p.y;
  }
#pragma unroll
  for (int off = ROWS / 2; off >= 1; off >>= 1) {
    sa += __shfl_xor(sa, off);
    sb += __shfl_xor(sb, off);
  }
  if (row == 0) {
    const double S = (double)s.S();
    const int i = n * s.C + c;
    if (mode == 0) {
      const double mu = sa / S;
      double var = sb / S - mu * mu;
      if (var < 0) var = 0;
      out0[i] = (float)mu;
      out1[i] = (float)(1.0 / sqrt(var + (double)kInEps));
    } else {
      out0[2 * i] = (float)(sa / S);
      out0[2 * i + 1] = (float)(sb / S);
    }
  }
}

// four values → the 16-bit operand words a bf16 (mode 2) / fp16 (mode 3) MFMA consumer would
// round them to (RNE, as prec.h's staging conversion): the 16-bit operand plane of a tensor
__device__ __forceinline__ uint2 f4_op16(float4 v, int mode) {
  typedef float f32x4_t __attribute__((ext_vector_type(4)));
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  typedef _Float16 f16x4_t __attribute__((ext_vector_type(4)));
  const f32x4_t f = {v.x, v.y, v.z, v.w};
  if (mode == 3) return __builtin_bit_cast(uint2, __builtin_convertvector(f, f16x4_t));
  return __builtin_bit_cast(uint2, __builtin_convertvector(f, bf16x4_t));
}

__device__ __forceinline__ float4 f4_act(float4 v, int act) {
  return make_float4(act_fwd(v.x, act), act_fwd(v.y, act), act_fwd(v.z, act), act_fwd(v.w, act));
}

__device__ __forceinline__ float dact_from_xhat(float xh, int act) {
  if (act == kActRelu) return xh > 0.f ? 1.f : 0.f;
  if (act == kActLrelu) return xh > 0.f ? 1.f : kLreluSlope;
  return 1.f;
}

// ---- forward statistics: partials[n][chunk][C][2] (Σx, Σx²) --------------------------------
// Rows (d, h) of one instance per block; thread = (voxel slot wt, channel quad q), q fixed per
// thread, the row's voxels dealt to the 256 / (C/4) slots: no per-element 64-bit index math.
__device__ __forceinline__ void in_block_reduce(double (&s0)[4], double (&s1)[4], int CQ, double* __restrict__ out) {
  __shared__ double red[2][256 * 4];
  const int tid = threadIdx.x;
  for (int j = 0; j < 4; ++j) { red[0][tid * 4 + j] = s0[j]; red[1][tid * 4 + j] = s1[j]; }
  __syncthreads();
  if (tid < CQ) {
    const int R = 256 / CQ;
    double a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
    for (int rr = 0; rr < R; ++rr)
      for (int j = 0; j < 4; ++j) { a[j] += red[0][(rr * CQ + tid) * 4 + j]; b[j] += red[1][(rr * CQ + tid) * 4 + j]; }
    for (int j = 0; j < 4; ++j) { out[8 * tid + 2 * j] = a[j]; out[8 * tid + 2 * j + 1] = b[j]; }
  }
}

__device__ __forceinline__ void in_rows(const InShape& s, int chunks, int chunk, int& r0, int& r1) {
  const int rows = s.D * s.H, per = (rows + chunks - 1) / chunks;
  r0 = chunk * per;
  r1 = min(rows, r0 + per);
}

__global__ void __launch_bounds__(256) in_stats_kernel(const float* __restrict__ x, InShape s, int chunks,
                                                       double* __restrict__ part) {
  const int n = blockIdx.y, chunk = blockIdx.x;
  const int CQ = s.C / 4, tid = threadIdx.x, q = tid % CQ, WS = 256 / CQ;
  const int wt = tid / CQ < WS ? tid / CQ : (1 << 30);   // C/4 not dividing 256: spare threads idle
  const int rowq = s.W * CQ;                       // float4s per row
  int r0, r1;
  in_rows(s, chunks, chunk, r0, r1);
  double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
  const float4* base = reinterpret_cast<const float4*>(x) + (size_t)n * s.D * s.H * rowq + q;
  for (int r = r0; r < r1; ++r) {
    const float4* row = base + (size_t)r * rowq;
    for (int w = wt; w < s.W; w += WS) {
      const float4 v = row[w * CQ];
      s0[0] += v.x; s0[1] += v.y; s0[2] += v.z; s0[3] += v.w;
      s1[0] += (double)v.x * v.x; s1[1] += (double)v.y * v.y; s1[2] += (double)v.z * v.z; s1[3] += (double)v.w * v.w;
    }
  }
  in_block_reduce(s0, s1, CQ, part + ((size_t)n * chunks + chunk) * s.C * 2);
}

// one block per instance (kernel boundary = coherence point for the partials of all XCDs; an
// in-kernel last-block reduction needs agent-scope release fences, i.e. L2 write-backs, per block)
__global__ void __launch_bounds__(256) in_finalize_kernel(const double* __restrict__ part, InShape s, int chunks,
                                                          float* __restrict__ mean, float* __restrict__ rstd, int lds) {
  if (lds) in_finalize_group_lds(part, s, chunks, blockIdx.y, blockIdx.x, 0, mean, rstd);
  else in_finalize_group(part, s, chunks, blockIdx.y, blockIdx.x, 0, mean, rstd);
}
static const int g_in_fin_lds = getenv("MRAGAN_IN_FIN_LDS") ? 1 : 0;

// ---- forward apply: y (padded by ypad) = act((x − μ)·rstd) + resid(interior of rpad-padded) --
// One output row (n, dp, hp) of the padded y per block iteration; source row and the residual
// row are fixed per row, each thread walks its float4s (q fixed per thread).
// y (fp32) and / or y16 (the 16-bit operand plane, precision mode `mode`) may be written
__global__ void __launch_bounds__(256) in_apply_kernel(const float* __restrict__ x, InShape s, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, int act,
                                                       const float* __restrict__ resid, int rpad, float* __restrict__ y,
                                                       int ypad, uint2* __restrict__ y16, int mode) {
  const int CQ = s.C / 4, tid = threadIdx.x, q = tid % CQ, WS = 256 / CQ;
  const int wt = tid / CQ < WS ? tid / CQ : (1 << 30);   // C/4 not dividing 256: spare threads idle
  const int Dp = s.D + 2 * ypad, Hp = s.H + 2 * ypad, Wp = s.W + 2 * ypad;
  const int Dr = s.D + 2 * rpad, Hr = s.H + 2 * rpad, Wr = s.W + 2 * rpad;
  const int rows = s.N * Dp * Hp, rowq = Wp * CQ;
  const float4* xv = reinterpret_cast<const float4*>(x);
  const float4* rv = reinterpret_cast<const float4*>(resid);
  float4* yv = reinterpret_cast<float4*>(y);
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const int hp = row % Hp, t = row / Hp, dp = t % Dp, n = t / Dp;
    const int sd = min(max(dp - ypad, 0), s.D - 1), sh = min(max(hp - ypad, 0), s.H - 1);
    const float4 mu = reinterpret_cast<const float4*>(mean + n * s.C)[q];
    const float4 rs = reinterpret_cast<const float4*>(rstd + n * s.C)[q];
    const float4* xrow = xv + (size_t)((n * s.D + sd) * s.H + sh) * s.W * CQ;
    const float4* rrow = resid ? rv + ((size_t)((n * Dr + sd + rpad) * Hr + sh + rpad) * Wr + rpad) * CQ : nullptr;
    float4* yrow = yv + (size_t)row * rowq + q;
    uint2* y16row = y16 + (size_t)row * rowq + q;
    for (int wp = wt; wp < Wp; wp += WS) {
      const int sw = min(max(wp - ypad, 0), s.W - 1);
      float4 v = xrow[sw * CQ + q];
      v = make_float4((v.x - mu.x) * rs.x, (v.y - mu.y) * rs.y, (v.z - mu.z) * rs.z, (v.w - mu.w) * rs.w);
      v = f4_act(v, act);
      if (resid) {
        const float4 r = rrow[sw * CQ + q];
        v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
      }
      if (y) yrow[wp * CQ] = v;
      if (y16) y16row[wp * CQ] = f4_op16(v, mode);
    }
  }
}

// ---- backward -----------------------------------------------------------------------------
// g = fold_pad(dy) (+ dy_add) · act'(x̂).  Per row (n, d, h) the padded rows folded into it are
// fixed ([d0, d1] × [h0, h1], one each inside the volume); per voxel w the padded columns
// [w0, w1].  32-bit offsets (the host checks the sizes).
struct InRow {
  const float4* dy;    // first padded row (d0, h0) of the fold, at column 0
  int nd, nh;          // rows folded along d and h
  int dstride, hstride;  // float4 strides between folded rows
  const float4* x;     // x row
  const float4* add;   // dy_add row or null
  float4 mu, rs;
};

__device__ __forceinline__ InRow in_bwd_row(const InBwdArgs& a, const InShape& s, int n, int d, int h, int q) {
  const int CQ = s.C / 4, p = a.dypad;
  const int Hp = s.H + 2 * p, Wp = s.W + 2 * p, Dp = s.D + 2 * p;
  const int d0 = d == 0 ? 0 : d + p, d1 = d == s.D - 1 ? s.D - 1 + 2 * p : d + p;
  const int h0 = h == 0 ? 0 : h + p, h1 = h == s.H - 1 ? s.H - 1 + 2 * p : h + p;
  InRow r;
  r.dy = reinterpret_cast<const float4*>(a.dy) + ((size_t)(n * Dp + d0) * Hp + h0) * Wp * CQ + q;
  r.nd = d1 - d0 + 1;
  r.nh = h1 - h0 + 1;
  r.hstride = Wp * CQ;
  r.dstride = Hp * Wp * CQ;
  const size_t xo = ((size_t)(n * s.D + d) * s.H + h) * s.W * CQ + q;
  r.x = reinterpret_cast<const float4*>(a.x) + xo;
  r.add = a.dy_add ? reinterpret_cast<const float4*>(a.dy_add) + xo : nullptr;
  r.mu = reinterpret_cast<const float4*>(a.mean + n * s.C)[q];
  r.rs = reinterpret_cast<const float4*>(a.rstd + n * s.C)[q];
  return r;
}

__device__ __forceinline__ void f4_add(float4& g, const float4& v) {
  g.x += v.x; g.y += v.y; g.z += v.z; g.w += v.w;
}

// fold of one padded row at voxel w: its column w + P, plus columns 0 … P−1 at w = 0 and
// W+P … W+2P−1 at w = W−1.  P is a template parameter so the border columns are a fixed, unrolled
// run of loads issued together (a runtime-bound loop made the w = 0 / W−1 lanes walk P+1 dependent
// loads, and their waves — hence every row — took ~P+1 load latencies: the pad-3 backward of the
// 64³ C32 norm ran at 2.5× the time of the pad-0 one)
template <int P>
__device__ __forceinline__ float4 in_fold_row(const float4* rowp, int w, int W, int CQ) {
  float4 g = rowp[(w + P) * CQ];
  if constexpr (P > 0) {
    if (w == 0) {
#pragma unroll
      for (int c = 0; c < P; ++c) f4_add(g, rowp[c * CQ]);
    }
    if (w == W - 1) {
#pragma unroll
      for (int c = 0; c < P; ++c) f4_add(g, rowp[(W + P + c) * CQ]);
    }
  }
  return g;
}

template <int P>
__device__ __forceinline__ void in_bwd_voxel(const InBwdArgs& a, const InShape& s, const InRow& r, int w, float4& g,
                                             float4& xh, float4* graw = nullptr) {
  const int CQ = s.C / 4;
  if constexpr (P < 0) {                               // any pad (runtime): the generic fold
    const int p = a.dypad;
    const int w0 = w == 0 ? 0 : w + p, w1 = w == s.W - 1 ? s.W - 1 + 2 * p : w + p;
    g = r.dy[w0 * CQ];
    if (p && (r.nd > 1 || r.nh > 1 || w1 > w0)) {      // border: sum the folded padded voxels
      g = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int i = 0; i < r.nd; ++i)
        for (int j = 0; j < r.nh; ++j) {
          const float4* rowp = r.dy + i * r.dstride + j * r.hstride;
          for (int c = w0; c <= w1; ++c) f4_add(g, rowp[c * CQ]);
        }
    }
  } else {
    // rows folded along d / h (nd, nh > 1 only on border rows: uniform per block row)
    g = in_fold_row<P>(r.dy, w, s.W, CQ);
    if (P > 0 && (r.nd > 1 || r.nh > 1)) {
      for (int i = 0; i < r.nd; ++i)
        for (int j = 0; j < r.nh; ++j)
          if (i | j) f4_add(g, in_fold_row<P>(r.dy + i * r.dstride + j * r.hstride, w, s.W, CQ));
    }
  }
  if (r.add) {
    const float4 e = r.add[w * CQ];
    g.x += e.x; g.y += e.y; g.z += e.z; g.w += e.w;
  }
  if (graw) *graw = g;
  const float4 xv = r.x[w * CQ];
  xh = make_float4((xv.x - r.mu.x) * r.rs.x, (xv.y - r.mu.y) * r.rs.y, (xv.z - r.mu.z) * r.rs.z,
                   (xv.w - r.mu.w) * r.rs.w);
  g.x *= dact_from_xhat(xh.x, a.act); g.y *= dact_from_xhat(xh.y, a.act);
  g.z *= dact_from_xhat(xh.z, a.act); g.w *= dact_from_xhat(xh.w, a.act);
}

template <int P>
__global__ void __launch_bounds__(256) in_bwd_stats_kernel(InBwdArgs a, InShape s, int chunks, double* __restrict__ part) {
  const int n = blockIdx.y, chunk = blockIdx.x;
  const int CQ = s.C / 4, tid = threadIdx.x, q = tid % CQ, WS = 256 / CQ;
  const int wt = tid / CQ < WS ? tid / CQ : (1 << 30);   // C/4 not dividing 256: spare threads idle
  int r0, r1;
  in_rows(s, chunks, chunk, r0, r1);
  double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
  for (int r = r0; r < r1; ++r) {
    const InRow row = in_bwd_row(a, s, n, r / s.H, r % s.H, q);
    for (int w = wt; w < s.W; w += WS) {
      float4 g, xh;
      in_bwd_voxel<P>(a, s, row, w, g, xh);
      s0[0] += g.x; s0[1] += g.y; s0[2] += g.z; s0[3] += g.w;
      s1[0] += (double)g.x * xh.x; s1[1] += (double)g.y * xh.y; s1[2] += (double)g.z * xh.z; s1[3] += (double)g.w * xh.w;
    }
  }
  in_block_reduce(s0, s1, CQ, part + ((size_t)n * chunks + chunk) * s.C * 2);
}

__global__ void __launch_bounds__(256) in_bwd_finalize_kernel(const double* __restrict__ part, InShape s, int chunks,
                                                              float* __restrict__ coef, int lds) {
  if (lds) in_finalize_group_lds(part, s, chunks, blockIdx.y, blockIdx.x, 1, coef, nullptr);
  else in_finalize_group(part, s, chunks, blockIdx.y, blockIdx.x, 1, coef, nullptr);
}

template <int P>
__global__ void __launch_bounds__(256) in_bwd_apply_kernel(InBwdArgs a, InShape s, const float* __restrict__ coef) {
  const int CQ = s.C / 4, tid = threadIdx.x, q = tid % CQ, WS = 256 / CQ;
  const int wt = tid / CQ < WS ? tid / CQ : (1 << 30);   // C/4 not dividing 256: spare threads idle
  const int rows = s.N * s.D * s.H;
  float4* dx = reinterpret_cast<float4*>(a.dx);
  for (int rr = blockIdx.x; rr < rows; rr += gridDim.x) {
    const int h = rr % s.H, t = rr / s.H, d = t % s.D, n = t / s.D;
    const InRow row = in_bwd_row(a, s, n, d, h, q);
    const float4 c0 = reinterpret_cast<const float4*>(coef + 2 * (n * s.C + 4 * q))[0];   // (mg0, mgx0, mg1, mgx1)
    const float4 c1 = reinterpret_cast<const float4*>(coef + 2 * (n * s.C + 4 * q))[1];
    float4* out = dx + (size_t)rr * s.W * CQ + q;
    uint2* out16 = reinterpret_cast<uint2*>(a.dx16) + (size_t)rr * s.W * CQ + q;
    float4* gout = a.g_out ? reinterpret_cast<float4*>(a.g_out) + (size_t)rr * s.W * CQ + q : nullptr;
    for (int w = wt; w < s.W; w += WS) {
      float4 g, xh, graw;
      in_bwd_voxel<P>(a, s, row, w, g, xh, &graw);
      if (gout) gout[w * CQ] = graw;
      float4 o;
      o.x = row.rs.x * (g.x - c0.x - xh.x * c0.y);
      o.y = row.rs.y * (g.y - c0.z - xh.y * c0.w);
      o.z = row.rs.z * (g.z - c1.x - xh.z * c1.y);
      o.w = row.rs.w * (g.w - c1.z - xh.w * c1.w);
      if (dx) out[w * CQ] = o;
      if (a.dx16) out16[w * CQ] = f4_op16(o, a.mode16);
    }
  }
}

// ---- fused finalize + apply ------------------------------------------------------------------
// The separate finalize launches (one per InstanceNorm and direction, ~5 µs each plus the
// dependency gap: 234 launches per 64³ b2 step, r04i trace) fold into the apply: every block of
// instance n reduces the instance's partials [chunks][C][2] (≤ kFuseMaxBytes, L2-resident) in the
// same fixed order — identical statistics in every block, deterministic — then applies them to its
// rows.  Grid (Bi, N): block (bi, n) owns rows [bi·per, (bi+1)·per) of instance n.
// mode 0: μ / rstd into sa / sb; mode 1: the backward coefficients mean(g), mean(g·x̂).
__device__ void in_stats_block(const double* __restrict__ part, const InShape& s, int chunks, int n, int mode,
                               float* sa, float* sb) {
  __shared__ double fr[2][256];
  const int tid = threadIdx.x;
  int tpc = 1;                                   // threads per channel (power of two)
  while (tpc * 2 * s.C <= 256) tpc *= 2;
  const int cpp = 256 / tpc;                     // channels per pass
  const double S = (double)s.S();
  for (int c0 = 0; c0 < s.C; c0 += cpp) {
    const int c = c0 + tid / tpc, j = tid % tpc;
    double a = 0, b = 0;
    if (c < s.C) {
#pragma unroll 4
      for (int k = j; k < chunks; k += tpc) {
        const double2 p = *reinterpret_cast<const double2*>(part + (((int64_t)n * chunks + k) * s.C + c) * 2);
        a += p.x; b += p.y;
      }
    }
    fr[0][tid] = a; fr[1][tid] = b;
    __syncthreads();
    if (j == 0 && c < s.C) {
      double A = 0, B = 0;
      for (int r = 0; r < tpc; ++r) { A += fr[0][tid + r]; B += fr[1][tid + r]; }
      if (mode == 0) {
        const double mu = A / S;
        double var = B / S - mu * mu;
        if (var < 0) var = 0;
        sa[c] = (float)mu;
        sb[c] = (float)(1.0 / sqrt(var + (double)kInEps));
      } else {
        sa[c] = (float)(A / S);
        sb[c] = (float)(B / S);
      }
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) in_apply_fused_kernel(const float* __restrict__ x, InShape s,
                                                             const double* __restrict__ part, int chunks,
                                                             float* __restrict__ mean, float* __restrict__ rstd,
                                                             int act, const float* __restrict__ resid, int rpad,
                                                             float* __restrict__ y, int ypad, uint2* __restrict__ y16,
                                                             int mode, int per) {
  __shared__ __attribute__((aligned(16))) float smu[1024], srs[1024];
  const int n = blockIdx.y, bi = blockIdx.x, tid = threadIdx.x;
  in_stats_block(part, s, chunks, n, 0, smu, srs);
  if (bi == 0)
    for (int c = tid; c < s.C; c += 256) { mean[n * s.C + c] = smu[c]; rstd[n * s.C + c] = srs[c]; }
  const int CQ = s.C / 4, q = tid % CQ, WS = 256 / CQ;
  const int wt = tid / CQ < WS ? tid / CQ : (1 << 30);   // C/4 not dividing 256: spare threads idle
  const int Dp = s.D + 2 * ypad, Hp = s.H + 2 * ypad, Wp = s.W + 2 * ypad;
  const int Dr = s.D + 2 * rpad, Hr = s.H + 2 * rpad, Wr = s.W + 2 * rpad;
  const int rowq = Wp * CQ;
  const float4 mu = reinterpret_cast<const float4*>(smu)[q];
  const float4 rs = reinterpret_cast<const float4*>(srs)[q];
  const float4* xv = reinterpret_cast<const float4*>(x);
  const float4* rv = reinterpret_cast<const float4*>(resid);
  float4* yv = reinterpret_cast<float4*>(y);
  const int r1 = min(Dp * Hp, (bi + 1) * per);
  for (int rr = bi * per; rr < r1; ++rr) {
    const int hp = rr % Hp, dp = rr / Hp;
    const int row = n * Dp * Hp + rr;
    const int sd = min(max(dp - ypad, 0), s.D - 1), sh = min(max(hp - ypad, 0), s.H - 1);
    const float4* xrow = xv + (size_t)((n * s.D + sd) * s.H + sh) * s.W * CQ;
    const float4* rrow = resid ? rv + ((size_t)((n * Dr + sd + rpad) * Hr + sh + rpad) * Wr + rpad) * CQ : nullptr;
    float4* yrow = yv + (size_t)row * rowq + q;
    uint2* y16row = y16 + (size_t)row * rowq + q;
    for (int wp = wt; wp < Wp; wp += WS) {
      const int sw = min(max(wp - ypad, 0), s.W - 1);
      float4 v = xrow[sw * CQ + q];
      v = make_float4((v.x - mu.x) * rs.x, (v.y - mu.y) * rs.y, (v.z - mu.z) * rs.z, (v.w - mu.w) * rs.w);
      v = f4_act(v, act);
      if (resid) {
        const float4 r = rrow[sw * CQ + q];
        v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
      }
      if (y) yrow[wp * CQ] = v;
      if (y16) y16row[wp * CQ] = f4_op16(v, mode);
    }
  }
}

template <int P>
__global__ void __launch_bounds__(256) in_bwd_apply_fused_kernel(InBwdArgs a, InShape s, const double* __restrict__ part,
                                                                 int chunks, int per) {
  __shared__ __attribute__((aligned(16))) float sg[1024], sgx[1024];
  const int n = blockIdx.y, bi = blockIdx.x, tid = threadIdx.x;
  in_stats_block(part, s, chunks, n, 1, sg, sgx);
  const int CQ = s.C / 4, q = tid % CQ, WS = 256 / CQ;
  const int wt = tid / CQ < WS ? tid / CQ : (1 << 30);   // C/4 not dividing 256: spare threads idle
  const float4 mg = reinterpret_cast<const float4*>(sg)[q], mgx = reinterpret_cast<const float4*>(sgx)[q];
  float4* dx = reinterpret_cast<float4*>(a.dx);
  const int r1 = min(s.D * s.H, (bi + 1) * per);
  for (int r = bi * per; r < r1; ++r) {
    const int h = r % s.H, d = r / s.H;
    const int rr = n * s.D * s.H + r;
    const InRow row = in_bwd_row(a, s, n, d, h, q);
    float4* out = dx + (size_t)rr * s.W * CQ + q;
    uint2* out16 = reinterpret_cast<uint2*>(a.dx16) + (size_t)rr * s.W * CQ + q;
    float4* gout = a.g_out ? reinterpret_cast<float4*>(a.g_out) + (size_t)rr * s.W * CQ + q : nullptr;
    for (int w = wt; w < s.W; w += WS) {
      float4 g, xh, graw;
      in_bwd_voxel<P>(a, s, row, w, g, xh, &graw);
      if (gout) gout[w * CQ] = graw;
      float4 o;
      o.x = row.rs.x * (g.x - mg.x - xh.x * mgx.x);
      o.y = row.rs.y * (g.y - mg.y - xh.y * mgx.y);
      o.z = row.rs.z * (g.z - mg.z - xh.z * mgx.z);
      o.w = row.rs.w * (g.w - mg.w - xh.w * mgx.w);
      if (dx) out[w * CQ] = o;
      if (a.dx16) out16[w * CQ] = f4_op16(o, a.mode16);
    }
  }
}

// fused grid: whole rows, never straddling instances; at least one block per CU in total, and
// about 256 KB of traffic per block for the large (64³-class) norms, whose blocks then stay few
// against their rows (each block re-reads the instance's partials once: ≤ 64 KB)
static void fused_grid(int N, int rows, int64_t bytes_per_row, int& bi, int& per) {
  int64_t want = (256 + N - 1) / N;
  const int64_t by_bytes = (rows * bytes_per_row + (256 << 10) - 1) / (256 << 10);
  if (want < by_bytes) want = by_bytes;
  if (want > rows) want = rows;
  if (want < 1) want = 1;
  per = (rows + want - 1) / want;
  bi = (rows + per - 1) / per;
}

static int launch_in_apply(const float* x, const InShape& s, const double* part, int chunks, float* mean, float* rstd,
                           int act, const float* resid, int rpad, float* y, int ypad, void* y16, int mode16,
                           hipStream_t st) {
  if (in_fusable(chunks, s.C) && !g_in_unfused) {
    int bi, per;
    // per padded row: the source row read, the fp32 / 16-bit output rows written
    const int64_t bpr = (int64_t)s.C * ((int64_t)s.W * 4 * (resid ? 2 : 1) + (int64_t)(s.W + 2 * ypad) * ((y ? 4 : 0) + (y16 ? 2 : 0)));
    fused_grid(s.N, (s.D + 2 * ypad) * (s.H + 2 * ypad), bpr, bi, per);
    hipLaunchKernelGGL(in_apply_fused_kernel, dim3(bi, s.N), dim3(256), 0, st, x, s, part, chunks, mean, rstd, act,
                       resid, rpad, y, ypad, static_cast<uint2*>(y16), mode16, per);
    return check_launch(y16 ? "in_apply_fused(op16)" : "in_apply_fused");
  }
  hipLaunchKernelGGL(in_finalize_kernel, dim3(ceil_div(s.C, 4), s.N), dim3(256), 0, st, part, s, chunks, mean, rstd, g_in_fin_lds);
  int rc = check_launch("in_finalize");
  if (rc) return rc;
  const int rows = s.N * (s.D + 2 * ypad) * (s.H + 2 * ypad);
  hipLaunchKernelGGL(in_apply_kernel, dim3(rows < 16384 ? rows : 16384), dim3(256), 0, st, x, s, mean, rstd, act, resid,
                     rpad, y, ypad, static_cast<uint2*>(y16), mode16);
  return check_launch(y16 ? "in_apply(op16)" : "in_apply");
}

static int launch_in_bwd_apply(const InBwdArgs& a, const InShape& s, const double* part, int chunks, float* coef,
                               hipStream_t st) {
  if (in_fusable(chunks, s.C) && !g_in_unfused) {
    int bi, per;
    // per row: dy (padded rows folded in: ≈ the row), x, dx / dx16, g_out
    const int64_t bpr = (int64_t)s.C * s.W * (4 + 4 + (a.dx ? 4 : 0) + (a.dx16 ? 2 : 0) + (a.g_out ? 4 : 0) + (a.dy_add ? 4 : 0));
    fused_grid(s.N, s.D * s.H, bpr, bi, per);
    const dim3 g(bi, s.N);
    switch (a.dypad) {
      case 0: hipLaunchKernelGGL(in_bwd_apply_fused_kernel<0>, g, dim3(256), 0, st, a, s, part, chunks, per); break;
      case 1: hipLaunchKernelGGL(in_bwd_apply_fused_kernel<1>, g, dim3(256), 0, st, a, s, part, chunks, per); break;
      case 3: hipLaunchKernelGGL(in_bwd_apply_fused_kernel<3>, g, dim3(256), 0, st, a, s, part, chunks, per); break;
      default: hipLaunchKernelGGL(in_bwd_apply_fused_kernel<-1>, g, dim3(256), 0, st, a, s, part, chunks, per); break;
    }
    return check_launch(a.dx16 ? "in_bwd_apply_fused(op16)" : "in_bwd_apply_fused");
  }
  hipLaunchKernelGGL(in_bwd_finalize_kernel, dim3(ceil_div(s.C, 4), s.N), dim3(256), 0, st, part, s, chunks, coef, g_in_fin_lds);
  int rc = check_launch("in_bwd_finalize");
  if (rc) return rc;
  const int rows = s.N * s.D * s.H;
  const dim3 ga(rows < 16384 ? rows : 16384);
  switch (a.dypad) {
    case 0: hipLaunchKernelGGL(in_bwd_apply_kernel<0>, ga, dim3(256), 0, st, a, s, coef); break;
    case 1: hipLaunchKernelGGL(in_bwd_apply_kernel<1>, ga, dim3(256), 0, st, a, s, coef); break;
    case 3: hipLaunchKernelGGL(in_bwd_apply_kernel<3>, ga, dim3(256), 0, st, a, s, coef); break;
    default: hipLaunchKernelGGL(in_bwd_apply_kernel<-1>, ga, dim3(256), 0, st, a, s, coef); break;
  }
  return check_launch(a.dx16 ? "in_bwd_apply(op16)" : "in_bwd_apply");
}

// ---- small instances: statistics and apply in ONE launch ----------------------------------
// The three-launch form (statistics partials → finalize → apply) costs three dependent launches
// whatever the size; on the small tensors (the UNet's 8³ / 4³ / 2³ levels, the PatchGAN's 8³ / 7³
// layers, ≤ 64 KB per channel group) each launch is a few µs of dispatch and ramp for a few KB of
// data, and the chain of a lane is what the step waits for (UNet 64³ b1 step: 240 of its ≈ 680
// launches were InstanceNorm).  Here a block owns 4·CQB channels of one instance: pass 1 sums
// (Σx, Σx²) — or the backward's (Σg, Σg·x̂) — in fp64 over every voxel, a fixed xor butterfly
// over the wave's voxel slots and a fixed 4-wave sum give the statistics (deterministic), pass 2
// re-reads the block's (L2-resident) slice and applies.  No partials, no finalize launch.
// Thread = (voxel slot vt, channel quad q of the block), q fastest: lane = vt·CQB + q.
constexpr int kInSmallBytes = 64 * 1024;          // per block and pass
constexpr int kInSmallU = 8;                      // voxels per thread whose loads are in flight together
static int in_small_cqb(const InShape& s) {
  static const int64_t max_s = [] {                 // A/B: MRAGAN_IN_SMALL=0 off, =S the largest S
    const char* e = getenv("MRAGAN_IN_SMALL");
    return e ? (int64_t)atoll(e) : (int64_t)1 << 20;
  }();
  // a block reads whole 128-B lines of each voxel (32 channels, or all of a narrower tensor): with
  // fewer channels per block every line is fetched by several blocks on different XCDs — the
  // 4-channel slices of a 16³ C128 norm ran the 64³ b2 step at 13.2 instead of 11.1 ms (r05o)
  const int CQ = s.C / 4;
  int cqb = 8;
  while (cqb > 1 && (cqb > CQ || CQ % cqb)) cqb >>= 1;           // narrower tensors: 4, 2 or 1 quads
  if (s.S() > max_s || s.N < 1 || (cqb < 8 && s.C >= 32)) return 0;
  return s.S() * cqb * 16 <= kInSmallBytes ? cqb : 0;
}

// fixed-order block sum of 4 channel values (per thread: its quad's 4 components) over the voxel
// slots: xor butterfly over the lane bits above the quad index, then the 4 waves in order
template <int CQB>
__device__ __forceinline__ void in_small_reduce(double (&a)[4], double (&b)[4], double* red /* [4][CQB*4][2] */) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = tid % CQB;
#pragma unroll
  for (int off = CQB; off < 64; off <<= 1)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] += __shfl_xor(a[j], off);
      b[j] += __shfl_xor(b[j], off);
    }
  if (lane < CQB)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      red[((wave * CQB + q) * 4 + j) * 2] = a[j];
      red[((wave * CQB + q) * 4 + j) * 2 + 1] = b[j];
    }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    double A = 0, B = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      A += red[((w * CQB + q) * 4 + j) * 2];
      B += red[((w * CQB + q) * 4 + j) * 2 + 1];
    }
    a[j] = A;
    b[j] = B;
  }
}

template <int CQB>
__global__ void __launch_bounds__(256) in_small_fwd_kernel(const float* __restrict__ x, InShape s, float* __restrict__ mean,
                                                           float* __restrict__ rstd, int act,
                                                           const float* __restrict__ resid, int rpad,
                                                           float* __restrict__ y, int ypad, uint2* __restrict__ y16,
                                                           int mode) {
  __shared__ double red[4 * CQB * 4 * 2];
  constexpr int VS = 256 / CQB;
  const int n = blockIdx.y, tid = threadIdx.x, q = tid % CQB, vt = tid / CQB;
  const int CQ = s.C / 4, qg = blockIdx.x * CQB + q;              // this thread's channel quad
  const int S = (int)s.S();
  const float4* xv = reinterpret_cast<const float4*>(x) + (size_t)n * S * CQ + qg;
  double sa[4] = {0, 0, 0, 0}, sb[4] = {0, 0, 0, 0};
#pragma unroll 4
  for (int v = vt; v < S; v += VS) {
    const float4 t = xv[(size_t)v * CQ];
    sa[0] += t.x; sa[1] += t.y; sa[2] += t.z; sa[3] += t.w;
    sb[0] += (double)t.x * t.x; sb[1] += (double)t.y * t.y; sb[2] += (double)t.z * t.z; sb[3] += (double)t.w * t.w;
  }
  in_small_reduce<CQB>(sa, sb, red);
  float mu[4], rs[4];
  const double Sd = (double)S;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const double m = sa[j] / Sd;
    double var = sb[j] / Sd - m * m;
    if (var < 0) var = 0;
    mu[j] = (float)m;
    rs[j] = (float)(1.0 / sqrt(var + (double)kInEps));
  }
  if (vt == 0) {
    reinterpret_cast<float4*>(mean + n * s.C)[qg] = make_float4(mu[0], mu[1], mu[2], mu[3]);
    reinterpret_cast<float4*>(rstd + n * s.C)[qg] = make_float4(rs[0], rs[1], rs[2], rs[3]);
  }
  const int Dp = s.D + 2 * ypad, Hp = s.H + 2 * ypad, Wp = s.W + 2 * ypad, P = Dp * Hp * Wp;
  const int Dr = s.D + 2 * rpad, Hr = s.H + 2 * rpad, Wr = s.W + 2 * rpad;
  const float4* rv = resid ? reinterpret_cast<const float4*>(resid) + (size_t)n * Dr * Hr * Wr * CQ + qg : nullptr;
  float4* yv = y ? reinterpret_cast<float4*>(y) + (size_t)n * P * CQ + qg : nullptr;
  uint2* y16v = y16 ? y16 + (size_t)n * P * CQ + qg : nullptr;
  // kInSmallU voxels' loads issued before their stores (the stores may alias the loads as far as
  // the compiler knows: a one-voxel loop waited a full load latency per voxel)
  const float4* rvp = rv ? rv : xv;
  for (int pv0 = vt; pv0 < P; pv0 += kInSmallU * VS) {
    float4 v[kInSmallU], r[kInSmallU];
#pragma unroll
    for (int u = 0; u < kInSmallU; ++u) {
      const int pv = min(pv0 + u * VS, P - 1);
      const int wp = pv % Wp, t = pv / Wp, hp = t % Hp, dp = t / Hp;
      const int sd = min(max(dp - ypad, 0), s.D - 1), sh = min(max(hp - ypad, 0), s.H - 1), sw = min(max(wp - ypad, 0), s.W - 1);
      v[u] = xv[(size_t)((sd * s.H + sh) * s.W + sw) * CQ];
      r[u] = rvp[(size_t)(rv ? ((sd + rpad) * Hr + sh + rpad) * Wr + sw + rpad : 0) * CQ];   // (no branch)
    }
#pragma unroll
    for (int u = 0; u < kInSmallU; ++u) {
      const int pv = pv0 + u * VS;
      if (pv >= P) break;
      float4 t = make_float4((v[u].x - mu[0]) * rs[0], (v[u].y - mu[1]) * rs[1], (v[u].z - mu[2]) * rs[2],
                             (v[u].w - mu[3]) * rs[3]);
      t = f4_act(t, act);
      if (rv) { t.x += r[u].x; t.y += r[u].y; t.z += r[u].z; t.w += r[u].w; }
      if (yv) yv[(size_t)pv * CQ] = t;
      if (y16v) y16v[(size_t)pv * CQ] = f4_op16(t, mode);
    }
  }
}

// the unpadded backward (P = 0: dY on the voxel grid) for kInSmallU voxels: every load first, in
// straight-line code (no branch between them: the add operand's pointer is a select, its value
// zeroed when absent), then the arithmetic — the compiler waited for each voxel's loads before the
// next voxel's act / add branches otherwise (vmcnt(0) per voxel)
template <int U>
__device__ __forceinline__ void in_small_voxels0(const InBwdArgs& a, const float4* dyp, const float4* xp,
                                                 const float4* addp, bool has_add, const size_t (&o)[U],
                                                 const float4& mu, const float4& rs, float4 (&g)[U],
                                                 float4 (&xh)[U], float4 (&graw)[U]) {
  float4 dv[U], xv[U], ev[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    dv[u] = dyp[o[u]];
    xv[u] = xp[o[u]];
    ev[u] = addp[o[u]];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float4 t = dv[u];
    if (has_add) f4_add(t, ev[u]);
    graw[u] = t;
    xh[u] = make_float4((xv[u].x - mu.x) * rs.x, (xv[u].y - mu.y) * rs.y, (xv[u].z - mu.z) * rs.z,
                        (xv[u].w - mu.w) * rs.w);
    t.x *= dact_from_xhat(xh[u].x, a.act); t.y *= dact_from_xhat(xh[u].y, a.act);
    t.z *= dact_from_xhat(xh[u].z, a.act); t.w *= dact_from_xhat(xh[u].w, a.act);
    g[u] = t;
  }
}

template <int CQB, int P>
__global__ void __launch_bounds__(256) in_small_bwd_kernel(InBwdArgs a, InShape s) {
  __shared__ double red[4 * CQB * 4 * 2];
  constexpr int VS = 256 / CQB;
  const int n = blockIdx.y, tid = threadIdx.x, q = tid % CQB, vt = tid / CQB;
  const int CQ = s.C / 4, qg = blockIdx.x * CQB + q;
  const int S = (int)s.S();
  double sa[4] = {0, 0, 0, 0}, sb[4] = {0, 0, 0, 0};
  const float4* dyp = reinterpret_cast<const float4*>(a.dy);
  const float4* xp = reinterpret_cast<const float4*>(a.x);
  const bool has_add = a.dy_add != nullptr;
  const float4* addp = has_add ? reinterpret_cast<const float4*>(a.dy_add) : dyp;
  const float4 mu = reinterpret_cast<const float4*>(a.mean + n * s.C)[qg];
  const float4 rsq = reinterpret_cast<const float4*>(a.rstd + n * s.C)[qg];
  // kInSmallU voxels' loads together, summed in voxel order (the one-voxel loop's order)
  auto voxels = [&](int v0, float4 (&g)[kInSmallU], float4 (&xh)[kInSmallU], float4 (&graw)[kInSmallU])
      __attribute__((always_inline)) {
    if constexpr (P == 0) {
      size_t o[kInSmallU];
#pragma unroll
      for (int u = 0; u < kInSmallU; ++u) o[u] = ((size_t)n * S + min(v0 + u * VS, S - 1)) * CQ + qg;
      in_small_voxels0<kInSmallU>(a, dyp, xp, addp, has_add, o, mu, rsq, g, xh, graw);
    } else {
#pragma unroll
      for (int u = 0; u < kInSmallU; ++u) {
        const int v = min(v0 + u * VS, S - 1);
        const int w = v % s.W, t = v / s.W, h = t % s.H, d = t / s.H;
        in_bwd_voxel<P>(a, s, in_bwd_row(a, s, n, d, h, qg), w, g[u], xh[u], &graw[u]);
      }
    }
  };
  for (int v0 = vt; v0 < S; v0 += kInSmallU * VS) {
    float4 g[kInSmallU], xh[kInSmallU], graw[kInSmallU];
    voxels(v0, g, xh, graw);
#pragma unroll
    for (int u = 0; u < kInSmallU; ++u) {
      if (v0 + u * VS >= S) break;
      sa[0] += g[u].x; sa[1] += g[u].y; sa[2] += g[u].z; sa[3] += g[u].w;
      sb[0] += (double)g[u].x * xh[u].x; sb[1] += (double)g[u].y * xh[u].y;
      sb[2] += (double)g[u].z * xh[u].z; sb[3] += (double)g[u].w * xh[u].w;
    }
  }
  in_small_reduce<CQB>(sa, sb, red);
  const double Sd = (double)S;
  float mg[4], mgx[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    mg[j] = (float)(sa[j] / Sd);
    mgx[j] = (float)(sb[j] / Sd);
  }
  float4* dx = reinterpret_cast<float4*>(a.dx);
  uint2* dx16 = reinterpret_cast<uint2*>(a.dx16);
  float4* gout = reinterpret_cast<float4*>(a.g_out);
  for (int v0 = vt; v0 < S; v0 += kInSmallU * VS) {
    float4 g[kInSmallU], xh[kInSmallU], graw[kInSmallU];
    voxels(v0, g, xh, graw);
#pragma unroll
    for (int u = 0; u < kInSmallU; ++u) {
      const int v = v0 + u * VS;
      if (v >= S) break;
      const size_t o = ((size_t)n * S + v) * CQ + qg;
      if (gout) gout[o] = graw[u];
      float4 r;
      r.x = rsq.x * (g[u].x - mg[0] - xh[u].x * mgx[0]);
      r.y = rsq.y * (g[u].y - mg[1] - xh[u].y * mgx[1]);
      r.z = rsq.z * (g[u].z - mg[2] - xh[u].z * mgx[2]);
      r.w = rsq.w * (g[u].w - mg[3] - xh[u].w * mgx[3]);
      if (dx) dx[o] = r;
      if (dx16) dx16[o] = f4_op16(r, a.mode16);
    }
  }
}

static int launch_in_small_fwd(int cqb, const float* x, const InShape& s, float* mean, float* rstd, int act,
                               const float* resid, int rpad, float* y, int ypad, void* y16, int mode16, hipStream_t st) {
  const dim3 g(s.C / 4 / cqb, s.N);
  uint2* o16 = static_cast<uint2*>(y16);
  switch (cqb) {
    case 8: hipLaunchKernelGGL(in_small_fwd_kernel<8>, g, dim3(256), 0, st, x, s, mean, rstd, act, resid, rpad, y, ypad, o16, mode16); break;
    case 4: hipLaunchKernelGGL(in_small_fwd_kernel<4>, g, dim3(256), 0, st, x, s, mean, rstd, act, resid, rpad, y, ypad, o16, mode16); break;
    case 2: hipLaunchKernelGGL(in_small_fwd_kernel<2>, g, dim3(256), 0, st, x, s, mean, rstd, act, resid, rpad, y, ypad, o16, mode16); break;
    default: hipLaunchKernelGGL(in_small_fwd_kernel<1>, g, dim3(256), 0, st, x, s, mean, rstd, act, resid, rpad, y, ypad, o16, mode16); break;
  }
  return check_launch(y16 ? "in_small_fwd(op16)" : "in_small_fwd");
}

template <int CQB>
static void launch_in_small_bwd_c(const InBwdArgs& a, const InShape& s, hipStream_t st) {
  const dim3 g(s.C / 4 / CQB, s.N);
  switch (a.dypad) {
    case 0: hipLaunchKernelGGL((in_small_bwd_kernel<CQB, 0>), g, dim3(256), 0, st, a, s); break;
    case 1: hipLaunchKernelGGL((in_small_bwd_kernel<CQB, 1>), g, dim3(256), 0, st, a, s); break;
    case 3: hipLaunchKernelGGL((in_small_bwd_kernel<CQB, 3>), g, dim3(256), 0, st, a, s); break;
    default: hipLaunchKernelGGL((in_small_bwd_kernel<CQB, -1>), g, dim3(256), 0, st, a, s); break;
  }
}

static int launch_in_small_bwd(int cqb, const InBwdArgs& a, const InShape& s, hipStream_t st) {
  switch (cqb) {
    case 8: launch_in_small_bwd_c<8>(a, s, st); break;
    case 4: launch_in_small_bwd_c<4>(a, s, st); break;
    case 2: launch_in_small_bwd_c<2>(a, s, st); break;
    default: launch_in_small_bwd_c<1>(a, s, st); break;
  }
  return check_launch(a.dx16 ? "in_small_bwd(op16)" : "in_small_bwd");
}

// ---- running statistics (composite of the reference's sequential calls) ------------------
// One entry per IN layer: the segments (one per reference call, in call order) of per-instance
// mean/rstd.  r ← (1−m)·r + m·avg_call(μ_n + bias), rv ← (1−m)·rv + m·avg_call(σ²_n · S/(S−1)).
struct RunningSeg { const float* mean; const float* rstd; int count; };
struct RunningEntry {
  float* rm; float* rv; const float* bias; int C; int nseg; long long S;
  RunningSeg seg[8];
};

__global__ void in_running_kernel(const RunningEntry* __restrict__ tab, float momentum) {
  const RunningEntry& e = tab[blockIdx.x];
  for (int c = threadIdx.x; c < e.C; c += blockDim.x) {
    double rm = e.rm[c], rv = e.rv[c];
    const double b = e.bias ? e.bias[c] : 0.0;
    const double corr = e.S > 1 ? (double)e.S / (double)(e.S - 1) : 1.0;
    for (int k = 0; k < e.nseg; ++k) {
      double am = 0, av = 0;
      for (int i = 0; i < e.seg[k].count; ++i) {
        const double mu = e.seg[k].mean[i * e.C + c];
        const double rs = e.seg[k].rstd[i * e.C + c];
        double var = 1.0 / (rs * rs) - (double)kInEps;
        if (var < 0) var = 0;
        am += mu + b;
        av += var * corr;
      }
      am /= e.seg[k].count; av /= e.seg[k].count;
      rm = (1.0 - momentum) * rm + momentum * am;
      rv = (1.0 - momentum) * rv + momentum * av;
    }
    e.rm[c] = (float)rm;
    e.rv[c] = (float)rv;
  }
}

// ---- host entry points -------------------------------------------------------------------
static int grid_for(int64_t work, int cap = 8192) {
  int64_t b = (work + 255) / 256;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

int instnorm_fwd(const float* x, InShape s, float* y, int ypad, int act, const float* resid, int rpad, float* mean,
                 float* rstd, void* ws, size_t ws_bytes, hipStream_t st, void* y16, int mode16) {
  MRAGAN_CHECK_ARG(s.C % 4 == 0 && s.C <= 1024, "instnorm: C=%d must be a multiple of 4 (≤1024)", s.C);
  MRAGAN_CHECK_ARG(in_fits(s, ypad > rpad ? ypad : rpad), "instnorm: tensor of %d×%d×%d×%d×%d too large", s.N, s.D, s.H, s.W, s.C);
  if (s.S() <= 1) {
    set_error("Expected more than 1 spatial element when training, got input size [%d, %d, %d, %d, %d]", s.N, s.C, s.D,
              s.H, s.W);
    return kBadArg;
  }
  const int chunks = in_chunks(s);
  if (instnorm_ws_bytes(s.N, s.D, s.H, s.W, s.C) > ws_bytes) { set_error("instnorm: workspace too small"); return kWorkspace; }
  if (const int cqb = in_small_cqb(s)) return launch_in_small_fwd(cqb, x, s, mean, rstd, act, resid, rpad, y, ypad, y16, mode16, st);
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(in_stats_kernel, dim3(chunks, s.N), dim3(256), 0, st, x, s, chunks, part);
  int rc = check_launch("in_stats");
  if (rc) return rc;
  return launch_in_apply(x, s, part, chunks, mean, rstd, act, resid, rpad, y, ypad, y16, mode16, st);
}

// Forward from statistics partials a producer conv already accumulated (conv_brick_x3 epilogue:
// [N][chunks][C][2] = Σy, Σy² per brick): the statistics pass is skipped.
int instnorm_fwd_partials(const float* x, InShape s, float* y, int ypad, int act, const float* resid, int rpad,
                          float* mean, float* rstd, const double* part, int chunks, hipStream_t st, void* y16,
                          int mode16) {
  MRAGAN_CHECK_ARG(s.C % 4 == 0 && s.C <= 1024, "instnorm: C=%d must be a multiple of 4 (≤1024)", s.C);
  MRAGAN_CHECK_ARG(in_fits(s, ypad > rpad ? ypad : rpad), "instnorm: tensor of %d×%d×%d×%d×%d too large", s.N, s.D, s.H, s.W, s.C);
  MRAGAN_CHECK_ARG(part && chunks > 0, "instnorm_fwd_partials: no partials");
  if (s.S() <= 1) {
    set_error("Expected more than 1 spatial element when training, got input size [%d, %d, %d, %d, %d]", s.N, s.C, s.D,
              s.H, s.W);
    return kBadArg;
  }
  return launch_in_apply(x, s, part, chunks, mean, rstd, act, resid, rpad, y, ypad, y16, mode16, st);
}

// ABI 15: the apply passes alone, the statistics already finalized by the producing conv
int instnorm_apply(const float* x, InShape s, float* y, int ypad, int act, const float* resid, int rpad,
                   const float* mean, const float* rstd, hipStream_t st, void* y16, int mode16) {
  MRAGAN_CHECK_ARG(s.C % 4 == 0 && s.C <= 1024, "instnorm: C=%d must be a multiple of 4 (≤1024)", s.C);
  MRAGAN_CHECK_ARG(in_fits(s, ypad > rpad ? ypad : rpad), "instnorm: tensor of %d×%d×%d×%d×%d too large", s.N, s.D, s.H, s.W, s.C);
  const int rows = s.N * (s.D + 2 * ypad) * (s.H + 2 * ypad);
  hipLaunchKernelGGL(in_apply_kernel, dim3(rows < 16384 ? rows : 16384), dim3(256), 0, st, x, s, mean, rstd, act, resid,
                     rpad, y, ypad, static_cast<uint2*>(y16), mode16);
  return check_launch(y16 ? "in_apply(op16)" : "in_apply");
}

int instnorm_bwd_apply(const InBwdArgs& a, InShape s, const float* coef, hipStream_t st) {
  MRAGAN_CHECK_ARG(s.C % 4 == 0 && s.C <= 1024, "instnorm_bwd: C=%d must be a multiple of 4", s.C);
  MRAGAN_CHECK_ARG(in_fits(s, a.dypad), "instnorm_bwd: tensor of %d×%d×%d×%d×%d too large", s.N, s.D, s.H, s.W, s.C);
  const int rows = s.N * s.D * s.H;
  const dim3 ga(rows < 16384 ? rows : 16384);
  switch (a.dypad) {
    case 0: hipLaunchKernelGGL(in_bwd_apply_kernel<0>, ga, dim3(256), 0, st, a, s, coef); break;
    case 1: hipLaunchKernelGGL(in_bwd_apply_kernel<1>, ga, dim3(256), 0, st, a, s, coef); break;
    case 3: hipLaunchKernelGGL(in_bwd_apply_kernel<3>, ga, dim3(256), 0, st, a, s, coef); break;
    default: hipLaunchKernelGGL(in_bwd_apply_kernel<-1>, ga, dim3(256), 0, st, a, s, coef); break;
  }
  return check_launch(a.dx16 ? "in_bwd_apply(op16)" : "in_bwd_apply");
}

int instnorm_bwd(const InBwdArgs& a, InShape s, void* ws, size_t ws_bytes, hipStream_t st) {
  MRAGAN_CHECK_ARG(s.C % 4 == 0 && s.C <= 1024, "instnorm_bwd: C=%d must be a multiple of 4", s.C);
  MRAGAN_CHECK_ARG(in_fits(s, a.dypad), "instnorm_bwd: tensor of %d×%d×%d×%d×%d too large", s.N, s.D, s.H, s.W, s.C);
  const int chunks = in_chunks(s);
  const size_t need = instnorm_ws_bytes(s.N, s.D, s.H, s.W, s.C) + (size_t)s.N * s.C * 2 * sizeof(float);
  if (need > ws_bytes) { set_error("instnorm_bwd: workspace too small"); return kWorkspace; }
  if (const int cqb = in_small_cqb(s)) return launch_in_small_bwd(cqb, a, s, st);
  double* part = static_cast<double*>(ws);
  float* coef = reinterpret_cast<float*>(static_cast<char*>(ws) + instnorm_ws_bytes(s.N, s.D, s.H, s.W, s.C));
  const int rows = s.N * s.D * s.H;
  const dim3 gs(chunks, s.N), ga(rows < 16384 ? rows : 16384);
  // the pads of the hot path get a compile-time fold (ResnetBlock 1, k7 layers 3, plain 0)
  switch (a.dypad) {
    case 0: hipLaunchKernelGGL(in_bwd_stats_kernel<0>, gs, dim3(256), 0, st, a, s, chunks, part); break;
    case 1: hipLaunchKernelGGL(in_bwd_stats_kernel<1>, gs, dim3(256), 0, st, a, s, chunks, part); break;
    case 3: hipLaunchKernelGGL(in_bwd_stats_kernel<3>, gs, dim3(256), 0, st, a, s, chunks, part); break;
    default: hipLaunchKernelGGL(in_bwd_stats_kernel<-1>, gs, dim3(256), 0, st, a, s, chunks, part); break;
  }
  int rc = check_launch("in_bwd_stats");
  if (rc) return rc;
  return launch_in_bwd_apply(a, s, part, chunks, coef, st);
}

// Backward from statistics partials the producer of dy already accumulated (conv_brick_x3's
// backward-statistics epilogue: [N][chunks][C][2] = Σg, Σg·x̂ per brick): finalize + apply only.
int instnorm_bwd_partials(const InBwdArgs& a, InShape s, const double* part, int chunks, void* ws, size_t ws_bytes,
                          hipStream_t st) {
  MRAGAN_CHECK_ARG(s.C % 4 == 0 && s.C <= 1024, "instnorm_bwd: C=%d must be a multiple of 4", s.C);
  MRAGAN_CHECK_ARG(in_fits(s, a.dypad), "instnorm_bwd: tensor of %d×%d×%d×%d×%d too large", s.N, s.D, s.H, s.W, s.C);
  MRAGAN_CHECK_ARG(part && chunks > 0, "instnorm_bwd_partials: no partials");
  const size_t need = (size_t)s.N * s.C * 2 * sizeof(float);
  if (need > ws_bytes) { set_error("instnorm_bwd_partials: workspace too small"); return kWorkspace; }
  float* coef = static_cast<float*>(ws);
  return launch_in_bwd_apply(a, s, part, chunks, coef, st);
}

int instnorm_running(const void* table, int nentries, float momentum, hipStream_t st) {
  if (nentries <= 0) return kOk;
  hipLaunchKernelGGL(in_running_kernel, dim3(nentries), dim3(256), 0, st, static_cast<const RunningEntry*>(table), momentum);
  return check_launch("in_running");
}

size_t instnorm_running_entry_bytes() { return sizeof(RunningEntry); }

}  // namespace mragan
