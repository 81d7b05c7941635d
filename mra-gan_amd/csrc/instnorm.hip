// InstanceNorm3d(affine=False, track_running_stats=True), train mode, on NDHWC fp32
// (reference networks3D.py:15-24: get_norm_layer('instance'); used after every conv of G and
// the three middle convs of D).  Fusions:
//   forward : y = act((x − μ)·rstd) + residual, written straight into a replication-padded
//             output (the ReplicationPad3d that precedes the next conv, networks3D.py:185/211/
//             233/249) — so neither the pad nor the activation costs a separate pass.
//   backward: g = fold(dy_padded) (+ dy_add) (ReplicationPad3d backward), × act'(x̂),
//             dx = rstd·(g − mean(g) − x̂·mean(g·x̂)).
// Statistics are accumulated in fp64 from fp32 data (per-thread → block → chunk partials),
// so the single-pass Σx / Σx² form keeps full fp32 accuracy.
#include "kernels.h"

namespace mragan {

constexpr float kInEps = 1e-5f;


// voxel chunks per instance: ≈2048 blocks per launch, but ≥ 4 voxel rows per thread
static int in_chunks(const InShape& s) {
  const int CQ = s.C / 4;
  const int R = CQ >= 256 ? 1 : 256 / CQ;
  int64_t want = (2048 + s.N - 1) / s.N;
  int64_t cap = s.S() / (4 * R);
  if (want > cap) want = cap;
  if (want < 1) want = 1;
  return (int)want;
}

size_t instnorm_ws_bytes(int N, int D, int H, int W, int C) {
  InShape s{N, D, H, W, C};
  return (size_t)N * in_chunks(s) * C * 2 * sizeof(double) + 16;
}

// Σ over chunks of partials[n][chunk][C][2] in fixed order (deterministic).  Block = 4
// channels × 64 chunk rows; grid (ceil(C/4), N): each thread sums ≤ chunks/64 partials with its
// loads in flight together (16 rows × 32 sequential partials took ~5 µs of dependent latency).
// mode 0: mean / rstd (out0, out1); mode 1: backward coefficients (out0 = coef[2C]).
__device__ void in_finalize_group(const double* __restrict__ part, const InShape& s, int chunks, int n, int cgroup,
                                  int mode, float* __restrict__ out0, float* __restrict__ out1) {
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

__device__ __forceinline__ float4 f4_act(float4 v, int act) {
  return make_float4(act_fwd(v.x, act), act_fwd(v.y, act), act_fwd(v.z, act), act_fwd(v.w, act));
}

__device__ __forceinline__ float dact_from_xhat(float xh, int act) {
  if (act == kActRelu) return xh > 0.f ? 1.f : 0.f;
  if (act == kActLrelu) return xh > 0.f ? 1.f : kLreluSlope;
  return 1.f;
}

// ---- forward statistics: partials[n][chunk][C][2] (Σx, Σx²) --------------------------------
__global__ void __launch_bounds__(256) in_stats_kernel(const float* __restrict__ x, InShape s, int chunks,
                                                       double* __restrict__ part) {
  __shared__ double red[2][256 * 4];
  const int n = blockIdx.y, chunk = blockIdx.x;
  const int CQ = s.C / 4, R = 256 / CQ;
  const int tid = threadIdx.x;
  const int q = tid % CQ, r = tid / CQ;
  const int64_t S = s.S();
  const int64_t per = (S + chunks - 1) / chunks;
  const int64_t v0 = chunk * per, v1 = min(S, v0 + per);
  double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
  if (r < R) {
    const float* base = x + (int64_t)n * S * s.C + 4 * q;
    for (int64_t v = v0 + r; v < v1; v += R) {
      float4 val = *reinterpret_cast<const float4*>(base + v * s.C);
      s0[0] += val.x; s0[1] += val.y; s0[2] += val.z; s0[3] += val.w;
      s1[0] += (double)val.x * val.x; s1[1] += (double)val.y * val.y;
      s1[2] += (double)val.z * val.z; s1[3] += (double)val.w * val.w;
    }
  }
  for (int j = 0; j < 4; ++j) { red[0][tid * 4 + j] = s0[j]; red[1][tid * 4 + j] = s1[j]; }
  __syncthreads();
  if (tid < CQ) {
    double a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
    for (int rr = 0; rr < R; ++rr)
      for (int j = 0; j < 4; ++j) { a[j] += red[0][(rr * CQ + tid) * 4 + j]; b[j] += red[1][(rr * CQ + tid) * 4 + j]; }
    double* out = part + (((int64_t)n * chunks + chunk) * s.C + 4 * tid) * 2;
    for (int j = 0; j < 4; ++j) { out[2 * j] = a[j]; out[2 * j + 1] = b[j]; }
  }
}

// one block per instance (kernel boundary = coherence point for the partials of all XCDs; an
// in-kernel last-block reduction needs agent-scope release fences, i.e. L2 write-backs, per block)
__global__ void __launch_bounds__(256) in_finalize_kernel(const double* __restrict__ part, InShape s, int chunks,
                                                          float* __restrict__ mean, float* __restrict__ rstd) {
  in_finalize_group(part, s, chunks, blockIdx.y, blockIdx.x, 0, mean, rstd);
}

// ---- forward apply: y (padded by ypad) = act((x − μ)·rstd) + resid(interior of rpad-padded) --
__global__ void __launch_bounds__(256) in_apply_kernel(const float* __restrict__ x, InShape s, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, int act,
                                                       const float* __restrict__ resid, int rpad, float* __restrict__ y,
                                                       int ypad) {
  const int CQ = s.C / 4;
  const int Dp = s.D + 2 * ypad, Hp = s.H + 2 * ypad, Wp = s.W + 2 * ypad;
  const int64_t total = (int64_t)s.N * Dp * Hp * Wp * CQ;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(e % CQ); int64_t u = e / CQ;
    const int w = (int)(u % Wp); u /= Wp;
    const int h = (int)(u % Hp); u /= Hp;
    const int d = (int)(u % Dp); const int n = (int)(u / Dp);
    const int sd = min(max(d - ypad, 0), s.D - 1), sh = min(max(h - ypad, 0), s.H - 1), sw = min(max(w - ypad, 0), s.W - 1);
    const int64_t src = (((int64_t)n * s.D + sd) * s.H + sh) * s.W + sw;
    float4 v = *reinterpret_cast<const float4*>(x + src * s.C + 4 * q);
    const float4 mu = *reinterpret_cast<const float4*>(mean + n * s.C + 4 * q);
    const float4 rs = *reinterpret_cast<const float4*>(rstd + n * s.C + 4 * q);
    v = make_float4((v.x - mu.x) * rs.x, (v.y - mu.y) * rs.y, (v.z - mu.z) * rs.z, (v.w - mu.w) * rs.w);
    v = f4_act(v, act);
    if (resid) {
      const int Dr = s.D + 2 * rpad, Hr = s.H + 2 * rpad, Wr = s.W + 2 * rpad;
      const float4 r = *reinterpret_cast<const float4*>(
          resid + ((((int64_t)n * Dr + sd + rpad) * Hr + sh + rpad) * Wr + sw + rpad) * s.C + 4 * q);
      v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
    }
    *reinterpret_cast<float4*>(y + u * 0 + e * 4) = v;   // e*4 == (((n*Dp+d)*Hp+h)*Wp+w)*C + 4q
  }
}

// ---- backward -----------------------------------------------------------------------------
__device__ __forceinline__ float4 fold_read(const float* __restrict__ dy, int pad, const InShape& s, int n, int d, int h,
                                            int w, int q) {
  if (pad == 0) return *reinterpret_cast<const float4*>(dy + ((((int64_t)n * s.D + d) * s.H + h) * s.W + w) * s.C + 4 * q);
  const int Dp = s.D + 2 * pad, Hp = s.H + 2 * pad, Wp = s.W + 2 * pad;
  const int d0 = d == 0 ? 0 : d + pad, d1 = d == s.D - 1 ? s.D - 1 + 2 * pad : d + pad;
  const int h0 = h == 0 ? 0 : h + pad, h1 = h == s.H - 1 ? s.H - 1 + 2 * pad : h + pad;
  const int w0 = w == 0 ? 0 : w + pad, w1 = w == s.W - 1 ? s.W - 1 + 2 * pad : w + pad;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int a = d0; a <= d1; ++a)
    for (int b = h0; b <= h1; ++b)
      for (int c = w0; c <= w1; ++c) {
        const float4 v = *reinterpret_cast<const float4*>(dy + ((((int64_t)n * Dp + a) * Hp + b) * Wp + c) * s.C + 4 * q);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
  return acc;
}


__device__ __forceinline__ void in_bwd_g(const InBwdArgs& a, const InShape& s, int n, int64_t v, int q, float4& g,
                                         float4& xh) {
  const int w = (int)(v % s.W); const int64_t u = v / s.W;
  const int h = (int)(u % s.H); const int d = (int)(u / s.H);
  g = fold_read(a.dy, a.dypad, s, n, d, h, w, q);
  const int64_t idx = ((int64_t)n * s.S() + v) * s.C + 4 * q;
  if (a.dy_add) {
    const float4 e = *reinterpret_cast<const float4*>(a.dy_add + idx);
    g.x += e.x; g.y += e.y; g.z += e.z; g.w += e.w;
  }
  const float4 xv = *reinterpret_cast<const float4*>(a.x + idx);
  const float4 mu = *reinterpret_cast<const float4*>(a.mean + n * s.C + 4 * q);
  const float4 rs = *reinterpret_cast<const float4*>(a.rstd + n * s.C + 4 * q);
  xh = make_float4((xv.x - mu.x) * rs.x, (xv.y - mu.y) * rs.y, (xv.z - mu.z) * rs.z, (xv.w - mu.w) * rs.w);
  g.x *= dact_from_xhat(xh.x, a.act); g.y *= dact_from_xhat(xh.y, a.act);
  g.z *= dact_from_xhat(xh.z, a.act); g.w *= dact_from_xhat(xh.w, a.act);
}

__global__ void __launch_bounds__(256) in_bwd_stats_kernel(InBwdArgs a, InShape s, int chunks, double* __restrict__ part) {
  __shared__ double red[2][256 * 4];
  const int n = blockIdx.y, chunk = blockIdx.x;
  const int CQ = s.C / 4, R = 256 / CQ;
  const int tid = threadIdx.x, q = tid % CQ, r = tid / CQ;
  const int64_t S = s.S(), per = (S + chunks - 1) / chunks;
  const int64_t v0 = chunk * per, v1 = min(S, v0 + per);
  double s0[4] = {0, 0, 0, 0}, s1[4] = {0, 0, 0, 0};
  if (r < R) {
    for (int64_t v = v0 + r; v < v1; v += R) {
      float4 g, xh;
      in_bwd_g(a, s, n, v, q, g, xh);
      s0[0] += g.x; s0[1] += g.y; s0[2] += g.z; s0[3] += g.w;
      s1[0] += (double)g.x * xh.x; s1[1] += (double)g.y * xh.y; s1[2] += (double)g.z * xh.z; s1[3] += (double)g.w * xh.w;
    }
  }
  for (int j = 0; j < 4; ++j) { red[0][tid * 4 + j] = s0[j]; red[1][tid * 4 + j] = s1[j]; }
  __syncthreads();
  if (tid < CQ) {
    double a0[4] = {0, 0, 0, 0}, b0[4] = {0, 0, 0, 0};
    for (int rr = 0; rr < R; ++rr)
      for (int j = 0; j < 4; ++j) { a0[j] += red[0][(rr * CQ + tid) * 4 + j]; b0[j] += red[1][(rr * CQ + tid) * 4 + j]; }
    double* out = part + (((int64_t)n * chunks + chunk) * s.C + 4 * tid) * 2;
    for (int j = 0; j < 4; ++j) { out[2 * j] = a0[j]; out[2 * j + 1] = b0[j]; }
  }
}

__global__ void __launch_bounds__(256) in_bwd_finalize_kernel(const double* __restrict__ part, InShape s, int chunks,
                                                              float* __restrict__ coef) {
  in_finalize_group(part, s, chunks, blockIdx.y, blockIdx.x, 1, coef, nullptr);
}

__global__ void __launch_bounds__(256) in_bwd_apply_kernel(InBwdArgs a, InShape s, const float* __restrict__ coef) {
  const int CQ = s.C / 4;
  const int64_t S = s.S();
  const int64_t total = (int64_t)s.N * S * CQ;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(e % CQ); const int64_t u = e / CQ;
    const int64_t v = u % S; const int n = (int)(u / S);
    float4 g, xh;
    in_bwd_g(a, s, n, v, q, g, xh);
    const float* cf = coef + 2 * ((int64_t)n * s.C + 4 * q);
    const float4 rs = *reinterpret_cast<const float4*>(a.rstd + n * s.C + 4 * q);
    float4 o;
    o.x = rs.x * (g.x - cf[0] - xh.x * cf[1]);
    o.y = rs.y * (g.y - cf[2] - xh.y * cf[3]);
    o.z = rs.z * (g.z - cf[4] - xh.z * cf[5]);
    o.w = rs.w * (g.w - cf[6] - xh.w * cf[7]);
    *reinterpret_cast<float4*>(a.dx + e * 4) = o;
  }
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
                 float* rstd, void* ws, size_t ws_bytes, hipStream_t st) {
  MRAGAN_CHECK_ARG(s.C % 4 == 0 && s.C <= 1024, "instnorm: C=%d must be a multiple of 4 (≤1024)", s.C);
  if (s.S() <= 1) {
    set_error("Expected more than 1 spatial element when training, got input size [%d, %d, %d, %d, %d]", s.N, s.C, s.D,
              s.H, s.W);
    return kBadArg;
  }
  const int chunks = in_chunks(s);
  if (instnorm_ws_bytes(s.N, s.D, s.H, s.W, s.C) > ws_bytes) { set_error("instnorm: workspace too small"); return kWorkspace; }
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(in_stats_kernel, dim3(chunks, s.N), dim3(256), 0, st, x, s, chunks, part);
  int rc = check_launch("in_stats");
  if (rc) return rc;
  hipLaunchKernelGGL(in_finalize_kernel, dim3(ceil_div(s.C, 4), s.N), dim3(256), 0, st, part, s, chunks, mean, rstd);
  if ((rc = check_launch("in_finalize"))) return rc;
  const int64_t total = (int64_t)s.N * (s.D + 2 * ypad) * (s.H + 2 * ypad) * (s.W + 2 * ypad) * (s.C / 4);
  hipLaunchKernelGGL(in_apply_kernel, dim3(grid_for(total)), dim3(256), 0, st, x, s, mean, rstd, act, resid, rpad, y, ypad);
  return check_launch("in_apply");
}

int instnorm_bwd(const InBwdArgs& a, InShape s, void* ws, size_t ws_bytes, hipStream_t st) {
  MRAGAN_CHECK_ARG(s.C % 4 == 0 && s.C <= 1024, "instnorm_bwd: C=%d must be a multiple of 4", s.C);
  const int chunks = in_chunks(s);
  const size_t need = instnorm_ws_bytes(s.N, s.D, s.H, s.W, s.C) + (size_t)s.N * s.C * 2 * sizeof(float);
  if (need > ws_bytes) { set_error("instnorm_bwd: workspace too small"); return kWorkspace; }
  double* part = static_cast<double*>(ws);
  float* coef = reinterpret_cast<float*>(static_cast<char*>(ws) + instnorm_ws_bytes(s.N, s.D, s.H, s.W, s.C));
  hipLaunchKernelGGL(in_bwd_stats_kernel, dim3(chunks, s.N), dim3(256), 0, st, a, s, chunks, part);
  int rc = check_launch("in_bwd_stats");
  if (rc) return rc;
  hipLaunchKernelGGL(in_bwd_finalize_kernel, dim3(ceil_div(s.C, 4), s.N), dim3(256), 0, st, part, s, chunks, coef);
  if ((rc = check_launch("in_bwd_finalize"))) return rc;
  const int64_t total = (int64_t)s.N * s.S() * (s.C / 4);
  hipLaunchKernelGGL(in_bwd_apply_kernel, dim3(grid_for(total)), dim3(256), 0, st, a, s, coef);
  return check_launch("in_bwd_apply");
}

int instnorm_running(const void* table, int nentries, float momentum, hipStream_t st) {
  if (nentries <= 0) return kOk;
  hipLaunchKernelGGL(in_running_kernel, dim3(nentries), dim3(256), 0, st, static_cast<const RunningEntry*>(table), momentum);
  return check_launch("in_running");
}

size_t instnorm_running_entry_bytes() { return sizeof(RunningEntry); }

}  // namespace mragan
