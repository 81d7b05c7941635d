// Thin-channel 3D convolutions (one side has the image channel count nc = 1..2):
//   * G stem   Conv3d(nc→ngf, k7) on the RPad3 input      (networks3D.py:185-189)  fwd: thin_k
//   * G head   Conv3d(ngf→nc, k7) + Tanh                   (networks3D.py:211-213)  fwd: thin_n
//   * D first  Conv3d(nc→ndf, k4 s2 p1) + LeakyReLU        (networks3D.py:389-390)  fwd: thin_k
//   * D last   Conv3d(8ndf→1, k4 s1 p1) (+ Sigmoid)        (networks3D.py:417-420)  fwd: thin_dot
// and their data / weight gradients.  In the bf16 / fp16 modes every operand is rounded to that
// type as it is loaded (op_round), like the MFMA kernels' fragments.  On fp32 the VALU FMA rate equals the f32 MFMA rate
// (157 TF both), and these GEMMs have N or K of 1-2, so they are written as VALU direct
// convolutions with the input halo staged in LDS and the per-tap weights read as
// wave-uniform (scalar) loads.
#include "kernels.h"

namespace mragan {


// ---------------------------------------------------------------------------------------
// thin_k: contraction channels cx ≤ 4, many output channels.  One thread = one output voxel ×
// 32 output channels (grid.y walks channel groups).  Forward (any stride) or transposed s = 1.
// ---------------------------------------------------------------------------------------
constexpr int TK_OD = 4, TK_OH = 8, TK_OW = 8;   // 256 voxels per block
constexpr int TK_NB = 32;

// NB: output channels per block (32, or 8 / 4 when ny is that small: the [T][NB][CX] weight
// slice of a k7 layer then still fits LDS — 343·32·4·4 B alone would not, at cx = 4)
template <int CX, int NB>
__global__ void __launch_bounds__(256) thin_k_kernel(ThinArgs a, int tiles_d, int tiles_h, int tiles_w, int RD, int RH,
                                                     int RW) {
  constexpr int TK_NB = NB;
  extern __shared__ __attribute__((aligned(16))) float xs[];   // [RD][RH][RW][CX]
  const int tid = threadIdx.x;
  int tile = blockIdx.x;
  const int tw_ = tile % tiles_w; tile /= tiles_w;
  const int th_ = tile % tiles_h; tile /= tiles_h;
  const int td_ = tile % tiles_d; const int nb = tile / tiles_d;
  const int o0d = td_ * TK_OD, o0h = th_ * TK_OH, o0w = tw_ * TK_OW;
  const int n0 = blockIdx.y * TK_NB;
  // region origin in input coordinates
  int r0d, r0h, r0w;
  if (!a.trans) { r0d = o0d * a.s - a.p; r0h = o0h * a.s - a.p; r0w = o0w * a.s - a.p; }
  else { r0d = o0d + a.p - (a.k - 1); r0h = o0h + a.p - (a.k - 1); r0w = o0w + a.p - (a.k - 1); }
  const int R = RD * RH * RW;
  for (int e = tid; e < R; e += 256) {
    int rw = e % RW, rh = (e / RW) % RH, rd = e / (RW * RH);
    int id = r0d + rd, ih = r0h + rh, iw = r0w + rw;
    bool ok = (unsigned)id < (unsigned)a.Di && (unsigned)ih < (unsigned)a.Hi && (unsigned)iw < (unsigned)a.Wi;
    const float* src = a.x + ((((int64_t)nb * a.Di + id) * a.Hi + ih) * a.Wi + iw) * CX;
#pragma unroll
    for (int c = 0; c < CX; ++c) xs[e * CX + c] = ok ? op_round(src[c], a.rnd) : 0.f;
  }
  // the block's weight slice for every tap, [t][32][CX], zero beyond ny (broadcast reads)
  const int T = a.k * a.k * a.k;
  float* wsl = xs + ((R * CX + 3) & ~3);
  for (int e = tid; e < T * TK_NB * CX; e += 256) {
    const int c = e % CX, j = (e / CX) % TK_NB, t = e / (CX * TK_NB);
    wsl[e] = (n0 + j < a.ny) ? op_round(a.w[((int64_t)t * a.ny + n0 + j) * CX + c], a.rnd) : 0.f;
  }
  __syncthreads();
  const int ow = tid % TK_OW, oh = (tid / TK_OW) % TK_OH, od = tid / (TK_OW * TK_OH);
  const int gd = o0d + od, gh = o0h + oh, gw = o0w + ow;
  float acc[TK_NB];
#pragma unroll
  for (int j = 0; j < TK_NB; ++j) acc[j] = 0.f;
  // local origin of this voxel's window inside the region
  const int ld = a.trans ? od : od * a.s, lh = a.trans ? oh : oh * a.s, lw = a.trans ? ow : ow * a.s;
  const int k = a.k;
  const int nvalid = min(TK_NB, a.ny - n0);
  for (int jd = 0; jd < k; ++jd)
    for (int jh = 0; jh < k; ++jh)
      for (int jw = 0; jw < k; ++jw) {
        // forward: tap t = j at offset j; transposed (s=1): offset j ↔ tap k-1-j
        int t = a.trans ? (((k - 1 - jd) * k + (k - 1 - jh)) * k + (k - 1 - jw)) : ((jd * k + jh) * k + jw);
        const float* xv = xs + (((ld + jd) * RH + (lh + jh)) * RW + (lw + jw)) * CX;
        const float* wt = wsl + t * TK_NB * CX;
        float xr[CX];
#pragma unroll
        for (int c = 0; c < CX; ++c) xr[c] = xv[c];
#pragma unroll
        for (int j = 0; j < TK_NB; ++j)
#pragma unroll
          for (int c = 0; c < CX; ++c) acc[j] = fmaf(xr[c], wt[j * CX + c], acc[j]);
      }
  if (gd < a.Do && gh < a.Ho && gw < a.Wo) {
    float* dst = a.y + ((((int64_t)nb * a.Do + gd) * a.Ho + gh) * a.Wo + gw) * a.ny + n0;
#pragma unroll
    for (int j = 0; j < TK_NB; ++j)
      if (j < nvalid) dst[j] = act_fwd(acc[j] + (a.bias ? a.bias[n0 + j] : 0.f), a.act);
  }
}

// ---------------------------------------------------------------------------------------
// thin_n: few output channels (ny ≤ 4), contraction channels a multiple of 8; stride 1
// (G head Conv3d(ngf→nc, k7) forward, G stem data gradient).
// Block = one output plane d × 16 rows h × 64 columns w; thread = 4 consecutive w outputs of
// one row.  The kernel sweeps td (plane offset) and 8-channel chunks: each stage fills LDS
// with the (16+K−1) × (64+K−1) × 8-channel input slab of plane d+td (float4 loads, two per
// position), then every thread slides a (4+K−1)-wide register window along its row for each
// th, K taps each: 4·K·8·NY FMAs per 2(4+K−1) ds_read_b128.  Weights of a (t, chunk) are
// wave-uniform (scalar loads).
// ---------------------------------------------------------------------------------------
constexpr int TN_TH = 16, TN_OW = 64, TN_VW = 4, TN_CC = 8;

// LDS image of one slab row: position p's two float4 at p*2 + p/4 (+half); one 16-B pad after
// every 4 positions makes the 16 lanes of a ds_read_b128 group (positions 4·vw + i) land on
// slots 9·vw mod 16 — all distinct — and the row stride is a multiple of 256 B so lanes of
// neighbouring rows inside a group stay distinct too.
__host__ __device__ constexpr int tn_row_stride(int rw) { return ((rw * 2 + rw / 4 + 1) + 15) / 16 * 16; }
__device__ __forceinline__ int tn_slot(int p) { return p * 2 + (p >> 2); }

template <int NY, int K>
__global__ void __launch_bounds__(256) thin_n_kernel(ThinArgs a, int tiles_h, int tiles_w) {
  extern __shared__ __attribute__((aligned(16))) float4 slab[];   // [RH][RS] float4
  constexpr int RH = TN_TH + K - 1, RW = TN_OW + K - 1;
  constexpr int RS = tn_row_stride(RW);
  constexpr int WL = TN_VW + K - 1;
  const int tid = threadIdx.x;
  int tile = blockIdx.x;
  const int tw_ = tile % tiles_w; tile /= tiles_w;
  const int th_ = tile % tiles_h; tile /= tiles_h;
  const int od = tile % a.Do; const int nb = tile / a.Do;
  const int o0h = th_ * TN_TH, o0w = tw_ * TN_OW;
  // input coordinate of local offset j along a dim: fwd o - p + j (tap j); trans o + p - (K-1) + j (tap K-1-j)
  const int sh = a.trans ? a.p - (K - 1) : -a.p;
  const int r0h = o0h + sh, r0w = o0w + sh;
  const int vw = tid % (TN_OW / TN_VW), hr = tid / (TN_OW / TN_VW);
  const int ow0 = vw * TN_VW;
  float acc[NY][TN_VW];
#pragma unroll
  for (int n = 0; n < NY; ++n)
#pragma unroll
    for (int v = 0; v < TN_VW; ++v) acc[n][v] = 0.f;
  constexpr int R = RH * RW * 2;   // float4 pieces per stage
  // this stage's weights [jh][jw][n][8] (broadcast reads), after the input slab
  float4* wsl = slab + RH * RS;
  for (int jd = 0; jd < K; ++jd) {
    const int id = od + sh + jd;
    if ((unsigned)id >= (unsigned)a.Di) continue;           // whole plane is zero padding
    const int td = a.trans ? K - 1 - jd : jd;
    for (int c0 = 0; c0 < a.cx; c0 += TN_CC) {
      __syncthreads();
      for (int e = tid; e < K * K * NY * 2; e += 256) {
        const int half = e & 1, n = (e >> 1) % NY, jj = (e >> 1) / NY;
        const int jw = jj % K, jh = jj / K;
        const int th = a.trans ? K - 1 - jh : jh, tw = a.trans ? K - 1 - jw : jw;
        wsl[e] = op_round4(*reinterpret_cast<const float4*>(a.w + ((int64_t)((td * K + th) * K + tw) * NY + n) * a.cx +
                                                            c0 + 4 * half),
                           a.rnd);
      }
      for (int e = tid; e < R; e += 256) {
        const int half = e & 1, pos = e >> 1;
        const int rw = pos % RW, rh = pos / RW;
        const int ih = r0h + rh, iw = r0w + rw;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if ((unsigned)ih < (unsigned)a.Hi && (unsigned)iw < (unsigned)a.Wi)
          v = *reinterpret_cast<const float4*>(a.x + ((((int64_t)nb * a.Di + id) * a.Hi + ih) * a.Wi + iw) * a.cx + c0 +
                                               4 * half);
        slab[rh * RS + tn_slot(rw) + half] = op_round4(v, a.rnd);
      }
      __syncthreads();
      for (int jh = 0; jh < K; ++jh) {
        const float4* row = slab + (hr + jh) * RS;
        float4 lo[WL], hi[WL];
#pragma unroll
        for (int i = 0; i < WL; ++i) {
          const int sl = tn_slot(ow0 + i);
          lo[i] = row[sl];
          hi[i] = row[sl + 1];
        }
#pragma unroll
        for (int jw = 0; jw < K; ++jw) {
#pragma unroll
          for (int n = 0; n < NY; ++n) {
            const float4 wa = wsl[((jh * K + jw) * NY + n) * 2], wb = wsl[((jh * K + jw) * NY + n) * 2 + 1];
            const float w0 = wa.x, w1 = wa.y, w2 = wa.z, w3 = wa.w, w4 = wb.x, w5 = wb.y, w6 = wb.z, w7 = wb.w;
#pragma unroll
            for (int v = 0; v < TN_VW; ++v) {
              const float4 a0 = lo[v + jw], a1 = hi[v + jw];
              float s = acc[n][v];
              s = fmaf(a0.x, w0, s); s = fmaf(a0.y, w1, s); s = fmaf(a0.z, w2, s); s = fmaf(a0.w, w3, s);
              s = fmaf(a1.x, w4, s); s = fmaf(a1.y, w5, s); s = fmaf(a1.z, w6, s); s = fmaf(a1.w, w7, s);
              acc[n][v] = s;
            }
          }
        }
      }
    }
  }
  const int gh = o0h + hr;
  if (gh < a.Ho) {
#pragma unroll
    for (int v = 0; v < TN_VW; ++v) {
      const int gw = o0w + ow0 + v;
      if (gw >= a.Wo) continue;
      float* dst = a.y + ((((int64_t)nb * a.Do + od) * a.Ho + gh) * a.Wo + gw) * NY;
#pragma unroll
      for (int n = 0; n < NY; ++n) dst[n] = act_fwd(acc[n][v] + (a.bias ? a.bias[n] : 0.f), a.act);
    }
  }
}

// ---------------------------------------------------------------------------------------
// thin_n_class: few output channels, transposed form with stride s > 1 (D-first data
// gradient, k4 s2 p1): one parity class per blockIdx.y, so the (≤ ceil(k/s)³) taps of a block
// are uniform; one thread per output voxel reads each tap's channel row with float4 loads.
// ---------------------------------------------------------------------------------------
template <int NY>
__global__ void __launch_bounds__(256) thin_n_class_kernel(ThinArgs a) {
  const int s = a.s, k = a.k;
  const int cls = blockIdx.y;
  const int cw = cls % s, ch = (cls / s) % s, cd = cls / (s * s);
  const int Qd = (a.Do - cd + s - 1) / s, Qh = (a.Ho - ch + s - 1) / s, Qw = (a.Wo - cw + s - 1) / s;
  const int64_t M = (int64_t)a.N * Qd * Qh * Qw;
  const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (m >= M) return;
  int qw = (int)(m % Qw); int64_t u = m / Qw;
  int qh = (int)(u % Qh); u /= Qh;
  int qd = (int)(u % Qd); int nb = (int)(u / Qd);
  const int od = qd * s + cd, oh = qh * s + ch, ow = qw * s + cw;
  const int t0d = (cd + a.p) % s, t0h = (ch + a.p) % s, t0w = (cw + a.p) % s;
  float acc[NY];
#pragma unroll
  for (int n = 0; n < NY; ++n) acc[n] = 0.f;
  for (int td = t0d; td < k; td += s) {
    const int id = (od + a.p - td) / s;
    if ((unsigned)id >= (unsigned)a.Di) continue;
    for (int th = t0h; th < k; th += s) {
      const int ih = (oh + a.p - th) / s;
      if ((unsigned)ih >= (unsigned)a.Hi) continue;
      for (int tw = t0w; tw < k; tw += s) {
        const int iw = (ow + a.p - tw) / s;
        if ((unsigned)iw >= (unsigned)a.Wi) continue;
        const float* xr = a.x + ((((int64_t)nb * a.Di + id) * a.Hi + ih) * a.Wi + iw) * a.cx;
        const float* wt = a.w + (int64_t)((td * k + th) * k + tw) * NY * a.cx;
        for (int c = 0; c < a.cx; c += 4) {
          const float4 xv = op_round4(*reinterpret_cast<const float4*>(xr + c), a.rnd);
#pragma unroll
          for (int n = 0; n < NY; ++n) {
            const float4 wn = op_round4(*reinterpret_cast<const float4*>(wt + n * a.cx + c), a.rnd);
            acc[n] = fmaf(xv.x, wn.x, fmaf(xv.y, wn.y, fmaf(xv.z, wn.z, fmaf(xv.w, wn.w, acc[n]))));
          }
        }
      }
    }
  }
  float* dst = a.y + ((((int64_t)nb * a.Do + od) * a.Ho + oh) * a.Wo + ow) * NY;
#pragma unroll
  for (int n = 0; n < NY; ++n) dst[n] = act_fwd(acc[n] + (a.bias ? a.bias[n] : 0.f), a.act);
}

// ---------------------------------------------------------------------------------------
// thin_n_class8: the same parity-class form for ceil(k/s) = 2 (k3/k4, s2: the D-first data
// gradient) with 8 lanes per output voxel.  Lane j of a group reads channel quads j, j+8 of each
// tap's input row, so 8 lanes read one voxel's 32-channel row as 128 contiguous bytes (the
// one-thread-per-voxel form above made every load instruction touch 64 different lines: ~3 TF/s);
// the class's ≤ 8 tap weights for those quads live in registers for the whole grid-stride walk;
// the 8 partial dots are summed with three xor-shuffles in a fixed order.  Products accumulate
// in fp64 (rounded once): the step's G gradients pass this through ~10 InstanceNorm backwards
// whose mean-subtraction cancels, so the fp32 rounding order of this sum is visible in them.
// ---------------------------------------------------------------------------------------
template <int NY, int QPL>
__global__ void __launch_bounds__(256) thin_n_class8_kernel(ThinArgs a) {
  const int s = a.s, k = a.k;
  const int cls = blockIdx.y;
  const int cw = cls % s, ch = (cls / s) % s, cd = cls / (s * s);
  const int Qd = (a.Do - cd + s - 1) / s, Qh = (a.Ho - ch + s - 1) / s, Qw = (a.Wo - cw + s - 1) / s;
  const int M = a.N * Qd * Qh * Qw;                   // < 2^31 (host check)
  const int t0d = (cd + a.p) % s, t0h = (ch + a.p) % s, t0w = (cw + a.p) % s;
  const int j = threadIdx.x & 7;
  const int CQ = a.cx / 4;
  float4 wr[8][QPL][NY];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int td = t0d + s * (t >> 2), th = t0h + s * ((t >> 1) & 1), tw = t0w + s * (t & 1);
    const bool tok = td < k && th < k && tw < k;
    const float* wt = a.w + (int64_t)((min(td, k - 1) * k + min(th, k - 1)) * k + min(tw, k - 1)) * NY * a.cx;
#pragma unroll
    for (int u = 0; u < QPL; ++u) {
      const int q = j + 8 * u;
#pragma unroll
      for (int n = 0; n < NY; ++n)
        wr[t][u][n] = (tok && q < CQ) ? op_round4(*reinterpret_cast<const float4*>(wt + n * a.cx + 4 * q), a.rnd)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  const int HWi = a.Hi * a.Wi;
  for (int m = blockIdx.x * 32 + (threadIdx.x >> 3); m < M; m += gridDim.x * 32) {
    const int qw = m % Qw;
    int u_ = m / Qw;
    const int qh = u_ % Qh; u_ /= Qh;
    const int qd = u_ % Qd;
    const int nb = u_ / Qd;
    const int od = qd * s + cd, oh = qh * s + ch, ow = qw * s + cw;
    double acc[NY];
#pragma unroll
    for (int n = 0; n < NY; ++n) acc[n] = 0.0;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int td = t0d + s * (t >> 2), th = t0h + s * ((t >> 1) & 1), tw = t0w + s * (t & 1);
      const int id = (od + a.p - td) / s, ih = (oh + a.p - th) / s, iw = (ow + a.p - tw) / s;
      if (td >= k || th >= k || tw >= k || (unsigned)id >= (unsigned)a.Di || (unsigned)ih >= (unsigned)a.Hi ||
          (unsigned)iw >= (unsigned)a.Wi)
        continue;
      const float* xr = a.x + ((int64_t)nb * a.Di * HWi + (id * a.Hi + ih) * a.Wi + iw) * a.cx;
#pragma unroll
      for (int u = 0; u < QPL; ++u) {
        const int q = j + 8 * u;
        if (q < CQ) {
          const float4 xv = op_round4(*reinterpret_cast<const float4*>(xr + 4 * q), a.rnd);
#pragma unroll
          for (int n = 0; n < NY; ++n) {
            const float4 wv = wr[t][u][n];
            acc[n] = fma((double)xv.x, (double)wv.x, fma((double)xv.y, (double)wv.y,
                         fma((double)xv.z, (double)wv.z, fma((double)xv.w, (double)wv.w, acc[n]))));
          }
        }
      }
    }
#pragma unroll
    for (int n = 0; n < NY; ++n) {
      acc[n] += __shfl_xor(acc[n], 4, 8);
      acc[n] += __shfl_xor(acc[n], 2, 8);
      acc[n] += __shfl_xor(acc[n], 1, 8);
    }
    if (j == 0) {
      float* dst = a.y + ((((int64_t)nb * a.Do + od) * a.Ho + oh) * a.Wo + ow) * NY;
#pragma unroll
      for (int n = 0; n < NY; ++n) dst[n] = act_fwd((float)acc[n] + (a.bias ? a.bias[n] : 0.f), a.act);
    }
  }
}

// ---------------------------------------------------------------------------------------
// thin_n_tile8: thin_n_class8 for stride 2 with the input halo of an 8×8×8 output tile staged in
// LDS once (7³ rows: every input row serves up to 64 outputs of the tile, which thin_n_class8 each
// re-read through L1/L2 — 537 MB of L2 reads for the 64³ b2 D-first data gradient, 75 µs).  Lane
// groups of 8 (lane j = channel quad j) walk the tile's outputs of one parity class each; taps,
// skip conditions, fp64 product order and the xor-shuffle sum are thin_n_class8's, so results are
// bit-identical to it.
// ---------------------------------------------------------------------------------------
constexpr int kT8 = 8, kT8Halo = kT8 / 2 + 3;

__device__ __forceinline__ int floor_div2(int v) { return v >= 0 ? v / 2 : -((1 - v) / 2); }

// QPL = 2: 64 contraction channels (the UNet outermost upconv in the MFMA modes), lane j holds
// channel quads j and j + 8 — the halo takes 88 KB of LDS (one block per CU)
template <int NY, int QPL>
__global__ void __launch_bounds__(256) thin_n_tile8_kernel(ThinArgs a, int tiles_d, int tiles_h, int tiles_w) {
  constexpr int s = 2, HE = kT8Halo;
  extern __shared__ float4 hx[];                      // [HE³][CQ], zero outside the input volume
  const int k = a.k, CQ = a.cx / 4;
  int b = blockIdx.x;
  const int tw_ = b % tiles_w; b /= tiles_w;
  const int th_ = b % tiles_h; b /= tiles_h;
  const int td_ = b % tiles_d;
  const int nb = b / tiles_d;
  const int o0d = td_ * kT8, o0h = th_ * kT8, o0w = tw_ * kT8;
  // lowest input index any output of the tile reads: floor((o0 + p − (k − 1)) / 2)
  const int ild = floor_div2(o0d + a.p - (k - 1)), ilh = floor_div2(o0h + a.p - (k - 1)),
            ilw = floor_div2(o0w + a.p - (k - 1));
  const float* xn = a.x + (int64_t)nb * a.Di * a.Hi * a.Wi * a.cx;
  for (int e = threadIdx.x; e < HE * HE * HE * CQ; e += 256) {
    const int q = e % CQ, r = e / CQ;
    const int id = ild + r / (HE * HE), ih = ilh + (r / HE) % HE, iw = ilw + r % HE;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if ((unsigned)id < (unsigned)a.Di && (unsigned)ih < (unsigned)a.Hi && (unsigned)iw < (unsigned)a.Wi)
      v = op_round4(*reinterpret_cast<const float4*>(xn + ((int64_t)(id * a.Hi + ih) * a.Wi + iw) * a.cx + 4 * q), a.rnd);
    hx[e] = v;
  }
  const int j = threadIdx.x & 7, grp = threadIdx.x >> 3;
  const int cls = grp & 7, gi = grp >> 3;             // 4 lane groups per parity class
  const int cw = cls % s, ch = (cls / s) % s, cd = cls / (s * s);
  const int t0d = (cd + a.p) % s, t0h = (ch + a.p) % s, t0w = (cw + a.p) % s;
  float4 wr[8][QPL][NY];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int td = t0d + s * (t >> 2), th = t0h + s * ((t >> 1) & 1), tw = t0w + s * (t & 1);
    const bool tok = td < k && th < k && tw < k;
    const float* wt = a.w + (int64_t)((min(td, k - 1) * k + min(th, k - 1)) * k + min(tw, k - 1)) * NY * a.cx;
#pragma unroll
    for (int u = 0; u < QPL; ++u)
#pragma unroll
      for (int n = 0; n < NY; ++n)
        wr[t][u][n] = (tok && j + 8 * u < CQ)
                          ? op_round4(*reinterpret_cast<const float4*>(wt + n * a.cx + 4 * (j + 8 * u)), a.rnd)
                          : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __syncthreads();
  constexpr int QT = kT8 / s;                         // class outputs per tile dim
  for (int idx = gi; idx < QT * QT * QT; idx += 4) {
    const int od = o0d + s * (idx / (QT * QT)) + cd, oh = o0h + s * ((idx / QT) % QT) + ch,
              ow = o0w + s * (idx % QT) + cw;
    if (od >= a.Do || oh >= a.Ho || ow >= a.Wo) continue;        // uniform per lane group
    double acc[NY];
#pragma unroll
    for (int n = 0; n < NY; ++n) acc[n] = 0.0;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int td = t0d + s * (t >> 2), th = t0h + s * ((t >> 1) & 1), tw = t0w + s * (t & 1);
      const int id = (od + a.p - td) / s, ih = (oh + a.p - th) / s, iw = (ow + a.p - tw) / s;
      if (td >= k || th >= k || tw >= k || (unsigned)id >= (unsigned)a.Di || (unsigned)ih >= (unsigned)a.Hi ||
          (unsigned)iw >= (unsigned)a.Wi)
        continue;
#pragma unroll
      for (int u = 0; u < QPL; ++u) {
        if (j + 8 * u < CQ) {
          const float4 xv = hx[(((id - ild) * HE + (ih - ilh)) * HE + (iw - ilw)) * CQ + j + 8 * u];
#pragma unroll
          for (int n = 0; n < NY; ++n) {
            const float4 wv = wr[t][u][n];
            acc[n] = fma((double)xv.x, (double)wv.x, fma((double)xv.y, (double)wv.y,
                         fma((double)xv.z, (double)wv.z, fma((double)xv.w, (double)wv.w, acc[n]))));
          }
        }
      }
    }
#pragma unroll
    for (int n = 0; n < NY; ++n) {
      acc[n] += __shfl_xor(acc[n], 4, 8);
      acc[n] += __shfl_xor(acc[n], 2, 8);
      acc[n] += __shfl_xor(acc[n], 1, 8);
    }
    if (j == 0) {
      float* dst = a.y + ((((int64_t)nb * a.Do + od) * a.Ho + oh) * a.Wo + ow) * NY;
#pragma unroll
      for (int n = 0; n < NY; ++n) dst[n] = act_fwd((float)acc[n] + (a.bias ? a.bias[n] : 0.f), a.act);
    }
  }
}

// ---------------------------------------------------------------------------------------
// naive: one wave per output voxel (lanes split taps × channels), any stride / transposed
// form.  Used for the tiny D-last convolution and the D-first data gradient.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) thin_naive_kernel(ThinArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t o = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t total = (int64_t)a.N * a.Do * a.Ho * a.Wo;
  if (o >= total) return;
  int ow = (int)(o % a.Wo); int64_t u = o / a.Wo;
  int oh = (int)(u % a.Ho); u /= a.Ho;
  int od = (int)(u % a.Do); int nb = (int)(u / a.Do);
  const int k = a.k, T = k * k * k;
  for (int n = 0; n < a.ny; ++n) {
    float s = 0.f;
    for (int e = lane; e < T * a.cx; e += 64) {
      int c = e % a.cx, t = e / a.cx;
      int tw = t % k, th = (t / k) % k, td = t / (k * k);
      int id, ih, iw;
      if (!a.trans) { id = od * a.s - a.p + td; ih = oh * a.s - a.p + th; iw = ow * a.s - a.p + tw; }
      else {
        int nd = od + a.p - td, nh = oh + a.p - th, nw = ow + a.p - tw;
        if (nd < 0 || nh < 0 || nw < 0 || nd % a.s || nh % a.s || nw % a.s) continue;
        id = nd / a.s; ih = nh / a.s; iw = nw / a.s;
      }
      if ((unsigned)id >= (unsigned)a.Di || (unsigned)ih >= (unsigned)a.Hi || (unsigned)iw >= (unsigned)a.Wi) continue;
      s = fmaf(op_round(a.x[((((int64_t)nb * a.Di + id) * a.Hi + ih) * a.Wi + iw) * a.cx + c], a.rnd),
               op_round(a.w[((int64_t)t * a.ny + n) * a.cx + c], a.rnd), s);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0) a.y[o * a.ny + n] = act_fwd(s + (a.bias ? a.bias[n] : 0.f), a.act);
  }
}

// ---------------------------------------------------------------------------------------
// thin_dot: ny ≤ 4 outputs from a wide contraction on a SMALL output grid (the D-last layer
// at 64³: 8ndf = 512 channels × 64 taps into 6³ voxels per patch).  One block per output
// voxel: the 256 threads sweep the block's (tap, channel-quad) elements with float4 loads of
// the input row and the weight row (both contiguous in cx), then a fixed-order block
// reduction (deterministic).  Forward form, any stride.  Replaces one-wave-per-voxel
// scalar loads (thin_naive, ≈10× slower on this shape).
// ---------------------------------------------------------------------------------------
template <int NY>
__global__ void __launch_bounds__(256) thin_dot_kernel(ThinArgs a) {
  __shared__ float red[NY][4];
  const int tid = threadIdx.x;
  int64_t o = blockIdx.x;
  const int ow = (int)(o % a.Wo); o /= a.Wo;
  const int oh = (int)(o % a.Ho); o /= a.Ho;
  const int od = (int)(o % a.Do); const int nb = (int)(o / a.Do);
  const int k = a.k, T = k * k * k, c4n = a.cx >> 2;
  float acc[NY];
#pragma unroll
  for (int n = 0; n < NY; ++n) acc[n] = 0.f;
  for (int e = tid; e < T * c4n; e += 256) {
    const int t = e / c4n, c = (e - t * c4n) * 4;
    const int tw = t % k, th = (t / k) % k, td = t / (k * k);
    const int id = od * a.s - a.p + td, ih = oh * a.s - a.p + th, iw = ow * a.s - a.p + tw;
    if ((unsigned)id >= (unsigned)a.Di || (unsigned)ih >= (unsigned)a.Hi || (unsigned)iw >= (unsigned)a.Wi) continue;
    const float4 xv = op_round4(
        *reinterpret_cast<const float4*>(a.x + ((((int64_t)nb * a.Di + id) * a.Hi + ih) * a.Wi + iw) * a.cx + c), a.rnd);
#pragma unroll
    for (int n = 0; n < NY; ++n) {
      const float4 wv = op_round4(*reinterpret_cast<const float4*>(a.w + ((int64_t)t * NY + n) * a.cx + c), a.rnd);
      acc[n] = fmaf(xv.x, wv.x, fmaf(xv.y, wv.y, fmaf(xv.z, wv.z, fmaf(xv.w, wv.w, acc[n]))));
    }
  }
#pragma unroll
  for (int n = 0; n < NY; ++n) {
    float s = acc[n];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((tid & 63) == 0) red[n][tid >> 6] = s;
  }
  __syncthreads();
  if (tid < NY) {
    const float s = ((red[tid][0] + red[tid][1]) + red[tid][2]) + red[tid][3];
    a.y[(int64_t)blockIdx.x * NY + tid] = act_fwd(s + (a.bias ? a.bias[tid] : 0.f), a.act);
  }
}

template <int NY>
static void launch_thin_n(const ThinArgs& a, dim3 grid, size_t lds, hipStream_t st, int th, int tw) {
  switch (a.k) {
    case 3: hipLaunchKernelGGL((thin_n_kernel<NY, 3>), grid, dim3(256), lds, st, a, th, tw); break;
    case 4: hipLaunchKernelGGL((thin_n_kernel<NY, 4>), grid, dim3(256), lds, st, a, th, tw); break;
    default: hipLaunchKernelGGL((thin_n_kernel<NY, 7>), grid, dim3(256), lds, st, a, th, tw); break;
  }
}

int conv_thin(ThinArgs a, hipStream_t st) {
  MRAGAN_CHECK_ARG(a.k >= 1 && a.k <= 7, "conv_thin: k=%d unsupported", a.k);
  if (a.N == 0 || a.ny == 0) return kOk;
  const bool s1 = a.s == 1;
  // the one-plane modes: k4 s2 p1 convs from 1-2 channels (the PatchGAN first layer, the UNet
  // outermost downconv and upconv data gradient) on MFMA (conv_down4.hip, round 5)
  if (down4_mfma_applicable(a)) return conv_down4_mfma(a, st);
  if (a.cx <= 4 && (!a.trans || s1)) {
    int td = ceil_div(a.Do, TK_OD), th = ceil_div(a.Ho, TK_OH), tw = ceil_div(a.Wo, TK_OW);
    int RD, RH, RW;
    if (!a.trans) { RD = (TK_OD - 1) * a.s + a.k; RH = (TK_OH - 1) * a.s + a.k; RW = (TK_OW - 1) * a.s + a.k; }
    else { RD = TK_OD + a.k - 1; RH = TK_OH + a.k - 1; RW = TK_OW + a.k - 1; }
    const int nb = a.ny <= 4 ? 4 : a.ny <= 8 ? 8 : TK_NB;
    size_t lds = ((((size_t)RD * RH * RW * a.cx + 3) & ~(size_t)3) + (size_t)a.k * a.k * a.k * nb * a.cx) *
                 sizeof(float);
    MRAGAN_CHECK_ARG(lds <= 160 * 1024, "thin_k: LDS %zu too large", lds);
    dim3 grid(a.N * td * th * tw, ceil_div(a.ny, nb));
#define MRAGAN_THIN_K(NBV)                                                                                      \
  switch (a.cx) {                                                                                              \
    case 1: hipLaunchKernelGGL((thin_k_kernel<1, NBV>), grid, dim3(256), lds, st, a, td, th, tw, RD, RH, RW); break; \
    case 2: hipLaunchKernelGGL((thin_k_kernel<2, NBV>), grid, dim3(256), lds, st, a, td, th, tw, RD, RH, RW); break; \
    case 3: hipLaunchKernelGGL((thin_k_kernel<3, NBV>), grid, dim3(256), lds, st, a, td, th, tw, RD, RH, RW); break; \
    default: hipLaunchKernelGGL((thin_k_kernel<4, NBV>), grid, dim3(256), lds, st, a, td, th, tw, RD, RH, RW); break; \
  }
    if (nb == 4) { MRAGAN_THIN_K(4) }
    else if (nb == 8) { MRAGAN_THIN_K(8) }
    else { MRAGAN_THIN_K(TK_NB) }
#undef MRAGAN_THIN_K
    return check_launch("thin_k");
  }
  const int64_t total = (int64_t)a.N * a.Do * a.Ho * a.Wo;
  // the row-sweep kernel is the k7 head's (ngf ≤ 64 contraction channels); a wide contraction
  // (the PatchGAN last layer, 8·ndf channels) goes to thin_dot at any output count — at 128³ the
  // D-last forward (256 → 1, 5,488 outputs) took 535 µs on thin_n
  if (a.ny <= 4 && s1 && a.cx % TN_CC == 0 && a.cx <= 64 && (a.k == 3 || a.k == 4 || a.k == 7) && total >= 4096) {
    int th = ceil_div(a.Ho, TN_TH), tw = ceil_div(a.Wo, TN_OW);
    size_t lds = ((size_t)(TN_TH + a.k - 1) * tn_row_stride(TN_OW + a.k - 1) + (size_t)a.k * a.k * a.ny * 2) *
                 sizeof(float4);
    dim3 grid(a.N * a.Do * th * tw);
    switch (a.ny) {
      case 1: launch_thin_n<1>(a, grid, lds, st, th, tw); break;
      case 2: launch_thin_n<2>(a, grid, lds, st, th, tw); break;
      case 3: launch_thin_n<3>(a, grid, lds, st, th, tw); break;
      default: launch_thin_n<4>(a, grid, lds, st, th, tw); break;
    }
    return check_launch("thin_n");
  }
  // ≤ 32 contraction channels (one quad per lane, 8 taps × NY float4 of weights in registers):
  // the D-first data gradient (ndf ≤ 32).  The UNet outermost upconv (2·ngf = 64 channels: two
  // quads per lane) joins it in the 16-bit MFMA modes (262 µs per 2×32³ → 64³ launch on
  // thin_n_class, r04final); in exact f32 it stays on thin_n_class — a forward layer, and the f32
  // step-parity envelopes of the 64³ UNet fixture were measured with its summation order (§2).
  // the one-plane modes: k4 s2 p1 transposed convs to ≤ 2 channels (the UNet outermost upconv, the
  // D-first data gradient) run input-centric on MFMA (conv_up4.hip, round 5)
  if (up4_mfma_applicable(a)) return conv_up4_mfma(a, st);
  const bool wide8 = a.cx > 32 && a.cx <= 64 && a.rnd != 0 && a.ny <= 2;   // ≤ 2 outputs: no spill
  if (a.ny <= 4 && a.trans && a.s > 1 && a.cx % 4 == 0 && (a.cx <= 32 || wide8) && ceil_div(a.k, a.s) == 2 &&
      (int64_t)a.N * a.Do * a.Ho * a.Wo < ((int64_t)1 << 31) &&
      (int64_t)a.N * a.Di * a.Hi * a.Wi * a.cx < ((int64_t)1 << 31)) {
    static const bool no_tile8 = getenv("MRAGAN_NO_TILE8") != nullptr;   // A/B switch
    if (a.s == 2 && !no_tile8) {
      const int tiles_d = ceil_div(a.Do, kT8), tiles_h = ceil_div(a.Ho, kT8), tiles_w = ceil_div(a.Wo, kT8);
      const int64_t blocks = (int64_t)a.N * tiles_d * tiles_h * tiles_w;
      const size_t lds = (size_t)kT8Halo * kT8Halo * kT8Halo * (a.cx / 4) * sizeof(float4);
      if (blocks < ((int64_t)1 << 31)) {
        static bool attr[2][4] = {};   // one flag per kernel: every instantiation has the same pointer type
        const int ai = a.ny < 4 ? a.ny - 1 : 3;
        auto go = [&](void (*kern)(ThinArgs, int, int, int)) {
          if (!attr[wide8][ai]) {
            (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)(kT8Halo * kT8Halo * kT8Halo * 16 * sizeof(float4)));
            attr[wide8][ai] = true;
          }
          hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), lds, st, a, tiles_d, tiles_h, tiles_w);
        };
        if (wide8) {
          if (a.ny == 1) go(thin_n_tile8_kernel<1, 2>);
          else go(thin_n_tile8_kernel<2, 2>);
        } else {
          switch (a.ny) {
            case 1: go(thin_n_tile8_kernel<1, 1>); break;
            case 2: go(thin_n_tile8_kernel<2, 1>); break;
            case 3: go(thin_n_tile8_kernel<3, 1>); break;
            default: go(thin_n_tile8_kernel<4, 1>); break;
          }
        }
        return check_launch("thin_n_tile8");
      }
    }
    const int64_t maxq = (int64_t)a.N * ceil_div(a.Do, a.s) * ceil_div(a.Ho, a.s) * ceil_div(a.Wo, a.s);
    int64_t gx = ceil_div(maxq, 32 * 4);             // ≈ 4 voxels per lane group: the weights load once per 4
    if (gx > 4096) gx = 4096;
    dim3 grid((unsigned)gx, a.s * a.s * a.s);
    if (wide8) {
      if (a.ny == 1) hipLaunchKernelGGL((thin_n_class8_kernel<1, 2>), grid, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((thin_n_class8_kernel<2, 2>), grid, dim3(256), 0, st, a);
      return check_launch("thin_n_class8");
    }
    switch (a.ny) {
      case 1: hipLaunchKernelGGL((thin_n_class8_kernel<1, 1>), grid, dim3(256), 0, st, a); break;
      case 2: hipLaunchKernelGGL((thin_n_class8_kernel<2, 1>), grid, dim3(256), 0, st, a); break;
      case 3: hipLaunchKernelGGL((thin_n_class8_kernel<3, 1>), grid, dim3(256), 0, st, a); break;
      default: hipLaunchKernelGGL((thin_n_class8_kernel<4, 1>), grid, dim3(256), 0, st, a); break;
    }
    return check_launch("thin_n_class8");
  }
  if (a.ny <= 4 && a.trans && a.s > 1 && a.cx % 4 == 0) {
    const int64_t maxq = (int64_t)a.N * ceil_div(a.Do, a.s) * ceil_div(a.Ho, a.s) * ceil_div(a.Wo, a.s);
    dim3 grid(ceil_div(maxq, 256), a.s * a.s * a.s);
    switch (a.ny) {
      case 1: hipLaunchKernelGGL(thin_n_class_kernel<1>, grid, dim3(256), 0, st, a); break;
      case 2: hipLaunchKernelGGL(thin_n_class_kernel<2>, grid, dim3(256), 0, st, a); break;
      case 3: hipLaunchKernelGGL(thin_n_class_kernel<3>, grid, dim3(256), 0, st, a); break;
      default: hipLaunchKernelGGL(thin_n_class_kernel<4>, grid, dim3(256), 0, st, a); break;
    }
    return check_launch("thin_n_class");
  }
  if (a.ny <= 4 && !a.trans && a.cx % 4 == 0 && a.cx >= 32) {
    dim3 grid((unsigned)total);
    switch (a.ny) {
      case 1: hipLaunchKernelGGL(thin_dot_kernel<1>, grid, dim3(256), 0, st, a); break;
      case 2: hipLaunchKernelGGL(thin_dot_kernel<2>, grid, dim3(256), 0, st, a); break;
      case 3: hipLaunchKernelGGL(thin_dot_kernel<3>, grid, dim3(256), 0, st, a); break;
      default: hipLaunchKernelGGL(thin_dot_kernel<4>, grid, dim3(256), 0, st, a); break;
    }
    return check_launch("thin_dot");
  }
  hipLaunchKernelGGL(thin_naive_kernel, dim3(ceil_div(total, 4)), dim3(256), 0, st, a);
  return check_launch("thin_naive");
}

// ---------------------------------------------------------------------------------------
// Thin weight gradient:  dW[dn][gn][t] = Σ_m D[m][dn] · G[m*s − p + t][gn]  (one side ≤ 4 ch)
// Used for the G stem / head, D first / last layers (dn or gn = image channels).
// Block = one channel group of the narrow side (grid.y) × a grid-stride walk over 4×4×16
// tiles of D's grid; D's tile and G's halo are staged in LDS.  A "role" = (4 channels of the
// wide side, or one channel of D when the vector runs over G, td, th) owns all K taps along w.
// Per tile row a role loads the G row window into registers once and sweeps the 16 voxels:
// one LDS read of D per voxel feeding 4K FMAs.  One role per thread (block = roles rounded up
// to 64, ≤ 512 threads); with fewer roles than 256 threads the tile rows are split over RS
// threads and combined through LDS.  Per-block partials go to a slab that a second kernel sums
// in fixed order (deterministic).
// ---------------------------------------------------------------------------------------
constexpr int TW_D = 4, TW_H = 4, TW_W = 16, TW_M = TW_D * TW_H * TW_W;

template <int K, int S, bool VDN, bool BIG = false>
__global__ void __launch_bounds__(BIG ? 1024 : 512) thin_wgrad_kernel(ThinWgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int RD = (TW_D - 1) * S + K, RH = (TW_H - 1) * S + K, RW = (TW_W - 1) * S + K;
  constexpr int WLEN = (TW_W - 1) * S + K;      // G row window of one tile row
  constexpr int Rn = RD * RH * RW;
  constexpr int GCH = VDN ? 1 : 4;              // G channels staged
  const int goff = VDN ? blockIdx.y : 4 * blockIdx.y;
  float* Dt = sm;                               // [TW_M][Cd]
  float* Gt = sm + TW_M * a.Cd;                 // [Rn][GCH]
  float* red = Gt + Rn * GCH;
  const int T = K * K * K;
  const int nroles = a.nroles, RS = a.RS;
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int role = tid % nroles, split = tid / nroles;
  const bool active = split < RS;
  const int th = role % K, td = (role / K) % K, ch = role / (K * K);
  float acc[4][K];
#pragma unroll
  for (int v = 0; v < 4; ++v)
#pragma unroll
    for (int t = 0; t < K; ++t) acc[v][t] = 0.f;

  for (int tile = blockIdx.x; tile < a.ntiles; tile += gridDim.x) {
    int tt = tile;
    const int tw_ = tt % a.tiles_w; tt /= a.tiles_w;
    const int th_ = tt % a.tiles_h; tt /= a.tiles_h;
    const int td_ = tt % a.tiles_d; const int nb = tt / a.tiles_d;
    const int m0d = td_ * TW_D, m0h = th_ * TW_H, m0w = tw_ * TW_W;
    __syncthreads();
    for (int e = tid; e < TW_M * a.Cd; e += nthr) {
      const int c = e % a.Cd, mi = e / a.Cd;
      const int mw = mi % TW_W, mh = (mi / TW_W) % TW_H, md = mi / (TW_W * TW_H);
      const int gd = m0d + md, gh = m0h + mh, gw = m0w + mw;
      const bool ok = gd < a.Dd && gh < a.Hd && gw < a.Wd;
      Dt[e] = ok ? op_round(a.D[((((int64_t)nb * a.Dd + gd) * a.Hd + gh) * a.Wd + gw) * a.Cd + c], a.rnd) : 0.f;
    }
    const int r0d = m0d * S - a.p, r0h = m0h * S - a.p, r0w = m0w * S - a.p;
    for (int e = tid; e < Rn * GCH; e += nthr) {
      const int c = e % GCH, ri = e / GCH;
      const int rw = ri % RW, rh = (ri / RW) % RH, rd = ri / (RW * RH);
      const int id = r0d + rd, ih = r0h + rh, iw = r0w + rw;
      const bool ok = (unsigned)id < (unsigned)a.Dg && (unsigned)ih < (unsigned)a.Hg && (unsigned)iw < (unsigned)a.Wg;
      Gt[e] = ok ? op_round(a.G[((((int64_t)nb * a.Dg + id) * a.Hg + ih) * a.Wg + iw) * a.Cg + goff + c], a.rnd) : 0.f;
    }
    __syncthreads();
    if (!active) continue;
    for (int row = split; row < TW_D * TW_H; row += RS) {
      const int mh = row % TW_H, md = row / TW_H;
      const int mi0 = (md * TW_H + mh) * TW_W;
      const float* grow = Gt + (((md * S + td) * RH + (mh * S + th)) * RW) * GCH;
      if constexpr (VDN) {
        float gw[WLEN];
#pragma unroll
        for (int i = 0; i < WLEN; ++i) gw[i] = grow[i];
#pragma unroll
        for (int mw = 0; mw < TW_W; ++mw) {
          const float4 dv = *reinterpret_cast<const float4*>(Dt + (mi0 + mw) * a.Cd + 4 * ch);
#pragma unroll
          for (int t = 0; t < K; ++t) {
            const float g = gw[mw * S + t];
            acc[0][t] = fmaf(dv.x, g, acc[0][t]);
            acc[1][t] = fmaf(dv.y, g, acc[1][t]);
            acc[2][t] = fmaf(dv.z, g, acc[2][t]);
            acc[3][t] = fmaf(dv.w, g, acc[3][t]);
          }
        }
      } else if constexpr (S == 1) {
        float4 gw[WLEN];
#pragma unroll
        for (int i = 0; i < WLEN; ++i) gw[i] = *reinterpret_cast<const float4*>(grow + 4 * i);
#pragma unroll
        for (int mw = 0; mw < TW_W; ++mw) {
          const float d = Dt[(mi0 + mw) * a.Cd + ch];
#pragma unroll
          for (int t = 0; t < K; ++t) {
            const float4 g = gw[mw + t];
            acc[0][t] = fmaf(d, g.x, acc[0][t]);
            acc[1][t] = fmaf(d, g.y, acc[1][t]);
            acc[2][t] = fmaf(d, g.z, acc[2][t]);
            acc[3][t] = fmaf(d, g.w, acc[3][t]);
          }
        }
      } else {
        for (int mw = 0; mw < TW_W; ++mw) {
          const float d = Dt[(mi0 + mw) * a.Cd + ch];
#pragma unroll
          for (int t = 0; t < K; ++t) {
            const float4 g = *reinterpret_cast<const float4*>(grow + 4 * (mw * S + t));
            acc[0][t] = fmaf(d, g.x, acc[0][t]);
            acc[1][t] = fmaf(d, g.y, acc[1][t]);
            acc[2][t] = fmaf(d, g.z, acc[2][t]);
            acc[3][t] = fmaf(d, g.w, acc[3][t]);
          }
        }
      }
    }
  }
  float* out = a.slab + (int64_t)blockIdx.x * a.Cd * a.Cg * T;
  auto out_index = [&](int rl, int v, int t) -> int64_t {
    const int th_ = rl % K, td_ = (rl / K) % K, ch_ = rl / (K * K);
    int dn, gn;
    if (VDN) { dn = 4 * ch_ + v; gn = goff; } else { dn = ch_; gn = goff + v; }
    return ((int64_t)dn * a.Cg + gn) * T + (td_ * K + th_) * K + t;
  };
  if (RS > 1) {
    __syncthreads();
    if (active) {
#pragma unroll
      for (int v = 0; v < 4; ++v)
#pragma unroll
        for (int t = 0; t < K; ++t) red[((split * nroles + role) * 4 + v) * K + t] = acc[v][t];
    }
    __syncthreads();
    for (int e = tid; e < nroles * 4 * K; e += nthr) {
      const int t = e % K, v = (e / K) % 4, rl = e / (4 * K);
      float sum = 0.f;
      for (int z = 0; z < RS; ++z) sum += red[((z * nroles + rl) * 4 + v) * K + t];
      out[out_index(rl, v, t)] = sum;
    }
  } else if (active) {
#pragma unroll
    for (int v = 0; v < 4; ++v)
#pragma unroll
      for (int t = 0; t < K; ++t) out[out_index(role, v, t)] = acc[v][t];
  }
}

// Block = 32 outputs (lanes: 128 contiguous bytes per slab) × 8 slab groups; group g sums the
// slabs z ≡ g (mod 8) in increasing z, the 8 partials are added in g order (fixed order,
// deterministic).  One thread per output over every slab ran 62 µs on 8 blocks (E = 2048).
__global__ void __launch_bounds__(256) slab_reduce_kernel(const float* __restrict__ slab, float* __restrict__ out,
                                                          int64_t E, int nslab, int accumulate) {
  __shared__ float part[8][32];
  const int l = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int64_t e = (int64_t)blockIdx.x * 32 + l;
  float s = 0.f;
  if (e < E) {
#pragma unroll 8
    for (int z = g; z < nslab; z += 8) s += slab[(int64_t)z * E + e];
  }
  part[g][l] = s;
  __syncthreads();
  if (g == 0 && e < E) {
    float r = part[0][l];
#pragma unroll
    for (int k = 1; k < 8; ++k) r += part[k][l];
    out[e] = accumulate ? out[e] + r : r;
  }
}

struct ThinWgradPlan { int gx, gy, threads; size_t lds; };

static int thin_wgrad_setup(ThinWgradArgs& a, ThinWgradPlan* pl) {
  a.vec_dn = (a.Cd % 4 == 0 && a.Cd >= a.Cg) ? 1 : 0;
  MRAGAN_CHECK_ARG(a.vec_dn || (a.Cg % 4 == 0 && a.Cd <= 64), "thin_wgrad: unsupported channels (%d,%d)", a.Cd, a.Cg);
  MRAGAN_CHECK_ARG(a.k == 3 || a.k == 4 || a.k == 7, "thin_wgrad: k=%d unsupported", a.k);
  MRAGAN_CHECK_ARG(a.s == 1 || (a.s == 2 && a.k != 7), "thin_wgrad: stride %d with k=%d unsupported", a.s, a.k);
  const int K = a.k;
  a.nroles = a.vec_dn ? (a.Cd / 4) * K * K : a.Cd * K * K;
  MRAGAN_CHECK_ARG(a.nroles <= 512, "thin_wgrad: %d roles > 512", a.nroles);
  // ≤ 256 roles: 512 threads (round 6 — the UNet's outermost k4 s2 weight gradients, 32 / 64 × 1
  // channels: one tile per block, so the tile rows split over RS ≥ 2 threads halve each thread's
  // serial FMA chain; A/B switch MRAGAN_THIN_WGRAD_T=256 restores 256 threads, =1024 tries 1024 on
  // the k4 layers)
  static const int nthr = [] {
    const char* e = getenv("MRAGAN_THIN_WGRAD_T");
    const int v = e ? atoi(e) : 512;
    return v == 256 || v == 1024 ? v : 512;
  }();
  if (a.nroles <= 256) {
    a.RS = (nthr > 512 && K != 4 ? 512 : nthr) / a.nroles;      // (1024 threads: the k4 instances only)
    if (a.RS > TW_D * TW_H) a.RS = TW_D * TW_H;
    pl->threads = (a.nroles * a.RS + 63) / 64 * 64;
    if (pl->threads < 256) pl->threads = 256;
  } else {
    pl->threads = (a.nroles + 63) / 64 * 64;
    a.RS = 1;
  }
  a.tiles_d = ceil_div(a.Dd, TW_D); a.tiles_h = ceil_div(a.Hd, TW_H); a.tiles_w = ceil_div(a.Wd, TW_W);
  a.ntiles = a.N * a.tiles_d * a.tiles_h * a.tiles_w;
  pl->gy = a.vec_dn ? a.Cg : a.Cg / 4;
  int want = 1024 / pl->gy;
  if (want < 16) want = 16;
  pl->gx = a.ntiles < want ? a.ntiles : want;
  if (pl->gx < 1) pl->gx = 1;
  const int s = a.s;
  const int RD = (TW_D - 1) * s + K, RH = (TW_H - 1) * s + K, RW = (TW_W - 1) * s + K;
  const int gch = a.vec_dn ? 1 : 4;
  pl->lds = ((size_t)TW_M * a.Cd + (size_t)RD * RH * RW * gch + (a.RS > 1 ? (size_t)a.RS * a.nroles * 4 * K : 0)) *
            sizeof(float);
  MRAGAN_CHECK_ARG(pl->lds <= 160 * 1024, "thin_wgrad: LDS %zu too large", pl->lds);
  return kOk;
}

size_t conv_thin_wgrad_ws_bytes(int N, int Dd, int Hd, int Wd, int Cd, int Cg, int k, int s) {
  ThinWgradArgs a{};
  a.N = N; a.Dd = Dd; a.Hd = Hd; a.Wd = Wd; a.Cd = Cd; a.Cg = Cg; a.k = k; a.s = s;
  ThinWgradPlan pl;
  if (thin_wgrad_setup(a, &pl)) return 0;
  return (size_t)pl.gx * Cd * Cg * k * k * k * sizeof(float);
}

template <int K, int S>
static void launch_thin_wgrad(const ThinWgradArgs& a, const ThinWgradPlan& pl, hipStream_t st) {
  dim3 grid(pl.gx, pl.gy);
  if constexpr (K == 4) {
    if (pl.threads > 512) {            // the 1024-thread A/B form (MRAGAN_THIN_WGRAD_T=1024)
      if (a.vec_dn) hipLaunchKernelGGL((thin_wgrad_kernel<K, S, true, true>), grid, dim3(pl.threads), pl.lds, st, a);
      else hipLaunchKernelGGL((thin_wgrad_kernel<K, S, false, true>), grid, dim3(pl.threads), pl.lds, st, a);
      return;
    }
  }
  if (a.vec_dn) hipLaunchKernelGGL((thin_wgrad_kernel<K, S, true>), grid, dim3(pl.threads), pl.lds, st, a);
  else hipLaunchKernelGGL((thin_wgrad_kernel<K, S, false>), grid, dim3(pl.threads), pl.lds, st, a);
}

int conv_thin_wgrad(ThinWgradArgs a, float* out, int accumulate, float* ws, size_t ws_bytes, hipStream_t st) {
  ThinWgradPlan pl;
  int rc = thin_wgrad_setup(a, &pl);
  if (rc) return rc;
  const int K = a.k;
  const int64_t E = (int64_t)a.Cd * a.Cg * K * K * K;
  size_t need = (size_t)pl.gx * E * sizeof(float);
  if (need > ws_bytes) { set_error("thin_wgrad: workspace %zu < %zu", ws_bytes, need); return kWorkspace; }
  if (a.ntiles == 0) return kOk;
  a.slab = ws;
  switch (K * 10 + a.s) {
    case 31: launch_thin_wgrad<3, 1>(a, pl, st); break;
    case 32: launch_thin_wgrad<3, 2>(a, pl, st); break;
    case 41: launch_thin_wgrad<4, 1>(a, pl, st); break;
    case 42: launch_thin_wgrad<4, 2>(a, pl, st); break;
    default: launch_thin_wgrad<7, 1>(a, pl, st); break;
  }
  rc = check_launch("thin_wgrad");
  if (rc) return rc;
  hipLaunchKernelGGL(slab_reduce_kernel, dim3((unsigned)((E + 31) / 32)), dim3(256), 0, st, ws, out, E, pl.gx,
                     accumulate);
  return check_launch("thin_wgrad_reduce");
}

}  // namespace mragan
