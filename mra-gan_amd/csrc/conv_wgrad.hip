// Weight gradient of a 3D convolution on gfx950 fp32 MFMA.
//
//   dW[dn][gn][t] = Σ_m  D[m][dn] · G[m*s - p + t][gn]          (zero fill outside G)
//
// Conv3d wgrad  : D = dY (output grid), G = X   → dW[Cout][Cin][k³]   (torch Conv3d layout)
// ConvT3d wgrad : D = X  (input grid),  G = dY  → dW[Cin][Cout][k³]   (torch ConvTranspose3d layout)
// (reference: the conv weights of networks3D.py:186-212, 241-257, 389-414 and
//  autograd's convolution_backward weight branch.)
//
// GEMM per tap: rows = dn, cols = gn, contraction = voxels m.  Split-K over m across
// blockIdx.z; every split writes its tile to a slab ws[z][t][dn][gn] (coalesced) and a second
// kernel sums the splits in a fixed order into the torch-layout gradient (deterministic; no
// float atomics).  LDS tiles are [m][ch] rows straight from NDHWC memory; the MFMA fragments
// are read with ds_read_b32 (lane = channel → consecutive banks, conflict-free).
#include "kernels.h"
#include "prec.h"

namespace mragan {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// Logical (tile, tap, split) of this block.  Workgroups are dispatched round-robin over the 8
// XCDs in flattened-id order; remapping id L → (L mod 8)·(B/8) + L/8 gives each XCD a contiguous
// range of splits with all their taps, so its L2 holds 1/8 of the voxel range instead of
// every XCD streaming all of it (the taps re-read the same dy/x rows).
__device__ __forceinline__ void wgrad_block(int& bx, int& by, int& bz) {
  const int gx = gridDim.x, gy = gridDim.y;
  const int B = gx * gy * gridDim.z;
  int L = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  if ((B & 7) == 0) L = (L & 7) * (B >> 3) + (L >> 3);
  bx = L % gx;
  by = (L / gx) % gy;
  bz = L / (gx * gy);
}


template <int WM, int WN, int TM, int TN>
__global__ void __launch_bounds__(256)
conv_wgrad_f32_kernel(WgradArgs a) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int BKm = 32;
  constexpr int LPR_D = BM / 4, LPR_G = BN / 4;
  constexpr int RPP_D = 256 / LPR_D, RPP_G = 256 / LPR_G;
  constexpr int D_LOADS = (BKm * LPR_D + 255) / 256;
  constexpr int G_LOADS = (BKm * LPR_G + 255) / 256;
  __shared__ __attribute__((aligned(16))) float smem[2 * BKm * (BM + BN)];
  float* Ds = smem;                   // [2][BKm][BM]
  float* Gs = smem + 2 * BKm * BM;    // [2][BKm][BN]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm0 = (wave / WN) * TM * 32, wn0 = (wave % WN) * TN * 32;
  const int ntn = (a.Cg + BN - 1) / BN;
  int bx, by, bz;
  wgrad_block(bx, by, bz);
  const int dn0 = (bx / ntn) * BM, gn0 = (bx % ntn) * BN;
  const int t = by;
  const int tw = t % a.k, th = (t / a.k) % a.k, td = t / (a.k * a.k);
  const int64_t M = (int64_t)a.N * a.Dd * a.Hd * a.Wd;
  const int64_t mb = (int64_t)bz * a.chunk;
  const int64_t me = min(M, mb + a.chunk);
  const int nK = (int)((me - mb + BKm - 1) / BKm);

  const int qd = tid % LPR_D, qg = tid % LPR_G;
  float4 rd[D_LOADS], rg[G_LOADS];

  auto load_tiles = [&](int ks) {
    int64_t mk = mb + (int64_t)ks * BKm;
#pragma unroll
    for (int i = 0; i < D_LOADS; ++i) {
      int r = tid / LPR_D + i * RPP_D;
      int64_t m = mk + r;
      int c = dn0 + 4 * qd;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < BKm && m < me && c < a.Cd) v = *reinterpret_cast<const float4*>(a.D + m * a.Cd + c);
      rd[i] = v;
    }
#pragma unroll
    for (int i = 0; i < G_LOADS; ++i) {
      int r = tid / LPR_G + i * RPP_G;
      int64_t m = mk + r;
      int c = gn0 + 4 * qg;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < BKm && m < me && c < a.Cg) {
        int mw = (int)(m % a.Wd); int64_t u = m / a.Wd;
        int mh = (int)(u % a.Hd); u /= a.Hd;
        int md = (int)(u % a.Dd); int nb = (int)(u / a.Dd);
        int gd = md * a.s - a.p + td, gh = mh * a.s - a.p + th, gw = mw * a.s - a.p + tw;
        if ((unsigned)gd < (unsigned)a.Dg && (unsigned)gh < (unsigned)a.Hg && (unsigned)gw < (unsigned)a.Wg)
          v = *reinterpret_cast<const float4*>(a.G + ((((int64_t)nb * a.Dg + gd) * a.Hg + gh) * a.Wg + gw) * a.Cg + c);
      }
      rg[i] = v;
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < D_LOADS; ++i) {
      int r = tid / LPR_D + i * RPP_D;
      if (r < BKm) *reinterpret_cast<float4*>(Ds + (buf * BKm + r) * BM + 4 * qd) = op_round4(rd[i], a.x3);
    }
#pragma unroll
    for (int i = 0; i < G_LOADS; ++i) {
      int r = tid / LPR_G + i * RPP_G;
      if (r < BKm) *reinterpret_cast<float4*>(Gs + (buf * BKm + r) * BN + 4 * qg) = op_round4(rg[i], a.x3);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  if (nK > 0) { load_tiles(0); store_tiles(0); }
  __syncthreads();
  const int li = lane & 31, lh = lane >> 5;
  for (int ks = 0; ks < nK; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nK) load_tiles(ks + 1);
    const float* Db = Ds + buf * BKm * BM;
    const float* Gb = Gs + buf * BKm * BN;
#pragma unroll
    for (int kc = 0; kc < BKm / 2; ++kc) {
      const int kr = 2 * kc + lh;   // lane half h supplies k = 2kc + h
      float av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) av[i] = Db[kr * BM + wm0 + i * 32 + li];
#pragma unroll
      for (int j = 0; j < TN; ++j) bv[j] = Gb[kr * BN + wn0 + j * 32 + li];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (ks + 1 < nK) store_tiles(buf ^ 1);
    __syncthreads();
  }

  const int T = a.k * a.k * a.k;
  float* slab = a.ws + ((int64_t)bz * T + t) * a.Cd * a.Cg;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    int col = gn0 + wn0 + j * 32 + li;
    if (col >= a.Cg) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int row = dn0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row < a.Cd) slab[(int64_t)row * a.Cg + col] = acc[i][j][r];
      }
  }
}

// ---- bf16x3 variant ------------------------------------------------------------------------
// Same split-K structure; the contraction (voxels) becomes the MFMA K.  Tiles are staged
// TRANSPOSED into LDS, one row per channel holding 32 voxels as [hi 32 × bf16][lo 32 × bf16]
// (144-B rows, the brick/igemm_x3 format), so the 32x32x16 fragments are plain ds_read_b128.
// Staging unit = 4 voxels × 4 channels per thread: lanes run over voxel quads first, so the
// 16 lanes of a ds_write_b64 group cover two rows 4 apart (144 dwords ≡ 16 mod 32 banks) and
// 8 consecutive 8-byte slots: conflict-free.  Every load is unconditional (clamped address,
// selected to 0) so vmcnt stays static across the register-staged double buffer.
typedef float f32x2w __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2w __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4w __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8w __attribute__((ext_vector_type(8)));
typedef float f32x4w __attribute__((ext_vector_type(4)));
constexpr int kWRow = 144;

// hi/lo of 4 voxel values of one channel → two 8-byte quads, stored at row (hi) and row + 64 (lo)
template <int PM>
__device__ __forceinline__ void wsplit4_store(char* row, float a, float b, float c, float d) {
  uint2 hi, lo;
  prec::split2<PM>(a, b, hi.x, lo.x);
  prec::split2<PM>(c, d, hi.y, lo.y);
  *reinterpret_cast<uint2*>(row) = hi;
  if constexpr (prec::has_lo<PM>()) *reinterpret_cast<uint2*>(row + 64) = lo;
}

template <int WM, int WN, int TM, int TN, int PM>
__global__ void __launch_bounds__(256)
conv_wgrad_x3_kernel(WgradArgs a) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  constexpr int BKm = 32;
  constexpr int UD = BM / 4 * 8, UG = BN / 4 * 8;          // staging units (4 voxels × 4 channels)
  static_assert(UD <= 256 && UG <= 256, "one unit per thread");
  constexpr int STAGE = (BM + BN) * kWRow;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm0 = (wave / WN) * TM * 32, wn0 = (wave % WN) * TN * 32;
  const int li = lane & 31, lh = lane >> 5;
  const int ntn = (a.Cg + BN - 1) / BN;
  int bx, by, bz;
  wgrad_block(bx, by, bz);
  const int dn0 = (bx / ntn) * BM, gn0 = (bx % ntn) * BN;
  const int t = by;
  const int tw = t % a.k, th = (t / a.k) % a.k, td = t / (a.k * a.k);
  const int64_t M = (int64_t)a.N * a.Dd * a.Hd * a.Wd;
  const int64_t mb = (int64_t)bz * a.chunk;
  const int64_t me = min(M, mb + a.chunk);
  const int nK = (int)((me - mb + BKm - 1) / BKm);

  // this thread's staging unit: voxel quad vq (4 voxels), channel quad cq
  const int vq = tid & 7, cq = tid >> 3;
  const bool do_d = tid < UD, do_g = tid < UG;
  const int cd = dn0 + 4 * (do_d ? cq : 0), cg = gn0 + 4 * (do_g ? cq : 0);
  const bool cd_ok = do_d && cd < a.Cd, cg_ok = do_g && cg < a.Cg;

  float4 rd[4], rg[4];
  // voxel coordinates of this thread's first voxel of the current K-step, advanced by BKm per
  // step with carries (32-bit index math: conv_wgrad checks that every offset fits)
  int cm = (int)min(mb + 4 * vq, M - 1);
  int cw = cm % a.Wd, ch_ = (cm / a.Wd) % a.Hd, cdd = (cm / (a.Wd * a.Hd)) % a.Dd, cn = cm / (a.Wd * a.Hd * a.Dd);
  int m_base = (int)mb + 4 * vq;
  const int me32 = (int)me;
  auto load = [&]() __attribute__((always_inline)) {
    int mw = cw, mh = ch_, md = cdd, nb = cn;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int m = m_base + s;
      const bool m_ok = m < me32;
      const float4 dv = *reinterpret_cast<const float4*>(a.D + (m_ok ? m : (int)mb) * a.Cd + (cd_ok ? cd : 0));
      rd[s] = (m_ok && cd_ok) ? dv : make_float4(0.f, 0.f, 0.f, 0.f);
      const int gd = md * a.s - a.p + td, gh = mh * a.s - a.p + th, gw = mw * a.s - a.p + tw;
      const bool g_in = m_ok && cg_ok && (unsigned)gd < (unsigned)a.Dg && (unsigned)gh < (unsigned)a.Hg &&
                        (unsigned)gw < (unsigned)a.Wg;
      const int goff = g_in ? (((nb * a.Dg + gd) * a.Hg + gh) * a.Wg + gw) * a.Cg + cg : 0;
      const float4 gv = *reinterpret_cast<const float4*>(a.G + goff);
      rg[s] = g_in ? gv : make_float4(0.f, 0.f, 0.f, 0.f);
      if (++mw == a.Wd) { mw = 0; if (++mh == a.Hd) { mh = 0; if (++md == a.Dd) { md = 0; ++nb; } } }
    }
  };
  auto advance = [&]() __attribute__((always_inline)) {
    m_base += BKm;
    cw += BKm;
    while (cw >= a.Wd) {
      cw -= a.Wd;
      if (++ch_ == a.Hd) { ch_ = 0; if (++cdd == a.Dd) { cdd = 0; ++cn; } }
    }
  };
  auto store = [&](int buf) __attribute__((always_inline)) {
    char* A = smem + buf * STAGE;
    char* B = A + BM * kWRow;
    if (do_d) {
      const int r = 4 * cq;
      wsplit4_store<PM>(A + (r + 0) * kWRow + 8 * vq, rd[0].x, rd[1].x, rd[2].x, rd[3].x);
      wsplit4_store<PM>(A + (r + 1) * kWRow + 8 * vq, rd[0].y, rd[1].y, rd[2].y, rd[3].y);
      wsplit4_store<PM>(A + (r + 2) * kWRow + 8 * vq, rd[0].z, rd[1].z, rd[2].z, rd[3].z);
      wsplit4_store<PM>(A + (r + 3) * kWRow + 8 * vq, rd[0].w, rd[1].w, rd[2].w, rd[3].w);
    }
    if (do_g) {
      const int r = 4 * cq;
      wsplit4_store<PM>(B + (r + 0) * kWRow + 8 * vq, rg[0].x, rg[1].x, rg[2].x, rg[3].x);
      wsplit4_store<PM>(B + (r + 1) * kWRow + 8 * vq, rg[0].y, rg[1].y, rg[2].y, rg[3].y);
      wsplit4_store<PM>(B + (r + 2) * kWRow + 8 * vq, rg[0].z, rg[1].z, rg[2].z, rg[3].z);
      wsplit4_store<PM>(B + (r + 3) * kWRow + 8 * vq, rg[0].w, rg[1].w, rg[2].w, rg[3].w);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  load();
  store(0);
  __syncthreads();
  for (int ks = 0; ks < nK; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nK) advance();
    load();                                   // unconditional (last step reloads itself, unused)
    const char* A = smem + buf * STAGE;
    const char* B = A + BM * kWRow;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8w ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const char* row = A + (wm0 + i * 32 + li) * kWRow + kk * 32 + lh * 16;
        ah[i] = *reinterpret_cast<const bf16x8w*>(row);
        al[i] = prec::has_lo<PM>() ? *reinterpret_cast<const bf16x8w*>(row + 64) : ah[i];
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const char* row = B + (wn0 + j * 32 + li) * kWRow + kk * 32 + lh * 16;
        bh[j] = *reinterpret_cast<const bf16x8w*>(row);
        bl[j] = prec::has_lo<PM>() ? *reinterpret_cast<const bf16x8w*>(row + 64) : bh[j];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = prec::mma<PM>(ah[i], al[i], bh[j], bl[j], acc[i][j]);
        }
    }
    if (ks + 1 < nK) store(buf ^ 1);
    __syncthreads();
  }

  const int T = a.k * a.k * a.k;
  float* slab = a.ws + ((int64_t)bz * T + t) * a.Cd * a.Cg;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    int col = gn0 + wn0 + j * 32 + li;
    if (col >= a.Cg) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int row = dn0 + wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row < a.Cd) slab[(int64_t)row * a.Cg + col] = acc[i][j][r];
      }
  }
}

// out[dn][gn][t] (=|+=) Σ_z ws[z][t][dn][gn].  Block = one dn × 64 gn × 4 t, one output per
// thread: every thread's `splits` slab loads are in flight together (a block walking several
// outputs per thread waits out the slab latency once per output), the slab reads run along gn
// (64 contiguous floats per (z, t)), and the sums are transposed through LDS so each gn's run of
// 4 taps is stored contiguously (a store per thread strided by T, plus 64-bit index math per
// element, took 7.7 µs for a 128×128×27 gradient).  Summation order over z is fixed (groups of
// four, pairwise): bit-reproducible.
constexpr int kRedG = 64, kRedT = 4;
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ ws, float* __restrict__ out, int Cd,
                                                           int Cg, int T, int splits, int accumulate) {
  __shared__ float tile[kRedG][kRedT + 1];
  const int dn = blockIdx.x, g0 = blockIdx.y * kRedG, t0 = blockIdx.z * kRedT;
  const int tid = threadIdx.x;
  const int gl = tid % kRedG, tl = tid / kRedG;
  const int plane = T * Cd * Cg;                      // < 2^31 (host check)
  if (g0 + gl < Cg && t0 + tl < T) {
    const float* src = ws + ((t0 + tl) * Cd + dn) * Cg + g0 + gl;
    float v = 0.f;
    int z = 0;
    for (; z + 4 <= splits; z += 4)
      v += (src[(int64_t)z * plane] + src[(int64_t)(z + 1) * plane]) +
           (src[(int64_t)(z + 2) * plane] + src[(int64_t)(z + 3) * plane]);
    for (; z < splits; ++z) v += src[(int64_t)z * plane];
    tile[gl][tl] = v;
  }
  __syncthreads();
  const int g2 = tid / kRedT, t2 = tid % kRedT;
  if (g0 + g2 < Cg && t0 + t2 < T) {
    float* dst = out + ((int64_t)dn * Cg + g0 + g2) * T + t0 + t2;
    const float v = tile[g2][t2];
    *dst = accumulate ? *dst + v : v;
  }
}

static int launch_wgrad_reduce(const float* ws, float* out, int Cd, int Cg, int T, int splits, int accumulate,
                               hipStream_t st) {
  MRAGAN_CHECK_ARG((int64_t)T * Cd * Cg < ((int64_t)1 << 31), "wgrad_reduce: %d x %d x %d too large", Cd, Cg, T);
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(Cd, ceil_div(Cg, kRedG), ceil_div(T, kRedT)), dim3(256), 0, st, ws, out,
                     Cd, Cg, T, splits, accumulate);
  return check_launch("wgrad_reduce");
}

// Short-contraction weight gradient (round 6): the UNet's innermost layers
// (networks3D.py:300-330 — Conv3d / ConvTranspose3d(8ngf, 8ngf, k4 s2) on 4³ / 2³ grids, the k4 s2
// layers on 4³) contract over M = N·Dd·Hd·Wd ≤ 128 voxels but write Cd·Cg·64 outputs (16.8 MB at
// 256 × 256).  On the split-K path that is one MFMA K-step per block, a 4-B-strided slab write of
// the whole gradient and a reduce that reads it back: 26-30 µs per launch, launch-latency and
// store bound at 0.001-0.002 of peak.  Here one thread owns one (gn, tap) column of the torch layout
// [dn][gn][t] for kSmR consecutive dn: per contraction voxel one gathered G load feeds kSmR FMAs
// whose D values come from an LDS broadcast, and the block stores kSmR runs of 256 contiguous
// floats straight into `out` — no slab, no reduce.  One-plane modes (bf16 / fp16) only: the
// operands are rounded RNE exactly as the MFMA staging rounds them and a product of two rounded
// operands is exact in fp32, so this is the MFMA kernel's arithmetic in another (fixed) summation
// order; the fp32-grade modes keep their kernels (their fixtures' emulation follows those).
constexpr int kSmR = 16;       // dn rows per thread
constexpr int kSmMaxM = 128;   // longest contraction this kernel takes
__global__ void __launch_bounds__(256) wgrad_small_kernel(WgradArgs a, float* __restrict__ out, int accumulate) {
  __shared__ __attribute__((aligned(16))) float dcol[kSmMaxM][kSmR];     // D[m][dn0 + r], rounded
  const int T = a.k * a.k * a.k;
  const int J = a.Cg * T;                                                 // outputs per dn row
  const int dn0 = blockIdx.y * kSmR;
  const int M = a.N * a.Dd * a.Hd * a.Wd;
  for (int e = threadIdx.x; e < M * kSmR; e += 256) {
    const int m = e / kSmR, r = e % kSmR;
    dcol[m][r] = op_round(a.D[(int64_t)m * a.Cd + dn0 + r], a.x3);
  }
  __syncthreads();
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= J) return;
  const int gn = j / T, t = j - gn * T;
  const int tw = t % a.k, th = (t / a.k) % a.k, td = t / (a.k * a.k);
  float acc[kSmR];
#pragma unroll
  for (int r = 0; r < kSmR; ++r) acc[r] = 0.f;
  int m = 0;
  for (int nb = 0; nb < a.N; ++nb)
    for (int md = 0; md < a.Dd; ++md) {
      const int gd = md * a.s - a.p + td;
      for (int mh = 0; mh < a.Hd; ++mh) {
        const int gh = mh * a.s - a.p + th;
        const bool okdh = (unsigned)gd < (unsigned)a.Dg && (unsigned)gh < (unsigned)a.Hg;
        for (int mw = 0; mw < a.Wd; ++mw, ++m) {
          const int gw = mw * a.s - a.p + tw;
          if (!okdh || (unsigned)gw >= (unsigned)a.Wg) continue;     // zero fill: the product adds 0
          const float g = op_round(a.G[((((int64_t)nb * a.Dg + gd) * a.Hg + gh) * a.Wg + gw) * a.Cg + gn], a.x3);
          const float4* dp = reinterpret_cast<const float4*>(dcol[m]);
#pragma unroll
          for (int q = 0; q < kSmR / 4; ++q) {
            const float4 d = dp[q];
            acc[4 * q] = fmaf(d.x, g, acc[4 * q]);
            acc[4 * q + 1] = fmaf(d.y, g, acc[4 * q + 1]);
            acc[4 * q + 2] = fmaf(d.z, g, acc[4 * q + 2]);
            acc[4 * q + 3] = fmaf(d.w, g, acc[4 * q + 3]);
          }
        }
      }
    }
#pragma unroll
  for (int r = 0; r < kSmR; ++r) {
    float* dst = out + (int64_t)(dn0 + r) * J + j;
    *dst = accumulate ? *dst + acc[r] : acc[r];
  }
}

// the short-contraction kernel takes this launch (A/B switch MRAGAN_WGRAD_SMALL_M: the longest
// contraction it takes, 0 = off)
static bool wgrad_small_applicable(const WgradArgs& a) {
  static const int max_m = [] {
    const char* e = getenv("MRAGAN_WGRAD_SMALL_M");
    const int v = e ? atoi(e) : 64;
    return v < kSmMaxM ? v : kSmMaxM;
  }();
  const int64_t M = (int64_t)a.N * a.Dd * a.Hd * a.Wd;
  return (a.x3 == kPrecBf16 || a.x3 == kPrecF16) && !a.in16 && !a.in16g && a.N2 == 0 && M <= max_m &&
         a.Cd % kSmR == 0 && (int64_t)a.Cd * a.Cg * a.k * a.k * a.k < ((int64_t)1 << 31);
}

static int launch_wgrad_small(const WgradArgs& a, float* out, int accumulate, hipStream_t st) {
  const int J = a.Cg * a.k * a.k * a.k;
  hipLaunchKernelGGL(wgrad_small_kernel, dim3(ceil_div(J, 256), a.Cd / kSmR), dim3(256), 0, st, a, out, accumulate);
  return check_launch("wgrad_small");
}

static int wgrad_plan(int Cd, int Cg, int T, int64_t M, int* splits, int64_t* chunk, bool* big) {
  *big = (Cd >= 128 && Cg >= 128);
  int bm = *big ? 128 : 64, bn = *big ? 128 : 64;
  int64_t tiles = (int64_t)ceil_div(Cd, bm) * ceil_div(Cg, bn) * T;
  int64_t want = (1024 + tiles - 1) / tiles;
  int64_t maxs = (M + 32 * 16 - 1) / (32 * 16);    // ≥16 K-steps per split
  int64_t s = want < maxs ? want : maxs;
  if (s < 1) s = 1;
  int64_t ch = (M + s - 1) / s;
  ch = (ch + 31) / 32 * 32;
  s = (M + ch - 1) / ch;
  if (s < 1) s = 1;
  *splits = (int)s;
  *chunk = ch;
  return 0;
}

size_t conv_wgrad_ws_bytes(int N, int Dd, int Hd, int Wd, int Cd, int Cg, int k) {
  int splits; int64_t chunk; bool big;
  int T = k * k * k;
  wgrad_plan(Cd, Cg, T, (int64_t)N * Dd * Hd * Wd, &splits, &chunk, &big);
  return (size_t)splits * T * Cd * Cg * sizeof(float);
}

int conv_wgrad(WgradArgs a, float* out, int accumulate, size_t ws_bytes, hipStream_t st) {
  MRAGAN_CHECK_ARG(a.Cd % 4 == 0 && a.Cg % 4 == 0, "conv_wgrad: channels must be multiples of 4 (%d,%d)", a.Cd, a.Cg);
  if (a.N2 > 0) {
    // two instance sets into one gradient (ABI 19): one wgrad3_x3 launch + one reduce where the
    // aligned operand-plane path takes both, else set 1 then set 2 accumulating
    WgradArgs b = a;
    b.D2 = b.G2 = nullptr; b.N2 = 0;
    WgradArgs c = b;
    c.D = a.D2; c.G = a.G2; c.N = a.N2;
    MRAGAN_CHECK_ARG(a.D2 && a.G2, "conv_wgrad: null second instance set");
    static const bool no_pair = getenv("MRAGAN_NO_WGRAD_PAIR") != nullptr;   // A/B switch
    if (!no_pair && a.in16 && getenv("MRAGAN_NO_WGRAD3") == nullptr && wgrad3_x3_applicable(b) &&
        wgrad3_x3_applicable(c)) {
      const int T = a.k * a.k * a.k;
      bool big;
      wgrad_plan(a.Cd, a.Cg, T, (int64_t)(a.N + a.N2) * a.Dd * a.Hd * a.Wd, &a.splits, &a.chunk, &big);
      const size_t need = (size_t)a.splits * T * a.Cd * a.Cg * sizeof(float);
      if (need > ws_bytes) {
        set_error("conv_wgrad: workspace %zu < %zu", ws_bytes, need);
        return kWorkspace;
      }
      const int used = conv_wgrad3_x3(a, wgrad3_x3_splits(a, a.splits), st);
      if (used != -kUnsupported) {
        if (used < 0) return -used;
        int rc = check_launch("wgrad3_x3(op16)");
        if (rc) return rc;
        return launch_wgrad_reduce(a.ws, out, a.Cd, a.Cg, T, used, accumulate, st);
      }
    }
    const int rc = conv_wgrad(b, out, accumulate, ws_bytes, st);
    return rc ? rc : conv_wgrad(c, out, 1, ws_bytes, st);
  }
  if (a.x3 && a.N > 1) {
    // the 16-bit MFMA kernels address their operands with 32-bit byte offsets: a batch whose
    // tensors exceed 2 GiB runs as consecutive instance ranges accumulating into `out` (each
    // range's plan needs at most the whole batch's workspace)
    const int64_t dper = (int64_t)a.Dd * a.Hd * a.Wd * a.Cd, gper = (int64_t)a.Dg * a.Hg * a.Wg * a.Cg;
    const int64_t per = 4 * (dper > gper ? dper : gper), lim = ((int64_t)1 << 31) - 1;
    if (per * a.N > lim && per <= lim) {
      MRAGAN_CHECK_ARG(!a.in16, "conv_wgrad: 16-bit operand planes of more than 2 GiB");
      const int nb = (int)(lim / per);
      for (int n0 = 0; n0 < a.N; n0 += nb) {
        WgradArgs c = a;
        c.N = nb < a.N - n0 ? nb : a.N - n0;
        c.D = a.D + n0 * dper;
        c.G = a.G + n0 * gper;
        const int rc = conv_wgrad(c, out, n0 == 0 ? accumulate : 1, ws_bytes, st);
        if (rc) return rc;
      }
      return kOk;
    }
  }
  if (wgrad_small_applicable(a)) return launch_wgrad_small(a, out, accumulate, st);
  const int T = a.k * a.k * a.k;
  const int64_t M = (int64_t)a.N * a.Dd * a.Hd * a.Wd;
  bool big;
  wgrad_plan(a.Cd, a.Cg, T, M, &a.splits, &a.chunk, &big);
  size_t need = (size_t)a.splits * T * a.Cd * a.Cg * sizeof(float);
  if (need > ws_bytes) {
    set_error("conv_wgrad: workspace %zu < %zu", ws_bytes, need);
    return kWorkspace;
  }
  static const bool no_w3 = getenv("MRAGAN_NO_WGRAD3") != nullptr;   // A/B switch
  const bool w3 = !no_w3 && wgrad3_x3_applicable(a), w3s2 = !no_w3 && !w3 && wgrad3s2_x3_applicable(a);
  MRAGAN_CHECK_ARG(!a.in16 || w3 || w3s2, "conv_wgrad: 16-bit operand planes are supported by the k3 s1 valid weight "
                   "gradient (wgrad3_x3) and the k3 s2 one (wgrad3s2_x3) only");
  MRAGAN_CHECK_ARG(!a.in16g || w3s2, "conv_wgrad: a 16-bit gathered-operand plane is supported by the k3 s2 weight "
                   "gradient (wgrad3s2_x3) only");
  if (w3 || w3s2) {
    const int used = w3 ? conv_wgrad3_x3(a, wgrad3_x3_splits(a, a.splits), st)
                        : conv_wgrad3s2_x3(a, wgrad3s2_x3_splits(a, a.splits), st);
    if (used < 0) return -used;
    int rc = check_launch(a.in16 ? "wgrad3_x3(op16)" : "wgrad3_x3");
    if (rc) return rc;
    return launch_wgrad_reduce(a.ws, out, a.Cd, a.Cg, T, used, accumulate, st);
  }
  const bool idx32 = M * a.Cd < ((int64_t)1 << 31) &&
                     (int64_t)a.N * a.Dg * a.Hg * a.Wg * a.Cg < ((int64_t)1 << 31);
  const bool x3 = a.x3 && a.Cd % 32 == 0 && a.Cg % 32 == 0 && idx32;
  if (x3) {
    auto grid_of = [&](int bm, int bn) { return dim3(ceil_div(a.Cd, bm) * ceil_div(a.Cg, bn), T, a.splits); };
    MRAGAN_PREC_DISPATCH(a.x3, {
      if (a.Cd >= 128 && a.Cg >= 128)
        hipLaunchKernelGGL((conv_wgrad_x3_kernel<2, 2, 2, 2, PM>), grid_of(128, 128), dim3(256), 0, st, a);
      else if (a.Cd >= 128)
        hipLaunchKernelGGL((conv_wgrad_x3_kernel<2, 2, 2, 1, PM>), grid_of(128, 64), dim3(256), 0, st, a);
      else if (a.Cg >= 128)
        hipLaunchKernelGGL((conv_wgrad_x3_kernel<2, 2, 1, 2, PM>), grid_of(64, 128), dim3(256), 0, st, a);
      // 32-channel side (G down1 / up2 at full resolution): a 64×32 tile on two waves instead of
      // a half-empty 64×64 one
      else if (a.Cg == 32 && a.Cd >= 64)
        hipLaunchKernelGGL((conv_wgrad_x3_kernel<2, 1, 1, 1, PM>), grid_of(64, 32), dim3(128), 0, st, a);
      else if (a.Cd == 32 && a.Cg >= 64)
        hipLaunchKernelGGL((conv_wgrad_x3_kernel<1, 2, 1, 1, PM>), grid_of(32, 64), dim3(128), 0, st, a);
      else
        hipLaunchKernelGGL((conv_wgrad_x3_kernel<2, 2, 1, 1, PM>), grid_of(64, 64), dim3(256), 0, st, a);
      break;
    })
  } else if (big) {
    dim3 grid(ceil_div(a.Cd, 128) * ceil_div(a.Cg, 128), T, a.splits);
    hipLaunchKernelGGL((conv_wgrad_f32_kernel<2, 2, 2, 2>), grid, dim3(256), 0, st, a);
  } else {
    dim3 grid(ceil_div(a.Cd, 64) * ceil_div(a.Cg, 64), T, a.splits);
    hipLaunchKernelGGL((conv_wgrad_f32_kernel<2, 2, 1, 1>), grid, dim3(256), 0, st, a);
  }
  int rc = check_launch(x3 ? "conv_wgrad_x3" : "conv_wgrad_f32");
  if (rc) return rc;
  return launch_wgrad_reduce(a.ws, out, a.Cd, a.Cg, T, a.splits, accumulate, st);
}

}  // namespace mragan
