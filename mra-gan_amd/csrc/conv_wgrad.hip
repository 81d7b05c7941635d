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

namespace mragan {

typedef float f32x16 __attribute__((ext_vector_type(16)));


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
  const int dn0 = (blockIdx.x / ntn) * BM, gn0 = (blockIdx.x % ntn) * BN;
  const int t = blockIdx.y;
  const int tw = t % a.k, th = (t / a.k) % a.k, td = t / (a.k * a.k);
  const int64_t M = (int64_t)a.N * a.Dd * a.Hd * a.Wd;
  const int64_t mb = (int64_t)blockIdx.z * a.chunk;
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
      if (r < BKm) *reinterpret_cast<float4*>(Ds + (buf * BKm + r) * BM + 4 * qd) = rd[i];
    }
#pragma unroll
    for (int i = 0; i < G_LOADS; ++i) {
      int r = tid / LPR_G + i * RPP_G;
      if (r < BKm) *reinterpret_cast<float4*>(Gs + (buf * BKm + r) * BN + 4 * qg) = rg[i];
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
  float* slab = a.ws + ((int64_t)blockIdx.z * T + t) * a.Cd * a.Cg;
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

// out[dn][gn][t] (=|+=) Σ_z ws[z][t][dn][gn]
__global__ void wgrad_reduce_kernel(const float* __restrict__ ws, float* __restrict__ out, int Cd, int Cg, int T,
                                    int splits, int accumulate) {
  int64_t total = (int64_t)Cd * Cg * T;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    int t = (int)(e % T); int64_t u = e / T;
    int gn = (int)(u % Cg); int dn = (int)(u / Cg);
    float s = 0.f;
    for (int z = 0; z < splits; ++z) s += ws[(((int64_t)z * T + t) * Cd + dn) * Cg + gn];
    out[e] = accumulate ? out[e] + s : s;
  }
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
  const int T = a.k * a.k * a.k;
  const int64_t M = (int64_t)a.N * a.Dd * a.Hd * a.Wd;
  bool big;
  wgrad_plan(a.Cd, a.Cg, T, M, &a.splits, &a.chunk, &big);
  size_t need = (size_t)a.splits * T * a.Cd * a.Cg * sizeof(float);
  if (need > ws_bytes) {
    set_error("conv_wgrad: workspace %zu < %zu", ws_bytes, need);
    return kWorkspace;
  }
  if (big) {
    dim3 grid(ceil_div(a.Cd, 128) * ceil_div(a.Cg, 128), T, a.splits);
    hipLaunchKernelGGL((conv_wgrad_f32_kernel<2, 2, 2, 2>), grid, dim3(256), 0, st, a);
  } else {
    dim3 grid(ceil_div(a.Cd, 64) * ceil_div(a.Cg, 64), T, a.splits);
    hipLaunchKernelGGL((conv_wgrad_f32_kernel<2, 2, 1, 1>), grid, dim3(256), 0, st, a);
  }
  int rc = check_launch("conv_wgrad_f32");
  if (rc) return rc;
  int64_t total = (int64_t)a.Cd * a.Cg * T;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, a.ws, out, a.Cd, a.Cg, T, a.splits, accumulate);
  return check_launch("wgrad_reduce");
}

}  // namespace mragan
