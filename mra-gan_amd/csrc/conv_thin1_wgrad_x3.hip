// bf16x3 MFMA weight gradient of the 1-channel k7 s1 convolutions (gfx950):
//
//   G stem  Conv3d(1 → 32, k7)   dW[c][t] = Σ_v dH[v][c] · Xpad[v + t]          networks3D.py:185-189
//   G head  Conv3d(32 → 1, k7)   dW[c][t] = Σ_m dZ[m] · Hpad[m + t][c]          networks3D.py:211-212
//
// Both are   Out[c][t] = Σ_v  P[v][c] · Q[v + τ(t) − pe]     (Q zero outside its grid)
// with P the 32-channel operand on its own grid and Q the single channel: the stem directly
// (P = dH, Q = Xpad, pe = p, τ = id), the head after u = m + t (P = Hpad, Q = dZ, pe = k−1−p,
// τ = the tap mirror).  As a GEMM: rows = taps (7·7·8 with kw padded, 13 tiles of 32), cols =
// the 32 channels, contraction = voxels.  A k-group of 8 is 8 w-consecutive voxels, so the A
// fragment Q[v + t][8 consecutive w] is a 16-B read from the same X8 image as conv_thin1_x3
// (X8[d][h][w] = Q[d][h][w..w+7], planar bf16 hi/lo), and the B fragment is a 16-B read from P
// staged transposed ([c][h][w], planar hi/lo).
//
// Persistent blocks (one per CU) walk 1 × 8 × 32-voxel bricks of P's grid and keep their 13
// tap tiles × 32 channels in accumulators across bricks; each block writes one partial
// [343][32] slab, and a second kernel sums the slabs in fixed order (deterministic).
#include "kernels.h"
#include "prec.h"

namespace mragan {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

constexpr int kK = 7;
constexpr int kT = kK * kK * kK;       // 343 taps
constexpr int kMT = 13;                // tap tiles: 7·7·8 = 392 padded rows → 13 × 32 (416)
constexpr int kBH = 8, kBW = 32;       // brick (BD = 1)
constexpr int kNV = kBH * kBW;         // voxels per brick = 16 K-steps of 16
constexpr int kRD = kK, kRH = kBH + kK - 1, kRW = 40;   // Q halo: 7 × 14 × (32+6 → 40)
constexpr int kC = 32;
constexpr int kPS = kNV + 8;           // P^T channel-row stride (bf16): 33 16-B slots, so the
                                       // 32 lanes (channels) of a B read hit distinct bank quads

}  // namespace

struct Thin1WArgs {
  const float* P; int N, Dp, Hp, Wp;          // [N][Dp][Hp][Wp][32]
  const float* Q; int Dq, Hq, Wq;             // [N][Dq][Hq][Wq]
  int pe, flip;
  int nbd, nbh, nbw;
  float* slab;                                // [gridDim.x][343][32]
};

// tap row m of tile `tile` (0..415) → tap index (kd·7 + kh)·7 + kw, or −1 for padding rows
__device__ __forceinline__ int tap_of_row(int m) {
  const int kw = m & 7, g = m >> 3;
  return (kw < kK && g < kK * kK) ? g * kK + kw : -1;
}

template <int PM>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
thin1_wgrad_x3_kernel(Thin1WArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* raw = reinterpret_cast<float*>(smem);                                   // [7][14][40]
  bf16x8* x8h = reinterpret_cast<bf16x8*>(smem + kRD * kRH * kRW * sizeof(float)); // [7][14][32]
  bf16x8* x8l = x8h + kRD * kRH * kBW;
  __bf16* pth = reinterpret_cast<__bf16*>(x8l + kRD * kRH * kBW);                // [32][8][32] hi
  __bf16* ptl = pth + kC * kPS;                                                   // lo

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  // tap tiles of this wave: 0-3 | 4-6 | 7-9 | 10-12
  const int t0 = wave == 0 ? 0 : 1 + 3 * wave;
  const int ntile = wave == 0 ? 4 : 3;
  // A row of each tile: tap (kd, kh, kw) → X8 offset (kd·14 + kh)·32 + kw (padding rows: 0)
  int aoff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = (t0 + i) * 32 + li;
    const int kw = m & 7, g = m >> 3;
    aoff[i] = (kw < kK && g < kK * kK) ? ((g / kK) * kRH + g % kK) * kBW + kw : 0;
  }
  f32x16 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x16{};

  const int nbricks = a.N * a.nbd * a.nbh * a.nbw;
  for (int b = blockIdx.x; b < nbricks; b += gridDim.x) {
    int r = b;
    const int bw_i = r % a.nbw; r /= a.nbw;
    const int bh_i = r % a.nbh; r /= a.nbh;
    const int vd = r % a.nbd;
    const int nb = r / a.nbd;
    const int vh0 = bh_i * kBH, vw0 = bw_i * kBW;
    __syncthreads();                 // previous brick's MFMA reads are done
    // 1a. Q halo raw: Q[vd + kd − pe][vh0 + hh − pe][vw0 + ww − pe], hh < 14, ww < 38
    {
      const float* qb = a.Q + (int64_t)nb * a.Dq * a.Hq * a.Wq;
      constexpr int NR = kRD * kRH * kRW;
      constexpr int NL = (NR + 255) / 256;
      float v[NL];
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        const int e = l * 256 + tid;
        const int ww = e % kRW, hh = (e / kRW) % kRH, dd = e / (kRW * kRH);
        const int qd = vd + dd - a.pe, qh = vh0 + hh - a.pe, qw = vw0 + ww - a.pe;
        const bool ok = e < NR && ww < kBW + kK - 1 && (unsigned)qd < (unsigned)a.Dq && (unsigned)qh < (unsigned)a.Hq &&
                        (unsigned)qw < (unsigned)a.Wq;
        const float t = qb[ok ? ((int64_t)qd * a.Hq + qh) * a.Wq + qw : 0];
        v[l] = ok ? t : 0.f;
      }
      // 1b. P brick transposed: thread → 2 w-consecutive voxels × 4 channels (bf16 pairs)
      const float* pb = a.P + (int64_t)nb * a.Dp * a.Hp * a.Wp * kC;
      float4 pv[4][2];
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        const int e = l * 256 + tid;            // 1024 units = 128 voxel pairs × 8 channel quads
        const int cq = e & 7, vp = e >> 3;
        const int vh = vp / (kBW / 2), vw = (vp % (kBW / 2)) * 2;
        const int ph = vh0 + vh, pw = vw0 + vw;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bool ok = vd < a.Dp && ph < a.Hp && pw + s < a.Wp;
          const float4 t = *reinterpret_cast<const float4*>(
              pb + (ok ? (((int64_t)vd * a.Hp + ph) * a.Wp + pw + s) * kC : 0) + 4 * cq);
          pv[l][s] = ok ? t : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int l = 0; l < NL; ++l) {
        const int e = l * 256 + tid;
        if (e < NR) raw[e] = v[l];
      }
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        const int e = l * 256 + tid;
        const int cq = e & 7, vp = e >> 3;
        const int vox = (vp / (kBW / 2)) * kBW + (vp % (kBW / 2)) * 2;   // brick voxel of the pair
        const float c0[4] = {pv[l][0].x, pv[l][0].y, pv[l][0].z, pv[l][0].w};
        const float c1[4] = {pv[l][1].x, pv[l][1].y, pv[l][1].z, pv[l][1].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t h, lo;
          prec::split2<PM>(c0[q], c1[q], h, lo);
          const int idx = (4 * cq + q) * kPS + vox;
          *reinterpret_cast<uint32_t*>(pth + idx) = h;
          if constexpr (prec::has_lo<PM>()) *reinterpret_cast<uint32_t*>(ptl + idx) = lo;
        }
      }
    }
    __syncthreads();
    // 2. X8 expansion (as conv_thin1_x3, but identity positions: here the A operand's lanes are
    // taps, 8 consecutive kw per k-group row)
    for (int gq = tid; gq < kRD * kRH * (kBW / 4); gq += 256) {
      const int row = gq / (kBW / 4), w0 = (gq % (kBW / 4)) * 4;
      const float4* src = reinterpret_cast<const float4*>(raw + row * kRW + w0);
      const float4 p0 = src[0], p1 = src[1], p2 = src[2];
      const float rr[12] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w, p2.x, p2.y, p2.z, p2.w};
#pragma unroll
      for (int dw = 0; dw < 4; ++dw) {
        const f32x8 v = {rr[dw], rr[dw + 1], rr[dw + 2], rr[dw + 3], rr[dw + 4], rr[dw + 5], rr[dw + 6], rr[dw + 7]};
        bf16x8 hi, lo;
        prec::split8v<PM>(v, hi, lo);
        x8h[row * kBW + w0 + dw] = hi;
        if constexpr (prec::has_lo<PM>()) x8l[row * kBW + w0 + dw] = lo;
      }
    }
    __syncthreads();
    // 3. MFMA: 16 K-steps of 16 voxels (h row ks/2, w 16·(ks mod 2) + 8·lh … +7)
#pragma unroll
    for (int ks = 0; ks < kNV / 16; ++ks) {
      const int bh = ks >> 1, w8 = 16 * (ks & 1) + 8 * lh;
      const int pidx = li * kPS + bh * kBW + w8;
      const bf16x8 bhv = *reinterpret_cast<const bf16x8*>(pth + pidx);
      const bf16x8 blv = prec::has_lo<PM>() ? *reinterpret_cast<const bf16x8*>(ptl + pidx) : bhv;
      const int xo = bh * kBW + w8;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i < ntile) {
          const bf16x8 ah = x8h[aoff[i] + xo];
          const bf16x8 al = prec::has_lo<PM>() ? x8l[aoff[i] + xo] : ah;
          acc[i] = prec::mma<PM>(ah, al, bhv, blv, acc[i]);
        }
      }
    }
  }
  // 4. this block's partial sums: slab[block][t][c] (rows = taps, cols = channels)
  float* slab = a.slab + (int64_t)blockIdx.x * kT * kC;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i >= ntile) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = (t0 + i) * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      const int t = tap_of_row(m);
      if (t >= 0) slab[t * kC + li] = acc[i][r];
    }
  }
}

// out[c][t] (=|+=) Σ_blocks slab[z][τ(t)][c]   (τ = tap mirror for the head form)
// One block per tap: 8 groups of 32 lanes (lane = channel: 128 contiguous bytes per slab row),
// group g sums slabs z ≡ g (mod 8) in increasing z, then the 8 partials are added in g order —
// fixed order, deterministic.  (One thread per output summing all slabs serially ran 83 µs on
// 43 blocks.)
__global__ void __launch_bounds__(256) thin1_wgrad_reduce_kernel(const float* __restrict__ slab, int nz, int flip,
                                                                 float* __restrict__ out, int accumulate) {
  __shared__ float part[8][kC];
  const int t = blockIdx.x, c = threadIdx.x % kC, g = threadIdx.x / kC;
  const int ts = flip ? kT - 1 - t : t;
  float s = 0.f;
#pragma unroll 8
  for (int z = g; z < nz; z += 8) s += slab[((int64_t)z * kT + ts) * kC + c];
  part[g][c] = s;
  __syncthreads();
  if (g == 0) {
    float r = part[0][c];
#pragma unroll
    for (int k = 1; k < 8; ++k) r += part[k][c];
    const int e = c * kT + t;
    out[e] = accumulate ? out[e] + r : r;
  }
}

static int thin1w_grid() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  return ncu;
}

bool thin1_wgrad_x3_applicable(int Cd, int Cg, int k, int s) {
  return k == kK && s == 1 && ((Cd == kC && Cg == 1) || (Cd == 1 && Cg == kC));
}

size_t thin1_wgrad_x3_ws_bytes() { return (size_t)thin1w_grid() * kT * kC * sizeof(float); }

// Same argument convention as conv_wgrad: dW[dn][gn][t] = Σ_m D[m][dn] · G[m − p + t][gn]
int conv_thin1_wgrad_x3(const float* D, int N, int Dd, int Hd, int Wd, int Cd, const float* G, int Dg, int Hg, int Wg,
                        int Cg, int p, float* out, int accumulate, int mode, void* ws, size_t ws_bytes, hipStream_t st) {
  Thin1WArgs a{};
  if (Cg == 1) {          // stem: P = D (32 ch), Q = G
    a.P = D; a.Dp = Dd; a.Hp = Hd; a.Wp = Wd;
    a.Q = G; a.Dq = Dg; a.Hq = Hg; a.Wq = Wg;
    a.pe = p; a.flip = 0;
  } else {                // head: P = G (32 ch), Q = D, u = m − p + t
    a.P = G; a.Dp = Dg; a.Hp = Hg; a.Wp = Wg;
    a.Q = D; a.Dq = Dd; a.Hq = Hd; a.Wq = Wd;
    a.pe = kK - 1 - p; a.flip = 1;
  }
  a.N = N;
  a.nbd = a.Dp; a.nbh = ceil_div(a.Hp, kBH); a.nbw = ceil_div(a.Wp, kBW);
  const int64_t bricks = (int64_t)N * a.nbd * a.nbh * a.nbw;
  int grid = thin1w_grid();
  if (bricks < grid) grid = (int)(bricks > 0 ? bricks : 1);
  const size_t need = (size_t)grid * kT * kC * sizeof(float);
  if (!ws || ws_bytes < need) {
    set_error("thin1_wgrad_x3: workspace %zu < %zu", ws_bytes, need);
    return kWorkspace;
  }
  a.slab = static_cast<float*>(ws);
  const size_t lds = (size_t)kRD * kRH * kRW * sizeof(float) + (size_t)2 * kRD * kRH * kBW * 16 +
                     (size_t)2 * kC * kPS * sizeof(__bf16);
  int rc = kOk;
  MRAGAN_PREC_DISPATCH(mode, {
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(thin1_wgrad_x3_kernel<PM>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr_set = true;
    }
    hipLaunchKernelGGL(thin1_wgrad_x3_kernel<PM>, dim3(grid), dim3(256), lds, st, a);
    rc = check_launch("thin1_wgrad_x3");
    break;
  })
  if (rc) return rc;
  static_assert(kC * 8 == 256, "reduce block = 8 groups of kC lanes");
  hipLaunchKernelGGL(thin1_wgrad_reduce_kernel, dim3(kT), dim3(256), 0, st, a.slab, grid, a.flip, out, accumulate);
  return check_launch("thin1_wgrad_reduce");
}

}  // namespace mragan
