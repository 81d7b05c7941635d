// Depth-streaming MFMA kernels for the ONE-channel k = 7, stride-1 convolutions (gfx950):
//
//   G stem   Conv3d(1 → ngf, k7) on the RPad3 input             networks3D.py:185-189 (forward)
//   G head   data gradient of Conv3d(ngf → 1, k7)                networks3D.py:211-212 (transposed
//            form s = 1 = forward form with pad 6 − p and the taps flipped)
//   both     weight gradients (dW[c][t] = Σ_v P[v][c] · Q[v + t − pe], P the 32-channel operand)
//
// The single-channel operand Q enters every product through an "X8" image: X8[d][h][w] =
// Q[d][h][w..w+7], split into planar bf16 hi / lo 16-B entries, so that one MFMA k-group of 8
// is one w-row of taps (kw padded to 8 with a zero tap) and every fragment is one aligned 16-B
// LDS read.  A block owns a column of the output (forward) or of P's grid (weight gradient) —
// 8 rows × 16 columns — and walks it along depth: the 7 X8 planes a depth step reads stay
// resident in an 8-slot ring, and each step expands exactly ONE new plane (the one 7 steps
// ahead) into the slot the previous step retired, while its MFMAs run.  One barrier per step.
// (A 7-deep halo re-expanded per brick cost more than the MFMAs: thin1_x3 of round 1.)
//
//   forward  rows = 32 output channels (the weights, all 25 K-steps held in registers),
//            cols = 32 voxels (2 rows × 16 columns per wave), K = 50 (kd, kh) groups × 8 kw;
//            the weight rows are permuted so a lane's 16 accumulators are 16 consecutive
//            channels of one voxel (64 contiguous bytes stored per lane);
//   wgrad    rows = 13 tiles of 32 taps (7·7·8 with kw padded), cols = 32 channels, K = the
//            step's 128 voxels split over the 4 waves (2 brick rows each), accumulators kept
//            across the block's whole work list; P's brick is staged transposed ([c][voxel],
//            double-buffered).  The 4 waves' partial sums are added in LDS in wave order and
//            each block writes one [343][32] slab; a second kernel sums the slabs in fixed
//            order (deterministic).
//
// Work items = (column, depth chunk of L steps); L is chosen on the host so that the items
// divide evenly over the CUs (one 4-wave block per CU, grid ≤ CU count, items strided).
#include "kernels.h"
#include "lane_ops.h"
#include "prec.h"

#include <type_traits>

namespace mragan {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kK = 7;
constexpr int kT = kK * kK * kK;        // 343 taps
constexpr int kC = 32;                  // channels of the wide side
constexpr int kGroups = 50;             // 49 (kd, kh) rows + 1 zero group
constexpr int kKS = kGroups / 2;        // forward K-steps (two groups each: lane halves)
constexpr int kMT = 13;                 // wgrad tap tiles: 7·7·8 rows → 13 × 32
constexpr int kBH = 8, kBW = 16;        // brick: rows × columns per depth step
constexpr int kRH = kBH + kK - 1;       // X8 rows per plane
constexpr int kRing = 8;                // X8 planes resident
constexpr int kPlaneE = kRH * kBW;      // 224 X8 entries per plane (hi or lo)
constexpr int kPS = kBH * kBW + 8;      // P^T channel-row stride (bf16): 272 B, 17 16-B slots
constexpr int kMaxItemsStamped = 4096;

// X8 entry of (row, pos) in a plane slot.  The forward reads (lanes = 16 columns of 2 rows)
// are conflict-free on the identity layout.  The weight-gradient reads (lanes = taps: 8 kw of
// one (kd, kh) row per lane octet, consecutive (kd, kh) rows on neighbouring octets) need the
// octets' column halves to alternate: odd (row + slot) swaps them — rows alternate within a
// plane, and the slot term keeps the alternation across the kh = 6 → 0 plane change.
template <int SW>
__device__ __forceinline__ int x8_entry(int row, int pos, int slot) {
  return row * kBW + (SW ? (pos ^ (((row + slot) & 1) << 3)) : pos);
}

// eight consecutive w of one Q row (zero outside Q) through the volume's range-checked
// descriptor: out-of-range elements get an offset past the end and read 0.  Q is channels-last
// with C channels; this reads channel c.
__device__ __forceinline__ void load_row8(__amdgpu_buffer_rsrc_t q, int D, int H, int W, int d, int h, int w0,
                                          float (&v)[8], int C = 1, int c = 0) {
  const bool okdh = (unsigned)d < (unsigned)D && (unsigned)h < (unsigned)H;
  const uint32_t rowb = ((uint32_t)(((int64_t)d * H + h) * W) * C + c) * 4u;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int w = w0 + j;
    const bool ok = okdh && (unsigned)w < (unsigned)W;
    v[j] = buf_load_f32(q, ok ? rowb + 4u * C * (uint32_t)w : kOobOffset);
  }
}

// both channels of a two-channel Q row (one 8-B load per voxel): channel 0 → v, channel 1 → u
__device__ __forceinline__ void load_row8x2(__amdgpu_buffer_rsrc_t q, int D, int H, int W, int d, int h, int w0,
                                            float (&v)[8], float (&u)[8]) {
  const bool okdh = (unsigned)d < (unsigned)D && (unsigned)h < (unsigned)H;
  const uint32_t rowb = (uint32_t)(((int64_t)d * H + h) * W) * 8u;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int w = w0 + j;
    const bool ok = okdh && (unsigned)w < (unsigned)W;
    const uint2 p = buf_load_8b(q, (int)(ok ? rowb + 8u * (uint32_t)w : kOobOffset), 0);
    v[j] = __uint_as_float(p.x);
    u[j] = __uint_as_float(p.y);
  }
}

// load_row8 / load_row8x2 by channel count (C2: channel 1 → u)
template <int C2>
__device__ __forceinline__ void load_rows(__amdgpu_buffer_rsrc_t q, int D, int H, int W, int d, int h, int w0,
                                          float (&v)[8], float (&u)[8]) {
  if constexpr (C2) load_row8x2(q, D, H, W, d, h, w0, v, u);
  else load_row8(q, D, H, W, d, h, w0, v);
}

// X8 entry e of a plane (rows of kBW entries) from its 8 raw values, split hi / lo
__device__ __forceinline__ f32x8 load_row8v(__amdgpu_buffer_rsrc_t q, int D, int H, int W, int d, int h, int w0,
                                            int C = 1, int c = 0) {
  float v[8];
  load_row8(q, D, H, W, d, h, w0, v, C, c);
  return f32x8{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
}

template <int PM, int SW>
__device__ __forceinline__ void store_x8v(bf16x8* ringH, bf16x8* ringL, int plane_e, int slot, int e, const f32x8 f) {
  bf16x8 hi, lo;
  prec::split8v<PM>(f, hi, lo);
  const int idx = slot * plane_e + x8_entry<SW>(e / kBW, e % kBW, slot);
  ringH[idx] = hi;
  if constexpr (prec::has_lo<PM>()) ringL[idx] = lo;
}

template <int PM, int SW>
__device__ __forceinline__ void store_x8(bf16x8* ringH, bf16x8* ringL, int plane_e, int slot, int e,
                                         const float (&v)[8]) {
  const f32x8 f = {v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
  bf16x8 hi, lo;
  prec::split8v<PM>(f, hi, lo);
  const int idx = slot * plane_e + x8_entry<SW>(e / kBW, e % kBW, slot);
  ringH[idx] = hi;
  if constexpr (prec::has_lo<PM>()) ringL[idx] = lo;
}

// X8 entry of a two-channel Q in a one-plane mode: channel 0 → the hi ring, channel 1 → the
// ring the lo planes of bf16x3 occupy (one-plane modes leave it free)
template <int PM, int C2>
__device__ __forceinline__ void store_x8c(bf16x8* ringH, bf16x8* ringL, int plane_e, int slot, int e,
                                          const float (&v)[8], const float (&u)[8]) {
  if constexpr (C2) {
    static_assert(!prec::has_lo<PM>(), "two-channel X8 rings use the lo ring: one-plane modes only");
    const f32x8 fv = {v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7]};
    const f32x8 fu = {u[0], u[1], u[2], u[3], u[4], u[5], u[6], u[7]};
    bf16x8 h0, l0, h1, l1;
    prec::split8v<PM>(fv, h0, l0);
    prec::split8v<PM>(fu, h1, l1);
    const int idx = slot * plane_e + x8_entry<0>(e / kBW, e % kBW, slot);
    ringH[idx] = h0;
    ringL[idx] = h1;
  } else {
    store_x8<PM, 0>(ringH, ringL, plane_e, slot, e, v);
  }
}

// the depth-chunk length: items = columns × ⌈D / L⌉ spread over ≤ ncu blocks; cost ≈ rounds ×
// (steps + the 7 prologue plane expansions, ≈ 1.5 steps)
void pick_chunk(int64_t columns, int D, int ncu, int& L, int& nch, int& grid) {
  double best = 1e30;
  L = D; nch = 1; grid = 1;
  for (int l = 4; l <= 32; ++l) {
    const int ll = l < D ? l : D;
    const int n = ceil_div(D, ll);
    const int64_t items = columns * n;
    const int g = (int)(items < ncu ? items : ncu);
    const int64_t rounds = (items + g - 1) / g;
    const double cost = (double)rounds * (ll + 1.5);
    if (cost < best - 1e-9) { best = cost; L = ll; nch = n; grid = g; }
    if (ll == D) break;
  }
}

int cu_count() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  return ncu;
}

// wp: packed [343][ny][cx] (cx = 1, or 2 in the one-plane modes) → out[(g·2 + hl)·ny + co][8]
// bf16, e = kw (e = 7 and g = 49: 0); hl = 1 holds the lo split (bf16x3) or channel 1 (cx = 2)
template <int PM>
__global__ void thin1_pack_kernel(const float* __restrict__ wp, int ny, int cx, int flip, __bf16* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kGroups * ny) return;
  const int co = i % ny, g = i / ny;
  f32x8 v, u;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float w = 0.f, w1 = 0.f;
    if (g < kK * kK && e < kK) {
      const int t = g * kK + e;
      const int64_t o = ((int64_t)(flip ? kT - 1 - t : t) * ny + co) * cx;
      w = wp[o];
      if (cx == 2) w1 = wp[o + 1];
    }
    v[e] = w;
    u[e] = w1;
  }
  bf16x8 hi, lo;
  prec::split8v<PM>(v, hi, lo);
  if (cx == 2) {
    bf16x8 l1;
    prec::split8v<PM>(u, lo, l1);
  }
  *reinterpret_cast<bf16x8*>(out + ((int64_t)(g * 2 + 0) * ny + co) * 8) = hi;
  *reinterpret_cast<bf16x8*>(out + ((int64_t)(g * 2 + 1) * ny + co) * 8) = lo;
}

}  // namespace

// diagnostic stamps (MRAGAN_STAMPS=1): s_memtime at item start / after the prologue / item end
__device__ unsigned long long g_thin1_stamps[kMaxItemsStamped * 3];

struct Thin1RArgs {
  int stamp;
  const float* x; int N, Di, Hi, Wi;      // [N][Di][Hi][Wi]
  const __bf16* wx;
  const float* bias;
  float* y; int Do, Ho, Wo;               // [N][Do][Ho][Wo][32]
  int pe, act;
  int nbh, nbw, L, nch, items;
  double* part;                           // optional: the next InstanceNorm's Σy / Σy² per item
  // optional (with part, transposed form = a data gradient): backward statistics of the
  // InstanceNorm(+act) whose output, replication-padded by sfold, was the conv's input — x̂ at the
  // clamped voxel c(o) = clamp(o − sfold) of every padded output: Σ g, Σ g·x̂ with g = y·act'(x̂)
  const float* sx; const float* smean; const float* srstd; int sact, sfold;
};

// forward brick: 16 rows × 16 columns per depth step, 4 rows (2 tiles) per wave
constexpr int kFH = 16;
constexpr int kFRH = kFH + kK - 1;      // 22 X8 rows per plane
constexpr int kFPlaneE = kFRH * kBW;    // 352 entries per plane (hi or lo)
constexpr int kFLds = 2 * kRing * kFPlaneE * 16 + kGroups * 2 * kC * 16;   // ring + weights: 141 312 B
constexpr int kFRed = 4 * kC * 2 * 8 + 2 * kC * 4;   // + [4 waves][32 ch][Σ, Σ²] doubles (a.part), μ / rstd of sx
// TW = 2 (one-plane modes, one input channel): no lo ring, hi weights only — 69 KB, so two blocks
// share a CU (two waves per SIMD: one block's loads and barrier waits under the other's MFMAs)
constexpr int kFLdsC = kRing * kFPlaneE * 16 + kGroups * kC * 16;              // 70 656 B

// C2: a two-channel input (one-plane modes): channel 1's X8 planes and weights sit where the lo
// splits of bf16x3 do, and each K-step issues one MFMA per channel
// EPI (compile-time epilogue, round 5): 0 = bias (+ activation); 1 = the next InstanceNorm's Σy, Σy²
// (a.part); 2 = backward statistics (a.part with a.sx).  With the three in one body the compiler
// kept every path's registers live (accumulator-file spills, 11 VALU per MFMA: PMC r05g).
template <int PM, int C2, int EPI, int TW>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(TW, TW))) thin1r_fwd_kernel(Thin1RArgs a) {
  static_assert(TW == 1 || (!prec::has_lo<PM>() && !C2), "two waves per SIMD: one-plane, one channel");
  constexpr bool CMP = TW == 2;                          // compact LDS: hi ring and hi weights only
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16x8* ringH = reinterpret_cast<bf16x8*>(smem);       // [kRing][kFPlaneE]
  bf16x8* ringL = CMP ? ringH : ringH + kRing * kFPlaneE;
  bf16x8* wsm = ringH + (CMP ? 1 : 2) * kRing * kFPlaneE;  // [kGroups][hi|lo][kC] (CMP: [kGroups][kC])
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  auto wsel = [&](int g, int hl, int c) __attribute__((always_inline)) { return CMP ? g * kC + c : (g * 2 + hl) * kC + c; };

  if constexpr (CMP) {
    for (int e = tid; e < kGroups * kC; e += 256) wsm[e] = reinterpret_cast<const bf16x8*>(a.wx)[(e / kC) * 2 * kC + e % kC];
  } else {
    for (int e = tid; e < kGroups * 2 * kC; e += 256) wsm[e] = reinterpret_cast<const bf16x8*>(a.wx)[e];
  }
  // A row li (weights) holds channel perm(li) = 16·((li>>2)&1) + 4·(li>>3) + (li&3), so
  // accumulator 4q + e of lane (li, lh) is channel 16·lh + 4q + e: 64 contiguous bytes per lane
  const int co = ((li >> 2) & 1) * 16 + (li >> 3) * 4 + (li & 3);
  // WREG (one-plane, one channel): the 25 A fragments live in registers for the whole kernel
  // (100 VGPRs; one wave per SIMD leaves room) — per MFMA only the ring's B fragment is read from
  // LDS.  The r05 form re-read the weights from LDS every K-step and issued each MFMA right behind
  // its two reads (s_waitcnt lgkmcnt(0) per MFMA: one LDS latency per 32-cycle MFMA, ≈ 8 k cycles
  // per depth step against 1.6 k of MFMA, stamps r05g).
  // (EPI 2: its registers go to the statistics; TW 2: 256 registers per wave in all)
  constexpr bool WREG = !prec::has_lo<PM>() && !C2 && EPI != 2 && TW == 1;
  bf16x8 wreg[WREG ? kKS : 1];
  if constexpr (WREG) {
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < kKS; ++ks) wreg[ks] = wsm[wsel(2 * ks + lh, 0, co)];
  }
  float bias[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) bias[q] = (EPI == 0 && a.bias) ? a.bias[16 * lh + q] : 0.f;
  // this lane's voxels (B columns): brick rows 4·wave + 2i + li/16 (tile i), column li % 16
  const int bh0 = 4 * wave + (li >> 4), bw = li & 15;
  // store layout (quad transposes): lane 4m + k handles piece k (channels 16·lh + 4k …) of the
  // voxels 4m … 4m + 3 — the same tile row as its own voxel, columns bwq … bwq + 3
  const int kq4 = li & 3, bwq = bw & ~3;

  for (int item = blockIdx.x; item < a.items; item += gridDim.x) {
    int r = item;
    const int cw = r % a.nbw; r /= a.nbw;
    const int chh = r % a.nbh; r /= a.nbh;
    const int chunk = r % a.nch;
    const int nb = r / a.nch;
    const int od0 = chunk * a.L, oh0 = chh * kFH, ow0 = cw * kBW;
    const int nsteps = min(a.L, a.Do - od0);
    const int nplanes = nsteps + kK - 1;
    constexpr int CX = C2 ? 2 : 1;
    const __amdgpu_buffer_rsrc_t xr =
        make_rsrc(a.x + (int64_t)nb * a.Di * a.Hi * a.Wi * CX, (uint32_t)a.Di * a.Hi * a.Wi * (4u * CX));
    const int d0 = od0 - a.pe, h0 = oh0 - a.pe, w0 = ow0 - a.pe;
    // this thread's X8 entries of a plane: tid and tid + 256 (< 352)
    const bool e1 = tid + 256 < kFPlaneE;
    const int er0 = tid / kBW, er1 = (tid + 256) / kBW, ep = tid % kBW;
    if (a.stamp && tid == 0 && item < kMaxItemsStamped) g_thin1_stamps[item * 3 + 0] = __builtin_amdgcn_s_memtime();

    // the item's instance's μ / rstd of the backward statistics' x̂ (EPI 2), staged through LDS;
    // each lane keeps its 4 store-layout channels' values in registers (below)
    float* sstat = reinterpret_cast<float*>(smem + (CMP ? kFLdsC : kFLds) + 4 * kC * 2 * 8);
    if constexpr (EPI == 2) {
      if (tid < 2 * kC) sstat[tid] = tid < kC ? a.smean[nb * kC + tid] : a.srstd[nb * kC + tid - kC];
    }
    // prologue: planes 0..6 → slots 0..6, every load in flight before the first store (one load
    // latency per item instead of seven)
    // (in batches of PB planes: all 7 at once for one wave per SIMD and one channel)
    constexpr int PB = (TW == 2 || C2) ? 4 : kK;
#pragma unroll
    for (int b0 = 0; b0 < kK; b0 += PB) {
      float v0[PB][8], v1[PB][8], u0[PB][8], u1[PB][8];
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        if (b0 + j < kK) {
          load_rows<C2>(xr, a.Di, a.Hi, a.Wi, d0 + b0 + j, h0 + er0, w0 + ep, v0[j], u0[j]);
          if (e1) load_rows<C2>(xr, a.Di, a.Hi, a.Wi, d0 + b0 + j, h0 + er1, w0 + ep, v1[j], u1[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        if (b0 + j < kK) {
          store_x8c<PM, C2>(ringH, ringL, kFPlaneE, b0 + j, tid, v0[j], u0[j]);
          if (e1) store_x8c<PM, C2>(ringH, ringL, kFPlaneE, b0 + j, tid + 256, v1[j], u1[j]);
        }
      }
    }
    __syncthreads();
    if (a.stamp && tid == 0 && item < kMaxItemsStamped) g_thin1_stamps[item * 3 + 1] = __builtin_amdgcn_s_memtime();
    // EPI 2: μ / rstd of this lane's 4 store-layout channels 16·lh + 4·kq4 + c (8 registers per item)
    float smu[4], srs[4];
    if constexpr (EPI == 2) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        smu[c] = sstat[16 * lh + 4 * kq4 + c];
        srs[c] = sstat[kC + 16 * lh + 4 * kq4 + c];
      }
    }

    // InstanceNorm partials of this item (a.part): lane (li, lh) holds channels 16·lh + q of its
    // voxels; fp64 throughout, y² formed in fp64 as the other producers do (fp32 sums of y and y²
    // lose var = E[y²] − E[y]² to cancellation by mean² / var — the stem reads a non-centred
    // volume).  One wave per SIMD by design: the 32 extra registers cost no occupancy.
    // The backward statistics (EPI 2: Σg, Σg·x̂ — no variance formula, nothing cancels against a
    // square) accumulate in fp32 over the item's ≤ 32 values per lane and channel and join the fp64
    // sums at the item's end: 4 VALU fewer per value than fp64 throughout (r05i PMC: 10 VALU per MFMA)
    // (EPI 2, round 6: in the store layout — 4 channels per lane, see the epilogue)
    constexpr int NS = EPI == 1 ? 16 : EPI == 2 ? 4 : 1;
    using AccT = typename std::conditional<EPI == 2, float, double>::type;
    AccT ps[NS], pq[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) ps[q] = pq[q] = AccT(0);
    for (int s = 0; s < nsteps; ++s) {
      const bool more = s + kK < nplanes;
      float n0[8], n1[8], m0[8], m1[8];
      if (more) {
#ifdef MRAGAN_EXP_NOLOAD            // bottleneck experiments (variant builds only, tools/)
#pragma unroll
        for (int j = 0; j < 8; ++j) n0[j] = n1[j] = m0[j] = m1[j] = 0.f;
#else
        load_rows<C2>(xr, a.Di, a.Hi, a.Wi, d0 + s + kK, h0 + er0, w0 + ep, n0, m0);
        if (e1) load_rows<C2>(xr, a.Di, a.Hi, a.Wi, d0 + s + kK, h0 + er1, w0 + ep, n1, m1);
#endif
      }
      // backward statistics: this step's x̂ operands, loaded before the MFMAs so their latency hides
      // under them (loaded in the epilogue they stalled every depth step: +0.17 ms per step)
      // Loaded in the store layout (below): lane (4m + k, lh) reads the 16-B piece k of the four
      // voxels 4m … 4m + 3 of its tile row — each load instruction then covers 8 voxels' whole
      // 128-B rows instead of 16-B pieces of 32 rows — and the statistics are formed in that layout
      // against the quad-transposed accumulators the stores use
      float4 sxv[2][EPI == 2 ? 4 : 1];
      if constexpr (EPI == 2) {
        const int Sd = a.Do - 2 * a.sfold, Sh = a.Ho - 2 * a.sfold, Sw = a.Wo - 2 * a.sfold;
        const int cd = min(max(od0 + s - a.sfold, 0), Sd - 1);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int ch = min(max(oh0 + bh0 + 2 * i - a.sfold, 0), Sh - 1);
          const float* xrow = a.sx + (((int64_t)nb * Sd + cd) * Sh + ch) * (int64_t)Sw * kC + 16 * lh + 4 * kq4;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int cw = min(max(ow0 + bwq + j - a.sfold, 0), Sw - 1);
            sxv[i][j] = *reinterpret_cast<const float4*>(xrow + (int64_t)cw * kC);
          }
        }
      }
      f32x16 acc[2] = {f32x16{}, f32x16{}};
      // fragments of K-step ks: this lane's group 2ks + lh → (kd, kh) (the zero group 49 reads
      // group 48's ring entries); software-pipelined one K-step ahead, so each MFMA waits on reads
      // issued a whole K-step earlier
      constexpr bool kTwo = prec::has_lo<PM>() || C2;
      auto frag = [&](int ks, bf16x8& ah, bf16x8& al, bf16x8 (&xh)[2], bf16x8 (&xl)[2]) __attribute__((always_inline)) {
        // (EPI 2 at TW 2: lh made opaque per K-step, so the compiler forms this K-step's (kd, kh)
        // and addresses here — two multiply-adds — instead of hoisting all 25 steps' per-lane values
        // out of the item loop, where they spilled: 40 registers over the 256 budget)
        int lhv = lh;
        if constexpr (EPI == 2 && TW == 2) asm volatile("" : "+v"(lhv));
        const int g = 2 * ks + lhv;
        const int g0 = 2 * ks, g1 = 2 * ks + 1 < kK * kK ? 2 * ks + 1 : kK * kK - 1;
        const int kd = g0 / kK + lhv * (g1 / kK - g0 / kK), kh = g0 % kK + lhv * (g1 % kK - g0 % kK);
        if constexpr (!WREG) {
          ah = wsm[wsel(g, 0, co)];
          al = kTwo ? wsm[wsel(g, 1, co)] : ah;
        }
        const int base = ((s + kd) & (kRing - 1)) * kFPlaneE + x8_entry<0>(bh0 + kh, bw, 0);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          xh[i] = ringH[base + 2 * i * kBW];
          xl[i] = kTwo ? ringL[base + 2 * i * kBW] : xh[i];
        }
      };
      bf16x8 fah[2], fal[2], fxh[2][2], fxl[2][2];
      frag(0, fah[0], fal[0], fxh[0], fxl[0]);
#pragma unroll
      for (int ks = 0; ks < kKS; ++ks) {
#ifdef MRAGAN_EXP_NOMFMA
        if (ks > 0) break;
#endif
        const int c = ks & 1;
        if (ks + 1 < kKS) frag(ks + 1, fah[c ^ 1], fal[c ^ 1], fxh[c ^ 1], fxl[c ^ 1]);
        const bf16x8 ah = WREG ? wreg[WREG ? ks : 0] : fah[c];
        const bf16x8 al = WREG ? ah : fal[c];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if constexpr (C2) {
            acc[i] = prec::mma<PM>(ah, ah, fxh[c][i], fxh[c][i], acc[i]);
            acc[i] = prec::mma<PM>(al, al, fxl[c][i], fxl[c][i], acc[i]);
          } else {
            acc[i] = prec::mma<PM>(ah, al, fxh[c][i], fxl[c][i], acc[i]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (more) {
        store_x8c<PM, C2>(ringH, ringL, kFPlaneE, (s + kK) & (kRing - 1), tid, n0, m0);
        if (e1) store_x8c<PM, C2>(ringH, ringL, kFPlaneE, (s + kK) & (kRing - 1), tid + 256, n1, m1);
      }

      const int od = od0 + s, ow = ow0 + bw;
      // the statistics run on every lane (a voxel outside the output adds 0), all of them before
      // the first store, and only the stores are predicated: on gfx9 vmcnt counts stores too, so a
      // wait for an sx load issued before some output stores also waits for those stores (the r05
      // form interleaved them and made every depth step wait for its own output stores)
      bool in[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) in[i] = oh0 + bh0 + 2 * i < a.Ho && ow < a.Wo;
      if constexpr (EPI == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const float v = acc[i][e] + bias[e];
            acc[i][e] = a.act != kActNone ? act_fwd(v, a.act) : v;
          }
      } else if constexpr (EPI == 1) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int e = 0; e < 16; ++e) {
            const float u = in[i] ? acc[i][e] : 0.f;
            ps[e] += u;
            pq[e] += (double)u * u;
          }
      }
      if constexpr (EPI == 2) {
        // the compiler sinks the statistics below the stores; this empty asm reads the sx values
        // (so their wait is placed here) and the memory clobber keeps the stores after it
        asm volatile("" ::"v"(sxv[0][0].x), "v"(sxv[0][1].x), "v"(sxv[0][2].x), "v"(sxv[0][3].x), "v"(sxv[1][0].x),
                     "v"(sxv[1][1].x), "v"(sxv[1][2].x), "v"(sxv[1][3].x)
                     : "memory");
      }
      // stores in the store layout: after component-wise quad transposes lane (4m + k, lh) holds
      // piece k of voxels 4m … 4m + 3, so store j writes 8 voxels' whole 128-B rows (the lanes of
      // a quad: 64 contiguous bytes per half) instead of 16-B pieces of 32 rows — 4× fewer cache
      // lines per store instruction (the stores were a third of the stem forward's time, r05r)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        f32x4v t[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          f32x4v v;
#pragma unroll
          for (int q = 0; q < 4; ++q) v[q] = acc[i][4 * q + c];
          t[c] = quad_transpose(v, kq4);
        }
        const int oh = oh0 + bh0 + 2 * i;
        if constexpr (EPI == 2) {
          // backward statistics in the store layout (round 6): t[c][j] and sxv[i][j] are channel
          // 16·lh + 4·kq4 + c of voxel (oh, ow0 + bwq + j) — no transposes of x̂ to the lane's own
          // voxel, 8 accumulators instead of 32 (the two-blocks-per-CU form fits 256 registers)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const bool vin = oh < a.Ho && ow0 + bwq + j < a.Wo;
            const float xs[4] = {sxv[i][j].x, sxv[i][j].y, sxv[i][j].z, sxv[i][j].w};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
              const float vs = t[c][j];
              const float xh = (xs[c] - smu[c]) * srs[c];
              const float g0 = (a.sact == kActRelu && !(xh > 0.f)) ? 0.f
                               : (a.sact == kActLrelu && !(xh > 0.f)) ? vs * kLreluSlope : vs;
              const float gv = vin ? g0 : 0.f;
              ps[c] += gv;
              pq[c] = fmaf(gv, xh, pq[c]);
            }
          }
        }
        float* yrow = a.y + (((int64_t)nb * a.Do + od) * a.Ho + oh) * (int64_t)a.Wo * kC + 16 * lh + 4 * kq4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int owj = ow0 + bwq + j;
#ifdef MRAGAN_EXP_NOSTORE
          if (oh < a.Ho && owj < a.Wo && a.Do < 0)
#else
          if (oh < a.Ho && owj < a.Wo)
#endif
            *reinterpret_cast<float4*>(yrow + (int64_t)owj * kC) = make_float4(t[0][j], t[1][j], t[2][j], t[3][j]);
        }
      }
      __syncthreads();
    }
    if constexpr (EPI != 0) {
      // item = nb · (items per instance) + (chunk · nbh + chh) · nbw + cw: the partials' chunk order
      double* red = reinterpret_cast<double*>(smem + (CMP ? kFLdsC : kFLds));
#pragma unroll
      for (int q = 0; q < NS; ++q) {
        double s2 = (double)ps[q], q2 = (double)pq[q];
        // EPI 1: lane (li, lh) holds channels 16·lh + q; EPI 2: channels 16·lh + 4·(li & 3) + q
#pragma unroll
        for (int m = EPI == 2 ? 4 : 1; m < 32; m <<= 1) {
          s2 += __shfl_xor(s2, m);
          q2 += __shfl_xor(q2, m);
        }
        const int ch = EPI == 2 ? 16 * lh + 4 * li + q : 16 * lh + q;
        if (EPI == 2 ? li < 4 : li == 0) {
          red[(wave * kC + ch) * 2] = s2;
          red[(wave * kC + ch) * 2 + 1] = q2;
        }
      }
      __syncthreads();
      if (tid < kC) {
        double s2 = 0.0, q2 = 0.0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          s2 += red[(w * kC + tid) * 2];
          q2 += red[(w * kC + tid) * 2 + 1];
        }
        double* dst = a.part + ((int64_t)item * kC + tid) * 2;
        dst[0] = s2;
        dst[1] = q2;
      }
      __syncthreads();
    }
    if (a.stamp && tid == 0 && item < kMaxItemsStamped) g_thin1_stamps[item * 3 + 2] = __builtin_amdgcn_s_memtime();
  }
}

int thin1_debug_stamps(unsigned long long* host, int n) {
  if (n > kMaxItemsStamped * 3) n = kMaxItemsStamped * 3;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_thin1_stamps), (size_t)n * 8) == hipSuccess ? kOk : kLaunch;
}

// cx = 2 (nc = 2 volumes, BASELINE configs[4]) in the one-plane modes: the second channel takes
// the lo ring / weight rows bf16x3 would use
bool thin1_x3_applicable(int cx, int ny, int k, int s, int mode) {
  const bool one_plane = mode == kPrecBf16 || mode == kPrecF16;
  return (cx == 1 || (cx == 2 && one_plane)) && k == kK && s == 1 && ny == kC;
}

size_t thin1_x3_ws_bytes(int ny) { return (size_t)kGroups * 2 * ny * 8 * sizeof(__bf16); }

template <int PM, int C2, int EPI, int TW>
static void launch_thin1_fwd_e(const Thin1RArgs& a, int grid, hipStream_t st) {
  const size_t lds = (TW == 2 ? kFLdsC : kFLds) + kFRed;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(thin1r_fwd_kernel<PM, C2, EPI, TW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((thin1r_fwd_kernel<PM, C2, EPI, TW>), dim3(grid), dim3(256), lds, st, a);
}

template <int PM, int C2, int TW>
static void launch_thin1_fwd(const Thin1RArgs& a, int grid, hipStream_t st) {
  if (!a.part) launch_thin1_fwd_e<PM, C2, 0, TW>(a, grid, st);
  else if (!a.sx) launch_thin1_fwd_e<PM, C2, 1, TW>(a, grid, st);
  else launch_thin1_fwd_e<PM, C2, 2, TW>(a, grid, st);
}

// two blocks per CU in the one-plane one-channel case (A/B switch: MRAGAN_THIN1_TW=1)
static int thin1_tw() {
  static const int tw = [] {
    const char* e = getenv("MRAGAN_THIN1_TW");
    return e && atoi(e) == 1 ? 1 : 2;
  }();
  return tw;
}

template <int PM>
static int conv_thin1_pm(const ThinArgs& t, void* ws, size_t ws_bytes, hipStream_t st) {
  const size_t need = thin1_x3_ws_bytes(t.ny);
  if (!ws || ws_bytes < need) {
    set_error("thin1_x3: workspace %zu < %zu", ws_bytes, need);
    return kWorkspace;
  }
  const bool c2 = t.cx == 2;
  if (!(t.cx == 1 || (c2 && !prec::has_lo<PM>()))) {
    set_error("thin1_x3: %d input channels in precision mode %d", t.cx, PM);
    return kBadArg;
  }
  hipLaunchKernelGGL(thin1_pack_kernel<PM>, dim3(ceil_div(kGroups * t.ny, 256)), dim3(256), 0, st, t.w, t.ny, t.cx,
                     t.trans ? 1 : 0, static_cast<__bf16*>(ws));
  int rc = check_launch("thin1_x3_pack");
  if (rc) return rc;
  Thin1RArgs a{};
  static const int stamps = getenv("MRAGAN_STAMPS") ? 1 : 0;
  a.stamp = stamps;
  a.x = t.x; a.N = t.N; a.Di = t.Di; a.Hi = t.Hi; a.Wi = t.Wi;
  a.wx = static_cast<const __bf16*>(ws);
  a.bias = t.bias; a.y = t.y; a.Do = t.Do; a.Ho = t.Ho; a.Wo = t.Wo;
  a.pe = t.trans ? kK - 1 - t.p : t.p;       // transposed s = 1: forward form, flipped taps
  a.act = t.act;
  a.nbh = ceil_div(t.Ho, kFH); a.nbw = ceil_div(t.Wo, kBW);
  const int64_t columns = (int64_t)t.N * a.nbh * a.nbw;
  if (columns == 0 || t.Do == 0) return kOk;
  MRAGAN_CHECK_ARG((int64_t)t.Di * t.Hi * t.Wi * t.cx * 4 < (int64_t)kOobOffset, "thin1_x3: input volume too large");
  int grid = 1;
  static const bool no_stats = getenv("MRAGAN_NO_THIN1_STATS") != nullptr;   // A/B switch
  const bool stats = t.in_part && !no_stats && t.act == kActNone && !t.bias &&
                     (t.bs_x ? (t.trans && t.bs_fold >= 0 && t.Do > 2 * t.bs_fold && t.Ho > 2 * t.bs_fold && t.Wo > 2 * t.bs_fold)
                             : !t.trans);
  // two blocks per CU for the plain and forward-statistics forms (the backward-statistics one
  // needs more than 256 registers)
  // (the backward-statistics form too since round 6: its statistics in the store layout take 215
  // registers; A/B switch MRAGAN_THIN1_BS_TW1 keeps it at one block per CU)
  static const bool bs_tw1 = getenv("MRAGAN_THIN1_BS_TW1") != nullptr;
  const int tw = (!prec::has_lo<PM>() && !c2 && !(stats && t.bs_x && bs_tw1)) ? thin1_tw() : 1;
  pick_chunk(columns, t.Do, tw * cu_count(), a.L, a.nch, grid);
  a.items = (int)(columns * a.nch);
  if (stats) {
    // conv3d_in_stats: the stem InstanceNorm's partials; conv3d_dgrad_in_stats (the G head's data
    // gradient): the backward statistics of the InstanceNorm in front of the head
    a.part = t.in_part;
    a.sx = t.bs_x; a.smean = t.bs_mean; a.srstd = t.bs_rstd; a.sact = t.bs_act; a.sfold = t.bs_fold;
    if (t.in_chunks) *t.in_chunks = a.nch * a.nbh * a.nbw;
  }
  if constexpr (!prec::has_lo<PM>()) {
    if (c2) launch_thin1_fwd<PM, 1, 1>(a, grid, st);
    else if (tw == 2) launch_thin1_fwd<PM, 0, 2>(a, grid, st);
    else launch_thin1_fwd<PM, 0, 1>(a, grid, st);
  } else {
    launch_thin1_fwd<PM, 0, 1>(a, grid, st);
  }
  return check_launch("thin1_x3");
}

int conv_thin1_x3(const ThinArgs& t, int mode, void* ws, size_t ws_bytes, hipStream_t st) {
  MRAGAN_PREC_DISPATCH(mode, return conv_thin1_pm<PM>(t, ws, ws_bytes, st))
}

// ---------------------------------------------------------------------------------------
// weight gradient
// ---------------------------------------------------------------------------------------
struct Thin1RWArgs {
  int stamp;
  const float* P; int N, Dp, Hp, Wp;          // [N][Dp][Hp][Wp][32]
  const float* Q; int Dq, Hq, Wq;             // [N][Dq][Hq][Wq][qC], channel qc
  int qC, qc;
  int pe;
  int nbh, nbw, L, nch, items;
  float* slab;                                // [gridDim.x][343][32]
};

// 8 waves (2 per SIMD): tap-tile group tg = wave / 4 (tiles 0–6 | 7–12) × K quarter kq = wave % 4
// (brick rows 2kq, 2kq + 1 of each step)
constexpr int kWT0 = 7;                 // tiles of group 0 (group 1: kMT − 7 = 6)

// P16 (one-plane modes, round 5): P is the 16-bit operand plane of the 32-channel operand (the words
// the staging would round it to): 8-B loads, the channel pairs of two voxels re-packed by bit ops —
// bit-identical to the fp32 path (tests/test_kernels_gpu.py::test_k7_planes_bit_identical)
template <int PM, int P16>
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) thin1r_wgrad_kernel(Thin1RWArgs a) {
  static_assert(!P16 || !prec::has_lo<PM>(), "operand planes exist in the one-plane modes only");
  constexpr uint32_t PES = P16 ? 2u : 4u;     // bytes per P element
  using PV = typename std::conditional<P16 != 0, uint4, float4>::type;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16x8* ringH = reinterpret_cast<bf16x8*>(smem);                     // [kRing][kPlaneE]
  bf16x8* ringL = ringH + kRing * kPlaneE;
  __bf16* pt = reinterpret_cast<__bf16*>(ringL + kRing * kPlaneE);     // [2 buf][hi|lo][32][kPS]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int tg = wave >> 2, kq = wave & 3;
  const int t0 = tg ? kWT0 : 0, nt = tg ? kMT - kWT0 : kWT0;

  // A rows of the tap tiles: tap m = 32t + li → (kd, kh, kw); the padding rows (kw = 7, or
  // groups past 48) read the neighbouring real entries (their sums are dropped), which keeps
  // the bank pattern of a full octet.  The offset inside the slot is row·16 + (pos ^ 8·((row +
  // kd + s) & 1)) with row = 2·kq + kss + kh, pos = 8·lh + kw.
  const int kw_l = li & 7;
  f32x16 acc[kWT0];
#pragma unroll
  for (int i = 0; i < kWT0; ++i) acc[i] = f32x16{};

  // P staging unit of this thread: voxel pair vp = tid & 63 (voxels 2vp, 2vp + 1 of the brick:
  // row vp / 8, columns 2(vp % 8) …), channel quad cq = tid >> 6
  const int vp = tid & 63, cq = tid >> 6;
  // P16: thread = (voxel vi = tid / 4 of the brick, 16-B chunk ck = tid % 4 = channels 8ck … 8ck+7):
  // a wave's load is 16 voxels' whole 64-B rows (1 KB contiguous); the voxel-pair / channel-quad
  // form touched 64 lines per load instruction for 8 B each
  const int vi16 = tid >> 2, ck16 = tid & 3;
  auto p_load = [&](__amdgpu_buffer_rsrc_t pr, int vd, int vh0, int vw0, PV& v0, PV& v1)
                    __attribute__((always_inline)) {
    if constexpr (P16) {
      const int ph = vh0 + (vi16 >> 4), pw = vw0 + (vi16 & 15);
      const bool ok = vd < a.Dp && ph < a.Hp && pw < a.Wp;
      const uint32_t b = (uint32_t)((((int64_t)vd * a.Hp + ph) * a.Wp + pw) * kC + 8 * ck16) * PES;
      v0 = __builtin_bit_cast(uint4, buf_load_16b(pr, (int)(ok ? b : kOobOffset), 0));
      v1 = v0;
      return;
    }
    const int ph = vh0 + (vp >> 3), pw = vw0 + 2 * (vp & 7);
    const bool okr = vd < a.Dp && ph < a.Hp;
    const bool ok0 = okr && pw < a.Wp, ok1 = okr && pw + 1 < a.Wp;
    const uint32_t b0 = (uint32_t)((((int64_t)vd * a.Hp + ph) * a.Wp + pw) * kC + 4 * cq) * PES;
    if constexpr (!P16) {
      v0 = buf_load_f32x4(pr, ok0 ? b0 : kOobOffset);
      v1 = buf_load_f32x4(pr, ok1 ? b0 + kC * PES : kOobOffset);
    }
  };
  auto p_store = [&](int buf, const PV v0, const PV v1) __attribute__((always_inline)) {
    __bf16* ph = pt + (size_t)buf * 2 * kC * kPS;
    __bf16* pl = ph + kC * kPS;
    auto put = [&](int q, float x0, float x1) __attribute__((always_inline)) {
      uint32_t h, l;
      prec::split2<PM>(x0, x1, h, l);
      const int idx = (4 * cq + q) * kPS + 2 * vp;
      *reinterpret_cast<uint32_t*>(ph + idx) = h;
      if constexpr (prec::has_lo<PM>()) *reinterpret_cast<uint32_t*>(pl + idx) = l;
    };
    if constexpr (P16) {
      // channel 8ck + j of voxel vi: the 16-bit word j of the chunk
      uint16_t* col = reinterpret_cast<uint16_t*>(ph) + (8 * ck16) * kPS + vi16;
      const uint32_t w[4] = {v0.x, v0.y, v0.z, v0.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        col[(2 * j) * kPS] = (uint16_t)(w[j] & 0xffffu);
        col[(2 * j + 1) * kPS] = (uint16_t)(w[j] >> 16);
      }
    } else {
      put(0, v0.x, v1.x);
      put(1, v0.y, v1.y);
      put(2, v0.z, v1.z);
      put(3, v0.w, v1.w);
    }
  };

  for (int item = blockIdx.x; item < a.items; item += gridDim.x) {
    int r = item;
    const int cw = r % a.nbw; r /= a.nbw;
    const int chh = r % a.nbh; r /= a.nbh;
    const int chunk = r % a.nch;
    const int nb = r / a.nch;
    const int vd0 = chunk * a.L, vh0 = chh * kBH, vw0 = cw * kBW;
    const int nsteps = min(a.L, a.Dp - vd0);
    const int nplanes = nsteps + kK - 1;
    const __amdgpu_buffer_rsrc_t qr =
        make_rsrc(a.Q + (int64_t)nb * a.Dq * a.Hq * a.Wq * a.qC, (uint32_t)a.Dq * a.Hq * a.Wq * a.qC * 4u);
    const __amdgpu_buffer_rsrc_t pr = make_rsrc(reinterpret_cast<const char*>(a.P) + (int64_t)nb * a.Dp * a.Hp * a.Wp * kC * PES,
                                                (uint32_t)a.Dp * a.Hp * a.Wp * kC * PES);
    const int d0 = vd0 - a.pe, h0 = vh0 - a.pe, w0 = vw0 - a.pe;
    const int erow = tid / kBW, epos = tid % kBW;      // this thread's X8 entry (tid < 224)
    if (a.stamp && tid == 0 && item < kMaxItemsStamped) g_thin1_stamps[item * 3 + 0] = __builtin_amdgcn_s_memtime();

    // prologue: P of step 0 → buffer 0, Q planes 0..6 → slots 0..6
    {
      PV v0, v1;
      p_load(pr, vd0, vh0, vw0, v0, v1);
      if (tid < kPlaneE) {
        float v[7][8];
#pragma unroll
        for (int rp = 0; rp < kK; ++rp) load_row8(qr, a.Dq, a.Hq, a.Wq, d0 + rp, h0 + erow, w0 + epos, v[rp], a.qC, a.qc);
#pragma unroll
        for (int rp = 0; rp < kK; ++rp) store_x8<PM, 1>(ringH, ringL, kPlaneE, rp, tid, v[rp]);
      }
      p_store(0, v0, v1);
    }
    __syncthreads();
    if (a.stamp && tid == 0 && item < kMaxItemsStamped) g_thin1_stamps[item * 3 + 1] = __builtin_amdgcn_s_memtime();

    for (int s = 0; s < nsteps; ++s) {
      // P(s + 1) and Q plane s + 7 → registers before the MFMAs, → the free buffer / slot after
      const bool more_q = s + kK < nplanes && tid < kPlaneE, more_p = s + 1 < nsteps;
      PV v0 = {}, v1 = {};
      f32x8 q = {};
      if (more_q) q = load_row8v(qr, a.Dq, a.Hq, a.Wq, d0 + s + kK, h0 + erow, w0 + epos, a.qC, a.qc);
      if (more_p) p_load(pr, vd0 + s + 1, vh0, vw0, v0, v1);

      const __bf16* ph = pt + (size_t)(s & 1) * 2 * kC * kPS;
      const __bf16* pl = ph + kC * kPS;
      if constexpr (!prec::has_lo<PM>()) {
        // one-plane modes: both K-steps' fragments are read before their MFMAs (K-step 1's while
        // K-step 0's MFMAs run) instead of each MFMA waiting on its own ring read (r05 PMC: 13.6
        // VALU per MFMA, every MFMA behind an s_waitcnt lgkmcnt(0))
        bf16x8 fa[2][kWT0], fb[2];
        auto fragw = [&](int kss, bf16x8 (&A)[kWT0], bf16x8& B) __attribute__((always_inline)) {
          B = *reinterpret_cast<const bf16x8*>(ph + li * kPS + (2 * kq + kss) * kBW + 8 * lh);
#pragma unroll
          for (int i = 0; i < kWT0; ++i) {
            if (i < nt) {
              const int g = min(4 * (t0 + i) + (li >> 3), kK * kK - 1);
              const int kd = g / kK, kh = g - kd * kK;
              const int row = 2 * kq + kss + kh;
              A[i] = ringH[((s + kd) & (kRing - 1)) * kPlaneE + row * kBW +
                           ((8 * lh + kw_l) ^ (((row + kd + s) & 1) << 3))];
            }
          }
        };
        fragw(0, fa[0], fb[0]);
        fragw(1, fa[1], fb[1]);
#pragma unroll
        for (int kss = 0; kss < 2; ++kss) {
#pragma unroll
          for (int i = 0; i < kWT0; ++i)
            if (i < nt) acc[i] = prec::mma<PM>(fa[kss][i], fa[kss][i], fb[kss], fb[kss], acc[i]);
        }
      } else
#pragma unroll
      for (int kss = 0; kss < 2; ++kss) {
        // K-step: brick row 2·kq + kss, voxels 8·lh … +7 of its 16
        const int pidx = li * kPS + (2 * kq + kss) * kBW + 8 * lh;
        const bf16x8 bh = *reinterpret_cast<const bf16x8*>(ph + pidx);
        const bf16x8 bl = prec::has_lo<PM>() ? *reinterpret_cast<const bf16x8*>(pl + pidx) : bh;
#pragma unroll
        for (int i = 0; i < kWT0; ++i) {
          if (i < nt) {
            const int g = min(4 * (t0 + i) + (li >> 3), kK * kK - 1);
            const int kd = g / kK, kh = g - kd * kK;
            const int row = 2 * kq + kss + kh;
            const int idx = ((s + kd) & (kRing - 1)) * kPlaneE + row * kBW +
                            ((8 * lh + kw_l) ^ (((row + kd + s) & 1) << 3));
            const bf16x8 ah = ringH[idx];
            const bf16x8 al = prec::has_lo<PM>() ? ringL[idx] : ah;
            acc[i] = prec::mma<PM>(ah, al, bh, bl, acc[i]);
          }
        }
      }
      if (more_q) store_x8v<PM, 1>(ringH, ringL, kPlaneE, (s + kK) & (kRing - 1), tid, q);
      if (more_p) p_store((s + 1) & 1, v0, v1);
      __syncthreads();
    }
    if (a.stamp && tid == 0 && item < kMaxItemsStamped) g_thin1_stamps[item * 3 + 2] = __builtin_amdgcn_s_memtime();
  }

  // the K quarters' partial sums, added in quarter order in LDS ([416 rows][32] floats over the
  // ring; the two tile groups own disjoint rows), then this block's slab rows (taps) × 32 channels
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int rq = 0; rq < 4; ++rq) {
    if (kq == rq) {
#pragma unroll
      for (int i = 0; i < kWT0; ++i) {
        if (i < nt) {
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int m = 32 * (t0 + i) + 8 * (q >> 2) + 4 * lh + (q & 3);
            const int idx = m * kC + li;
            red[idx] = rq == 0 ? acc[i][q] : red[idx] + acc[i][q];
          }
        }
      }
    }
    __syncthreads();
  }
  float* slab = a.slab + (int64_t)blockIdx.x * kT * kC;
  for (int e = tid; e < kT * kC; e += 512) {
    const int tp = e / kC, c = e % kC;
    const int m = (tp / kK) * 8 + tp % kK;
    slab[e] = red[m * kC + c];
  }
}

// out[c·ocs + ooff + t] (=|+=) Σ_blocks slab[z][τ(t)][c]   (τ = tap mirror for the head form; ocs,
// ooff place the 32-channel side and the Q channel in dW[dn][gn][343])
// One block per tap: 8 groups of 32 lanes (lane = channel: 128 contiguous bytes per slab row),
// group g sums slabs z ≡ g (mod 8) in increasing z, then the 8 partials are added in g order —
// fixed order, deterministic.
__global__ void __launch_bounds__(256) thin1_wgrad_reduce_kernel(const float* __restrict__ slab, int nz, int flip,
                                                                 float* __restrict__ out, int ocs, int ooff,
                                                                 int accumulate) {
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
    const int64_t e = (int64_t)c * ocs + ooff + t;
    out[e] = accumulate ? out[e] + r : r;
  }
}

template <int PM, int P16>
static int launch_thin1w(const Thin1RWArgs& a, int grid, size_t lds, hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(thin1r_wgrad_kernel<PM, P16>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((thin1r_wgrad_kernel<PM, P16>), dim3(grid), dim3(512), lds, st, a);
  return check_launch(P16 ? "thin1_wgrad_x3(op16)" : "thin1_wgrad_x3");
}

// 2-channel single side (nc = 2) in the one-plane modes: one pass per channel of that side
bool thin1_wgrad_x3_applicable(int Cd, int Cg, int k, int s, int mode) {
  const bool one_plane = mode == kPrecBf16 || mode == kPrecF16;
  auto thin = [&](int c) { return c == 1 || (c == 2 && one_plane); };
  return k == kK && s == 1 && ((Cd == kC && thin(Cg)) || (thin(Cd) && Cg == kC));
}

size_t thin1_wgrad_x3_ws_bytes() { return (size_t)cu_count() * kT * kC * sizeof(float); }

// Same argument convention as conv_wgrad: dW[dn][gn][t] = Σ_m D[m][dn] · G[m − p + t][gn]
int conv_thin1_wgrad_x3(const float* D, int N, int Dd, int Hd, int Wd, int Cd, const float* G, int Dg, int Hg, int Wg,
                        int Cg, int p, float* out, int accumulate, int mode, void* ws, size_t ws_bytes, hipStream_t st,
                        int wide16) {
  MRAGAN_CHECK_ARG(!wide16 || mode == kPrecBf16 || mode == kPrecF16,
                   "thin1_wgrad_x3: a 16-bit operand plane needs the bf16 / fp16 mode");
  Thin1RWArgs a{};
  static const int stamps = getenv("MRAGAN_STAMPS") ? 1 : 0;
  a.stamp = stamps;
  int flip, nq, ocs, qstride;
  if (Cd == kC) {         // stem: P = D (32 ch), Q = G (Cg channels): dW[c][q][t]
    a.P = D; a.Dp = Dd; a.Hp = Hd; a.Wp = Wd;
    a.Q = G; a.Dq = Dg; a.Hq = Hg; a.Wq = Wg;
    a.pe = p; flip = 0;
    nq = Cg; ocs = Cg * kT; qstride = kT;
  } else {                // head: P = G (32 ch), Q = D (Cd channels), u = m − p + t: dW[q][c][t]
    a.P = G; a.Dp = Dg; a.Hp = Hg; a.Wp = Wg;
    a.Q = D; a.Dq = Dd; a.Hq = Hd; a.Wq = Wd;
    a.pe = kK - 1 - p; flip = 1;
    nq = Cd; ocs = kT; qstride = kC * kT;
  }
  MRAGAN_CHECK_ARG(nq == 1 || (nq == 2 && (mode == kPrecBf16 || mode == kPrecF16)),
                   "thin1_wgrad_x3: %d single-side channels in precision mode %d", nq, mode);
  a.N = N;
  a.qC = nq;
  MRAGAN_CHECK_ARG((int64_t)a.Dp * a.Hp * a.Wp * kC * (wide16 ? 2 : 4) < (int64_t)kOobOffset &&
                       (int64_t)a.Dq * a.Hq * a.Wq * nq * 4 < (int64_t)kOobOffset,
                   "thin1_wgrad_x3: volume too large");
  a.nbh = ceil_div(a.Hp, kBH); a.nbw = ceil_div(a.Wp, kBW);
  const int64_t columns = (int64_t)N * a.nbh * a.nbw;
  int grid = 1;
  if (columns > 0 && a.Dp > 0) pick_chunk(columns, a.Dp, cu_count(), a.L, a.nch, grid);
  else { a.L = 1; a.nch = 0; }
  a.items = (int)(columns * a.nch);
  const size_t need = (size_t)grid * kT * kC * sizeof(float);
  if (!ws || ws_bytes < need) {
    set_error("thin1_wgrad_x3: workspace %zu < %zu", ws_bytes, need);
    return kWorkspace;
  }
  a.slab = static_cast<float*>(ws);
  const size_t lds = (size_t)2 * kRing * kPlaneE * 16 + (size_t)2 * 2 * kC * kPS * sizeof(__bf16);
  static_assert(kMT * 32 * kC * 4 <= 2 * kRing * kPlaneE * 16, "the wave reduction fits the ring");
  static_assert(kC * 8 == 256, "reduce block = 8 groups of kC lanes");
  // one pass per channel of the single side (nc = 2: the 32-channel operand is read twice; the
  // slabs are reused, stream-ordered)
  for (int qc = 0; qc < nq; ++qc) {
    a.qc = qc;
    int rc = kOk;
    if (wide16) {
      rc = mode == kPrecF16 ? launch_thin1w<kPrecF16, 1>(a, grid, lds, st) : launch_thin1w<kPrecBf16, 1>(a, grid, lds, st);
    } else {
      MRAGAN_PREC_DISPATCH(mode, {
        rc = launch_thin1w<PM, 0>(a, grid, lds, st);
        break;
      })
    }
    if (rc) return rc;
    hipLaunchKernelGGL(thin1_wgrad_reduce_kernel, dim3(kT), dim3(256), 0, st, a.slab, grid, flip, out, ocs,
                       qc * qstride, accumulate);
    rc = check_launch("thin1_wgrad_reduce");
    if (rc) return rc;
  }
  return kOk;
}

}  // namespace mragan
