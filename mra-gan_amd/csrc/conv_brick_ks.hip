// K-split brick convolution for the one-plane modes (bf16 / fp16), gfx950: the ResnetBlock k3 s1
// convolutions (reference networks3D.py:241-243, 256-257: ReplicationPad3d(1) → Conv3d(4ngf, 4ngf,
// k3) twice per block) and their data gradients, when the contraction has a multiple of 128
// channels (ngf = 32: 128).
//
// Why a second brick kernel (profiles/r03w): conv_brick_x3 splits a 128×64
// output tile over its 4 waves by rows and columns (64×32 per wave).  In the one-plane modes a
// K-step is one MFMA per 32×32 tile, so every wave streams a 1 KB weight fragment from L1 per one
// or two MFMAs: at the MFMA rate that is 64–128 B/clk/CU against an L1 → SIMD return of ≈ 64, and
// the waves park on it (42 % of their cycles parked, 32 % issue-stalled, MFMA 0.15–0.24 of peak).
//
// Here the 4 waves split the CONTRACTION instead: wave w owns the channels [32w, 32w + 32) (+128
// per further chunk) of every tap, and the WHOLE 128 × BN output tile.  Per K-step (one tap × 16
// channels) a wave issues 4 × TN MFMAs from 4 A fragments (LDS) and TN B fragments (L1/L2): each
// weight byte is used by 128 output rows and each halo byte by BN columns.  The price is a 4-way
// reduction of the fp32 tiles through LDS after the main loop.
//
// No block barrier inside the main loop: a wave's halo is its own, and LDS executes one wave's
// instructions in order.  Halo rows are an odd number of 16-B slots (brick_row_perm's conflict-free
// A-read assignment).  The halo streams in half-chunks of 16 channels; the next half-chunk's
// slices are loaded during the current half's taps:
//   DB = 1: two half-slots per row (80-B rows, 128 KB per block, ONE block per CU): the slices are
//           stored into the idle half-slot kHD steps after their load;
//   DB = 0: one half-slot (48-B rows, 77 KB per block, TWO blocks per CU, ≤ 256 registers): the
//           slices wait in registers and are stored right after the half's last A reads — the
//           co-resident block's MFMAs cover this block's prologue, boundaries and epilogue
//           (tools/diag_ks.py phase stamps, r04b: with one block per CU the table set-up,
//           prologue, reduction and epilogue were 54 % of a wave's cycles).
// Weights are the pre-split fragment-order copy (brick_x3_pack / tr 2/3 packs: [tap][chunk][16-ch
// half][hi|lo][n][8-ch group][8]) through a buffer descriptor with wave-uniform per-step offsets,
// kPF steps ahead.
//
// Epilogue: wave w sums rows 32w … over the 4 waves' partials (order p0 + p1 + p2 + p3:
// deterministic, and the same for the fp32-input and the operand-plane input X16, so the two stay
// bit-identical — tests/test_kernels_gpu.py::test_op16_brick_conv_and_wgrad), then transposes each
// 4×4 block of its accumulator within lane quads (DPP) so that a lane holds 4 consecutive channels
// of one voxel: 16-B output stores (the 4-B column stores of the MFMA layout were store-issue bound:
// 11.8 k cycles of a 48 k-cycle wave, r04b) and 16-B loads of the backward-statistics operand.
#include "conv_geo.h"
#include "in_ticket.h"
#include "kernels.h"
#include "prec.h"
#include "lane_ops.h"

#include <cstdlib>
#include <type_traits>

// build-time knobs of the two-blocks-per-CU variant (≤ 256 registers): weight prefetch distance and
// A-fragment read distance, in steps (divisors of 27 and 27 / (kAD + 1) integral)
#ifndef MRAGAN_KS_PF0
#define MRAGAN_KS_PF0 3
#endif
#ifndef MRAGAN_KS_AD0
#define MRAGAN_KS_AD0 2
#endif

namespace mragan {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kTaps = 27;
constexpr int kKsBM = 128;    // GEMM rows per block (4 fragment rows of 32)
constexpr int kKsHmax = 400;  // halo positions per wave

template <int DB>
constexpr int ks_row_bytes() { return DB ? 80 : 48; }
constexpr size_t ks_tables_bytes() { return (size_t)(2 * kKsBM) * sizeof(int); }
template <int TN, int DB>
constexpr size_t ks_region_bytes() {
  // halos [4 waves][HMAX][row], later the reduction [4 tiles][4 waves][TN][4 quads][64 lanes] × 16 B
  return (size_t)4 * kKsHmax * ks_row_bytes<DB>() > (size_t)TN * 65536 ? (size_t)4 * kKsHmax * ks_row_bytes<DB>()
                                                                          : (size_t)TN * 65536;
}

// a double from the lane given by the DPP quad permutation CTRL (two 32-bit moves)
template <int CTRL>
__device__ __forceinline__ double dpp_xor_d(double x) {
  const uint64_t u = __builtin_bit_cast(uint64_t, x);
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

}  // namespace

// diagnostic stamps (MRAGAN_STAMPS=1): s_memtime per wave at entry / first half-chunk issued / tables
// ready / prologue done / main loop done / reduction done / exit — 8 slots per wave, 4 waves per
// block (mragan_debug_stamps, n < 0)
constexpr int kKsStampBlocks = 1024;
__device__ unsigned long long g_ks_stamps[kKsStampBlocks * 32];
#define KS_STAMP(i)                                                                                   \
  do {                                                                                                \
    if (a.stamp && lane == 0 && blockIdx.x < kKsStampBlocks)                                          \
      g_ks_stamps[blockIdx.x * 32 + wave * 8 + (i)] = __builtin_amdgcn_s_memtime();                   \
  } while (0)

template <int TN, int DB, int PM, int X16>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DB ? 1 : 2, DB ? 1 : 2)))
conv_brick_ks_kernel(BrickArgs a) {
  static_assert(!prec::has_lo<PM>(), "the K-split brick runs the one-plane modes");
  constexpr int TM = 4, BM = kKsBM, BN = TN * 32, HMAX = kKsHmax;
  constexpr int kRowB = ks_row_bytes<DB>();
  constexpr int ES = X16 ? 2 : 4;                   // bytes per input element
  constexpr int SPP = X16 ? 2 : 4;                  // 16-B global slices per position per half-chunk
  constexpr int CPS = 16 / SPP;                     // channels per slice
  constexpr int NSL = (HMAX * SPP + 63) / 64;       // slices per lane per half-chunk
  constexpr int LPS = X16 ? 1 : 2;                  // slices loaded per step
  constexpr int NLD = (NSL + LPS - 1) / LPS;        // steps that load
  constexpr int kHalf = kTaps;                      // steps per half-chunk (one tap each)
  // a slice is stored (DB) or packed into its staging register (DB = 0) kHD steps after its load
  constexpr int kHD = (X16 && DB) ? 8 : 2;
  constexpr int kPF = DB ? 9 : MRAGAN_KS_PF0;       // weight prefetch distance (steps)
  constexpr int kAD = DB ? 2 : MRAGAN_KS_AD0;       // A-fragment read distance (steps)
  static_assert(!DB || NLD + kHD <= kHalf, "halo stream does not fit a half-chunk");
  static_assert(DB || NLD + kHD <= kHalf - kAD, "halo stream does not fit a half-chunk");
  static_assert(kHalf % kPF == 0 && kHalf % (kAD + 1) == 0 && kHalf % (kHD + 1) == 0, "ring periods");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* out_off = reinterpret_cast<int*>(smem);      // [BM]
  int* xoff = out_off + BM;                         // [BM] (backward statistics)
  char* region = smem + ks_tables_bytes();          // halos, then the K reduction

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  KS_STAMP(0);

  // Small non-negative quotients (< 2^22 / divisor) through an fp32 reciprocal: (n + ½)·(1/d) lies
  // ≥ ½/d away from an integer and the product's relative error is ~2^-23, so the truncation is
  // exact here (every index below is < 2^20).  Replaces ~30-instruction integer divisions: the
  // block set-up (tables + prologue) took 9 k cycles of a 35 k-cycle wave (r04c phase stamps).
  auto qdiv = [](int n, float rd) __attribute__((always_inline)) { return (int)(((float)n + 0.5f) * rd); };

  // tile → (instance, brick, n-block); XCD-aware order (n fastest, then bricks)
  int L = blockIdx.x, tile = L;
  if ((a.ntiles & 7) == 0) tile = (L & 7) * (a.ntiles >> 3) + (L >> 3);
  const int nbk = tile % a.gn;
  int rest = tile / a.gn;
  const int bw_i = rest % a.nbw; rest /= a.nbw;
  const int bh_i = rest % a.nbh; rest /= a.nbh;
  const int bd_i = rest % a.nbd;
  const int nb = rest / a.nbd;
  const int od0 = bd_i * a.BD, oh0 = bh_i * a.BH, ow0 = bw_i * a.BW;
  const int n0 = nbk * BN;
  const int HP = a.HD * a.HH * a.HW;
  const float r_hw = 1.f / (float)a.HW, r_hplane = 1.f / (float)(a.HW * a.HH);
  const float r_bw = 1.f / (float)a.BW, r_bplane = 1.f / (float)(a.BW * a.BH);

  char* Hw = region + wave * (HMAX * kRowB);
  const int nch = __builtin_amdgcn_readfirstlane(a.C / 32);
  const int nck = __builtin_amdgcn_readfirstlane(a.C / 128);     // chunks of this wave: wave + 4k
  const int flip = __builtin_amdgcn_readfirstlane(a.flip);
  const int HH = __builtin_amdgcn_readfirstlane(a.HH), HWd = __builtin_amdgcn_readfirstlane(a.HW);
  const int blkb = a.ny * 16 * 2;                   // bytes of one (hi|lo) fragment block
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(reinterpret_cast<const char*>(a.x) + (int64_t)nb * a.Di * a.Hi * a.Wi * a.C * ES,
                                              (uint32_t)a.Di * a.Hi * a.Wi * a.C * (uint32_t)ES);
  // this lane's halo slices (the same positions for every half-chunk): element offset or −1,
  // computed per lane so that the first half-chunk's loads leave before anything else
  int ho[NSL];
#pragma unroll
  for (int sl = 0; sl < NSL; ++sl) {
    const int pos = (sl * 64 + lane) / SPP;
    const int hd = qdiv(pos, r_hplane), rem = pos - hd * a.HW * a.HH;
    const int hh = qdiv(rem, r_hw), hw = rem - hh * a.HW;
    const int id = od0 - a.p + hd, ih = oh0 - a.p + hh, iw = ow0 - a.p + hw;
    const bool ok = pos < HP && (unsigned)id < (unsigned)a.Di && (unsigned)ih < (unsigned)a.Hi && (unsigned)iw < (unsigned)a.Wi;
    ho[sl] = ok ? ((id * a.Hi + ih) * a.Wi + iw) * a.C : -1;
  }
  // half-chunk g = 2k + h (chunk k of this wave, half h): channels (wave + 4k)·32 + 16h …, LDS
  // half-slot h (DB) or the only slot (DB = 0)
  auto halo_ld = [&](int g, int sl) __attribute__((always_inline)) -> float4 {
    const int e = sl * 64 + lane;
    const int o = ho[sl];
    const int cb = (wave + 4 * (g >> 1)) * 32 + 16 * (g & 1);
    return buf_load_f32x4(xr, o < 0 ? kOobOffset : (uint32_t)(o + cb + CPS * (e % SPP)) * (uint32_t)ES);
  };
  // the first half-chunk's slices, in flight through the table set-up (one batch of ≤ kPB)
  constexpr int kPB = NSL < 13 ? NSL : 13;
  float4 pv0[kPB];
#pragma unroll
  for (int sl = 0; sl < kPB; ++sl) pv0[sl] = halo_ld(0, sl);
  KS_STAMP(1);

  for (int r = tid; r < BM; r += 256) {
    int off = -1;
    const int v = a.rowvox[r];
    if (v >= 0) {
      const int bd = qdiv(v, r_bplane), bh = qdiv(v - bd * a.BW * a.BH, r_bw), bw = v - (bd * a.BH + bh) * a.BW;
      const int od = od0 + bd, oh = oh0 + bh, ow = ow0 + bw;
      if (od < a.Do && oh < a.Ho && ow < a.Wo) {
        off = (int)((((int64_t)nb * a.Yd + od + a.ye) * a.Yh + oh + a.ye) * a.Yw + ow + a.ye);
        if (a.sx) {   // backward statistics: the interior voxel this padded output folds into
          const int cd = min(max(od - 1, 0), a.Do - 3), ch = min(max(oh - 1, 0), a.Ho - 3),
                    cw = min(max(ow - 1, 0), a.Wo - 3);
          xoff[r] = (int)((((int64_t)nb * (a.Do - 2) + cd) * (a.Ho - 2) + ch) * (a.Wo - 2) + cw);
          // bit 30: the padded output is the interior voxel's own (no clamp) — where sadd joins
          if (od >= 1 && od <= a.Do - 2 && oh >= 1 && oh <= a.Ho - 2 && ow >= 1 && ow <= a.Wo - 2) xoff[r] |= 1 << 30;
        }
      }
    }
    out_off[r] = off;
  }
  // A: byte offset of each fragment row in this wave's halo (tap 0, this lane's 8-channel half)
  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int v = a.rowvox[i * 32 + li];
    if (v < 0) v = -v - 1;
    const int bd = qdiv(v, r_bplane), bh = qdiv(v - bd * a.BW * a.BH, r_bw), bw = v - (bd * a.BH + bh) * a.BW;
    abase[i] = ((bd * a.HH + bh) * a.HW + bw) * kRowB + lh * 16;
  }
  // B: the pre-split weights through a descriptor (lane part fixed, step part wave-uniform)
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.wx3, (uint32_t)kTaps * a.C * a.ny * 4);
  int boff[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) boff[j] = ((n0 + j * 32 + li) * 16 + lh * 8) * 2;
  __syncthreads();
  KS_STAMP(2);

  // a loaded slice in its LDS format: the 16 B of a plane as they are, or 4 fp32 → 4 16-bit words
  typedef typename std::conditional<X16, f32x4v, uint2>::type Packed;
  auto halo_pack = [&](const float4& v) __attribute__((always_inline)) -> Packed {
    if constexpr (X16) {
      return f32x4v{v.x, v.y, v.z, v.w};
    } else {
      uint2 hi, lo;
      prec::split4<PM>(v, hi, lo);
      return hi;
    }
  };
  auto halo_put = [&](int g, int sl, const Packed& v) __attribute__((always_inline)) {
    const int e = sl * 64 + lane, pos = e / SPP;
    if (pos < HP) {
      char* row = Hw + pos * kRowB + (DB ? 32 * (g & 1) : 0);
      *reinterpret_cast<Packed*>(row + (X16 ? 16 : 8) * (e % SPP)) = v;
    }
  };
  auto halo_st = [&](int g, int sl, const float4& v) __attribute__((always_inline)) { halo_put(g, sl, halo_pack(v)); };
  // Per-step offsets are built from strides made opaque to the compiler once per step (an empty
  // asm on SGPR copies): left alone, LICM hoists all 27 taps' offsets out of the half-chunk loop
  // and the SGPR file overflows (spills to VGPR lanes and a scratch frame).
  const int tstride = flip ? -nch * 4 * blkb : nch * 4 * blkb;     // weight bytes per tap
  const int tbase = flip ? (kTaps - 1) * nch * 4 * blkb : 0;
  const int wgb = wave * 4 * blkb;                                    // this wave's chunk, half 0
  const int pstride = HH * HWd * kRowB, rstride = HWd * kRowB;       // halo bytes per d / h tap
  auto b_load = [&](int g, int t, bf16x8 (&dst)[TN]) __attribute__((always_inline)) {
    int ts = tstride, tb = tbase;
    asm volatile("" : "+s"(ts), "+s"(tb));
    const int sb = tb + t * ts + wgb + (g >> 1) * 16 * blkb + (g & 1) * 2 * blkb;
#pragma unroll
    for (int j = 0; j < TN; ++j) dst[j] = __builtin_bit_cast(bf16x8, buf_load_16b(wr, boff[j], sb));
  };
  auto a_read = [&](int g, int t, bf16x8 (&dst)[TM]) __attribute__((always_inline)) {
    int ps = pstride, rs = rstride;
    asm volatile("" : "+s"(ps), "+s"(rs));
    const int tap_off = (t / 9) * ps + ((t / 3) % 3) * rs + (t % 3) * kRowB + (DB ? (g & 1) * 32 : 0);
#pragma unroll
    for (int i = 0; i < TM; ++i) dst[i] = *reinterpret_cast<const bf16x8*>(Hw + abase[i] + tap_off);
  };

  // prologue: the weights of the first kPF steps, then half-chunk 0 (its first batch has been in
  // flight since the kernel began), the A fragments of the first kAD steps
  bf16x8 rb[kPF][TN];
#pragma unroll
  for (int u = 0; u < kPF; ++u) b_load(0, u, rb[u]);
#pragma unroll
  for (int sl = 0; sl < kPB; ++sl) halo_st(0, sl, pv0[sl]);
#pragma unroll
  for (int s0 = kPB; s0 < NSL; s0 += kPB) {
    float4 pv[kPB];
#pragma unroll
    for (int sl = 0; sl < kPB; ++sl)
      if (s0 + sl < NSL) pv[sl] = halo_ld(0, s0 + sl);
#pragma unroll
    for (int sl = 0; sl < kPB; ++sl)
      if (s0 + sl < NSL) halo_st(0, s0 + sl, pv[sl]);
  }
  bf16x8 af[kAD + 1][TM];
#pragma unroll
  for (int v = 0; v < kAD; ++v) a_read(0, v, af[v]);

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  KS_STAMP(3);
  // one loop iteration = one half-chunk (27 taps, unrolled: ring slots are compile-time because 9
  // and 3 divide 27); the next half-chunk streams in meanwhile
  const int nhalf = 2 * nck;
  for (int g = 0; g < nhalf; ++g) {
    const bool next = g + 1 < nhalf;
    const int gn = next ? g + 1 : g;          // past the last half: harmless re-reads, no stores
    constexpr int kRing = kHD + 1;
    float4 rh[kRing][LPS];
    Packed stg[DB ? 1 : NSL];                 // DB = 0: the next half-chunk, packed, until its store
#pragma unroll
    for (int t = 0; t < kHalf; ++t) {
      __builtin_amdgcn_sched_barrier(0);
      if (t < NLD && next) {
#pragma unroll
        for (int l = 0; l < LPS; ++l)
          if (t * LPS + l < NSL) rh[t % kRing][l] = halo_ld(gn, t * LPS + l);
      }
      if (t >= kHD && t - kHD < NLD && next) {
#pragma unroll
        for (int l = 0; l < LPS; ++l) {
          const int sl = (t - kHD) * LPS + l;
          if (sl < NSL) {
            if constexpr (DB) halo_st(gn, sl, rh[(t - kHD) % kRing][l]);
            else stg[sl] = halo_pack(rh[(t - kHD) % kRing][l]);
          }
        }
      }
      if constexpr (!DB) {
        // one slot: the next half-chunk overwrites it once this half's last A reads are issued
        // (they were, kAD steps ago: LDS runs this wave's instructions in order)
        if (t == kHalf - kAD && next) {
#pragma unroll
          for (int sl = 0; sl < NSL; ++sl) halo_put(gn, sl, stg[sl]);
        }
      }
      // B fragments of this step (loaded kPF steps ago); refill the slot with step + kPF
      bf16x8 bc[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) bc[j] = rb[t % kPF][j];
      if (t + kPF < kHalf) b_load(g, t + kPF, rb[t % kPF]);
      else b_load(gn, t + kPF - kHalf, rb[t % kPF]);
      // A fragments kAD steps ahead (into the next half-chunk near the end: stored by then)
      if (t + kAD < kHalf) a_read(g, t + kAD, af[(t + kAD) % (kAD + 1)]);
      else a_read(gn, t + kAD - kHalf, af[(t + kAD) % (kAD + 1)]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const bf16x8& A = af[t % (kAD + 1)][i];
          acc[i][j] = prec::mma<PM>(A, A, bc[j], bc[j], acc[i][j]);
        }
    }
  }

  KS_STAMP(4);
  // The epilogue's operands are loaded before the reduction so that their latency hides under it.
  // After the 4×4 quad transposes lane (li = 4m + k, lh) holds voxel row 32w + 8q + 4lh + k,
  // channels n0 + 32j + 4m … 4m + 3 (q = 0 … 3).
  const int k4 = li & 3, m4 = li >> 2;
  int orow[4], xrow[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = wave * 32 + 8 * q + 4 * lh + k4;
    orow[q] = out_off[row];
    xrow[q] = a.sx ? xoff[row] : 0;
  }
  float4 bq[TN], mu[TN], rsd[TN], xs[TN][4], xa[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int c0 = n0 + j * 32 + 4 * m4;
    bq[j] = a.bias ? *reinterpret_cast<const float4*>(a.bias + c0) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.sx) {
      mu[j] = *reinterpret_cast<const float4*>(a.smean + nb * a.ny + c0);
      rsd[j] = *reinterpret_cast<const float4*>(a.srstd + nb * a.ny + c0);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t xi = (int64_t)(xrow[q] & ((1 << 30) - 1)) * a.ny + c0;
        xs[j][q] = orow[q] >= 0 ? *reinterpret_cast<const float4*>(a.sx + xi) : make_float4(0.f, 0.f, 0.f, 0.f);
        xa[j][q] = (a.sadd && orow[q] >= 0 && (xrow[q] >> 30)) ? *reinterpret_cast<const float4*>(a.sadd + xi)
                                                               : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
  // K reduction: every wave leaves the partials of the three fragment rows it does not finish
  // (float4 quads, lane-contiguous: conflict-free 16-B stores / loads); wave w then sums rows
  // 32w … 32w + 31 over the waves in order 0, 1, 2, 3
  __syncthreads();
  f32x4v* red = reinterpret_cast<f32x4v*>(region);
  auto red_idx = [&](int i, int src, int j, int q) { return (((i * 4 + src) * TN + j) * 4 + q) * 64 + lane; };
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    if (i != wave) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        red[red_idx(i, wave, j, 0)] = __builtin_shufflevector(acc[i][j], acc[i][j], 0, 1, 2, 3);
        red[red_idx(i, wave, j, 1)] = __builtin_shufflevector(acc[i][j], acc[i][j], 4, 5, 6, 7);
        red[red_idx(i, wave, j, 2)] = __builtin_shufflevector(acc[i][j], acc[i][j], 8, 9, 10, 11);
        red[red_idx(i, wave, j, 3)] = __builtin_shufflevector(acc[i][j], acc[i][j], 12, 13, 14, 15);
      }
    }
  }
  f32x16 own[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) own[j] = acc[0][j];
#pragma unroll
  for (int i = 1; i < TM; ++i)
    if (i == wave) {
#pragma unroll
      for (int j = 0; j < TN; ++j) own[j] = acc[i][j];
    }
  __syncthreads();
  // fin[j][q]: quad q of column tile j — rows 8q + 4lh + {0..3}, column j·32 + li
  f32x4v fin[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) fin[j][q] = f32x4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int src = 0; src < 4; ++src) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (src == wave) {
        fin[j][0] += __builtin_shufflevector(own[j], own[j], 0, 1, 2, 3);
        fin[j][1] += __builtin_shufflevector(own[j], own[j], 4, 5, 6, 7);
        fin[j][2] += __builtin_shufflevector(own[j], own[j], 8, 9, 10, 11);
        fin[j][3] += __builtin_shufflevector(own[j], own[j], 12, 13, 14, 15);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) fin[j][q] += red[red_idx(wave, src, j, q)];
      }
    }
  }

  KS_STAMP(5);
  // epilogue: bias / activation or the backward-statistics operand, 16-B stores, per-lane fp64
  // statistics over its 4 voxels per channel
  double ps[TN][4], pq[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int c0 = n0 + j * 32 + 4 * m4;
    const float muv[4] = {mu[j].x, mu[j].y, mu[j].z, mu[j].w}, rsv[4] = {rsd[j].x, rsd[j].y, rsd[j].z, rsd[j].w};
    const float bv[4] = {bq[j].x, bq[j].y, bq[j].z, bq[j].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) ps[j][e] = pq[j][e] = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x4v t = quad_transpose(fin[j][q], k4);
      if (orow[q] < 0) continue;
      float v[4] = {t[0], t[1], t[2], t[3]};
      if (!a.sx) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = act_fwd(v[e] + bv[e], a.act);
          ps[j][e] += v[e];
          pq[j][e] += (double)v[e] * v[e];
        }
      } else {
        const float xv[4] = {xs[j][q].x, xs[j][q].y, xs[j][q].z, xs[j][q].w};
        const float av[4] = {xa[j][q].x, xa[j][q].y, xa[j][q].z, xa[j][q].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float xh = (xv[e] - muv[e]) * rsv[e];
          const float gin = v[e] + av[e];    // + 0 where no skip gradient joins: the same float
          const float gv = (a.sact == kActRelu && !(xh > 0.f)) ? 0.f : (a.sact == kActLrelu && !(xh > 0.f)) ? gin * kLreluSlope : gin;
          ps[j][e] += gv;
          pq[j][e] += (double)gv * xh;
        }
      }
      *reinterpret_cast<f32x4v*>(a.y + (int64_t)orow[q] * a.ny + c0) = f32x4v{v[0], v[1], v[2], v[3]};
    }
  }
  if (a.part) {
    // lanes k = 0 … 3 of a quad hold the same channels: sum over k by DPP (xor 1, 2 — two 32-bit
    // moves per double), then over the lane halves and the 4 waves through LDS, one double2 per
    // channel
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        ps[j][e] += dpp_xor_d<0xB1>(ps[j][e]);
        pq[j][e] += dpp_xor_d<0xB1>(pq[j][e]);
        ps[j][e] += dpp_xor_d<0x4E>(ps[j][e]);
        pq[j][e] += dpp_xor_d<0x4E>(pq[j][e]);
      }
    __syncthreads();
    double* red2 = reinterpret_cast<double*>(region);        // [4 waves][2 halves][BN][2]
    if (k4 == 0) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = j * 32 + 4 * m4 + e;
          red2[((wave * 2 + lh) * BN + c) * 2] = ps[j][e];
          red2[((wave * 2 + lh) * BN + c) * 2 + 1] = pq[j][e];
        }
    }
    __syncthreads();
    const int chunks = a.nbd * a.nbh * a.nbw;
    const int brick = (bd_i * a.nbh + bh_i) * a.nbw + bw_i;
    for (int c = tid; c < BN; c += 256) {
      double s2 = 0.0, q2 = 0.0;
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        s2 += red2[(w * BN + c) * 2];
        q2 += red2[(w * BN + c) * 2 + 1];
      }
      double* dst = a.part + (((int64_t)nb * chunks + brick) * a.ny + n0 + c) * 2;
      if (a.tick) {                     // write-through: the tile's reducer reads them (in_ticket.h)
        st_sc1(dst, s2);
        st_sc1(dst + 1, q2);
      } else {
        dst[0] = s2;
        dst[1] = q2;
      }
    }
    // ABI 15: the last block of this (instance, column tile) finalizes the tile's statistics
    if (a.tick && in_ticket_draw(a.tick + nb * a.gn + nbk, chunks, reinterpret_cast<int*>(region)))
      in_ticket_reduce<BN>(a.part, chunks, a.ny, nb, n0, a.fin_mode, a.fin_S, a.fin0, a.fin1);
  }
  KS_STAMP(6);
}

template <int TN, int DB, int PM, int X16>
static int launch_brick_ks_as(const BrickArgs& a, hipStream_t st) {
  const size_t lds = ks_tables_bytes() + ks_region_bytes<TN, DB>();
  auto kern = conv_brick_ks_kernel<TN, DB, PM, X16>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(a.ntiles), dim3(256), lds, st, a);
  return check_launch(X16 ? "conv_brick_ks(op16)" : "conv_brick_ks");
}

template <int PM>
static int brick_ks_launch_pm(BrickArgs a, int tn, int db, void* ws, size_t ws_bytes, const void* wsplit, hipStream_t st) {
  if constexpr (prec::has_lo<PM>()) {
    set_error("conv_brick_ks: the K-split brick runs the bf16 / fp16 modes only");
    return kBadArg;
  } else {
    if (wsplit) {
      a.wx3 = wsplit;
    } else {
      const size_t need = conv_brick_x3_ws_bytes(a.C, a.ny);
      if (!ws || ws_bytes < need) {
        set_error("conv_brick_ks: workspace %zu < %zu", ws_bytes, need);
        return kWorkspace;
      }
      const int rc = brick_x3_pack(a.w, a.ny, a.C, ws, PM, st);
      if (rc) return rc;
      a.wx3 = ws;
    }
    if (tn == 2 && db) return a.x16 ? launch_brick_ks_as<2, 1, PM, 1>(a, st) : launch_brick_ks_as<2, 1, PM, 0>(a, st);
    if (db) return a.x16 ? launch_brick_ks_as<1, 1, PM, 1>(a, st) : launch_brick_ks_as<1, 1, PM, 0>(a, st);
    // the fp32-input form of the two-per-CU variant would not fit 256 registers: it runs one per CU
    // (same per-element summation order — bit-identical results)
    return a.x16 ? launch_brick_ks_as<1, 0, PM, 1>(a, st) : launch_brick_ks_as<1, 1, PM, 0>(a, st);
  }
}

bool conv_brick_ks_applicable(const IgemmArgs& g) {
  static const bool off = [] {
    const char* e = getenv("MRAGAN_BRICK_KS");
    return e && atoi(e) == 0;
  }();
  return !off && (g.x3 == kPrecBf16 || g.x3 == kPrecF16) && g.cx % 128 == 0 && g.ny % 32 == 0;
}

// Brick shape and variant: the fewest rounds of the CU slots (DB = 1: one block per CU; DB = 0, TN
// = 1: two) × the block's MFMA time (∝ TN), then the fewest GEMM rows computed, then conflict-free
// A reads, then the smallest halo.  Every shape keeps bh ≥ 4 and bw ≥ 6 (the partials bound in capi.hip) and a halo ≤ 400
// positions.  MRAGAN_BRICK_KS=1|2|3 forces the variant (1: TN 1 two per CU, 2: TN 1 one per CU,
// 3: TN 2 one per CU) for A/B.
int conv_brick_ks(BrickArgs a, int ny, void* ws, size_t ws_bytes, const void* wsplit, int mode, int* in_chunks,
                  hipStream_t st) {
  static const int shapes[][3] = {{4, 4, 8}, {2, 8, 8}, {3, 6, 6}, {2, 6, 9}, {3, 4, 8}, {5, 4, 6}, {2, 6, 8}, {4, 4, 6}};
  static const int force = [] {
    const char* e = getenv("MRAGAN_BRICK_KS");
    return e ? atoi(e) : 0;
  }();
  struct Var { int tn, db, per_cu; };
  static const Var vars[] = {{1, 0, 2}, {1, 1, 1}, {2, 1, 1}};
  int best_v = -1, best_s = -1;
  double best[5] = {1e30, 1e30, 1e30, 1e30, 1e30};
  for (int vi = 0; vi < 3; ++vi) {
    const Var& V = vars[vi];
    if (force >= 1 && force <= 3 && force - 1 != vi) continue;
    if (ny % (32 * V.tn)) continue;
    for (int s = 0; s < (int)(sizeof(shapes) / sizeof(shapes[0])); ++s) {
      const int* b = shapes[s];
      const int64_t bricks = (int64_t)a.N * ceil_div(a.Do, b[0]) * ceil_div(a.Ho, b[1]) * ceil_div(a.Wo, b[2]);
      const int64_t blocks = bricks * (ny / (32 * V.tn));
      const int64_t slots = 256 * V.per_cu;
      // a round costs about the same in every variant (r04c: fixed per-block costs dominate — one
      // TN-1 block per CU took as long as two co-resident ones)
      const double round_t = 2.0;
      // A-read bank conflicts: brick_row_perm deals each residue class (halo position mod 16) over
      // the 8 lane groups of a 128-row tile — conflict-free iff no class has more than 8 voxels
      // (3×6×6 in an 8×8 halo plane has 9 per class: 2-way on every read)
      int cnt[16] = {0}, worst = 0;
      for (int v = 0; v < b[0] * b[1] * b[2]; ++v) {
        const int bd = v / (b[1] * b[2]), bh = (v / b[2]) % b[1], bw = v % b[2];
        const int r = (((bd * (b[1] + 2) + bh) * (b[2] + 2) + bw) % 16);
        worst = ++cnt[r] > worst ? cnt[r] : worst;
      }
      const double conflict = worst > kKsBM / 16 ? 1.0 : 0.0;
      const double key[5] = {(double)((blocks + slots - 1) / slots) * round_t, (double)blocks * V.tn, conflict,
                             (double)(b[0] + 2) * (b[1] + 2) * (b[2] + 2), (double)vi};
      bool better = false;
      for (int q = 0; q < 5; ++q) {
        if (key[q] < best[q]) { better = true; break; }
        if (key[q] > best[q]) break;
      }
      if (better) {
        for (int q = 0; q < 5; ++q) best[q] = key[q];
        best_v = vi;
        best_s = s;
      }
    }
  }
  MRAGAN_CHECK_ARG(best_s >= 0, "conv_brick_ks: %d output channels are not a multiple of 32", ny);
  // more than one round of CU slots (the 18³ data gradient at N = 4: 864 blocks): the r03 brick's
  // 128×128 eight-wave tiles are faster there (30.0 vs 36.2 µs, r04c) — the caller falls back
  // Large grids (≥ 3 rounds: the 128³ / 96³ configurations' 34³ / 26³ data gradients) with the
  // backward-statistics epilogue run here all the same: the K-split brick's epilogue beats the
  // 8-wave brick's there (125.6 vs 135.7 µs at 2 × 32³ → 34³, r05z); A/B switch MRAGAN_KS_BIG=0
  static const bool ks_big = [] {
    const char* e = getenv("MRAGAN_KS_BIG");
    return !(e && atoi(e) == 0);
  }();
  const bool big_bs = ks_big && a.sx && best[0] >= 6.0;
  if (!force && best[0] > 2.0 && !big_bs) return kUnsupported;
  const int* b = shapes[best_s];
  // experiment (A/B switch MRAGAN_KS_SMALL_DB1=1): a grid of at most one block per CU in the
  // two-per-CU variant (N = 2 at 16³: 256 blocks) may be packed two to a CU by the dispatcher,
  // leaving half the CUs idle; the one-per-CU variant cannot be
  static const bool small_db1 = getenv("MRAGAN_KS_SMALL_DB1") != nullptr;
  if (small_db1 && !force && best_v == 0 &&
      (int64_t)a.N * ceil_div(a.Do, b[0]) * ceil_div(a.Ho, b[1]) * ceil_div(a.Wo, b[2]) * (ny / 32) <= 256)
    best_v = 1;
  const Var& V = vars[best_v];
  a.BD = b[0]; a.BH = b[1]; a.BW = b[2];
  a.HD = b[0] + 2; a.HH = b[1] + 2; a.HW = b[2] + 2;
  a.nbd = ceil_div(a.Do, b[0]); a.nbh = ceil_div(a.Ho, b[1]); a.nbw = ceil_div(a.Wo, b[2]);
  a.gn = ny / (32 * V.tn);
  const int64_t ntiles = (int64_t)a.N * a.nbd * a.nbh * a.nbw * a.gn;
  MRAGAN_CHECK_ARG(ntiles < ((int64_t)1 << 31), "conv_brick_ks: grid too large");
  a.ntiles = (int)ntiles;
  static const int stamps = getenv("MRAGAN_STAMPS") ? 1 : 0;
  a.stamp = stamps;
  if (in_chunks && a.part) *in_chunks = a.nbd * a.nbh * a.nbw;
  if (a.tick && !a.part) a.tick = nullptr;
  if (a.tick && a.finalized) *a.finalized = 1;   // the launch below finalizes (in_ticket.h)
  if (a.ntiles == 0) return kOk;
  brick_row_perm(a.BD, a.BH, a.BW, a.HH, a.HW, kKsBM, a.rowvox);
  MRAGAN_PREC_DISPATCH(mode, return brick_ks_launch_pm<PM>(a, V.tn, V.db, ws, ws_bytes, wsplit, st))
}

int ks_debug_stamps(unsigned long long* host, int n) {
  if (n > kKsStampBlocks * 32) n = kKsStampBlocks * 32;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ks_stamps), (size_t)n * 8) == hipSuccess ? kOk : kLaunch;
}

}  // namespace mragan
