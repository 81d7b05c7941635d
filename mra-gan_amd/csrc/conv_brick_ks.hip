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
// weight byte is used by 128 output rows (4 MFMAs) and each halo byte by BN columns — at the MFMA
// rate 32 B/clk/CU of weights from L1 (TN = 2) and 64 B/clk/CU of LDS reads (of 256).  The price
// is a 4-way reduction of the fp32 tiles through LDS after the main loop (≈ 10 % of it).
//
// No block barrier inside the main loop: a wave's halo is its own (HMAX positions × [16 ch | 16
// ch] bf16 + 16-B pad = 80 B rows, an odd count of 16-B slots so brick_row_perm's conflict-free
// A-read assignment holds), and LDS executes one wave's instructions in order.  The halo streams
// in half-chunks of 16 channels: while a wave's 27 taps run on one half-slot of every row, the
// next half-chunk's 16 channels are loaded into the other half-slot (loads at steps 0…, stored
// kHD steps later).  Weights are the pre-split fragment-order copy (brick_x3_pack / tr 2/3 packs:
// [tap][chunk][16-ch half][hi|lo][n][8-ch group][8]), read through a buffer descriptor with
// wave-uniform per-step offsets, kPF steps ahead.
//
// The result per output element is p0 + p1 + p2 + p3 over the waves' fp32 partials in that order
// (deterministic); the same order serves the fp32-input and the operand-plane input (X16), so the
// two stay bit-identical (tests/test_kernels_gpu.py::test_op16_brick_conv_and_wgrad).
#include "conv_geo.h"
#include "kernels.h"
#include "prec.h"

#include <cstdlib>

namespace mragan {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kTaps = 27;
constexpr int kRowB = 80;     // per-wave halo row: 2 half-slots of 16 channels × 2 B + 16-B pad
constexpr int kKsBM = 128;    // GEMM rows per block (4 fragment rows of 32)
constexpr int kKsHmax = 400;  // halo positions per wave

constexpr size_t ks_tables_bytes() { return (size_t)(2 * kKsBM + kKsHmax) * sizeof(int); }
template <int TN>
constexpr size_t ks_region_bytes() {
  // halos [4 waves][HMAX][80 B], later the reduction [4 tiles][4 waves][TN][4 quads][64 lanes] × 16 B
  return (size_t)4 * kKsHmax * kRowB > (size_t)TN * 65536 ? (size_t)4 * kKsHmax * kRowB : (size_t)TN * 65536;
}

}  // namespace

// diagnostic stamps (MRAGAN_STAMPS=1): s_memtime per wave at entry / tables ready / prologue done /
// main loop done / reduction done / exit — 6 per wave, 4 waves per block (mragan_debug_stamps, n < 0)
constexpr int kKsStampBlocks = 1024;
__device__ unsigned long long g_ks_stamps[kKsStampBlocks * 24];
#define KS_STAMP(i)                                                                                   \
  do {                                                                                                \
    if (a.stamp && lane == 0 && blockIdx.x < kKsStampBlocks)                                          \
      g_ks_stamps[blockIdx.x * 24 + wave * 6 + (i)] = __builtin_amdgcn_s_memtime();                   \
  } while (0)

template <int TN, int PM, int X16>
__global__ void __launch_bounds__(256) conv_brick_ks_kernel(BrickArgs a) {
  static_assert(!prec::has_lo<PM>(), "the K-split brick runs the one-plane modes");
  constexpr int TM = 4, BM = kKsBM, BN = TN * 32, HMAX = kKsHmax;
  constexpr int ES = X16 ? 2 : 4;                   // bytes per input element
  constexpr int SPP = X16 ? 2 : 4;                  // 16-B global slices per position per half-chunk
  constexpr int CPS = 16 / SPP;                     // channels per slice
  constexpr int NSL = (HMAX * SPP + 63) / 64;       // slices per lane per half-chunk
  constexpr int LPS = X16 ? 1 : 2;                  // slices loaded per step
  constexpr int NLD = (NSL + LPS - 1) / LPS;        // steps that load
  constexpr int kHalf = kTaps;                      // steps per half-chunk (one tap each)
  constexpr int kHD = X16 ? 8 : 2;                  // a slice is stored kHD steps after its load
  constexpr int kPF = 9;                            // weight prefetch distance (steps)
  constexpr int kAD = 2;                            // A-fragment read distance (steps)
  static_assert(NLD + kHD <= kHalf, "halo stream does not fit a half-chunk");
  static_assert(kHalf % kPF == 0 && kHalf % (kAD + 1) == 0 && kHalf % (kHD + 1) == 0, "ring periods");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* out_off = reinterpret_cast<int*>(smem);      // [BM]
  int* xoff = out_off + BM;                         // [BM] (backward statistics)
  int* hoff = xoff + BM;                            // [HMAX]
  char* region = smem + ks_tables_bytes();          // halos, then the K reduction

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  KS_STAMP(0);

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

  for (int r = tid; r < BM; r += 256) {
    int off = -1;
    const int v = a.rowvox[r];
    if (v >= 0) {
      const int bd = v / (a.BH * a.BW), bh = (v / a.BW) % a.BH, bw = v % a.BW;
      const int od = od0 + bd, oh = oh0 + bh, ow = ow0 + bw;
      if (od < a.Do && oh < a.Ho && ow < a.Wo) {
        off = (int)((((int64_t)nb * a.Yd + od + a.ye) * a.Yh + oh + a.ye) * a.Yw + ow + a.ye);
        if (a.sx) {   // backward statistics: the interior voxel this padded output folds into
          const int cd = min(max(od - 1, 0), a.Do - 3), ch = min(max(oh - 1, 0), a.Ho - 3),
                    cw = min(max(ow - 1, 0), a.Wo - 3);
          xoff[r] = (int)((((int64_t)nb * (a.Do - 2) + cd) * (a.Ho - 2) + ch) * (a.Wo - 2) + cw);
        }
      }
    }
    out_off[r] = off;
  }
  for (int pos = tid; pos < HMAX; pos += 256) {
    int o = -1;
    if (pos < HP) {
      const int hw = pos % a.HW, hh = (pos / a.HW) % a.HH, hd = pos / (a.HW * a.HH);
      const int id = od0 - a.p + hd, ih = oh0 - a.p + hh, iw = ow0 - a.p + hw;
      if ((unsigned)id < (unsigned)a.Di && (unsigned)ih < (unsigned)a.Hi && (unsigned)iw < (unsigned)a.Wi)
        o = ((id * a.Hi + ih) * a.Wi + iw) * a.C;
    }
    hoff[pos] = o;
  }
  // A: byte offset of each fragment row in this wave's halo (tap 0, this lane's 8-channel half)
  char* Hw = region + wave * (HMAX * kRowB);
  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int v = a.rowvox[i * 32 + li];
    if (v < 0) v = -v - 1;
    const int bd = v / (a.BH * a.BW), bh = (v / a.BW) % a.BH, bw = v % a.BW;
    abase[i] = ((bd * a.HH + bh) * a.HW + bw) * kRowB + lh * 16;
  }
  // B: the pre-split weights through a descriptor (lane part fixed, step part wave-uniform)
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.wx3, (uint32_t)kTaps * a.C * a.ny * 4);
  int boff[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) boff[j] = ((n0 + j * 32 + li) * 16 + lh * 8) * 2;
  const int nch = __builtin_amdgcn_readfirstlane(a.C / 32);
  const int nck = __builtin_amdgcn_readfirstlane(a.C / 128);     // chunks of this wave: wave + 4k
  const int flip = __builtin_amdgcn_readfirstlane(a.flip);
  const int HH = __builtin_amdgcn_readfirstlane(a.HH), HWd = __builtin_amdgcn_readfirstlane(a.HW);
  const int blkb = a.ny * 16 * 2;                   // bytes of one (hi|lo) fragment block
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(reinterpret_cast<const char*>(a.x) + (int64_t)nb * a.Di * a.Hi * a.Wi * a.C * ES,
                                              (uint32_t)a.Di * a.Hi * a.Wi * a.C * (uint32_t)ES);
  __syncthreads();
  KS_STAMP(1);

  // this lane's halo slices (the same positions for every half-chunk): element offset or −1
  int ho[NSL];
#pragma unroll
  for (int sl = 0; sl < NSL; ++sl) {
    const int e = sl * 64 + lane, pos = e / SPP;
    ho[sl] = pos < HP ? hoff[pos] : -1;
  }
  // half-chunk (chunk k of this wave, half h): channels (wave + 4k)·32 + 16h …, LDS half-slot h
  auto halo_ld = [&](int k, int h, int sl) __attribute__((always_inline)) -> float4 {
    const int e = sl * 64 + lane;
    const int o = ho[sl];
    const int cb = (wave + 4 * k) * 32 + 16 * h;
    return buf_load_f32x4(xr, o < 0 ? kOobOffset : (uint32_t)(o + cb + CPS * (e % SPP)) * (uint32_t)ES);
  };
  auto halo_st = [&](int h, int sl, const float4& v) __attribute__((always_inline)) {
    const int e = sl * 64 + lane, pos = e / SPP;
    if (pos < HP) {
      char* row = Hw + pos * kRowB + 32 * h;
      if constexpr (X16) {
        *reinterpret_cast<f32x4v*>(row + 16 * (e % SPP)) = f32x4v{v.x, v.y, v.z, v.w};
      } else {
        uint2 hi, lo;
        prec::split4<PM>(v, hi, lo);
        *reinterpret_cast<uint2*>(row + 8 * (e % SPP)) = hi;
      }
    }
  };
  // step (half-chunk g = 2k + h, tap t): weights of tap t (flipped for the transposed form), channels
  // 16h … of chunk wave + 4k; the A fragments of tap t in half-slot h of the halo rows
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
    const int tap_off = (t / 9) * ps + ((t / 3) % 3) * rs + (t % 3) * kRowB + (g & 1) * 32;
#pragma unroll
    for (int i = 0; i < TM; ++i) dst[i] = *reinterpret_cast<const bf16x8*>(Hw + abase[i] + tap_off);
  };

  // prologue: half-chunk 0 (all loads in flight before the first store), weights of the first
  // kPF steps, A fragments of the first kAD
  constexpr int kPB = 13;                           // prologue slices in flight per batch
#pragma unroll
  for (int s0 = 0; s0 < NSL; s0 += kPB) {
    float4 pv[kPB];
#pragma unroll
    for (int sl = 0; sl < kPB; ++sl)
      if (s0 + sl < NSL) pv[sl] = halo_ld(0, 0, s0 + sl);
#pragma unroll
    for (int sl = 0; sl < kPB; ++sl)
      if (s0 + sl < NSL) halo_st(0, s0 + sl, pv[sl]);
  }
  bf16x8 rb[kPF][TN];
#pragma unroll
  for (int u = 0; u < kPF; ++u) b_load(0, u, rb[u]);
  bf16x8 af[kAD + 1][TM];
#pragma unroll
  for (int v = 0; v < kAD; ++v) a_read(0, v, af[v]);

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  KS_STAMP(2);
  // one loop iteration = one half-chunk (27 taps, unrolled: ring slots are compile-time because 9
  // and 3 divide 27); the next half-chunk streams into the other half-slot meanwhile
  const int nhalf = 2 * nck;
  for (int g = 0; g < nhalf; ++g) {
    const bool next = g + 1 < nhalf;
    const int gn = next ? g + 1 : g;          // past the last half: harmless re-reads, no stores
    float4 rh[kHD + 1][LPS];
#pragma unroll
    for (int t = 0; t < kHalf; ++t) {
      __builtin_amdgcn_sched_barrier(0);
      if (t < NLD && next) {
#pragma unroll
        for (int l = 0; l < LPS; ++l)
          if (t * LPS + l < NSL) rh[t % (kHD + 1)][l] = halo_ld(gn >> 1, gn & 1, t * LPS + l);
      }
      if (t >= kHD && t - kHD < NLD && next) {
#pragma unroll
        for (int l = 0; l < LPS; ++l)
          if ((t - kHD) * LPS + l < NSL) halo_st(gn & 1, (t - kHD) * LPS + l, rh[(t - kHD) % (kHD + 1)][l]);
      }
      // B fragments of this step (loaded kPF steps ago); refill the slot with step + kPF
      bf16x8 bc[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) bc[j] = rb[t % kPF][j];
      if (t + kPF < kHalf) b_load(g, t + kPF, rb[t % kPF]);
      else b_load(gn, t + kPF - kHalf, rb[t % kPF]);
      // A fragments kAD steps ahead (into the next half-chunk's slot near the end: stored at
      // steps kHD … kHD + NLD − 1 of this half, before these reads)
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

  KS_STAMP(3);
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
      for (int j = 0; j < TN; ++j)
      {
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
  f32x16 fin[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) fin[j] = f32x16{};
#pragma unroll
  for (int src = 0; src < 4; ++src) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (src == wave) {
        fin[j] += own[j];
      } else {
        const f32x4v r0 = red[red_idx(wave, src, j, 0)], r1 = red[red_idx(wave, src, j, 1)],
                     r2 = red[red_idx(wave, src, j, 2)], r3 = red[red_idx(wave, src, j, 3)];
        const f32x8 r01 = __builtin_shufflevector(r0, r1, 0, 1, 2, 3, 4, 5, 6, 7);
        const f32x8 r23 = __builtin_shufflevector(r2, r3, 0, 1, 2, 3, 4, 5, 6, 7);
        fin[j] += __builtin_shufflevector(r01, r23, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
      }
    }
  }

  KS_STAMP(4);
  // epilogue on rows 32w + …: bias / activation, output store, InstanceNorm partials
  const int wm0 = wave * 32;
  double ps[TN], pq[TN];
  if (!a.sx) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + j * 32 + li;
      const float bsum = a.bias ? a.bias[col] : 0.f;
      ps[j] = 0.0;
      pq[j] = 0.0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm0 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const int off = out_off[row];
        if (off >= 0) {
          const float v = act_fwd(fin[j][r] + bsum, a.act);
          a.y[(int64_t)off * a.ny + col] = v;
          ps[j] += v;
          pq[j] += (double)v * v;
        }
      }
    }
  } else {
    // backward statistics of the InstanceNorm in front of this conv (see conv_brick_x3.hip)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + j * 32 + li;
      const float mu = a.smean[nb * a.ny + col], rs = a.srstd[nb * a.ny + col];
      ps[j] = 0.0;
      pq[j] = 0.0;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm0 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const int off = out_off[row];
        if (off >= 0) {
          const float v = fin[j][r];
          a.y[(int64_t)off * a.ny + col] = v;
          const float xh = (a.sx[(int64_t)xoff[row] * a.ny + col] - mu) * rs;
          const float gv = (a.sact == kActRelu && !(xh > 0.f)) ? 0.f : (a.sact == kActLrelu && !(xh > 0.f)) ? v * kLreluSlope : v;
          ps[j] += gv;
          pq[j] += (double)gv * xh;
        }
      }
    }
  }
  if (a.part) {
    __syncthreads();
    double* red2 = reinterpret_cast<double*>(region);        // [4 waves][BN][2]
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const double s2 = ps[j] + __shfl_xor(ps[j], 32);
      const double q2 = pq[j] + __shfl_xor(pq[j], 32);
      if (lh == 0) {
        red2[(wave * BN + j * 32 + li) * 2] = s2;
        red2[(wave * BN + j * 32 + li) * 2 + 1] = q2;
      }
    }
    __syncthreads();
    const int chunks = a.nbd * a.nbh * a.nbw;
    const int brick = (bd_i * a.nbh + bh_i) * a.nbw + bw_i;
    for (int c = tid; c < BN; c += 256) {
      double s2 = 0.0, q2 = 0.0;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        s2 += red2[(w * BN + c) * 2];
        q2 += red2[(w * BN + c) * 2 + 1];
      }
      double* dst = a.part + (((int64_t)nb * chunks + brick) * a.ny + n0 + c) * 2;
      dst[0] = s2;
      dst[1] = q2;
    }
  }
  KS_STAMP(5);
}

template <int TN, int PM, int X16>
static int launch_brick_ks_as(const BrickArgs& a, hipStream_t st) {
  const size_t lds = ks_tables_bytes() + ks_region_bytes<TN>();
  auto kern = conv_brick_ks_kernel<TN, PM, X16>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(a.ntiles), dim3(256), lds, st, a);
  return check_launch(X16 ? "conv_brick_ks(op16)" : "conv_brick_ks");
}

template <int PM>
static int brick_ks_launch_pm(BrickArgs a, int tn, void* ws, size_t ws_bytes, const void* wsplit, hipStream_t st) {
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
    if (tn == 2) return a.x16 ? launch_brick_ks_as<2, PM, 1>(a, st) : launch_brick_ks_as<2, PM, 0>(a, st);
    return a.x16 ? launch_brick_ks_as<1, PM, 1>(a, st) : launch_brick_ks_as<1, PM, 0>(a, st);
  }
}

bool conv_brick_ks_applicable(const IgemmArgs& g) {
  static const bool off = [] {
    const char* e = getenv("MRAGAN_BRICK_KS");
    return e && atoi(e) == 0;
  }();
  return !off && (g.x3 == kPrecBf16 || g.x3 == kPrecF16) && g.cx % 128 == 0 && g.ny % 32 == 0;
}

// Brick shape and column tile: the fewest rounds of 256 blocks (one block per CU: 131 KB of LDS)
// × the block's time (∝ TN), then the fewest GEMM rows computed, then the smallest halo.  Every
// shape keeps bh ≥ 4 and bw ≥ 6 (the partials bound in capi.hip) and a halo ≤ 400 positions.
int conv_brick_ks(BrickArgs a, int ny, void* ws, size_t ws_bytes, const void* wsplit, int mode, int* in_chunks,
                  hipStream_t st) {
  static const int shapes[][3] = {{4, 4, 8}, {2, 8, 8}, {3, 6, 6}, {2, 6, 9}, {3, 4, 8}, {5, 4, 6}, {2, 6, 8}, {4, 4, 6}};
  int best_tn = 0, best_s = -1;
  double best[4] = {1e30, 1e30, 1e30, 1e30};
  for (int tn = 2; tn >= 1; --tn) {
    if (ny % (32 * tn)) continue;
    for (int s = 0; s < (int)(sizeof(shapes) / sizeof(shapes[0])); ++s) {
      const int* b = shapes[s];
      const int64_t bricks = (int64_t)a.N * ceil_div(a.Do, b[0]) * ceil_div(a.Ho, b[1]) * ceil_div(a.Wo, b[2]);
      const int64_t blocks = bricks * (ny / (32 * tn));
      const double key[4] = {(double)((blocks + 255) / 256) * tn, (double)blocks * tn, (double)(b[0] + 2) * (b[1] + 2) * (b[2] + 2),
                             (double)blocks};
      bool better = false;
      for (int q = 0; q < 4; ++q) {
        if (key[q] < best[q]) { better = true; break; }
        if (key[q] > best[q]) break;
      }
      if (better) {
        for (int q = 0; q < 4; ++q) best[q] = key[q];
        best_tn = tn;
        best_s = s;
      }
    }
  }
  MRAGAN_CHECK_ARG(best_s >= 0, "conv_brick_ks: %d output channels are not a multiple of 32", ny);
  const int* b = shapes[best_s];
  a.BD = b[0]; a.BH = b[1]; a.BW = b[2];
  a.HD = b[0] + 2; a.HH = b[1] + 2; a.HW = b[2] + 2;
  a.nbd = ceil_div(a.Do, b[0]); a.nbh = ceil_div(a.Ho, b[1]); a.nbw = ceil_div(a.Wo, b[2]);
  a.gn = ny / (32 * best_tn);
  const int64_t ntiles = (int64_t)a.N * a.nbd * a.nbh * a.nbw * a.gn;
  MRAGAN_CHECK_ARG(ntiles < ((int64_t)1 << 31), "conv_brick_ks: grid too large");
  a.ntiles = (int)ntiles;
  static const int stamps = getenv("MRAGAN_STAMPS") ? 1 : 0;
  a.stamp = stamps;
  if (in_chunks && a.part) *in_chunks = a.nbd * a.nbh * a.nbw;
  if (a.ntiles == 0) return kOk;
  brick_row_perm(a.BD, a.BH, a.BW, a.HH, a.HW, kKsBM, a.rowvox);
  MRAGAN_PREC_DISPATCH(mode, return brick_ks_launch_pm<PM>(a, best_tn, ws, ws_bytes, wsplit, st))
}

int ks_debug_stamps(unsigned long long* host, int n) {
  if (n > kKsStampBlocks * 24) n = kKsStampBlocks * 24;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ks_stamps), (size_t)n * 8) == hipSuccess ? kOk : kLaunch;
}

}  // namespace mragan
