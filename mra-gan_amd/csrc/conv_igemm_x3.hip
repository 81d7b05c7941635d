// Implicit-GEMM 3D convolution on gfx950 bf16 MFMA with a three-term fp32 split ("bf16x3").
//
// Same GEMM view, geometry and epilogue as conv_igemm.hip (forward form, transposed form per
// output parity class); only the inner product differs.  Every fp32 operand x is split once,
// when its tile is staged into LDS, into x = hi + lo + r with hi = bf16(x), lo = bf16(x − hi)
// (x − hi is exact in fp32, |r| ≤ 2⁻¹⁸|x|), and
//
//     a·b ≈ lo_a·hi_b + hi_a·lo_b + hi_a·hi_b
//
// is accumulated in fp32 by three v_mfma_f32_32x32x16_bf16 (the dropped lo·lo term and the
// residuals are ≤ 3·2⁻¹⁸ of |a·b|; bf16×bf16 products are exact in the fp32 accumulator).
// Three bf16 MFMAs cost 96 cycles per 32×32×16 block versus 512 for eight f32 32x32x2 MFMAs,
// so the contraction runs at up to 5.3× the exact-f32 MFMA rate.  Error measured against fp64
// is of the same order as fp32 accumulation over the K = 27·Cin taps (tests/test_kernels_gpu.py).
//
// LDS: hi and lo planes of the A tile [BM][BK] and B tile [BN][BK] in bf16, rows padded by
// 16 B (BK = 32 → 80-B rows, BK = 16 → 48-B rows: the 16 lanes of each ds_read_b128 phase hit
// disjoint bank quads); register-staged double buffer, one barrier per K-step.  Fragment of
// lane l for k-slice kk: row l&31, k = 16kk + 8(l>>5) … +7 — one ds_read_b128 per plane.
// Grid: 1-D, XCD-aware — consecutive tiles (the n-blocks sharing an A row-block, then the
// neighbouring row-blocks sharing input halo) are placed on the same XCD's L2.
//
// Precision modes (prec.h): the same kernel is instantiated for bf16x3 (three MFMAs, hi + lo
// planes), bf16 and fp16 (one MFMA per block product, hi planes only).
#include <type_traits>

#include <atomic>

#include "conv_geo.h"
#include "in_ticket.h"
#include "kernels.h"
#include "prec.h"

namespace mragan {

// Split-K reduction in the launch (round 6, opt-in: MRAGAN_SK_FUSE=1): the slices of an output tile
// store their partial tiles write-through, draw a ticket from the tile's counter (in_ticket.h's
// hand-off), and the block that draws the last one sums the tile's slabs in slice order and writes
// y = act(bias + Σ_z slab_z) — conv_splitk_reduce's arithmetic element for element (bit-identical),
// without its launch and the dependency gap in front of it — and, for forward statistics, the
// InstanceNorm partials of the tile.  Measured SLOWER on the UNet leg (same box, alternating:
// 3.62-3.63 against 3.55-3.57 ms with the reduce launch, profiles/r06/r06o_sk_fuse_ab.txt): one block
// per tile sums every slice of it (a 64×64 tile of a 16-way split: 256 loads per thread) while the
// reduce launch spreads the same sums over the whole chip, and a graph-replayed launch gap is short.
// Counters: a zeroed device pool, slots handed out round-robin per launch by the host; the reducer
// resets its counter.
constexpr int kSkSlots = 1 << 20;
__device__ unsigned g_sk_tickets[kSkSlots];

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// X16: the input is the producer's 16-bit operand plane (bf16 / fp16 words, rounded as the
// staging would round them; the one-plane modes): an A row's BK channels are BK / 8 16-B loads
// stored to LDS as they are — half the bytes of the fp32 input and no conversion.
// W16: the weights are the pre-split fragment copy (IgemmArgs::wx3, pack tr 2-5: per (tap, 32-channel
// chunk, 16-channel half) the hi words of every output row n, 8 channels in 16 B) instead of the fp32
// pack — the B row's BK channels are BK / 8 16-B loads of hi words stored to LDS as they are, bit for
// bit the RNE words the fp32 staging would produce.  The shell pass of the interior + shell data
// gradient runs this way, so it reads the same weights as the interior brick and the fp32 pack of a
// ResnetBlock conv is never needed in the one-plane modes (r05final2: a stale fp32 pack read here).
template <int WM, int WN, int TM, int TN, int BK, int PM, int DEPTH, int X16, int W16 = 0>
__global__ void __launch_bounds__(256)
conv_igemm_x3_kernel(IgemmArgs a, int gm, int gn, int ntiles, int ksplit) {
  static_assert(!X16 || !prec::has_lo<PM>(), "16-bit operand planes exist in the one-plane modes only");
  static_assert(!W16 || (!prec::has_lo<PM>() && BK == 32), "pre-split weights: one-plane modes, 32-channel chunks");
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int LDK = BK + 8;               // bf16 per padded row
  constexpr int LPR = BK / 4;               // float4 per row (global side)
  constexpr int LPRA = X16 ? BK / 8 : LPR;  // A loads per row (16 B each)
  constexpr int LPRB = W16 ? BK / 8 : LPR;  // B loads per row (16 B each)
  constexpr int A_LOADS = (BM * LPRA + 255) / 256;
  constexpr int B_LOADS = (BN * LPRB + 255) / 256;
  constexpr int ROWS_PER_PASS = 256 / LPRB;
  constexpr int ROWS_PER_PASS_A = 256 / LPRA;
  constexpr int PLANE_A = BM * LDK, PLANE_B = BN * LDK;   // bf16 elements per plane
  // hi (+ lo in bf16x3) planes of A and B.  The one-plane modes drop the lo planes of the 2-tile
  // waves' blocks: 128×64 at 31 instead of 62 KB, two more blocks per CU (G down1 [4×64³]: 64.6
  // vs 71.2 µs); the 64×64 tile keeps them — at 7 blocks per CU it ran 9 % slower
  // (profiles/r03u/)
#ifdef MRAGAN_IG_TWO_PLANES   // A/B baseline (build variant)
  constexpr int NPL = 2;
#else
  constexpr int NPL = (prec::has_lo<PM>() || TM * TN == 1) ? 2 : 1;
#endif
  constexpr int STAGE = NPL * (PLANE_A + PLANE_B);
  static_assert(WM * WN == 4, "4 waves");
  static_assert(BK % 16 == 0, "bf16 MFMA consumes K in 16s");

  __shared__ __attribute__((aligned(16))) __bf16 smem[2 * STAGE];
  __shared__ int out_off[BM];
  __shared__ int sk_flag;

  // XCD-aware tile order: hardware puts block L on XCD L % 8; give each XCD a contiguous range
  const int kz = blockIdx.x / ntiles;                 // split-K slice
  int L = blockIdx.x - kz * ntiles, tile = L;
  if ((ntiles & 7) == 0) tile = (L & 7) * (ntiles >> 3) + (L >> 3);
  // parity classes fastest (transposed s2): the classes of one output region read the same input
  // region, so each XCD's contiguous tile range holds every class — with the classes outermost, one
  // XCD got the 8-tap class (every dim odd) and another the 1-tap one: the kernel took as long as
  // 1/8 of the chip doing 8/27 of the work.  Heaviest class first within a group.
  int rest = tile;
  int cls = 0;
  if (a.nclass > 1) {
    cls = a.nclass - 1 - rest % a.nclass;
    rest /= a.nclass;
  }
  const int nb_idx = rest % gn;
  const int mb_idx = rest / gn;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm0 = (wave / WN) * TM * 32;
  const int wn0 = (wave % WN) * TN * 32;

  int cw = cls % a.s, ch = (cls / a.s) % a.s, cd = cls / (a.s * a.s);
  if (a.nclass == 1) { cd = ch = cw = 0; }
  const DimGeo gd = a.shell ? shell_geo(cls, 0, a.Do, a.k) : dim_geo(cd, a.Do, a.k, a.s, a.p, a.trans);
  const DimGeo gh = a.shell ? shell_geo(cls, 1, a.Ho, a.k) : dim_geo(ch, a.Ho, a.k, a.s, a.p, a.trans);
  const DimGeo gw = a.shell ? shell_geo(cls, 2, a.Wo, a.k) : dim_geo(cw, a.Wo, a.k, a.s, a.p, a.trans);
  const int64_t Mc = (int64_t)a.N * gd.Q * gh.Q * gw.Q;
  const int64_t m0 = (int64_t)mb_idx * BM;
  const int n0 = nb_idx * BN;
  if (m0 >= Mc) return;
  const int ntaps = gd.ntap * gh.ntap * gw.ntap;

  for (int r = tid; r < BM; r += 256) {
    int64_t m = m0 + r;
    int off = -1;
    if (m < Mc) {
      int qw = (int)(m % gw.Q); int64_t t = m / gw.Q;
      int qh = (int)(t % gh.Q); t /= gh.Q;
      int qd = (int)(t % gd.Q); int nb = (int)(t / gd.Q);
      int od = gd.o_mul * qd + gd.o_add, oh = gh.o_mul * qh + gh.o_add, ow = gw.o_mul * qw + gw.o_add;
      off = (int)((((int64_t)nb * a.Do + od) * a.Ho + oh) * a.Wo + ow);
    }
    out_off[r] = off;
  }

  const int q = tid % LPRB;                 // B: this thread's 16-B slice of a row
  const int qa = tid % LPRA;                // A: this thread's 16-B slice of a row
  int a_nb[A_LOADS], a_bd[A_LOADS], a_bh[A_LOADS], a_bw[A_LOADS];
#pragma unroll
  for (int i = 0; i < A_LOADS; ++i) {
    int r = tid / LPRA + i * ROWS_PER_PASS_A;
    int64_t m = m0 + r;
    if (r < BM && m < Mc) {
      int qw = (int)(m % gw.Q); int64_t t = m / gw.Q;
      int qh = (int)(t % gh.Q); t /= gh.Q;
      int qd = (int)(t % gd.Q); int nb = (int)(t / gd.Q);
      a_nb[i] = nb;
      a_bd[i] = gd.a_mul * qd + gd.base_add;
      a_bh[i] = gh.a_mul * qh + gh.base_add;
      a_bw[i] = gw.a_mul * qw + gw.base_add;
    } else {
      a_nb[i] = -1; a_bd[i] = a_bh[i] = a_bw[i] = 0;
    }
  }

  const int kchunks = a.cx / BK;
  const int nK_all = ntaps * kchunks;
  const int kper = (nK_all + ksplit - 1) / ksplit;
  const int ks0 = min(nK_all, kz * kper);
  const int nK = min(nK_all, ks0 + kper) - ks0;       // steps of this slice: ks0 … ks0+nK−1
  // DEPTH 2 (A/B only, measured slower): two register stages, the tiles of step ks + 2 loaded
  // while step ks runs and stored to LDS at the end of step ks + 1; DEPTH 1 (default): one stage
  using RegA = std::conditional_t<X16 != 0, uint4, float4>;   // X16: eight 16-bit words, else four fp32
  using RegB = std::conditional_t<W16 != 0, uint4, float4>;   // W16: eight hi words, else four fp32
  RegA ra[2][A_LOADS];
  RegB rb[2][B_LOADS];

  // Operands through buffer descriptors (byte offsets are 32-bit: the host checks the sizes).
  // A: per thread and row a fixed base offset of its (nb, bd, bh, bw) voxel + channel quad; a
  // K-step adds a wave-uniform tap / channel offset, and a tap outside the input (padding) reads
  // zeros through an out-of-range voffset.  B: the lane part is fixed, the step part is the
  // SGPR soffset.  K-steps advance (channel chunk, kw, kh, kd) with carries: no per-step
  // divisions, no 64-bit address arithmetic.
  constexpr int ESA = X16 ? 2 : 4;          // bytes per input element
  const __amdgpu_buffer_rsrc_t xrs = make_rsrc(a.x, __builtin_amdgcn_readfirstlane(a.N * a.Di * a.Hi * a.Wi * a.cx * ESA / (a.tmode == 2 ? 2 : 1)));
  // a.tmode (timing-only A/B, MRAGAN_IG_TIMING): 1 — the weight descriptor covers the first half
  // of the packed taps (the rest read as zeros: no memory traffic), 2 — the input's first half
  // (the pre-split copy has the fp32 pack's size: hi + lo words per weight)
  const __amdgpu_buffer_rsrc_t wrs = make_rsrc(W16 ? a.wx3 : a.w, __builtin_amdgcn_readfirstlane(a.k * a.k * a.k * a.ny * a.cx * 4 / (a.tmode == 1 ? 2 : 1)));
  int a_base[A_LOADS];
#pragma unroll
  for (int i = 0; i < A_LOADS; ++i)
    a_base[i] = ((((a_nb[i] < 0 ? 0 : a_nb[i]) * a.Di + a_bd[i]) * a.Hi + a_bh[i]) * a.Wi + a_bw[i]) * a.cx * ESA + 16 * qa;
  int b_voff[B_LOADS];
#pragma unroll
  for (int i = 0; i < B_LOADS; ++i) {
    const int r = tid / LPRB + i * ROWS_PER_PASS, n = n0 + r;
    // W16: slice q = 16-channel half (q >> 1) and 8-channel group (q & 1) of the chunk's fragments
    const int lane_off = W16 ? ((q >> 1) * 32 * a.ny + n * 16 + (q & 1) * 8) * 2 : n * a.cx * 4 + 16 * q;
    b_voff[i] = (r < BN && n < a.ny) ? lane_off : (int)kOobOffset;
  }
  int kc = ks0 % kchunks, tap0 = ks0 / kchunks;
  int kjw = tap0 % gw.ntap, kjh = (tap0 / gw.ntap) % gh.ntap, kjd = tap0 / gw.ntap / gh.ntap;
  // the step's tap offsets (input: toff bytes, weights: wso bytes) and tap displacements are kept
  // incrementally — one add per carry level instead of ~25 scalar multiplies per K-step (PMC r04:
  // 21.8 SALU per MFMA in G down1); the deltas are block constants
  const int rs_ = a.cx * ESA, rwo = a.ny * a.cx * 4;                       // one input voxel / weight tap
  const int dC_t = BK * ESA, dC_w = W16 ? BK * 4 * a.ny : BK * 4;       // W16: a chunk's fragments span every row
  const int rC_t = (kchunks - 1) * dC_t, rC_w = (kchunks - 1) * dC_w;      // chunk wrap
  const int dW_t = gw.sign * rs_, dW_w = gw.tstep * rwo;
  const int dH_t = gh.sign * a.Wi * rs_, dH_w = gh.tstep * a.k * rwo;
  const int dD_t = gd.sign * a.Hi * a.Wi * rs_, dD_w = gd.tstep * a.k * a.k * rwo;
  const int rW_t = (gw.ntap - 1) * dW_t, rW_w = (gw.ntap - 1) * dW_w;
  const int rH_t = (gh.ntap - 1) * dH_t, rH_w = (gh.ntap - 1) * dH_w;
  int dd = gd.sign * kjd, dh = gh.sign * kjh, dw = gw.sign * kjw;
  int toff = (((dd * a.Hi + dh) * a.Wi + dw) * a.cx + kc * BK) * ESA;
  int wso = ((((gd.t0 + gd.tstep * kjd) * a.k + gh.t0 + gh.tstep * kjh) * a.k + gw.t0 + gw.tstep * kjw) * a.ny * a.cx +
             kc * BK * (W16 ? a.ny : 1)) * 4;
  auto advance = [&]() __attribute__((always_inline)) {
    toff += dC_t; wso += dC_w;
    if (++kc == kchunks) {
      kc = 0;
      toff += dW_t - rC_t - dC_t; wso += dW_w - rC_w - dC_w; dw += gw.sign;
      if (++kjw == gw.ntap) {
        kjw = 0;
        toff += dH_t - rW_t - dW_t; wso += dH_w - rW_w - dW_w; dw = 0; dh += gh.sign;
        if (++kjh == gh.ntap) {
          kjh = 0;
          toff += dD_t - rH_t - dH_t; wso += dD_w - rH_w - dH_w; dh = 0; dd += gd.sign;
          ++kjd;
        }
      }
    }
  };

  auto load_tiles = [&](RegA (&ra_)[A_LOADS], RegB (&rb_)[B_LOADS]) __attribute__((always_inline)) {
    const int toffu = __builtin_amdgcn_readfirstlane(toff);
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
      const int id = a_bd[i] + dd, ih = a_bh[i] + dh, iw = a_bw[i] + dw;
      const bool ok = a_nb[i] >= 0 && (unsigned)id < (unsigned)a.Di && (unsigned)ih < (unsigned)a.Hi &&
                      (unsigned)iw < (unsigned)a.Wi;
      const buf_f32x4 v = buf_load_16b(xrs, ok ? a_base[i] + toffu : (int)kOobOffset, 0);
      if constexpr (X16) ra_[i] = __builtin_bit_cast(uint4, v);
      else ra_[i] = make_float4(v.x, v.y, v.z, v.w);
    }
    const int wsou = __builtin_amdgcn_readfirstlane(wso);
#pragma unroll
    for (int i = 0; i < B_LOADS; ++i) {
      const buf_f32x4 v = buf_load_16b(wrs, b_voff[i], wsou);
      if constexpr (W16) rb_[i] = __builtin_bit_cast(uint4, v);
      else rb_[i] = make_float4(v.x, v.y, v.z, v.w);
    }
    advance();
  };
  auto store_tiles = [&](int buf, const RegA (&ra_)[A_LOADS], const RegB (&rb_)[B_LOADS]) {
    __bf16* st = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
      int r = tid / LPRA + i * ROWS_PER_PASS_A;
      if (r < BM) {
        if constexpr (X16) {
          *reinterpret_cast<uint4*>(st + r * LDK + 8 * qa) = ra_[i];
        } else {
          uint2 hi, lo;
          prec::split4<PM>(ra_[i], hi, lo);
          *reinterpret_cast<uint2*>(st + r * LDK + 4 * qa) = hi;      // (LPRA = LPR: qa is the float4 slot)
          if constexpr (prec::has_lo<PM>()) *reinterpret_cast<uint2*>(st + PLANE_A + r * LDK + 4 * qa) = lo;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < B_LOADS; ++i) {
      int r = tid / LPRB + i * ROWS_PER_PASS;
      if constexpr (W16) {
        if (r < BN) *reinterpret_cast<uint4*>(st + NPL * PLANE_A + r * LDK + 8 * q) = rb_[i];
      } else if (r < BN) {
        uint2 hi, lo;
        prec::split4<PM>(rb_[i], hi, lo);
        *reinterpret_cast<uint2*>(st + NPL * PLANE_A + r * LDK + 4 * q) = hi;
        if constexpr (prec::has_lo<PM>())
          *reinterpret_cast<uint2*>(st + NPL * PLANE_A + PLANE_B + r * LDK + 4 * q) = lo;
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  if (nK > 0) {
    load_tiles(ra[0], rb[0]);
    if (DEPTH == 2 && nK > 1) load_tiles(ra[1], rb[1]);
    store_tiles(0, ra[0], rb[0]);
  }
  __syncthreads();

  const int li = lane & 31;
  const int lh = lane >> 5;
  for (int ks = 0; ks < nK; ++ks) {
    const int buf = ks & 1;
    // register stage ks & 1 was stored at the end of step ks − 1: refill it with step ks + 2
    // (DEPTH 1: one stage, step ks + 1 loaded here and stored at the end of this step)
    if constexpr (DEPTH == 2) {
      if (ks + 2 < nK) {
        if (buf) load_tiles(ra[1], rb[1]);
        else load_tiles(ra[0], rb[0]);
      }
    } else {
      if (ks + 1 < nK) load_tiles(ra[0], rb[0]);
    }
    const __bf16* Ah = smem + buf * STAGE;
    const __bf16* Al = Ah + PLANE_A;
    const __bf16* Bh = Ah + NPL * PLANE_A;
    const __bf16* Bl = Bh + PLANE_B;
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      bf16x8 ah[TM], al[TM], bh[TN], bl[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        int o = (wm0 + i * 32 + li) * LDK + kk * 16 + 8 * lh;
        ah[i] = *reinterpret_cast<const bf16x8*>(Ah + o);
        if constexpr (prec::has_lo<PM>()) al[i] = *reinterpret_cast<const bf16x8*>(Al + o);
        else al[i] = ah[i];
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int o = (wn0 + j * 32 + li) * LDK + kk * 16 + 8 * lh;
        bh[j] = *reinterpret_cast<const bf16x8*>(Bh + o);
        if constexpr (prec::has_lo<PM>()) bl[j] = *reinterpret_cast<const bf16x8*>(Bl + o);
        else bl[j] = bh[j];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = prec::mma<PM>(ah[i], al[i], bh[j], bl[j], acc[i][j]);
        }
    }
    if (ks + 1 < nK) {
      if (DEPTH == 1) store_tiles(buf ^ 1, ra[0], rb[0]);
      else if (buf) store_tiles(0, ra[0], rb[0]);
      else store_tiles(1, ra[1], rb[1]);
    }
    __syncthreads();
  }

  // epilogue: C/D map of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5).
  // Split-K slices write raw partial tiles to their slab; conv_splitk_reduce applies bias/act.
  if (ksplit > 1) {
    const int64_t E = (int64_t)a.N * a.Do * a.Ho * a.Wo * a.ny;     // one slab
    float* slab = a.ws + (int64_t)kz * E;
    const bool fused = a.sk_slot >= 0;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      int col = n0 + wn0 + j * 32 + li;
      if (col >= a.ny) continue;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          int off = out_off[wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh];
          if (off >= 0) {
            float* p = slab + (int64_t)off * a.ny + col;
            if (fused) __hip_atomic_store(p, acc[i][j][r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            else *p = acc[i][j][r];
          }
        }
    }
    if (!fused || !in_ticket_draw(&g_sk_tickets[a.sk_slot + L], ksplit, &sk_flag)) return;
    // the last slice of this tile: conv_splitk_reduce's sum for the tile's outputs (columns fastest;
    // per thread EB outputs × ZB slices of loads in flight at once, summed in slice order)
    constexpr int EB = 8, ZB = 4;
    static_assert(256 % BN == 0, "a reducer thread keeps one column");
    double rps = 0.0, rpq = 0.0;             // its column's Σy, Σy² (InstanceNorm partials, a.in_part)
    for (int e0 = tid; e0 < BM * BN; e0 += 256 * EB) {
      int64_t idx[EB];
      float v[EB];
#pragma unroll
      for (int u = 0; u < EB; ++u) {
        const int e = e0 + u * 256;
        const int r = e / BN, col = n0 + e % BN;
        const int off = e < BM * BN ? out_off[r] : -1;
        idx[u] = (off < 0 || col >= a.ny) ? -1 : (int64_t)off * a.ny + col;
        v[u] = (idx[u] >= 0 && a.bias) ? a.bias[col] : 0.f;
      }
      for (int z0 = 0; z0 < ksplit; z0 += ZB) {
        float t[ZB][EB];
#pragma unroll
        for (int zz = 0; zz < ZB; ++zz)
#pragma unroll
          for (int u = 0; u < EB; ++u)
            t[zz][u] = (z0 + zz < ksplit && idx[u] >= 0)
                           ? __hip_atomic_load(a.ws + (int64_t)(z0 + zz) * E + idx[u], __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)
                           : 0.f;
#pragma unroll
        for (int zz = 0; zz < ZB; ++zz)
#pragma unroll
          for (int u = 0; u < EB; ++u)
            if (z0 + zz < ksplit) v[u] += t[zz][u];
      }
#pragma unroll
      for (int u = 0; u < EB; ++u)
        if (idx[u] >= 0) {
          const float yv = act_fwd(v[u], a.act);
          a.y[idx[u]] = yv;
          rps += yv;
          rpq += (double)yv * yv;
        }
    }
    if (a.in_part) {
      // the tile's partial as the unsplit epilogue leaves it (same chunk index; the host allows it
      // for forward statistics without bias / activation): the 256 / BN threads of a column in order
      double* red = reinterpret_cast<double*>(smem);
      red[2 * tid] = rps;
      red[2 * tid + 1] = rpq;
      __syncthreads();
      if (tid < BN && n0 + tid < a.ny) {
        double s2 = 0.0, q2 = 0.0;
        for (int k = tid; k < 256; k += BN) {
          s2 += red[2 * k];
          q2 += red[2 * k + 1];
        }
        const int64_t qv = Mc / a.N;
        const int nb = (int)(m0 / qv);
        const int cpc = (int)(qv / BM);
        const int chunk = cls * cpc + (int)((m0 - (int64_t)nb * qv) / BM);
        double* dst = a.in_part + (((int64_t)nb * (a.nclass * cpc) + chunk) * a.ny + n0 + tid) * 2;
        dst[0] = s2;
        dst[1] = q2;
      }
    }
    return;
  }
  double ps[TN], pq[TN];                 // InstanceNorm statistics of the written values
  // backward statistics instead (a.bs_x, ABI 12): y is the gradient of the InstanceNorm(+act) of
  // bs_x (same shape, no fold): Σ g, Σ g·x̂ with g = y·act'(x̂)
  const int snb = a.bs_x ? (int)(m0 / (Mc / a.N)) : 0;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    int col = n0 + wn0 + j * 32 + li;
    ps[j] = pq[j] = 0.0;
    if (col >= a.ny) continue;
    float bsum = a.bias ? a.bias[col] : 0.f;
    const float smu = a.bs_x ? a.bs_mean[snb * a.ny + col] : 0.f, srs = a.bs_x ? a.bs_rstd[snb * a.ny + col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int row = wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        int off = out_off[row];
        if (off >= 0) {
          const float v = act_fwd(acc[i][j][r] + bsum, a.act);
          a.y[(int64_t)off * a.ny + col] = v;
          if (a.bs_x) {
            const float xh = (a.bs_x[(int64_t)off * a.ny + col] - smu) * srs;
            const float gv = (a.bs_act == kActRelu && !(xh > 0.f)) ? 0.f
                             : (a.bs_act == kActLrelu && !(xh > 0.f)) ? v * kLreluSlope : v;
            ps[j] += gv;
            pq[j] += (double)gv * xh;
          } else {
            ps[j] += v;
            pq[j] += (double)v * v;
          }
        }
      }
    }
  }
  // the consumer InstanceNorm's Σy / Σy² partial of this tile (the host guarantees that a tile's
  // rows lie in one instance and one class): chunk = class · (tiles per class and instance) +
  // tile within them; lanes li / li + 32 share a column, the WM waves of a column add through LDS
  if (a.in_part) {
    __syncthreads();                                  // the staging buffers are idle now
    double* red = reinterpret_cast<double*>(smem);    // [WM][BN][2]
    const int wmi = wave / WN;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const double s2 = ps[j] + __shfl_xor(ps[j], 32);
      const double q2 = pq[j] + __shfl_xor(pq[j], 32);
      if (lh == 0) {
        red[(wmi * BN + wn0 + j * 32 + li) * 2] = s2;
        red[(wmi * BN + wn0 + j * 32 + li) * 2 + 1] = q2;
      }
    }
    __syncthreads();
    const int64_t qv = Mc / a.N;                      // rows of this class per instance
    const int nb = (int)(m0 / qv);
    const int cpc = (int)(qv / BM);
    const int chunk = cls * cpc + (int)((m0 - (int64_t)nb * qv) / BM);
    const int chunks = a.nclass * cpc;
    for (int c = tid; c < BN; c += 256) {
      if (n0 + c >= a.ny) continue;
      double s2 = 0.0, q2 = 0.0;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        s2 += red[(w * BN + c) * 2];
        q2 += red[(w * BN + c) * 2 + 1];
      }
      double* dst = a.in_part + (((int64_t)nb * chunks + chunk) * a.ny + n0 + c) * 2;
      dst[0] = s2;
      dst[1] = q2;
    }
  }
}

// y[e] = act(bias[col] + Σ_z slab[z][e]), fixed order (deterministic)
__global__ void __launch_bounds__(256) conv_splitk_reduce_kernel(const float* __restrict__ ws, int64_t E, int ny,
                                                                 int splits, const float* __restrict__ bias, int act,
                                                                 float* __restrict__ y) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E; e += (int64_t)gridDim.x * blockDim.x) {
    float v = bias ? bias[e % ny] : 0.f;
    for (int z = 0; z < splits; ++z) v += ws[(int64_t)z * E + e];
    y[e] = act_fwd(v, act);
  }
}

// tile configurations of the dispatch, in preference order per output-channel class
struct X3Cfg { int bm, bn; };
static const X3Cfg kX3Cfg[] = {{128, 128}, {128, 64}, {64, 64}, {256, 32}, {128, 32}};

struct X3Plan { int cfg; int splits; };

// largest tile that still gives one block per CU (256 CUs), else the smallest; when even that
// leaves the chip under-filled and the contraction is long (PatchGAN layers: M ≤ 4k rows,
// K = 16·Cin), split K across ≤ 16 slices.
static X3Plan x3_plan(const IgemmArgs& a, int64_t total_m) {
  auto blocks = [&](int c) {
    return (int64_t)ceil_div(total_m, kX3Cfg[c].bm) * ceil_div(a.ny, kX3Cfg[c].bn);
  };
  // the largest tile with ≥ 512 blocks (two rounds of the 256 CUs at up to 3 blocks per CU: a
  // 256-block 128×64 grid left G's down2 at 61–66 µs, 64×64 tiles 49.6 µs); without one, 64×64
  // for > 64 outputs, and for ≤ 64 outputs the 128×64 tile whose short M is then split in K
  // (PatchGAN layer 2: 37.5 µs split 4 ways vs 47.1 µs on 64×64 tiles; tools/gpu_igcfg.sh)
  static const int64_t want = [] {                            // A/B switch: MRAGAN_IG_MINBLOCKS
    const char* e = getenv("MRAGAN_IG_MINBLOCKS");
    return (int64_t)(e ? atoi(e) : 512);
  }();
  int cfg;
  if (a.ny > 64) cfg = blocks(0) >= want ? 0 : blocks(1) >= want ? 1 : 2;
  else if (a.ny > 32) cfg = blocks(1) >= want ? 1 : blocks(2) >= want ? 2 : 1;
  else cfg = blocks(3) >= 256 ? 3 : 4;
  X3Plan pl{cfg, 1};
  const int64_t b = blocks(cfg);
  const int bk = a.cx % 32 == 0 ? 32 : 16;
  const int nk = (a.k * a.k * a.k + a.nclass - 1) / a.nclass * (a.cx / bk);   // K-steps per class (average)
  if (b < 256 && nk >= 32) {
    int64_t sp = (512 + b - 1) / b;
    if (sp > nk / 16) sp = nk / 16;
    if (sp > 16) sp = 16;
    if (sp > 1) pl.splits = (int)sp;
  }
  return pl;
}

size_t conv_igemm_x3_ws_bytes(const IgemmArgs& a, int64_t max_mc, int64_t total_m) {
  (void)max_mc;
  X3Plan pl = x3_plan(a, total_m);
  return pl.splits > 1 ? (size_t)pl.splits * total_m * a.ny * sizeof(float) : 0;
}

template <int WM, int WN, int TM, int TN, int BK, int PM, int DEPTH>
static void launch_x3_pm(const IgemmArgs& a, dim3 grid, int gm, int gn, int ntiles, int splits, hipStream_t st,
                         bool w16 = false) {
  if constexpr (prec::has_lo<PM>()) {
    // BK 64 runs the one-plane modes only (the host's use64): two planes would not fit the LDS
    if constexpr (BK != 64)
      hipLaunchKernelGGL((conv_igemm_x3_kernel<WM, WN, TM, TN, BK, PM, DEPTH, 0>), grid, dim3(256), 0, st, a, gm, gn,
                         ntiles, splits);
  } else if (w16) {
    // the pre-split weights (the shell pass, conv_igemm_x3_shell: BK 32, one stage)
    if constexpr (BK == 32 && DEPTH == 1) {
      if (a.x16)
        hipLaunchKernelGGL((conv_igemm_x3_kernel<WM, WN, TM, TN, BK, PM, DEPTH, 1, 1>), grid, dim3(256), 0, st, a, gm,
                           gn, ntiles, splits);
      else
        hipLaunchKernelGGL((conv_igemm_x3_kernel<WM, WN, TM, TN, BK, PM, DEPTH, 0, 1>), grid, dim3(256), 0, st, a, gm,
                           gn, ntiles, splits);
    }
  } else {
    if (a.x16)
      hipLaunchKernelGGL((conv_igemm_x3_kernel<WM, WN, TM, TN, BK, PM, DEPTH, 1>), grid, dim3(256), 0, st, a, gm, gn,
                         ntiles, splits);
    else
      hipLaunchKernelGGL((conv_igemm_x3_kernel<WM, WN, TM, TN, BK, PM, DEPTH, 0>), grid, dim3(256), 0, st, a, gm, gn,
                         ntiles, splits);
  }
}

template <int WM, int WN, int TM, int TN, int BK>
static int launch_x3(const IgemmArgs& a, int64_t max_mc, int splits, hipStream_t st, bool w16 = false) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  int gm = ceil_div(max_mc, BM), gn = ceil_div(a.ny, BN);
  int ntiles = gm * gn * a.nclass;
  // A/B switch, off: the two-stage register prefetch measured 15–20 % SLOWER than one stage on
  // every stride-2 / PatchGAN shape (bf16, r03h: down1 84.3 vs 70.8 µs, down2 52.6 vs 42.2, up1
  // 87.6 vs 72.8, D layer 2 28.8 vs 25.2 at N = 4) — the extra 24–32 VGPRs cost occupancy
  static const bool depth1 = getenv("MRAGAN_IG_DEPTH2") == nullptr;
  MRAGAN_PREC_DISPATCH(a.x3, {
    if (depth1 || w16) launch_x3_pm<WM, WN, TM, TN, BK, PM, 1>(a, dim3(ntiles * splits), gm, gn, ntiles, splits, st, w16);
    else launch_x3_pm<WM, WN, TM, TN, BK, PM, 2>(a, dim3(ntiles * splits), gm, gn, ntiles, splits, st);
    return check_launch(a.x16 ? "conv_igemm_x3(op16)" : "conv_igemm_x3");
  })
}

template <int BK>
static int dispatch_x3(const IgemmArgs& a, int64_t max_mc, int cfg, int splits, hipStream_t st, bool w16 = false) {
  switch (cfg) {
    case 0: return launch_x3<2, 2, 2, 2, BK>(a, max_mc, splits, st, w16);
    case 1: return launch_x3<2, 2, 2, 1, BK>(a, max_mc, splits, st, w16);
    case 2: return launch_x3<2, 2, 1, 1, BK>(a, max_mc, splits, st, w16);
    case 3: return launch_x3<4, 1, 2, 1, BK>(a, max_mc, splits, st, w16);
    default: return launch_x3<4, 1, 1, 1, BK>(a, max_mc, splits, st, w16);
  }
}

// the shell pass of a full k3 s1 transposed conv (see shell_geo): 6 classes, rows = shell outputs.
// In the one-plane modes it reads the pre-split weights the interior brick reads (W16): the fp32
// pack is then not needed at all, and a caller whose fp32 pack is stale passes none (w = null)
int conv_igemm_x3_shell(IgemmArgs a, hipStream_t st) {
  a.shell = 1;
  a.nclass = 6;
  const int O = a.Do;
  const int64_t max_mc = (int64_t)a.N * O * O;                       // classes 0/1: one plane
  const int64_t total_m = (int64_t)a.N * ((int64_t)O * O * O - (int64_t)(O - 2) * (O - 2) * (O - 2));
  X3Plan pl = x3_plan(a, total_m);
  const bool w16 = a.wx3 != nullptr && (a.x3 == kPrecBf16 || a.x3 == kPrecF16) && a.cx % 32 == 0;
  MRAGAN_CHECK_ARG(w16 || a.w, "conv: the shell pass needs the fp32 weight pack (no pre-split copy usable)");
  // no split-K: its reduce would rewrite every output of the grid, not only the shell
  return a.cx % 32 == 0 ? dispatch_x3<32>(a, max_mc, pl.cfg, 1, st, w16) : dispatch_x3<16>(a, max_mc, pl.cfg, 1, st);
}

int conv_igemm_x3(IgemmArgs a, int64_t max_mc, int64_t total_m, hipStream_t st) {
  MRAGAN_CHECK_ARG(a.w, "conv: this convolution needs the fp32 weight pack (only a pre-split copy was given)");
  MRAGAN_CHECK_ARG(!a.x16 || ((a.x3 == kPrecBf16 || a.x3 == kPrecF16) && a.cx % 32 == 0),
                   "conv (16-bit operand plane): the one-plane modes and multiples of 32 input channels only");
  // operand byte offsets are 32-bit (buffer descriptors)
  MRAGAN_CHECK_ARG((int64_t)a.N * a.Di * a.Hi * a.Wi * a.cx * 4 < ((int64_t)1 << 31) &&
                       (int64_t)a.k * a.k * a.k * a.ny * a.cx * 4 < ((int64_t)1 << 31),
                   "conv (16-bit MFMA modes): input of %d×%d×%d×%d×%d too large for one launch", a.N, a.Di, a.Hi, a.Wi,
                   a.cx);
  // a skip gradient joining the backward statistics (ABI 18) exists in the brick epilogues only:
  // no partials here (chunks stays 0, the caller runs the statistics pass)
  if (a.bs_add) a.in_part = nullptr;
  X3Plan pl = x3_plan(a, total_m);
  if (pl.splits > 1) {
    const size_t need = (size_t)pl.splits * total_m * a.ny * sizeof(float);
    if (a.ws == nullptr || a.ws_bytes < need) {
      set_error("conv: split-K workspace %zu < %zu bytes (query mragan_conv3d_workspace)", a.ws_bytes, need);
      return kWorkspace;
    }
  }
  // split-K reduced in the launch (opt-in MRAGAN_SK_FUSE=1, see g_sk_tickets); the tile counters of
  // one launch are consecutive pool slots, handed out round-robin
  static const bool sk_fuse = getenv("MRAGAN_SK_FUSE") != nullptr;
  a.sk_slot = -1;
  if (sk_fuse && pl.splits > 1) {
    const int bm = kX3Cfg[pl.cfg].bm, bn = kX3Cfg[pl.cfg].bn;
    const int64_t nt = (int64_t)ceil_div(max_mc, bm) * ceil_div(a.ny, bn) * a.nclass;
    if (nt <= kSkSlots / 4) {
      static std::atomic<int64_t> next{0};
      int64_t s0 = next.fetch_add(nt) % kSkSlots;
      if (s0 + nt > kSkSlots) s0 = 0;     // (a wrap skips the pool's tail: slots stay disjoint)
      a.sk_slot = (int)s0;
    }
  }
  // InstanceNorm partials from the epilogue: no K split (or one the launch reduces itself), every
  // tile inside one instance and one class, every class the same row count (forward convs, and
  // transposed ones whose output is a whole multiple of the stride)
  if (a.in_part) {
    const int bm = kX3Cfg[pl.cfg].bm;
    const int64_t per_cls = total_m / ((int64_t)a.N * a.nclass);
    const bool even = per_cls * a.N * a.nclass == total_m && per_cls == max_mc / a.N && max_mc % a.N == 0;
    // (split-K: where the launch reduces its slices itself, forward statistics only — the reducer
    // forms them from the summed outputs)
    const bool split_ok = pl.splits == 1 || (a.sk_slot >= 0 && a.bs_x == nullptr);
    if (split_ok && !a.shell && even && per_cls % bm == 0 && a.bias == nullptr && a.act == kActNone) {
      if (a.in_chunks) *a.in_chunks = (int)(a.nclass * (per_cls / bm));
    } else {
      a.in_part = nullptr;
    }
  }
  if (!a.in_part) a.bs_x = nullptr;     // no partials: the epilogue skips the backward-statistics reads
  // BK 64 (one-plane modes, a multiple of 64 input channels): 8 MFMAs per wave between barriers
  // instead of 4 — G down2 [4×32³] 32.0 → 27.1 µs, up1 / down2-dgrad [2×16³] 37.0 → 33.7 µs, the
  // UNet leg 5.34 → 5.21 ms (same box, profiles/r04/ab_same_box.json r04y); A/B switch MRAGAN_IG_BK32
  static const bool bk64 = getenv("MRAGAN_IG_BK32") == nullptr;
  static const int tmode = [] { const char* e = getenv("MRAGAN_IG_TIMING"); return e ? atoi(e) : 0; }();
  a.tmode = tmode;
  const bool use64 = bk64 && a.cx % 64 == 0 && (a.x3 == kPrecBf16 || a.x3 == kPrecF16);
  int rc = use64 ? dispatch_x3<64>(a, max_mc, pl.cfg, pl.splits, st)
           : a.cx % 32 == 0 ? dispatch_x3<32>(a, max_mc, pl.cfg, pl.splits, st)
                            : dispatch_x3<16>(a, max_mc, pl.cfg, pl.splits, st);
  if (rc || pl.splits == 1 || a.sk_slot >= 0) return rc;
  const int64_t E = total_m * a.ny;
  int blocks = (int)((E + 255) / 256);
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(conv_splitk_reduce_kernel, dim3(blocks), dim3(256), 0, st, a.ws, E, a.ny, pl.splits, a.bias, a.act,
                     a.y);
  return check_launch("conv_splitk_reduce");
}

}  // namespace mragan
