// bf16x3 weight gradient of a "valid" 3×3×3 stride-1 convolution whose input is the
// materialised replication-padded volume (every ResnetBlock conv, networks3D.py:241-257; the
// engine feeds them a padded input and runs the conv with p = 0):
//
//   dW[co][ci][kd][kh][kw] = Σ_{n,d,h,w} dY[n,d,h,w][co] · X[n, d+kd, h+kh, w+kw][ci]
//
// conv_wgrad_x3 runs one GEMM per tap, so every (dY, X) element is loaded, split to bf16 hi/lo
// and staged 27 times — VALU-bound at ~17 % MFMA (rocprofv3 PMC).  Here a block owns one
// (kd, kh) pair and all three kw taps of a 64(co) × 64(ci) tile: the contraction runs over
// "row segments" (n, d, h, 16 w-voxels), 8 segments per stage, with the K index ordered
// k = w·8 + r (r = segment of the stage).  Then the X rows a kw tap needs are the staged rows
// shifted by kw·8 K-entries = 16 B, so one staged X tile (18 w-positions) serves all three taps
// and one staged dY tile serves all three: staging cost and L2 traffic per FLOP drop 3×.
//
// LDS (one stage, 70 KB → two blocks per CU): dY as [co][w 16][r 8] bf16 (hi 256 B, lo 256 B,
// 16 B pad: 528-B rows), X as [ci][w' 18][r 8] (592-B rows); both row strides keep the 16-lane
// ds_read_b128 groups conflict-free.  The next stage's global loads are in registers during the
// MFMAs.  Partial tiles go to split-K slabs ws[z][t][co][ci], reduced by wgrad_reduce_kernel.
#include <type_traits>

#include "kernels.h"
#include "prec.h"

namespace mragan {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kTile = 64;                 // co and ci per block (4-wave variant)
constexpr int kR = 8;                     // row segments per stage
constexpr int kSegW = 16;                 // voxels per row segment
constexpr int kDRow = 2 * kSegW * 16 + 16;          // 528 B
constexpr int kGRow = 2 * (kSegW + 2) * 16 + 16;    // 592 B
constexpr int kDHalf = kSegW * 16;                  // lo part offset in a dY row
constexpr int kGHalf = (kSegW + 2) * 16;            // lo part offset in an X row
constexpr int kLds = kTile * kDRow + kTile * kGRow; // 71 680 B
constexpr int kLdsW = 128 * kDRow + 64 * kGRow;     // 105 472 B (8-wave 128 × 64 variant)

// 16-bit modes (bf16 / fp16: one plane, no lo half): the tiles are staged in their natural
// [K = w·8 + r][channel] order — each thread converts its float4 (4 channels of one voxel) and
// stores 8 B, no transpose in VALU — and the MFMA operands, which need 8 consecutive K per lane,
// come out of LDS through ds_read_b64_tr_b16 (gfx950's transposing read: lane 4q+p of a 16-lane
// group addresses row q, channels 4p…4p+3; lane i receives channel i of the 4 rows).  Rows are
// TC·2 (dY) / TI·2 (X) bytes; 16-B chunks are XOR-swizzled by the row so the 4 rows × 2 channel
// groups of a 32-lane half hit 16 distinct 16-B slots (conflict-free transposed reads; the
// ds_write_b64 of 16 contiguous lanes stays one 128-B run): chunk c of row k sits at
// c ^ tr_swz(k).  The kw-shifted X rows (k + 8kw) keep k's swizzle.
// (SW: voxels per row segment of the 16-bit paths — 16, or 24 for 24-wide volumes such as the
// 96³ configuration's ResnetBlocks, BASELINE configs[4]; the operand-plane path only)
template <int SW> constexpr int tr_rows_d() { return SW * kR; }          // 128 K rows of dY per stage (SW 16)
template <int SW> constexpr int tr_rows_g() { return (SW + 2) * kR; }    // 144 K rows of X (two extra w for kw = 1, 2)
constexpr int kTrRowsD = tr_rows_d<kSegW>();
constexpr int kTrRowsG = tr_rows_g<kSegW>();
template <int RB>
__device__ __forceinline__ int tr_swz(int row) {
  return RB == 256 ? (row & 3) << 2 : ((row >> 1) & 1) << 2;
}
// two stage buffers: the stage after next is loaded while this one's MFMAs run and stored right
// after them, so a load has a whole stage (not only the MFMA phase) to land
constexpr int kTrStage = kTrRowsD * 64 * 2 + kTrRowsG * 64 * 2;    // 34 816 B
constexpr int kTrStageW = kTrRowsD * 128 * 2 + kTrRowsG * 64 * 2;  // 51 200 B
constexpr int kLdsTr = 2 * kTrStage;
constexpr int kLdsTrW = 2 * kTrStageW;
template <int SW, int TC>
constexpr int lds_tr() { return 2 * (tr_rows_d<SW>() * TC * 2 + tr_rows_g<SW>() * 64 * 2); }
typedef short tr_v4s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ tr_v4s tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) tr_v4s*)(p));
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// one channel of the 8 segments → 16 B hi at p, 16 B lo at p + half (pairwise scalar splits: an
// 8-wide vector built from the register array makes LLVM read the array through memory)
template <int PM>
__device__ __forceinline__ void split8_store(char* p, int half, float v0, float v1, float v2, float v3, float v4,
                                             float v5, float v6, float v7) {
  uint4 hi, lo;
  prec::split2<PM>(v0, v1, hi.x, lo.x);
  prec::split2<PM>(v2, v3, hi.y, lo.y);
  prec::split2<PM>(v4, v5, hi.z, lo.z);
  prec::split2<PM>(v6, v7, hi.w, lo.w);
  *reinterpret_cast<uint4*>(p) = hi;
  if constexpr (prec::has_lo<PM>()) *reinterpret_cast<uint4*>(p + half) = lo;
}

}  // namespace

struct Wgrad3Args {
  const float* dy; int N, D, H, W, Cd;    // dY [N][D][H][W][Cd]
  const float* x; int Cg;                 // X  [N][D+2][H+2][W+2][Cg]
  float* ws;                              // slabs [splits][27][Cd][Cg]
  int nseg, seg_per_split;                // row segments in total / per split (multiple of kR)
  // second instance set (kW16 path): segments from nseg1 on are instances of dy2 / x2 (N2 of them);
  // without one dy2 = dy, x2 = x, N2 = 0, nseg1 = nseg
  const float* dy2; const float* x2; int N2, nseg1;
};

// TC × TI = 64 × 64: 4 waves (2 × 2 sub-tiles of 32 × 32), two blocks per CU.  128 × 64 (the
// 128-channel ResnetBlock convs): 8 waves (4 × 2), one block per CU — per staged element twice
// the MFMAs of the 64 × 64 tile; the split-to-bf16 staging, not the matrix pipe, bounds this
// kernel (PMC: VALU instructions ≈ 9× the MFMAs, ACTIVE 39 % vs MFMA busy 33 %).
// WM = 2 (128 × 64 on operand planes, aligned stages; opt-in, measured slower — see the launch):
// 4 waves of 64 × 32 instead of 8 of 32 × 32.  Per K-step a wave then reads 2 A + 3 B fragments
// for 6 MFMAs instead of 1 + 3 for 3 (0.85 instead of 1.37 KB of transposing LDS reads per MFMA).
// PF2 (round 6, operand-plane aligned path, opt-in MRAGAN_W3_PF2=1): two register sets for the staged
// operands — the loads of stage st + 3 leave at the end of stage st and are stored at the end of stage
// st + 2, two stages of MFMAs in between (one set leaves one stage, ≈ 1.5 k cycles, to cover an HBM /
// L2 round trip; PMC r06x: waves parked 32 % of their cycles).  Measured neutral (r06y): kept opt-in.
template <int TC, int TI, int PM, int X16, int AL, int SW, int WM, int PF2 = 0>
__global__ void __launch_bounds__(TC * TI / (16 * WM), TC == 64 ? 2 : 1) wgrad3_x3_kernel(Wgrad3Args a) {
  constexpr int NT = TC * TI / (16 * WM); // 32·WM × 32 sub-tile per wave
  constexpr int WC = TC / (32 * WM);      // waves along co
  constexpr bool kTr = !prec::has_lo<PM>();        // 16-bit modes: natural-order tiles + transposing reads
  // X16: dY and X are the producers' 16-bit operand planes (bf16 / fp16 words, rounded as the
  // staging below would round them): 8-B loads stored as they are, no conversion
  static_assert(!X16 || kTr, "16-bit operand planes exist in the one-plane modes only");
  constexpr int ES = X16 ? 2 : 4;         // bytes per operand element
  using RegT = std::conditional_t<X16 != 0, uint2, float4>;
  constexpr int RBD = TC * 2, RBG = TI * 2;         // tr image row bytes (dY, X)
  extern __shared__ __attribute__((aligned(16))) char smem[];
  static_assert(SW == kSegW || (X16 && AL), "24-voxel segments: the aligned operand-plane path only");
  constexpr int kSegW = SW;               // voxels per row segment (shadows the file constant)
  constexpr int kTrRowsD = tr_rows_d<SW>(), kTrRowsG = tr_rows_g<SW>();
  constexpr int kStage = kTrRowsD * RBD + kTrRowsG * RBG;            // tr: bytes of one stage buffer
  char* Ds = smem;
  char* Gs = smem + (kTr ? kTrRowsD * RBD : TC * kDRow);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int wm0 = (wave % WC) * 32 * WM, wn0 = (wave / WC) * 32;

  // logical block: (co tile, ci tile) fastest, then (kd, kh), then split; XCD-aware remap so an
  // XCD's blocks share a contiguous range of splits (their dY / X rows stay in its L2)
  const int nco = a.Cd / TC, nci = a.Cg / TI;
  const int B = gridDim.x;
  int L = blockIdx.x;
  if ((B & 7) == 0) L = (L & 7) * (B >> 3) + (L >> 3);
  const int tile = L % (nco * nci);
  const int kk9 = (L / (nco * nci)) % 9;
  const int z = L / (nco * nci * 9);
  const int co0 = (tile / nci) * TC, ci0 = (tile % nci) * TI;
  const int kd = kk9 / 3, kh = kk9 % 3;
  const int seg_lo = z * a.seg_per_split;
  if (seg_lo >= a.nseg) return;                    // grid padding (a multiple of 8 blocks)
  const int seg_hi = min(a.nseg, seg_lo + a.seg_per_split);
  const int nstage = (seg_hi - seg_lo + kR - 1) / kR;

  const int Dg = a.D + 2, Hg = a.H + 2, Wg = a.W + 2;
  const int nsw = a.W / kSegW;
  // staging units (w position, channel quad), quad fastest: 16 lanes read one voxel's 256
  // contiguous bytes (a w-fastest order, conflict-free for the LDS writes below, measured 35 %
  // slower overall).  dY: TC/4 quads × 16 w = one unit per thread.  X: TI/4 quads × 18 w'.
  constexpr int DQ = TC / 4, GQ = TI / 4;
  static_assert((X16 && AL) || SW != 16 || NT == 16 * DQ, "one dY unit per thread");
  static_assert(WM == 1 || (X16 && AL), "64-row waves: the aligned operand-plane path only");
  const int cq = tid % DQ, uw = tid / DQ;          // dY unit
  const int gcq = tid % GQ, gw = tid / GQ;         // X unit: w' = gw
  // TC == TI: threads own w' 0..15 and threads < 2·GQ also w' 16, 17 (rg2).  TC = 2·TI: threads
  // < 16·GQ own w' 0..15, the next 2·GQ own w' 16, 17, the rest no X unit.
  constexpr bool kSplitG = TC == TI;
  const bool g1 = kSplitG || tid < 18 * GQ;        // has an X unit in rg
  const bool g2 = kSplitG && tid < 2 * GQ;         // second X unit (w' 16, 17) in rg2
  const int uw2 = 16 + tid / GQ;

  RegT rd[kR], rg[kR], rg2[kR];
  // dY / X through buffer descriptors: the segment part of each offset is wave-uniform (SGPR
  // soffset), the lane part fixed per thread (VGPR) — no per-load 64-bit address arithmetic
  const __amdgpu_buffer_rsrc_t dyr = make_rsrc(a.dy, __builtin_amdgcn_readfirstlane(a.N * a.D * a.H * a.W * a.Cd * ES));
  const __amdgpu_buffer_rsrc_t xgr = make_rsrc(a.x, __builtin_amdgcn_readfirstlane(a.N * Dg * Hg * Wg * a.Cg * ES));
  const int dlane = (uw * a.Cd + co0 + 4 * cq) * ES;
  const int glane = ((g1 ? gw : 0) * a.Cg + ci0 + 4 * gcq) * ES;
  const int glane2 = ((g2 ? uw2 : gw) * a.Cg + ci0 + 4 * gcq) * ES;
  // Segments are 16-voxel runs of dY in (n, d, h, w) order, so a segment's dY offset is linear in
  // its index; its X offset (padded volume, shifted by (kd, kh)) is carried along with (h, d, n)
  // carries — no per-segment index arithmetic (divisions cost ~600 scalar instructions per
  // stage, the recomputed products ~100)
  const int dseg = kSegW * a.Cd * ES;                         // dY bytes per segment
  const int gw16 = kSegW * a.Cg * ES, grow = (Wg - a.W) * a.Cg * ES;
  const int gplane = (Hg - a.H) * Wg * a.Cg * ES, gvol = (Dg - a.D) * Hg * Wg * a.Cg * ES;
  const int gkdh = (kd * Hg + kh) * Wg * a.Cg * ES;
  int sw = seg_lo % nsw, sh = (seg_lo / nsw) % a.H, sd = (seg_lo / nsw / a.H) % a.D, sn = seg_lo / nsw / a.H / a.D;
  int sxo = (((sn * Dg + sd) * Hg + sh) * Wg + sw * kSegW) * a.Cg * ES;
  auto bump = [&](int& w_, int& h_, int& d_, int& xo) __attribute__((always_inline)) {
    xo += gw16;
    if (++w_ == nsw) {
      w_ = 0; xo += grow;
      if (++h_ == a.H) { h_ = 0; xo += gplane; if (++d_ == a.D) { d_ = 0; xo += gvol; } }
    }
  };
  // AL (aligned stages, the host checks): every stage's kR segments are whole w-runs of kR / nsw
  // consecutive rows of one (n, d) plane and every stage is full — the X offset of segment r is
  // the stage's plus a per-block constant, and a stage advances with one carry chain instead of
  // kR (the per-segment carries cost ~9 scalar instructions per MFMA, PMC r03e)
  const int rps = kR / nsw;                                   // rows per stage (AL)
  const int grow1 = Wg * a.Cg * ES;                            // X bytes per padded row
  int xro[kR];
#pragma unroll
  for (int r = 0; r < kR; ++r) xro[r] = AL ? __builtin_amdgcn_readfirstlane((r / nsw) * grow1 + (r % nsw) * gw16) : 0;
  auto adv_stage = [&]() __attribute__((always_inline)) {     // AL: the next stage's first segment
    if constexpr (AL) {
      sxo += rps * grow1;
      sh += rps;
      if (sh == a.H) {
        sh = 0; sxo += gplane;
        if (++sd == a.D) { sd = 0; sxo += gvol; }
      }
    } else {
#pragma unroll
      for (int r = 0; r < kR; ++r) bump(sw, sh, sd, sxo);
    }
  };
  // kW16 (16-bit planes, aligned stages): wave w stages segment(s) w (+ NW) of a stage, 16 B =
  // 8 channels per load and per LDS store (the 8-B quad units issued 3× the loads at 0.54–0.70×
  // the 16-B rate: the plane path ran 8 % slower than the fp32 one, r03f)
  constexpr bool kW16 = X16 && AL;
  constexpr int NW = NT / 64, SPW = kR / NW;                   // waves, segments per wave
  constexpr int DO8 = TC / 8, GO8 = TI / 8;                    // 16-B octets per voxel
  constexpr int DL = kSegW * DO8 / 64, GU = (kSegW + 2) * GO8, GL = (GU + 63) / 64;
  static_assert(kR % NW == 0 && (kSegW * DO8) % 64 == 0, "wave-per-segment staging");
  static_assert(!PF2 || kW16, "two register sets: the aligned operand-plane path only");
  uint4 d16[kW16 ? SPW : 1][kW16 ? DL : 1], g16[kW16 ? SPW : 1][kW16 ? GL : 1];
  uint4 d16b[PF2 ? SPW : 1][PF2 ? DL : 1], g16b[PF2 ? SPW : 1][PF2 ? GL : 1];
  int dlo[kW16 ? DL : 1], glo[kW16 ? GL : 1], rdo[kW16 ? SPW : 1], rgo[kW16 ? SPW : 1];
  if constexpr (kW16) {
#pragma unroll
    for (int j = 0; j < DL; ++j) {
      const int u = lane + 64 * j;
      dlo[j] = ((u / DO8) * a.Cd + co0 + 8 * (u % DO8)) * 2;
    }
#pragma unroll
    for (int j = 0; j < GL; ++j) {
      const int u = lane + 64 * j;
      glo[j] = u < GU ? ((u / GO8) * a.Cg + ci0 + 8 * (u % GO8)) * 2 : (int)kOobOffset;
    }
#pragma unroll
    for (int q = 0; q < SPW; ++q) {
      const int r = wave + NW * q;
      rdo[q] = __builtin_amdgcn_readfirstlane(r * dseg);
      rgo[q] = __builtin_amdgcn_readfirstlane((r / nsw) * grow1 + (r % nsw) * gw16);
    }
  }
  // the second instance set: a stage lies in one (n, d) plane, so in one set — the stage picks its
  // descriptors (wave-uniform) and rebases its offsets by set 1's bytes (segment / X offsets stay
  // linear across the set boundary)
  const int xoff1 = a.N * Dg * Hg * Wg * a.Cg * ES;
  auto load16x = [&](int st, auto& D16, auto& G16) __attribute__((always_inline)) {
    const int s0 = seg_lo + st * kR;
    const bool s2 = s0 >= a.nseg1;
    const __amdgpu_buffer_rsrc_t dr = s2 ? make_rsrc(a.dy2, a.N2 * a.D * a.H * a.W * a.Cd * ES) : dyr;
    const __amdgpu_buffer_rsrc_t gr = s2 ? make_rsrc(a.x2, a.N2 * Dg * Hg * Wg * a.Cg * ES) : xgr;
    const int dso0 = __builtin_amdgcn_readfirstlane((s0 - (s2 ? a.nseg1 : 0)) * dseg);
    const int gso0 = __builtin_amdgcn_readfirstlane(sxo - (s2 ? xoff1 : 0) + gkdh);
#pragma unroll
    for (int q = 0; q < SPW; ++q) {
#pragma unroll
      for (int j = 0; j < DL; ++j) D16[q][j] = __builtin_bit_cast(uint4, buf_load_16b(dr, dlo[j], dso0 + rdo[q]));
#pragma unroll
      for (int j = 0; j < GL; ++j) G16[q][j] = __builtin_bit_cast(uint4, buf_load_16b(gr, glo[j], gso0 + rgo[q]));
    }
  };
  auto load16 = [&](int st) __attribute__((always_inline)) { load16x(st, d16, g16); };
  auto load = [&](int st) __attribute__((always_inline)) {
    if constexpr (kW16) {
      load16(st);
      return;
    }
    int cw = sw, chh = sh, cdd = sd, cxo = sxo;
    const int dso0 = __builtin_amdgcn_readfirstlane((seg_lo + st * kR) * dseg);
    const int gso0 = __builtin_amdgcn_readfirstlane(sxo + gkdh);
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const int seg = seg_lo + st * kR + r;
      const bool ok = AL || seg < seg_hi;
      // past the split's end: re-read segment 0 (a valid row, masked to zero)
      const int dso = AL ? dso0 + r * dseg : __builtin_amdgcn_readfirstlane(ok ? seg * dseg : 0);
      const int gso = AL ? gso0 + xro[r] : __builtin_amdgcn_readfirstlane((ok ? cxo : 0) + gkdh);
      if constexpr (!AL) bump(cw, chh, cdd, cxo);
      // past the split's end: an out-of-range voffset reads zeros (no select on the values)
      if constexpr (X16) {
        rd[r] = buf_load_8b(dyr, ok ? dlane : (int)kOobOffset, dso);
        rg[r] = buf_load_8b(xgr, ok ? glane : (int)kOobOffset, gso);
        if constexpr (kSplitG) rg2[r] = buf_load_8b(xgr, ok ? glane2 : (int)kOobOffset, gso);
      } else {
        const buf_f32x4 dv = buf_load_16b(dyr, ok ? dlane : (int)kOobOffset, dso);
        const buf_f32x4 gv = buf_load_16b(xgr, ok ? glane : (int)kOobOffset, gso);
        rd[r] = make_float4(dv.x, dv.y, dv.z, dv.w);
        rg[r] = make_float4(gv.x, gv.y, gv.z, gv.w);
        // w' = 16, 17 (threads < 2·GQ; the others re-read their own unit: keeps rg2 a plain register
        // array, a conditionally written one goes to scratch)
        if constexpr (kSplitG) {
          const buf_f32x4 g = buf_load_16b(xgr, ok ? glane2 : (int)kOobOffset, gso);
          rg2[r] = make_float4(g.x, g.y, g.z, g.w);
        }
      }
    }
  };
  // one unit: 8 segments × 4 channels → 4 rows × (16 B hi + 16 B lo) at w-slot `w`.  Write j
  // of lane cq goes to channel (j + rot) & 3, rot = (cq >> 1) & 3: an 8-lane ds_write_b128 group
  // (cq = 8g … 8g+7) then covers 8 distinct 16-B bank groups for both row strides (528 B and
  // 592 B rows, banks mod 32 dwords); unrotated, rows 4 apart collide 4-way (PMC: 51 % of the
  // LDS cycles were conflicts)
  auto put = [&](char* base, int row_bytes, int half, int w, int q, const float4 (&v)[kR]) __attribute__((always_inline)) {
    const int rot = (q >> 1) & 3;
    auto rotv = [&](const float4& x) __attribute__((always_inline)) {
      const float4 t = (rot & 1) ? make_float4(x.y, x.z, x.w, x.x) : x;
      return (rot & 2) ? make_float4(t.z, t.w, t.x, t.y) : t;
    };
    float4 u[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) u[r] = rotv(v[r]);
    char* p = base + (4 * q) * row_bytes + w * 16;
    split8_store<PM>(p + ((0 + rot) & 3) * row_bytes, half, u[0].x, u[1].x, u[2].x, u[3].x, u[4].x, u[5].x, u[6].x, u[7].x);
    split8_store<PM>(p + ((1 + rot) & 3) * row_bytes, half, u[0].y, u[1].y, u[2].y, u[3].y, u[4].y, u[5].y, u[6].y, u[7].y);
    split8_store<PM>(p + ((2 + rot) & 3) * row_bytes, half, u[0].z, u[1].z, u[2].z, u[3].z, u[4].z, u[5].z, u[6].z, u[7].z);
    split8_store<PM>(p + ((3 + rot) & 3) * row_bytes, half, u[0].w, u[1].w, u[2].w, u[3].w, u[4].w, u[5].w, u[6].w, u[7].w);
  };
  // 16-bit modes: unit (voxel w, channel quad q) → rows w·8 + r, 8 B at chunk q/2 (swizzled), half q&1
  auto put16 = [&](char* base, auto rb_c, int w, int q, const RegT (&v)[kR]) __attribute__((always_inline)) {
    constexpr int RB = decltype(rb_c)::value;
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const int row = w * kR + r;
      uint2 h;
      if constexpr (X16) {
        h = v[r];
      } else {
        uint2 l;
        prec::split4<PM>(v[r], h, l);
      }
      *reinterpret_cast<uint2*>(base + row * RB + 16 * ((q >> 1) ^ tr_swz<RB>(row)) + 8 * (q & 1)) = h;
    }
  };
  auto store16x = [&](const auto& D16, const auto& G16) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < SPW; ++q) {
      const int r = wave + NW * q;
#pragma unroll
      for (int j = 0; j < DL; ++j) {
        const int u = lane + 64 * j, row = (u / DO8) * kR + r;
        *reinterpret_cast<uint4*>(Ds + row * RBD + 16 * ((u % DO8) ^ tr_swz<RBD>(row))) = D16[q][j];
      }
#pragma unroll
      for (int j = 0; j < GL; ++j) {
        const int u = lane + 64 * j, row = (u / GO8) * kR + r;
        if (u < GU) *reinterpret_cast<uint4*>(Gs + row * RBG + 16 * ((u % GO8) ^ tr_swz<RBG>(row))) = G16[q][j];
      }
    }
  };
  auto store16 = [&]() __attribute__((always_inline)) { store16x(d16, g16); };
  auto store = [&]() __attribute__((always_inline)) {
    if constexpr (kW16) {
      store16();
      return;
    }
    if constexpr (kTr) {
      put16(Ds, std::integral_constant<int, RBD>{}, uw, cq, rd);
      if (g1) put16(Gs, std::integral_constant<int, RBG>{}, gw, gcq, rg);
      if constexpr (kSplitG) {
        if (g2) put16(Gs, std::integral_constant<int, RBG>{}, uw2, gcq, rg2);
      }
    } else {
      put(Ds, kDRow, kDHalf, uw, cq, rd);
      if (g1) put(Gs, kGRow, kGHalf, gw, gcq, rg);
      if constexpr (kSplitG) {
        if (g2) put(Gs, kGRow, kGHalf, uw2, gcq, rg2);
      }
    }
  };
  // transposed-read lane offsets: lane 4q+p of its 16-lane group g (g = lane bit 4) addresses row
  // 8h + q (+ the read's K offset) and channels (sub-tile base + 16g + 4p … +3)
  const int tq = (lane & 15) >> 2, tp = lane & 3, tg = (lane >> 4) & 1;
  int trA[WM];
#pragma unroll
  for (int i = 0; i < WM; ++i)
    trA[i] = (8 * lh + tq) * RBD + 16 * (((wm0 + 32 * i + 16 * tg) / 8 + (tp >> 1)) ^ tr_swz<RBD>(tq)) + 8 * (tp & 1);
  const int trB = (8 * lh + tq) * RBG + 16 * (((wn0 + 16 * tg) / 8 + (tp >> 1)) ^ tr_swz<RBG>(tq)) + 8 * (tp & 1);

  f32x16 acc[3][WM];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < WM; ++i) acc[t][i] = f32x16{};

  auto use_buf = [&](int b) __attribute__((always_inline)) {       // tr: select stage buffer b
    Ds = smem + b * kStage;
    Gs = Ds + kTrRowsD * RBD;
  };
  // the MFMAs of one staged stage (Ds / Gs: its buffers)
  auto compute = [&]() __attribute__((always_inline)) {
    const char* arow = kTr ? Ds + trA[0] : Ds + (wm0 + li) * kDRow + lh * 16;
    const char* brow = kTr ? Gs + trB : Gs + (wn0 + li) * kGRow + lh * 16;
    // fragments of K-step ks: A hi/lo (dY) and B hi/lo for the three kw taps (X shifted by kw
    // slots); software-pipelined one K-step ahead so the LDS latency hides under the MFMAs
    bf16x8 fa[2][WM][2], fb[2][3][2];
    auto frag = [&](int ks, bf16x8 (&A)[WM][2], bf16x8 (&Bf)[3][2]) __attribute__((always_inline)) {
      if constexpr (kTr) {
        // K-step ks covers rows 16ks … 16ks+15: two 4-row reads per operand for this lane's 8 K
#pragma unroll
        for (int i = 0; i < WM; ++i) {
          const char* ar = Ds + trA[i];
          const tr_v4s a0 = tr_read(ar + (16 * ks) * RBD), a1 = tr_read(ar + (16 * ks + 4) * RBD);
          A[i][0] = A[i][1] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const tr_v4s b0 = tr_read(brow + (16 * ks + 8 * kw) * RBG), b1 = tr_read(brow + (16 * ks + 8 * kw + 4) * RBG);
          Bf[kw][0] = Bf[kw][1] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7));
        }
        return;
      }
      A[0][0] = *reinterpret_cast<const bf16x8*>(arow + ks * 32);
      A[0][1] = prec::has_lo<PM>() ? *reinterpret_cast<const bf16x8*>(arow + ks * 32 + kDHalf) : A[0][0];
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        Bf[kw][0] = *reinterpret_cast<const bf16x8*>(brow + ks * 32 + kw * 16);
        Bf[kw][1] = prec::has_lo<PM>() ? *reinterpret_cast<const bf16x8*>(brow + ks * 32 + kw * 16 + kGHalf) : Bf[kw][0];
      }
    };
    frag(0, fa[0], fb[0]);
#pragma unroll
    for (int ks = 0; ks < kSegW / 2; ++ks) {
      const int c = ks & 1;
      if (ks + 1 < kSegW / 2) frag(ks + 1, fa[c ^ 1], fb[c ^ 1]);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int i = 0; i < WM; ++i)
          acc[kw][i] = prec::mma<PM>(fa[c][i][0], fa[c][i][1], fb[c][kw][0], fb[c][kw][1], acc[kw][i]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  if constexpr (PF2) {
    // prologue: stage 0 staged; stages 1 and 2 in the register sets B and A
    use_buf(0);
    if (nstage > 0) {
      load16x(0, d16, g16);
      store16x(d16, g16);
    }
    if (nstage > 1) {
      adv_stage();
      load16x(1, d16b, g16b);
    }
    if (nstage > 2) {
      adv_stage();
      load16x(2, d16, g16);
    }
    // stage st: its MFMAs, then stage st + 1 from the set that holds it into the other buffer, and
    // stage st + 3 into that set (unrolled by two: the set is compile-time)
    auto step = [&](int st, auto& D16, auto& G16) __attribute__((always_inline)) {
      use_buf(st & 1);
      __syncthreads();              // stage st staged by every wave; buffer (st+1)&1 read by nobody now
      compute();
      if (st + 1 < nstage) {
        use_buf((st + 1) & 1);
        store16x(D16, G16);
        if (st + 3 < nstage) {
          adv_stage();
          load16x(st + 3, D16, G16);
        }
      }
    };
    for (int st = 0; st < nstage; st += 2) {
      step(st, d16b, g16b);
      if (st + 1 < nstage) step(st + 1, d16, g16);
    }
  } else {
  if constexpr (kTr) {
    // prologue: stage 0 staged, stage 1 in registers
    if (nstage > 0) {
      load(0);
      store();
    }
    if (nstage > 1) {
      adv_stage();
      load(1);
    }
  } else if (nstage > 0) {
    load(0);
  }
  for (int st = 0; st < nstage; ++st) {
    if constexpr (kTr) {
      use_buf(st & 1);
      __syncthreads();              // stage st staged by every wave; buffer (st+1)&1 read by nobody now
    } else {
      store();
      __syncthreads();
      if (st + 1 < nstage) {                        // lands during this stage's MFMAs
        adv_stage();
        load(st + 1);
      }
    }
    compute();
    if constexpr (kTr) {
      if (st + 1 < nstage) {
        use_buf((st + 1) & 1);
        store();                    // stage st+1 (loaded one stage ago) into the other buffer
        if (st + 2 < nstage) {
          adv_stage();
          load(st + 2);
        }
      }
    } else {
      __syncthreads();
    }
  }
  }

  // slab[z][t][co][ci]: lane li = ci column, register r = co row (r & 3) + 8 (r >> 2) + 4 lh
#pragma unroll
  for (int kw = 0; kw < 3; ++kw) {
    const int t = (kd * 3 + kh) * 3 + kw;
    float* slab = a.ws + ((int64_t)z * 27 + t) * a.Cd * a.Cg;
    const int col = ci0 + wn0 + li;
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = co0 + wm0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lh;
        slab[(int64_t)row * a.Cg + col] = acc[kw][i][r];
      }
  }
}

static bool w3_wide(const WgradArgs& a) { return a.Cd % 128 == 0 && a.Cg % 64 == 0; }

// segment width: 16, or 24 on the aligned operand-plane path (whole w-runs per 8-segment stage)
static int w3_segw(const WgradArgs& a) {
  if (a.Wd % kSegW == 0) return kSegW;
  if (a.in16 && a.Wd % 24 == 0) {
    const int nsw = a.Wd / 24;
    if (kR % nsw == 0 && a.Hd % (kR / nsw) == 0) return 24;
  }
  return 0;
}

bool wgrad3_x3_applicable(const WgradArgs& a) {
  return a.x3 && a.k == 3 && a.s == 1 && a.p == 0 && w3_segw(a) != 0 && a.Dg == a.Dd + 2 && a.Hg == a.Hd + 2 &&
         a.Wg == a.Wd + 2 && a.Cd % kTile == 0 && a.Cg % kTile == 0 &&
         (int64_t)a.N * a.Dg * a.Hg * a.Wg * a.Cg * 4 < ((int64_t)1 << 31) &&     // byte offsets are 32-bit
         (int64_t)a.N * a.Dd * a.Hd * a.Wd * a.Cd * 4 < ((int64_t)1 << 31);
}

// splits: at most 2 blocks per CU in total (one round: a 513th block doubles the time),
// ≥ 4 stages per block; never more than the generic plan's (its workspace query sizes the slabs)
int wgrad3_x3_splits(const WgradArgs& a, int max_splits) {
  const int nseg = (a.N + a.N2) * a.Dd * a.Hd * (a.Wd / w3_segw(a));
  const bool wide = w3_wide(a);
  const int tiles = (a.Cd / (wide ? 128 : kTile)) * (a.Cg / kTile) * 9;
  static const int budget = [] {                              // A/B switch: MRAGAN_W3_BLOCKS
    const char* e = getenv("MRAGAN_W3_BLOCKS");
    return e ? atoi(e) : 0;
  }();
  // wide tiles: a 192-block budget (10 splits for the 128-channel ResnetBlock convs) — in the
  // two-lane step fewer, longer blocks beat one block per CU (same box, r03k: 13.14 ms at 192,
  // 13.20 at 128, 13.36 at 256: the split-K slabs and their reduce shrink, the other lane
  // fills the CUs left)
  int s = (budget > 0 ? budget : (wide ? 192 : 512)) / tiles;
  const int by_len = nseg / (4 * kR);
  if (s > by_len) s = by_len;
  if (s > max_splits) s = max_splits;
  if (s < 1) s = 1;
  return s;
}

template <int TC, int TI, int PM, int X16, int AL, int SW = kSegW, int WM = 1, int PF2 = 0>
static void launch_wgrad3(const Wgrad3Args& a, int blocks, hipStream_t st) {
  if constexpr ((X16 && prec::has_lo<PM>()) || ((SW != kSegW || WM != 1 || PF2) && !(X16 && AL))) {
    return;                                     // rejected by the caller
  } else {
    constexpr bool tr = !prec::has_lo<PM>();
    constexpr bool wide = TC == 128;
    const int lds = SW != kSegW ? lds_tr<SW, TC>() : wide ? (tr ? kLdsTrW : kLdsW) : (tr ? kLdsTr : kLds);
    static_assert(SW == kSegW || lds_tr<SW, TC>() <= 160 * 1024, "LDS");
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(wgrad3_x3_kernel<TC, TI, PM, X16, AL, SW, WM, PF2>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      attr_set = true;
    }
    hipLaunchKernelGGL((wgrad3_x3_kernel<TC, TI, PM, X16, AL, SW, WM, PF2>), dim3(blocks), dim3(TC * TI / (16 * WM)), lds,
                       st, a);
  }
}

int conv_wgrad3_x3(const WgradArgs& g, int splits, hipStream_t st) {
  Wgrad3Args a{};
  a.dy = g.D; a.N = g.N; a.D = g.Dd; a.H = g.Hd; a.W = g.Wd; a.Cd = g.Cd;
  a.x = g.G; a.Cg = g.Cg;
  a.ws = g.ws;
  const int segw = w3_segw(g);
  if (!segw) {
    set_error("wgrad3_x3: width %d is not a multiple of 16 (or of 24 on the operand-plane path)", g.Wd);
    return -kBadArg;
  }
  a.nseg = (g.N + g.N2) * g.Dd * g.Hd * (g.Wd / segw);
  a.nseg1 = g.N * g.Dd * g.Hd * (g.Wd / segw);
  a.dy2 = g.N2 ? g.D2 : g.D; a.x2 = g.N2 ? g.G2 : g.G; a.N2 = g.N2;
  int per = (a.nseg + splits - 1) / splits;
  per = (per + kR - 1) / kR * kR;
  a.seg_per_split = per;
  const int nsplit = (a.nseg + per - 1) / per;
  const bool wide = w3_wide(g);
  const int blocks = ((g.Cd / (wide ? 128 : kTile)) * (g.Cg / kTile) * 9 * nsplit + 7) / 8 * 8;   // XCD remap needs % 8
  if (g.in16 && g.x3 != kPrecBf16 && g.x3 != kPrecF16) {
    set_error("wgrad3_x3: 16-bit operand planes need the bf16 or fp16 mode");
    return -kBadArg;
  }
  // aligned stages: whole w-runs of rows of one plane per stage, every stage full
  const int nsw = g.Wd / segw;
  static const bool no_al = getenv("MRAGAN_W3_NO_AL") != nullptr;   // A/B switch
  const bool al = !no_al && kR % nsw == 0 && g.Hd % (kR / nsw) == 0 && a.nseg % kR == 0 && per % kR == 0;
  if (segw != kSegW && !(al && g.in16)) {
    set_error("wgrad3_x3: 24-voxel segments need aligned stages on operand planes");
    return -kBadArg;
  }
  // two instance sets: the aligned operand-plane path only (the caller runs two passes otherwise)
  if (g.N2 && !(al && g.in16)) return -kUnsupported;
  MRAGAN_PREC_DISPATCH(g.x3, {
    // 64-row waves on the wide aligned operand-plane tiles: opt-in A/B (MRAGAN_W3_WM=2), measured
    // slower than the 8-wave tiles (res wgrad [4×16³] 34.2 vs 32.2 µs, [2×32³] 90.3 vs 81.9 µs,
    // r04r): the LDS reads were not the limiter, the two waves per SIMD are worth more
    static const bool wm2 = [] { const char* e = getenv("MRAGAN_W3_WM"); return e && atoi(e) == 2; }();
    // two register sets of staged operands on the wide operand-plane tiles: opt-in A/B
    // (MRAGAN_W3_PF2=1), measured neutral — res wgrad [4+2×16³] 37.5 vs 37.4 µs (rocprof), headline
    // 9.75-9.77 vs 9.71-9.78 ms, 128³ 28.50-28.52 vs 28.53-28.57 ms (r06y): the staged loads' latency
    // is not what parks these waves
    static const bool pf1 = getenv("MRAGAN_W3_PF2") == nullptr;
    if (segw != kSegW) {
      if (wide) {
        if (wm2) launch_wgrad3<128, 64, PM, 1, 1, 24, 2>(a, blocks, st);
        else if (!pf1) launch_wgrad3<128, 64, PM, 1, 1, 24, 1, 1>(a, blocks, st);
        else launch_wgrad3<128, 64, PM, 1, 1, 24>(a, blocks, st);
      } else {
        launch_wgrad3<64, 64, PM, 1, 1, 24>(a, blocks, st);
      }
      return nsplit;
    }
    if (wide) {
      if (g.in16 && al && wm2) launch_wgrad3<128, 64, PM, 1, 1, kSegW, 2>(a, blocks, st);
      else if (g.in16) {
        if (al && !pf1) launch_wgrad3<128, 64, PM, 1, 1, kSegW, 1, 1>(a, blocks, st);
        else if (al) launch_wgrad3<128, 64, PM, 1, 1>(a, blocks, st);
        else launch_wgrad3<128, 64, PM, 1, 0>(a, blocks, st);
      }
      else { if (al) launch_wgrad3<128, 64, PM, 0, 1>(a, blocks, st); else launch_wgrad3<128, 64, PM, 0, 0>(a, blocks, st); }
    } else {
      if (g.in16) { if (al) launch_wgrad3<64, 64, PM, 1, 1>(a, blocks, st); else launch_wgrad3<64, 64, PM, 1, 0>(a, blocks, st); }
      else { if (al) launch_wgrad3<64, 64, PM, 0, 1>(a, blocks, st); else launch_wgrad3<64, 64, PM, 0, 0>(a, blocks, st); }
    }
    return nsplit;
  })
}

}  // namespace mragan
