// bf16x3 weight gradient of the stride-2 k3 p1 convolutions of the generator (gfx950):
//
//   G down convs   Conv3d(c → 2c, k3, s2, p1)                 networks3D.py:192-197
//                  dW[co][ci][t] = Σ_m dY[m][co] · X[2m − 1 + t][ci]
//   G up convs     ConvTranspose3d(2c → c, k3, s2, p1, op1)   networks3D.py:203-210
//                  dW[ci][co][t] = Σ_i X[i][ci] · dY[2i − 1 + t][co]
//
// Both are  Out[dn][gn][t] = Σ_m D[m][dn] · G[2m − 1 + t][gn]  with D on the coarse grid and G
// on the fine grid (2× per axis).  conv_wgrad_x3 runs one GEMM per tap and re-reads D and G for
// each of the 27 taps (PMC: 4× the operands' bytes fetched from HBM, MFMA busy < 20 %).  Here, as
// in conv_wgrad3_x3.hip, a block owns one (kd, kh) pair and all three kw taps, the contraction
// runs over row segments (n, d, h, 16 coarse w) 8 per stage with K index k = w·8 + r, and one
// staged G tile serves all three taps: along w the taps read the fine positions 2w − 1, 2w,
// 2w + 1, so the G row is staged as its even phase E[j] = G[2(w0 + j)] (slots 0–15) and odd
// phase O[j] = G[2(w0 + j) + 1], j = −1 … 15 (slots 16–32): tap kw = 1 reads E[w], kw = 0 reads
// O[w − 1], kw = 2 reads O[w] — each a plain 16-B fragment read at a fixed slot offset.  The 33
// staged fine positions of a segment are contiguous in memory (2w0 − 1 … 2w0 + 31).
//
// Tiles: 64 D-channels × TG G-channels.  TG = 64: 4 waves as 2 × 2 32×32 sub-tiles.  TG = 32
// (the 32-channel side at full resolution): 4 waves as 2 sub-tiles × 2 K halves (even / odd
// K-steps), the halves added in LDS before the slab store.  Split-K partial tiles go to slabs
// ws[z][t][dn][gn], reduced in fixed order by wgrad_reduce_kernel (deterministic).
#include <type_traits>

#include "kernels.h"
#include "prec.h"

namespace mragan {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kTD = 64;                             // D channels per block
constexpr int kR = 8;                               // row segments per stage
constexpr int kSegW = 16;                           // coarse voxels per row segment
constexpr int kGPos = 2 * kSegW + 1;                // 33 fine positions per segment
constexpr int kDRow = 2 * kSegW * 16 + 16;          // 528 B: hi 16 slots, lo 16 slots, pad
constexpr int kGRow = 2 * kGPos * 16 + 16;          // 1072 B: hi 33 slots, lo 33 slots, pad
constexpr int kDHalf = kSegW * 16;
constexpr int kGHalf = kGPos * 16;

// fine position q (0 … 32) of a segment → its slot: odd positions (q even) are the O phase
__device__ __forceinline__ int gslot(int q) { return (q & 1) ? (q - 1) >> 1 : 16 + (q >> 1); }

// One-plane modes (bf16 / fp16), as conv_wgrad3_x3.hip's: the tiles are staged in natural
// [K row][channel] order — row = slot·8 + r (slot: the coarse w of D, the phase slot of G), each
// thread converts its float4 (4 channels of one voxel) and stores 8 B — and the MFMA operands come
// out of LDS through ds_read_b64_tr_b16 (lane 4q+p of a 16-lane group addresses row q, channels
// 4p … 4p+3).  Rows of ≥ 128 B XOR their 16-B chunks by the row so the transposed reads are
// conflict-free; the 64-B rows of a 32-channel G tile put a group's 4 rows on disjoint banks as
// they are.  No fp32 → bf16 hi/lo transposition in VALU (the split staging was 29 VALU + 38 SALU
// per MFMA, PMC r03v).
constexpr int kTrRowsD = kSegW * kR;        // 128
constexpr int kTrRowsG = kGPos * kR;        // 264
template <int RB>
__device__ __forceinline__ int tr_swz(int row) {
  return RB == 256 ? (row & 3) << 2 : RB == 128 ? ((row >> 1) & 1) << 2 : 0;
}
typedef short tr_v4s __attribute__((ext_vector_type(4)));
__device__ __forceinline__ tr_v4s tr_read(const char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) tr_v4s*)(p));
}
template <int TG>
constexpr int tr_stage() { return kTrRowsD * kTD * 2 + kTrRowsG * TG * 2; }

// KW = 4: the k4 s2 p1 convolutions (PatchGAN layers 2-3, networks3D.py:389-400; the UNet's down
// convs and, as G = dY, its k4 s2 p1 transposed up convs, networks3D.py:300-330), one-plane modes.
// Along w the four taps read the fine positions 2w − 1 … 2w + 2 = O[w − 1], E[w], O[w], E[w + 1]:
// the segment stages 34 fine positions (2w0 − 1 … 2w0 + 32), E in slots 0 … 16, O from slot 17.
// SW = 8: 8-voxel coarse segments for the 8-wide levels (the UNet's 8³, the PatchGAN's layer-3
// gradient), one-plane modes on fp32 operands; a stage is then 64 K rows (4 K-steps)
template <int KW, int SW = kSegW> constexpr int gpos() { return 2 * SW + KW - 2; }      // 33 | 34 (SW 16)
template <int KW, int SW = kSegW> constexpr int obase() { return SW + (KW == 4 ? 1 : 0); }   // first O-phase slot
template <int KW, int SW = kSegW> __device__ __forceinline__ int gslot_k(int q) {
  return (q & 1) ? (q - 1) >> 1 : obase<KW, SW>() + (q >> 1);
}
template <int TG, int KW, int SW = kSegW> constexpr int tr_stage_k() {
  return SW * kR * kTD * 2 + gpos<KW, SW>() * kR * TG * 2;
}

// one channel of the 8 segments → 16 B hi at p, 16 B lo at p + half
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

struct Wgrad3s2Args {
  const float* d; int N, D, H, W, Cd;     // D [N][D][H][W][Cd] (coarse)
  const float* g; int Cg;                 // G [N][2D][2H][2W][Cg] (fine; X16G: its 16-bit operand plane)
  float* ws;                              // slabs [splits][27][Cd][Cg]
  int nseg, seg_per_split;
};

// X16G: G is the producer's 16-bit operand plane (bf16 / fp16 words): its staging units are
// (fine position, 8-channel octet), one 16-B load each, stored as they are (one-plane modes);
// X16G = 2: D too (ABI 16: G down2's weight gradient, whose dY exists only as its plane) — D units
// (coarse w, octet, segment half): 4 segments × 16 B per thread
template <int TG, int PM, int AL, int X16G, int KW, int SW>
__global__ void __launch_bounds__(256) wgrad3s2_x3_kernel(Wgrad3s2Args a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool kTr = !prec::has_lo<PM>();
  static_assert(KW == 3 || (kTr && !X16G), "k4: the one-plane modes on fp32 operands");
  static_assert(SW == kSegW || (kTr && !X16G), "8-voxel segments: the one-plane modes on fp32 operands");
  constexpr int kGPos = gpos<KW, SW>();   // shadows the file constant (33) in this kernel
  constexpr int kSegW = SW;               // (and the segment width)
  constexpr int kTrRowsD = SW * kR;       // D rows per stage
  static_assert(!X16G || kTr, "16-bit operand planes exist in the one-plane modes only");
  constexpr bool kDp = X16G == 2;         // D as a 16-bit plane too
  constexpr int ESG = X16G ? 2 : 4;       // bytes per G element
  constexpr int ESD = kDp ? 2 : 4;        // bytes per D element
  constexpr int RBD = kTD * 2, RBG = TG * 2;        // tr: row bytes of the D / G images
  char* Ds = smem;
  char* Gs = smem + (kTr ? kTrRowsD * RBD : kTD * kDRow);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  // TG = 64: wave → (dn half, gn half); TG = 32: wave → (dn half, K half)
  const int wm0 = (wave >> 1) * 32;
  const int wn0 = TG == 64 ? (wave & 1) * 32 : 0;
  const int kpar = TG == 64 ? -1 : (wave & 1);

  // logical block: (dn tile, gn tile) fastest, then (kd, kh), then split; XCD-aware remap
  const int ndn = a.Cd / kTD, ngn = a.Cg / TG;
  const int B = gridDim.x;
  int L = blockIdx.x;
  if ((B & 7) == 0) L = (L & 7) * (B >> 3) + (L >> 3);
  const int tile = L % (ndn * ngn);
  const int kk9 = (L / (ndn * ngn)) % (KW * KW);
  const int z = L / (ndn * ngn * KW * KW);
  const int dn0 = (tile / ngn) * kTD, gn0 = (tile % ngn) * TG;
  const int kd = kk9 / KW, kh = kk9 % KW;
  const int seg_lo = z * a.seg_per_split;
  if (seg_lo >= a.nseg) return;                    // grid padding (a multiple of 8 blocks)
  const int seg_hi = min(a.nseg, seg_lo + a.seg_per_split);
  const int nstage = (seg_hi - seg_lo + kR - 1) / kR;

  const int Dg = 2 * a.D, Hg = 2 * a.H, Wg = 2 * a.W;
  const int nsw = a.W / kSegW;
  // staging units, channel quad fastest.  D: (w = tid >> 4, cq = tid & 15).
  // G: TG / 4 channel quads × 33 positions: q = tid / (TG/4) (+ 256/(TG/4) for the second pass)
  // and the last position(s) on the first threads (the others re-read their own unit).
  constexpr int GQ = TG / 4;                       // channel quads of G
  constexpr int GP = 256 / GQ;                     // positions per pass: 16 (TG 64) or 32 (TG 32)
  constexpr int GPASS = kGPos / GP;                // full passes: 2 or 1
  const int cq = tid & 15, uw = tid >> 4;
  const bool dact = uw < SW;                       // SW 8: threads 128 … 255 stage no D unit
  const int gcq = tid % GQ, gq = tid / GQ;
  const int gqx = GPASS * GP + gq;                 // the remainder pass (q = 32 …)
  const bool gx = gqx < kGPos;
  // X16G units: (q8 = tid / GO, octet go = tid % GO); TG 32: one pass covers the 33 positions,
  // TG 64: 32 of them, the last one (q8x = 32) on the first GO threads (wave 0 only: the other
  // waves branch round it)
  constexpr int GO = TG / 8;
  const int go = tid % GO, q8 = tid / GO;
  const bool g8 = q8 < kGPos;
  constexpr bool kG8X = X16G && 256 / GO < kGPos;
  const int q8x = 256 / GO + q8;
  const bool g8x = kG8X && q8x < kGPos;

  float4 rd[kR], rg[2][kR], rgx[kR];
  uint4 rd8[kDp ? kR / 2 : 1];
  const int uwd = (tid & 127) >> 3, od8 = tid & 7, rhd = __builtin_amdgcn_readfirstlane(tid >> 7);
  uint4 rg8[X16G ? kR : 1], rg8x[kG8X ? kR : 1];
  // D / G rows through buffer descriptors: segment / row parts of the offsets are wave-uniform
  // (SGPR soffset); out-of-range rows and positions read zeros through an out-of-range voffset
  // (no select on the loaded values, no 64-bit address arithmetic)
  const __amdgpu_buffer_rsrc_t dr = make_rsrc(a.d, __builtin_amdgcn_readfirstlane(a.N * a.D * a.H * a.W * a.Cd * ESD));
  const __amdgpu_buffer_rsrc_t gr = make_rsrc(a.g, __builtin_amdgcn_readfirstlane(a.N * Dg * Hg * Wg * a.Cg * ESG));
  const int dlane = dact ? (uw * a.Cd + dn0 + 4 * cq) * 4 : (int)kOobOffset;
  const int dlane8 = (uwd * a.Cd + dn0 + 8 * od8) * 2;             // kDp: octet od8 of coarse voxel uwd
  const int dseg = kSegW * a.Cd * ESD;
  int sw = seg_lo % nsw, sh = (seg_lo / nsw) % a.H, sd = (seg_lo / nsw / a.H) % a.D, sn = seg_lo / nsw / a.H / a.D;
  auto bump = [&](int& w_, int& h_, int& d_, int& n_) __attribute__((always_inline)) {
    if (++w_ == nsw) { w_ = 0; if (++h_ == a.H) { h_ = 0; if (++d_ == a.D) { d_ = 0; ++n_; } } }
  };
  // AL (aligned stages, the host checks): a stage's kR segments are whole coarse rows (kR / nsw of
  // them) of one (n, d) plane and every stage is full, so segment r's G row is the stage's first
  // fine row + 2·(r / nsw) and its w run starts 32·(r % nsw) fine voxels in — wave-uniform
  // constants; the only out-of-range G reads left are the fine row −1 (d or h = 0 with kd or kh =
  // 0) and the fine voxel −1 (lane q = 0 of a row's first segment).  The per-segment carries and
  // range checks were ~35 SALU per MFMA (PMC r04p).
  const int gplane_b = Wg * a.Cg * ESG;                             // G bytes per fine row
  const int glane_al = ((gq - 1) * a.Cg + gn0 + 4 * gcq) * 4;      // fine voxel q − 1 of a run
  const int glane_alx = (((gx ? gqx : gq) - 1) * a.Cg + gn0 + 4 * gcq) * 4;
  const int glane_al8 = ((q8 - 1) * a.Cg + gn0 + 8 * go) * 2;      // X16G: octet go of fine voxel q8 − 1
  const int glane_al8x = ((q8x - 1) * a.Cg + gn0 + 8 * go) * 2;
  auto load_al = [&](int st) __attribute__((always_inline)) {
    // stage base: (sn, sd, sh) is its first row (sw = 0)
    const int dso0 = __builtin_amdgcn_readfirstlane((seg_lo + st * kR) * dseg);
    const int gd = 2 * sd - 1 + kd;
    const bool dok = (unsigned)gd < (unsigned)Dg;
    const int gh0 = 2 * sh - 1 + kh;                                 // fine row of segment 0
    const int gbase = __builtin_amdgcn_readfirstlane(((sn * Dg + (dok ? gd : 0)) * Hg + (gh0 < 0 ? 0 : gh0)) * gplane_b);
    if constexpr (kDp) {
#pragma unroll
      for (int j = 0; j < kR / 2; ++j)
        rd8[j] = __builtin_bit_cast(uint4, buf_load_16b(dr, dlane8, dso0 + (kR / 2 * rhd + j) * dseg));
    }
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      if constexpr (!kDp) {
        const buf_f32x4 dv = buf_load_16b(dr, dlane, dso0 + r * dseg);
        rd[r] = make_float4(dv.x, dv.y, dv.z, dv.w);
      }
      const int rr = r / nsw, wr = r - rr * nsw;                     // coarse row / run of the segment
      // (KW 4: the fine row past the last, 2H, on the last coarse row with kh = 3)
      const bool rok = dok && (gh0 >= 0 || rr > 0) && (KW == 3 || gh0 + 2 * rr < Hg);
      // gh0 < 0 only for segment rows rr = 0 (then invalid): rows rr > 0 start at fine row gh0 + 2rr.
      // The soffset carries the row only; the run's w start goes into the (non-negative) voffset:
      // the range check must see the lane's real offset
      const int gso = __builtin_amdgcn_readfirstlane(gbase + (gh0 < 0 ? 2 * rr - 1 : 2 * rr) * gplane_b);
      const int wrun = 2 * SW * wr * a.Cg * ESG;
      const bool w_edge = wr == 0;                                   // fine voxel −1 is outside
      const bool w_redge = KW == 4 && wr == nsw - 1;                 // KW 4: fine voxel 2W too
      if constexpr (X16G) {
        const bool ok8 = rok && g8 && !(w_edge && q8 == 0);
        rg8[r] = __builtin_bit_cast(uint4, buf_load_16b(gr, ok8 ? glane_al8 + wrun : (int)kOobOffset, gso));
        continue;
      }
#pragma unroll
      for (int pass = 0; pass < GPASS; ++pass) {
        const int q = pass * GP + gq;
        const bool ok = rok && !(w_edge && q == 0) && !(w_redge && q == kGPos - 1);
        const buf_f32x4 v = buf_load_16b(gr, ok ? glane_al + wrun + pass * GP * a.Cg * 4 : (int)kOobOffset, gso);
        rg[pass][r] = make_float4(v.x, v.y, v.z, v.w);
      }
      const int qx = gx ? gqx : gq;
      const bool okx = rok && !(w_edge && qx == 0) && !(w_redge && qx == kGPos - 1);
      const buf_f32x4 v = buf_load_16b(gr, okx ? glane_alx + wrun : (int)kOobOffset, gso);
      rgx[r] = make_float4(v.x, v.y, v.z, v.w);
    }
    if constexpr (kG8X) {
      // the 33rd fine position (wave 0's first GO lanes): one branch for the stage's 8 loads
      if (g8x) {
#pragma unroll
        for (int r = 0; r < kR; ++r) {
          const int rr = r / nsw, wr = r - rr * nsw;
          const bool rok = dok && (gh0 >= 0 || rr > 0);
          const int gso = __builtin_amdgcn_readfirstlane(gbase + (gh0 < 0 ? 2 * rr - 1 : 2 * rr) * gplane_b);
          rg8x[r] = __builtin_bit_cast(uint4, buf_load_16b(gr, rok ? glane_al8x + 2 * SW * wr * a.Cg * ESG : (int)kOobOffset, gso));
        }
      }
    }
  };
  auto load = [&](int st) __attribute__((always_inline)) {
    if constexpr (AL) {
      load_al(st);
      return;
    }
    if constexpr (kDp) {
#pragma unroll
      for (int j = 0; j < kR / 2; ++j) {
        const int seg = seg_lo + st * kR + kR / 2 * rhd + j;
        const bool ok = seg < seg_hi;
        const int dso = __builtin_amdgcn_readfirstlane(ok ? seg * dseg : 0);
        rd8[j] = __builtin_bit_cast(uint4, buf_load_16b(dr, ok ? dlane8 : (int)kOobOffset, dso));
      }
    }
    int cw = sw, chh = sh, cdd = sd, cn = sn;
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const int seg = seg_lo + st * kR + r;
      const bool ok = seg < seg_hi;
      const int n = ok ? cn : 0, d = ok ? cdd : 0, h = ok ? chh : 0;
      const int w0 = (ok ? cw : 0) * kSegW;
      bump(cw, chh, cdd, cn);
      // D segments are contiguous 16-voxel runs: offset linear in the segment index
      if constexpr (!kDp) {
        const int dso = __builtin_amdgcn_readfirstlane(ok ? seg * dseg : 0);
        const buf_f32x4 dv = buf_load_16b(dr, ok ? dlane : (int)kOobOffset, dso);
        rd[r] = make_float4(dv.x, dv.y, dv.z, dv.w);
      }
      const int gd = 2 * d - 1 + kd, gh = 2 * h - 1 + kh;
      const bool rok = ok && (unsigned)gd < (unsigned)Dg && (unsigned)gh < (unsigned)Hg;
      const int gso = __builtin_amdgcn_readfirstlane(rok ? ((n * Dg + gd) * Hg + gh) * Wg * a.Cg * ESG : 0);
      if constexpr (X16G) {
        const int p = 2 * w0 - 1 + q8;
        const bool pok = rok && g8 && (unsigned)p < (unsigned)Wg;
        rg8[r] = __builtin_bit_cast(uint4, buf_load_16b(gr, pok ? (p * a.Cg + gn0 + 8 * go) * 2 : (int)kOobOffset, gso));
        if constexpr (kG8X) {
          if (g8x) {
            const int px = 2 * w0 - 1 + q8x;
            const bool pokx = rok && (unsigned)px < (unsigned)Wg;
            rg8x[r] = __builtin_bit_cast(uint4, buf_load_16b(gr, pokx ? (px * a.Cg + gn0 + 8 * go) * 2 : (int)kOobOffset, gso));
          }
        }
        continue;
      }
      auto gload = [&](int q) __attribute__((always_inline)) {
        const int p = 2 * w0 - 1 + q;
        const bool pok = rok && (unsigned)p < (unsigned)Wg;
        const buf_f32x4 v = buf_load_16b(gr, pok ? (p * a.Cg + gn0 + 4 * gcq) * 4 : (int)kOobOffset, gso);
        return make_float4(v.x, v.y, v.z, v.w);
      };
#pragma unroll
      for (int pass = 0; pass < GPASS; ++pass) rg[pass][r] = gload(pass * GP + gq);
      rgx[r] = gload(gx ? gqx : gq);
    }
  };
  // one unit: 8 segments × 4 channels → 4 rows × (16 B hi + 16 B lo) at `slot`; write j of a
  // lane goes to channel (j + rot) & 3, rot = (c >> 1) & 3 (conflict-free 8-lane write groups for
  // both row strides: 33 and 67 16-B units per row)
  auto put = [&](char* base, int row_bytes, int half, int slot, int c, const float4 (&v)[kR]) __attribute__((always_inline)) {
    const int rot = (c >> 1) & 3;
    auto rotv = [&](const float4& x) __attribute__((always_inline)) {
      const float4 t = (rot & 1) ? make_float4(x.y, x.z, x.w, x.x) : x;
      return (rot & 2) ? make_float4(t.z, t.w, t.x, t.y) : t;
    };
    float4 u[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) u[r] = rotv(v[r]);
    char* p = base + (4 * c) * row_bytes + slot * 16;
    split8_store<PM>(p + ((0 + rot) & 3) * row_bytes, half, u[0].x, u[1].x, u[2].x, u[3].x, u[4].x, u[5].x, u[6].x, u[7].x);
    split8_store<PM>(p + ((1 + rot) & 3) * row_bytes, half, u[0].y, u[1].y, u[2].y, u[3].y, u[4].y, u[5].y, u[6].y, u[7].y);
    split8_store<PM>(p + ((2 + rot) & 3) * row_bytes, half, u[0].z, u[1].z, u[2].z, u[3].z, u[4].z, u[5].z, u[6].z, u[7].z);
    split8_store<PM>(p + ((3 + rot) & 3) * row_bytes, half, u[0].w, u[1].w, u[2].w, u[3].w, u[4].w, u[5].w, u[6].w, u[7].w);
  };
  // tr: unit (slot, channel quad c) → rows slot·8 + r, 8 B at chunk c/2 (swizzled), half c&1
  auto put16 = [&](char* base, auto rb_c, int slot, int c, const float4 (&v)[kR]) __attribute__((always_inline)) {
    constexpr int RB = decltype(rb_c)::value;
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const int row = slot * kR + r;
      uint2 h, l;
      prec::split4<PM>(v[r], h, l);
      *reinterpret_cast<uint2*>(base + row * RB + 16 * ((c >> 1) ^ tr_swz<RB>(row)) + 8 * (c & 1)) = h;
    }
  };
  // X16G: unit (slot, octet o) → rows slot·8 + r, the 16 B at chunk o (swizzled)
  auto put8 = [&](char* base, int slot, int o, const uint4 (&v)[kR]) __attribute__((always_inline)) {
    if constexpr (X16G) {
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        const int row = slot * kR + r;
        *reinterpret_cast<uint4*>(base + row * RBG + 16 * (o ^ tr_swz<RBG>(row))) = v[r];
      }
    }
  };
  auto store = [&]() __attribute__((always_inline)) {
    if constexpr (kTr) {
      if constexpr (kDp) {
        // unit (coarse w uwd, octet od8) → rows uwd·8 + 4·rhd + j, the 16 B at chunk od8 (swizzled)
#pragma unroll
        for (int j = 0; j < kR / 2; ++j) {
          const int row = uwd * kR + kR / 2 * rhd + j;
          *reinterpret_cast<uint4*>(Ds + row * RBD + 16 * (od8 ^ tr_swz<RBD>(row))) = rd8[j];
        }
      } else {
        if (dact) put16(Ds, std::integral_constant<int, RBD>{}, uw, cq, rd);
      }
      if constexpr (X16G) {
        if (g8) put8(Gs, gslot_k<KW, SW>(q8), go, rg8);
        if constexpr (kG8X)
          if (g8x) put8(Gs, gslot_k<KW, SW>(q8x), go, rg8x);
        return;
      }
#pragma unroll
      for (int pass = 0; pass < GPASS; ++pass)
        put16(Gs, std::integral_constant<int, RBG>{}, gslot_k<KW, SW>(pass * GP + gq), gcq, rg[pass]);
      if (gx) put16(Gs, std::integral_constant<int, RBG>{}, gslot_k<KW, SW>(gqx), gcq, rgx);
      return;
    }
    put(Ds, kDRow, kDHalf, uw, cq, rd);
#pragma unroll
    for (int pass = 0; pass < GPASS; ++pass) put(Gs, kGRow, kGHalf, gslot_k<KW, SW>(pass * GP + gq), gcq, rg[pass]);
    if (gx) put(Gs, kGRow, kGHalf, gslot_k<KW, SW>(gqx), gcq, rgx);
  };
  // tr read offsets: lane 4q+p of its 16-lane group g (lane bit 4) reads row 8h + q (+ the read's
  // K offset) and channels (sub-tile base + 16g + 4p … +3)
  const int tq = (lane & 15) >> 2, tp = lane & 3, tgi = (lane >> 4) & 1;
  const int trA = (8 * lh + tq) * RBD + 16 * (((wm0 + 16 * tgi) / 8 + (tp >> 1)) ^ tr_swz<RBD>(tq)) + 8 * (tp & 1);
  const int trB = (8 * lh + tq) * RBG + 16 * (((wn0 + 16 * tgi) / 8 + (tp >> 1)) ^ tr_swz<RBG>(tq)) + 8 * (tp & 1);
  constexpr int KSTEP = TG == 32 ? 2 : 1, NKS = (kSegW / 2) / KSTEP;
  const int kp = TG == 32 ? __builtin_amdgcn_readfirstlane(kpar) : 0;
  const int trA_k = trA + 16 * kp * RBD, trB_k = trB + 16 * kp * RBG;
  auto use_buf = [&](int b) __attribute__((always_inline)) {       // tr: select stage buffer b
    Ds = smem + b * tr_stage_k<TG, KW, SW>();
    Gs = Ds + kTrRowsD * RBD;
  };

  f32x16 acc[KW];
#pragma unroll
  for (int t = 0; t < KW; ++t) acc[t] = f32x16{};

  auto advance = [&]() __attribute__((always_inline)) {
    if constexpr (AL) {           // whole rows: one carry chain per stage
      sh += kR / nsw;
      if (sh == a.H) { sh = 0; if (++sd == a.D) { sd = 0; ++sn; } }
      return;
    }
#pragma unroll
    for (int r = 0; r < kR; ++r) bump(sw, sh, sd, sn);
  };
  if constexpr (kTr) {
    // two stage buffers: the stage after next is loaded while this one's MFMAs run and stored
    // right after them, so a load has a whole stage to land
    if (nstage > 0) {
      use_buf(0);
      load(0);
      store();
    }
    if (nstage > 1) {
      advance();
      load(1);
    }
  } else if (nstage > 0) {
    load(0);
  }
  for (int st = 0; st < nstage; ++st) {
    if constexpr (kTr) {
      use_buf(st & 1);
      __syncthreads();              // stage st staged by every wave; the other buffer read by nobody now
    } else {
      store();
      __syncthreads();
      if (st + 1 < nstage) {                        // lands during this stage's MFMAs
        advance();
        load(st + 1);
      }
    }
    // TG = 32: this wave's K half is the K-steps ks ≡ kp (mod 2) — a loop over them with the
    // wave-uniform kp folded into the base offsets (a per-step `continue` on the wave index compiled
    // to exec-mask branches around every step: no LDS read could run ahead of the previous MFMAs)
#pragma unroll
    for (int ki = 0; ki < NKS; ++ki) {
      const int ks = KSTEP * ki;                    // + kp (in the bases)
      // K-step ks: coarse w = 2ks + lh × 8 segments
      bf16x8 fa[2], fb[KW][2];
      // tap kw: kw = 1 → E[w] (slot w), kw = 0 → O[w − 1] (slot ob + w), kw = 2 → O[w] (slot ob + 1 + w),
      // kw = 3 (KW 4) → E[w + 1] (slot w + 1); ob = the first O slot (16 | 17)
      if constexpr (kTr) {
        // rows 16ks … 16ks+15 (slots 2ks, 2ks+1 × 8 segments): two 4-row reads per operand
        const char* ar = Ds + trA_k + (16 * ks) * RBD;
        const tr_v4s a0 = tr_read(ar), a1 = tr_read(ar + 4 * RBD);
        fa[0] = fa[1] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7));
        constexpr int kslot[4] = {obase<KW, SW>(), 0, obase<KW, SW>() + 1, 1};
#pragma unroll
        for (int kw = 0; kw < KW; ++kw) {
          const char* br = Gs + trB_k + (16 * ks + kR * kslot[kw]) * RBG;
          const tr_v4s b0 = tr_read(br), b1 = tr_read(br + 4 * RBG);
          fb[kw][0] = fb[kw][1] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(b0, b1, 0, 1, 2, 3, 4, 5, 6, 7));
        }
      } else if constexpr (KW == 3) {
        const char* arow = Ds + (wm0 + li) * kDRow + lh * 16 + 32 * kp;
        const char* brow = Gs + (wn0 + li) * kGRow + lh * 16 + 32 * kp;
        fa[0] = *reinterpret_cast<const bf16x8*>(arow + ks * 32);
        fa[1] = prec::has_lo<PM>() ? *reinterpret_cast<const bf16x8*>(arow + ks * 32 + kDHalf) : fa[0];
        constexpr int koff[3] = {16 * 16, 0, 17 * 16};
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          fb[kw][0] = *reinterpret_cast<const bf16x8*>(brow + ks * 32 + koff[kw]);
          fb[kw][1] = prec::has_lo<PM>() ? *reinterpret_cast<const bf16x8*>(brow + ks * 32 + koff[kw] + kGHalf) : fb[kw][0];
        }
      }
#pragma unroll
      for (int kw = 0; kw < KW; ++kw) acc[kw] = prec::mma<PM>(fa[0], fa[1], fb[kw][0], fb[kw][1], acc[kw]);
    }
    if constexpr (kTr) {
      if (st + 1 < nstage) {
        use_buf((st + 1) & 1);
        store();                    // stage st+1 (loaded one stage ago) into the other buffer
        if (st + 2 < nstage) {
          advance();
          load(st + 2);
        }
      }
    } else {
      __syncthreads();
    }
  }

  // TG = 32: the odd-K waves' partial sums join the even-K waves' through LDS (fixed order)
  if constexpr (TG == 32) {
    if constexpr (kTr) __syncthreads();             // every wave is past its last stage's reads
    float* red = reinterpret_cast<float*>(smem);    // [2 dn halves][KW taps][16][64 lanes]
    if (kpar == 1) {
#pragma unroll
      for (int kw = 0; kw < KW; ++kw)
#pragma unroll
        for (int r = 0; r < 16; ++r) red[(((wave >> 1) * KW + kw) * 16 + r) * 64 + lane] = acc[kw][r];
    }
    __syncthreads();
    if (kpar == 1) return;
#pragma unroll
    for (int kw = 0; kw < KW; ++kw)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[kw][r] += red[(((wave >> 1) * KW + kw) * 16 + r) * 64 + lane];
  }

  // slab[z][t][dn][gn]: lane li = gn column, register r = dn row (r & 3) + 8 (r >> 2) + 4 lh
#pragma unroll
  for (int kw = 0; kw < KW; ++kw) {
    const int t = (kd * KW + kh) * KW + kw;
    float* slab = a.ws + ((int64_t)z * KW * KW * KW + t) * a.Cd * a.Cg;
    const int col = gn0 + wn0 + li;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = dn0 + wm0 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      slab[(int64_t)row * a.Cg + col] = acc[kw][r];
    }
  }
}

// coarse voxels per segment: 16, or 8 for the 8-wide levels (one-plane modes, fp32 operands;
// A/B switch MRAGAN_NO_W3S2_SW8)
static int s2_segw(const WgradArgs& a) {
  static const bool no_sw8 = getenv("MRAGAN_NO_W3S2_SW8") != nullptr;
  if (a.Wd % kSegW == 0) return kSegW;
  if (!no_sw8 && a.Wd % 8 == 0 && (a.x3 == kPrecBf16 || a.x3 == kPrecF16) && !a.in16 && !a.in16g) return 8;
  return 0;
}

bool wgrad3s2_x3_applicable(const WgradArgs& a) {
  static const bool no_k4 = getenv("MRAGAN_NO_W4S2") != nullptr;   // A/B switch
  const bool k4 = !no_k4 && a.k == 4 && (a.x3 == kPrecBf16 || a.x3 == kPrecF16) && !a.in16 && !a.in16g;
  return a.x3 && (a.k == 3 || k4) && a.s == 2 && a.p == 1 && s2_segw(a) != 0 && a.Dg == 2 * a.Dd && a.Hg == 2 * a.Hd &&
         a.Wg == 2 * a.Wd && a.Cd % kTD == 0 && (a.Cg % 64 == 0 || a.Cg == 32) &&
         (int64_t)a.N * a.Dg * a.Hg * a.Wg * a.Cg * 4 < ((int64_t)1 << 31) &&     // byte offsets are 32-bit
         (int64_t)a.N * a.Dd * a.Hd * a.Wd * a.Cd * 4 < ((int64_t)1 << 31);
}

static int s2_tg(const WgradArgs& a) { return a.Cg % 64 == 0 ? 64 : 32; }

static size_t s2_lds(int tg, bool tr, int kw, int sw) {
  if (tr && sw == 8) {
    if (kw == 4) return (size_t)2 * (tg == 64 ? tr_stage_k<64, 4, 8>() : tr_stage_k<32, 4, 8>());
    return (size_t)2 * (tg == 64 ? tr_stage_k<64, 3, 8>() : tr_stage_k<32, 3, 8>());
  }
  if (tr && kw == 4) return (size_t)2 * (tg == 64 ? tr_stage_k<64, 4>() : tr_stage_k<32, 4>());
  if (tr) return (size_t)2 * (tg == 64 ? tr_stage<64>() : tr_stage<32>());
  return (size_t)kTD * kDRow + (size_t)tg * kGRow;
}

// splits: one round of resident blocks (1 per CU at TG 64, 2 at TG 32), ≥ 4 stages per block;
// never more than the generic plan's (its workspace query sizes the slabs)
int wgrad3s2_x3_splits(const WgradArgs& a, int max_splits) {
  const int tg = s2_tg(a);
  const int nseg = a.N * a.Dd * a.Hd * (a.Wd / s2_segw(a));
  const int tiles = (a.Cd / kTD) * (a.Cg / tg) * a.k * a.k;
  static const int scale = [] {                               // A/B switch: MRAGAN_W3S2_BUDGET (percent)
    const char* e = getenv("MRAGAN_W3S2_BUDGET");
    return e ? atoi(e) : 100;
  }();
  int s = (tg == 64 ? 256 : 512) * scale / 100 / tiles;
  const int by_len = nseg / (4 * kR);
  if (s > by_len) s = by_len;
  if (s > max_splits) s = max_splits;
  if (s < 1) s = 1;
  return s;
}

template <int TG, int PM, int AL, int X16G, int KW, int SW = kSegW>
static void launch_w3s2_as(const Wgrad3s2Args& a, int blocks, size_t lds, hipStream_t st) {
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(wgrad3s2_x3_kernel<TG, PM, AL, X16G, KW, SW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((wgrad3s2_x3_kernel<TG, PM, AL, X16G, KW, SW>), dim3(blocks), dim3(256), lds, st, a);
}

template <int TG, int PM, int AL>
static void launch_w3s2(const Wgrad3s2Args& a, int blocks, size_t lds, int planes, int kw, int sw, hipStream_t st) {
  if constexpr (prec::has_lo<PM>()) {
    launch_w3s2_as<TG, PM, AL, 0, 3>(a, blocks, lds, st);   // (planes, k4 and 8-wide rejected by the caller)
  } else {
    if (sw == 8) {
      if (kw == 4) launch_w3s2_as<TG, PM, AL, 0, 4, 8>(a, blocks, lds, st);
      else launch_w3s2_as<TG, PM, AL, 0, 3, 8>(a, blocks, lds, st);
    } else if (kw == 4) launch_w3s2_as<TG, PM, AL, 0, 4>(a, blocks, lds, st);
    else if (planes == 2) launch_w3s2_as<TG, PM, AL, 2, 3>(a, blocks, lds, st);
    else if (planes == 1) launch_w3s2_as<TG, PM, AL, 1, 3>(a, blocks, lds, st);
    else launch_w3s2_as<TG, PM, AL, 0, 3>(a, blocks, lds, st);
  }
}

int conv_wgrad3s2_x3(const WgradArgs& g, int splits, hipStream_t st) {
  Wgrad3s2Args a{};
  a.d = g.D; a.N = g.N; a.D = g.Dd; a.H = g.Hd; a.W = g.Wd; a.Cd = g.Cd;
  a.g = g.G; a.Cg = g.Cg;
  a.ws = g.ws;
  const int segw = s2_segw(g);
  if (!segw) {
    set_error("wgrad3s2_x3: coarse width %d is not a multiple of 16 (8 in the one-plane modes)", g.Wd);
    return -kBadArg;
  }
  a.nseg = g.N * g.Dd * g.Hd * (g.Wd / segw);
  int per = (a.nseg + splits - 1) / splits;
  per = (per + kR - 1) / kR * kR;
  a.seg_per_split = per;
  const int nsplit = (a.nseg + per - 1) / per;
  const int tg = s2_tg(g);
  const int blocks = ((g.Cd / kTD) * (g.Cg / tg) * g.k * g.k * nsplit + 7) / 8 * 8;   // XCD remap needs % 8
  const size_t lds = s2_lds(tg, g.x3 == kPrecBf16 || g.x3 == kPrecF16, g.k, segw);
  // aligned stages: whole coarse rows of one plane per stage, every stage full
  const int nsw = g.Wd / segw;
  static const bool no_al = getenv("MRAGAN_W3S2_NO_AL") != nullptr;   // A/B switch
  const bool al = !no_al && kR % nsw == 0 && g.Hd % (kR / nsw) == 0 && a.nseg % kR == 0 && per % kR == 0;
  static_assert(2 * 3 * 16 * 64 * 4 <= kTD * kDRow, "the K-half reduction fits the D tile");
  static_assert(2 * 3 * 16 * 64 * 4 <= 2 * tr_stage<32>(), "the K-half reduction fits the tr stages");
  static_assert(2 * 4 * 16 * 64 * 4 <= 2 * tr_stage_k<32, 4>(), "the K-half reduction fits the tr stages (k4)");
  static_assert(2 * 4 * 16 * 64 * 4 <= 2 * tr_stage_k<32, 3, 8>(), "the K-half reduction fits the tr stages (8-wide)");
  if (g.k == 4 && (g.x3 == kPrecBf16x3 || g.in16 || g.in16g)) {
    set_error("wgrad3s2_x3: k4 runs the one-plane modes on fp32 operands");
    return -kBadArg;
  }
  if ((g.in16g || g.in16) && g.x3 != kPrecBf16 && g.x3 != kPrecF16) {
    set_error("wgrad3s2_x3: a 16-bit operand plane needs the bf16 or fp16 mode");
    return -kBadArg;
  }
  const int planes = g.in16 ? 2 : g.in16g ? 1 : 0;       // both operands / G only / none
  MRAGAN_PREC_DISPATCH(g.x3, {
    if (tg == 64) {
      if (al) launch_w3s2<64, PM, 1>(a, blocks, lds, planes, g.k, segw, st);
      else launch_w3s2<64, PM, 0>(a, blocks, lds, planes, g.k, segw, st);
    } else {
      if (al) launch_w3s2<32, PM, 1>(a, blocks, lds, planes, g.k, segw, st);
      else launch_w3s2<32, PM, 0>(a, blocks, lds, planes, g.k, segw, st);
    }
    return nsplit;
  })
}

}  // namespace mragan
