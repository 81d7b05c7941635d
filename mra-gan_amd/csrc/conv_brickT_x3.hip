// bf16x3 transposed 3D convolution with stride 2 (k = 3 or 4) from an LDS-resident input halo
// (gfx950).  Serves every stride-2 transposed form of the step:
//
//   G up-convs      ConvTranspose3d(k3 s2 p1 op1)                   networks3D.py:203-210
//   G down-convs    data gradient of Conv3d(k3 s2 p1)               networks3D.py:191-197
//   D layers 2, 3   data gradient of Conv3d(k4 s2 p1)               networks3D.py:395-405
//   UNet            ConvTranspose3d(k4 s2 p1) and down-conv dgrads   networks3D.py:307-343
//
// y[o] = Σ_t x[(o + p − t)/2] · W[t]   over the taps with o + p − t even (per dimension).
// The generic implicit GEMM (conv_igemm_x3) gathers every input row once per tap from L2 — for
// these layers (K = 27·Cin/8 per output parity class, 32–64 output channels) that re-read is the
// bound.  Here a block owns an output brick of 4 × 16 × 16 voxels; its input halo
// 4 × 10 × 10 × (32-channel chunk) sits in LDS (bf16 hi/lo 144-B rows, next chunk prefetched in
// registers), and wave w takes the 4 × 4 × 16 sub-brick at h = 4w…4w+3, which holds exactly one
// 32-voxel M-tile of each of the 8 output parity classes — so every wave runs all 27 (k = 3) or 64
// (k = 4) class taps and the waves stay balanced.  Within a class the input offset of a tap is a
// wave-uniform constant, so an A fragment is one 16-B LDS read at lane base + immediate.
// Weights come pre-split in fragment order from L2 (brickT_pack), used as the MFMA's A operand,
// through buffer loads whose step offset is a scalar (no per-load address VGPRs), D steps ahead.
// The next chunk's halo is read whole at the chunk's first step; out-of-volume positions get an
// offset past the descriptor's range, so the hardware returns the zero padding.  The epilogue
// transposes the accumulators through LDS into whole-voxel 16-B-per-lane non-temporal stores.
// Measured at 4 × 32³ × 64 → 4 × 64³ × 32 (k3): 132 µs (conv_igemm_x3: 304 µs); the store
// stream is the bound (the same kernel without stores: 60 µs).
#include "kernels.h"
#include "prec.h"

namespace mragan {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int kBK = 32;                    // channels per chunk
constexpr int kRow = 144;                  // LDS row: hi 64 B, lo 64 B, 16 B pad (also the epilogue's fp32 voxel row)
// halo row of the one-plane modes (bf16 / fp16): hi 64 B + 16 B pad — the halo buffers take 64 KB
// instead of 115 KB, so two blocks share a CU and one block's epilogue stores overlap the other's
// MFMAs (the store stream bounded the one-block-per-CU kernel: 132 µs with stores, 60 without)
template <int PM>
constexpr int halo_row() { return prec::has_lo<PM>() ? 144 : 80; }
// output brick 4 × 4·NW × 16 for NW waves (each wave 4 × 4 × 16: one 32-voxel tile of each parity
// class); NW = 4 on the large layers, 2 or 1 where 4-wave bricks would leave most CUs idle (the
// UNet's 16³ → 32³ up convs: 32 bricks at N = 1, 34.9 µs)
constexpr int kOD = 4, kOW = 16;
constexpr int kHD = 4, kHW = 10;           // input halo (k ≤ 4, p = 1): 4 × (2·NW + 2) × 10
template <int NW> constexpr int oh_t() { return 4 * NW; }
template <int NW> constexpr int hh_t() { return 2 * NW + 2; }
template <int NW> constexpr int hp_t() { return kHD * hh_t<NW>() * kHW; }   // 400 positions at NW 4

// packed [T][ny][C] fp32 → [T][chunk][kk][hi|lo][ny][lh][8] bf16 (one thread per 8 channels)
template <int PM>
__global__ void brickT_pack_kernel(const float* __restrict__ wp, int T, int ny, int C, __bf16* __restrict__ out) {
  const int nch = C / kBK;
  const int64_t total = (int64_t)T * ny * (C / 8);
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(e % (C / 8));
    const int64_t tn = e / (C / 8);
    const int n = (int)(tn % ny), tap = (int)(tn / ny);
    const float* src = wp + tn * C + g * 8;
    const float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 4);
    bf16x8 hi, lo;
    prec::split8<PM>(a, b, hi, lo);
    const int chunk = g >> 2, kk = (g >> 1) & 1, lh = g & 1;
    const int64_t base = ((((int64_t)tap * nch + chunk) * 2 + kk) * 2) * ny * 16 + (int64_t)n * 16 + lh * 8;
    *reinterpret_cast<bf16x8*>(out + base) = hi;
    if constexpr (prec::has_lo<PM>()) *reinterpret_cast<bf16x8*>(out + base + (int64_t)ny * 16) = lo;
  }
}

__device__ __forceinline__ int floordiv2(int v) { return v >= 0 ? v / 2 : -((1 - v) / 2); }

// Compile-time (class, tap) sequence for p = 1: class c = (cd, ch, cw) runs the taps t ≡ c + 1
// (mod 2) per dimension; its input offset inside the halo is (3 + c − t)/2 per dimension (the
// halo origin is o0/2 − 1 for k = 3 and 4).
struct TStep { signed char c, od, oh, ow; short tap; };
template <int K> struct TSteps {
  static constexpr int N = K == 3 ? 27 : 64;
  TStep s[N];
  constexpr TSteps() : s{} {
    int n = 0;
    for (int c = 0; c < 8; ++c) {
      const int cd = c >> 2, ch = (c >> 1) & 1, cw = c & 1;
      for (int td = (cd + 1) & 1; td < K; td += 2)
        for (int th = (ch + 1) & 1; th < K; th += 2)
          for (int tw = (cw + 1) & 1; tw < K; tw += 2) {
            s[n].c = (signed char)c;
            s[n].od = (signed char)((3 + cd - td) / 2);
            s[n].oh = (signed char)((3 + ch - th) / 2);
            s[n].ow = (signed char)((3 + cw - tw) / 2);
            s[n].tap = (short)((td * K + th) * K + tw);
            ++n;
          }
    }
  }
};

}  // namespace

struct BrickTArgs {
  const float* x; int N, Di, Hi, Wi, C;    // C = contraction channels (multiple of 32)
  const __bf16* wx;                        // brickT_pack output
  const float* bias;
  float* y; int Do, Ho, Wo, ny;            // ny: a multiple of 32, one 32-channel group per block
  int gn;                                  // channel groups (ny / 32)
  int k, p, act;
  int nbd, nbh, nbw;
  double* part;                            // optional: the next InstanceNorm's Σy / Σy² per brick
  // optional with part (ABI 12 form): backward statistics instead — y is the gradient of the
  // InstanceNorm(+sact) of sx (same grid, no fold): Σ g, Σ g·x̂ with g = y·act'(x̂)
  const float* sx; const float* smean; const float* srstd; int sact;
};

// X16 (round 4, one-plane modes): the input is the producer's 16-bit operand plane — a halo
// position's 32-channel chunk is four 16-B units copied to LDS as they are (G up2 on up1's IN plane,
// G down1's data gradient on the plane of its dY)
template <int K, int PM, int X16, int NW>
__global__ void __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(prec::has_lo<PM>() ? 1 : 2, prec::has_lo<PM>() ? 1 : 2)))
brickT_x3_kernel(BrickTArgs a) {
  static_assert(!X16 || !prec::has_lo<PM>(), "16-bit operand planes exist in the one-plane modes only");
  constexpr int NT = 64 * NW;                    // threads
  constexpr int kOH = oh_t<NW>(), kHH = hh_t<NW>(), kHP = hp_t<NW>();
  constexpr int kHRow = halo_row<PM>();
  constexpr int ES = X16 ? 2 : 4;                // bytes per input element
  constexpr int UPP = X16 ? 4 : 8;               // 16-B units per halo position and chunk
  constexpr int NSL = (kHP * UPP + NT - 1) / NT; // units per thread per chunk
  constexpr TSteps<K> ts{};
  constexpr int NS = 2 * TSteps<K>::N;          // (class tap, 16-channel half) steps per chunk
  // weight prefetch distance in steps (divides NS: a ring slot is compile-time in every chunk)
  constexpr int D = K == 3 ? 9 : 8;
  // next-chunk halo: all slices are loaded (from HBM) at step 0 and split + stored at step kHD.
  // vmcnt retires in issue order, so the first weight wait behind those loads (step D) absorbs
  // their latency once per chunk; streaming them in slices instead exposes it once per slice.
  constexpr int kHD = D + 1;
  static_assert(NS % D == 0, "prefetch ring");
  static_assert(kHD < NS / 2, "halo store step");
  extern __shared__ __attribute__((aligned(16))) char smem[];   // 2 × [kHP][kHRow] + [kHP] offsets
  int* hoff = reinterpret_cast<int*>(smem + 2 * kHP * kHRow);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  int blk = blockIdx.x;
  const int bw_i = blk % a.nbw; blk /= a.nbw;
  const int bh_i = blk % a.nbh; blk /= a.nbh;
  const int bd_i = blk % a.nbd; blk /= a.nbd;
  const int nb = blk % a.N;
  const int n0 = (blk / a.N) * 32;               // this block's 32 output channels
  const int o0d = bd_i * kOD, o0h = bh_i * kOH, o0w = bw_i * kOW;
  // halo origin: lowest input index any output of the brick reads (tap k−1)
  const int i0d = floordiv2(o0d + a.p - (a.k - 1)), i0h = floordiv2(o0h + a.p - (a.k - 1)),
            i0w = floordiv2(o0w + a.p - (a.k - 1));
  // byte offsets into this instance's volume; out-of-volume positions get an offset past the
  // descriptor's range, so the buffer load returns zeros (the transposed conv's implicit padding)
  for (int pos = tid; pos < kHP; pos += NT) {
    const int hw = pos % kHW, hh = (pos / kHW) % kHH, hd = pos / (kHW * kHH);
    const int id = i0d + hd, ih = i0h + hh, iw = i0w + hw;
    const bool ok = (unsigned)id < (unsigned)a.Di && (unsigned)ih < (unsigned)a.Hi && (unsigned)iw < (unsigned)a.Wi;
    hoff[pos] = ok ? ((id * a.Hi + ih) * a.Wi + iw) * a.C * ES : (int)0x80000000;
  }
  const int vol_bytes = a.Di * a.Hi * a.Wi * a.C * ES;    // < 2^31 (brickT_x3_applicable)
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(reinterpret_cast<const char*>(a.x)) + (int64_t)nb * vol_bytes, 0, vol_bytes, 0x00020000);
  // uniform scalars (readfirstlane: otherwise the chunk loop bound and every offset derived
  // from the chunk index live in VGPRs)
  const int nch = __builtin_amdgcn_readfirstlane(a.C / kBK);
  const int blkw = __builtin_amdgcn_readfirstlane(a.ny * 32);        // one (hi|lo) block, bytes
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<__bf16*>(a.wx), 0, K * K * K * nch * 4 * blkw, 0x00020000);
  __syncthreads();

  auto halo_off = [&](int s) __attribute__((always_inline)) {
    const int e = s * NT + tid, pos = e / UPP;
    const int o = pos < kHP ? hoff[pos] : (int)0x80000000;
    return o + 16 * (e % UPP);
  };
  auto halo_store = [&](char* buf, int s, const float4& v) __attribute__((always_inline)) {
    const int e = s * NT + tid, pos = e / UPP, q = e % UPP;
    if (pos < kHP) {
      if constexpr (X16) {
        *reinterpret_cast<float4*>(buf + pos * kHRow + 16 * q) = v;    // 8 channels' words, as they are
      } else {
        uint2 h, lo;
        prec::split4<PM>(v, h, lo);
        *reinterpret_cast<uint2*>(buf + pos * kHRow + 8 * q) = h;
        if constexpr (prec::has_lo<PM>()) *reinterpret_cast<uint2*>(buf + pos * kHRow + 64 + 8 * q) = lo;
      }
    }
  };
  auto bload = [&](const __amdgpu_buffer_rsrc_t& r, int voff, int soff) __attribute__((always_inline)) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
  };
  auto xload = [&](int voff, int soff) __attribute__((always_inline)) { return bload(xr, voff, soff); };

  // chunk 0's halo: all slices in flight before the first store
  {
    float4 pv[NSL];
#pragma unroll
    for (int s = 0; s < NSL; ++s) pv[s] = xload(halo_off(s), 0);
#pragma unroll
    for (int s = 0; s < NSL; ++s) halo_store(smem, s, pv[s]);
  }

  // lane li of a class tile = voxel (qd, qh, qw) = (li / 16, (li / 8) & 1, li & 7) of the class
  // sub-grid; output o = o0 + 2q + c (+ 4·wave along h).  Input index of tap t: (o + p − t)/2 =
  // i0 + [q + (o0 − 2·i0 + c + p − t)/2] → lane part q, the rest wave-uniform.
  const int qd = li >> 4, qh = (li >> 3) & 1, qw = li & 7;
  const int lane_row = ((qd * kHH) + qh + 2 * wave) * kHW + qw;     // halo position (tap part added)
  const int wlane = (n0 + li) * 32 + lh * 16;                        // this lane's 16 B of a fragment

  f32x16 acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = f32x16{};

  // weights of step i: tap ts.s[i/2], half i&1 — one 16-B hi and lo fragment per lane; the step
  // offset is wave-uniform (soffset), the lane part a constant voffset
  auto b_load = [&](int chunk, int i, bf16x8 (&dst)[2]) __attribute__((always_inline)) {
    const int so = __builtin_amdgcn_readfirstlane((((ts.s[i >> 1].tap * nch + chunk) * 2 + (i & 1)) * 2) * blkw);
    dst[0] = __builtin_bit_cast(bf16x8, bload(wr, wlane, so));
    if constexpr (prec::has_lo<PM>()) dst[1] = __builtin_bit_cast(bf16x8, bload(wr, wlane, so + blkw));
    else dst[1] = dst[0];
  };
  bf16x8 rb[D][2];
#pragma unroll
  for (int i = 0; i < D; ++i) b_load(0, i, rb[i]);
  __syncthreads();

  for (int chunk = 0; chunk < nch; ++chunk) {
    const char* H = smem + (chunk & 1) * kHP * kHRow + lh * 16 + lane_row * kHRow;
    char* Hn = smem + ((chunk + 1) & 1) * kHP * kHRow;
    const int cn = chunk + 1 < nch ? chunk + 1 : chunk;
    auto a_read = [&](int i, bf16x8 (&dst)[2]) __attribute__((always_inline)) {
      const TStep st = ts.s[i >> 1];
      const char* arow = H + ((st.od * kHH + st.oh) * kHW + st.ow) * kHRow + (i & 1) * 32;
      dst[0] = *reinterpret_cast<const bf16x8*>(arow);
      if constexpr (prec::has_lo<PM>()) dst[1] = *reinterpret_cast<const bf16x8*>(arow + 64);
      else dst[1] = dst[0];
    };
    // the next chunk's halo in NB batches (one-plane modes: two, so the 256-register budget of
    // two blocks per CU holds half of it at a time)
    // (one-wave blocks: four — their lanes carry 20 fp32 slices per chunk)
    constexpr int NB = prec::has_lo<PM>() ? 1 : NW == 1 ? 4 : 2, BS = (NSL + NB - 1) / NB;
    float4 pv[BS];
    bf16x8 af[2][2];
    a_read(0, af[0]);
#pragma clang loop unroll(full)
    for (int i = 0; i < NS; ++i) {
      // (unconditional: on the last chunk this re-reads chunk cn = chunk into the idle buffer —
      // a branch here makes the compiler unswitch the loop and serialize the copy without it)
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        if (i == b * (NS / NB)) {
#pragma unroll
          for (int sl = 0; sl < BS; ++sl)
            if (b * BS + sl < NSL) pv[sl] = xload(halo_off(b * BS + sl), __builtin_amdgcn_readfirstlane(cn * kBK * ES));
        }
        if (i == b * (NS / NB) + kHD) {
#pragma unroll
          for (int sl = 0; sl < BS; ++sl)
            if (b * BS + sl < NSL) halo_store(Hn, b * BS + sl, pv[sl]);
        }
      }
      const int c = ts.s[i >> 1].c;
      const bf16x8 bh = rb[i % D][0], bl = rb[i % D][1];
      if (i + D < NS) b_load(chunk, i + D, rb[i % D]);
      else b_load(cn, i + D - NS, rb[i % D]);
      if (i + 1 < NS) a_read(i + 1, af[(i + 1) & 1]);
      const bf16x8 ah = af[i & 1][0], al = af[i & 1][1];
      // weights as the A operand (rows = output channels), voxels as B (cols)
      acc[c] = prec::mma<PM>(bh, bl, ah, al, acc[c]);
      // pin each step's loads to their step: under register pressure the scheduler otherwise
      // sinks the prefetches next to their uses (load → vmcnt(0) → MFMA, measured 8× slower)
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();
  }

  // epilogue through LDS (the halo buffers are free after the last chunk's barrier): in the MFMA
  // layout a store instruction writes 32 B into each of 32 voxel lines; transposed, each lane
  // stores 16 B and 8 lanes a whole 128-B voxel, 64 lanes 8 w-consecutive voxels (1 KB).
  // NP passes of 8 / NP classes: two halves (output depth parity cd, 128 voxels × 144-B rows per
  // wave each) in the bf16x3 mode; four quarters (cd, ch; 64 voxels per wave) in the one-plane
  // modes, whose LDS is the 64 KB of the halo buffers
  constexpr int NP = prec::has_lo<PM>() ? 2 : 4, CPP = 8 / NP, VPW = 32 * CPP;
  char* ew = smem + wave * (VPW * kRow);
  const int q = lane & 7;                                   // read-back: channel quad 4q … 4q+3
  float4 bq = make_float4(0.f, 0.f, 0.f, 0.f);
  if (a.bias) bq = *reinterpret_cast<const float4*>(a.bias + n0 + 4 * q);
  float4 smu = make_float4(0.f, 0.f, 0.f, 0.f), srs = smu;
  if (a.sx) {
    smu = *reinterpret_cast<const float4*>(a.smean + nb * a.ny + n0 + 4 * q);
    srs = *reinterpret_cast<const float4*>(a.srstd + nb * a.ny + n0 + 4 * q);
  }
  double ps[4] = {0.0, 0.0, 0.0, 0.0}, pq[4] = {0.0, 0.0, 0.0, 0.0};   // InstanceNorm partials (a.part)
#pragma unroll
  for (int pass = 0; pass < NP; ++pass) {
    // pass classes c = pass·CPP …: cd = c >> 2 (and, in quarters, ch = (c >> 1) & 1) fixed
#pragma unroll
    for (int c = pass * CPP; c < pass * CPP + CPP; ++c) {
      // voxel of the pass's (VPW) rows: (dq, h, w) with h over the pass's h parities
      const int v = NP == 2 ? (qd * 4 + 2 * qh + ((c >> 1) & 1)) * 16 + 2 * qw + (c & 1)
                            : (qd * 2 + qh) * 16 + 2 * qw + (c & 1);
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(ew + v * kRow + (8 * g + 4 * lh) * 4) =
            f32x4{acc[c][4 * g], acc[c][4 * g + 1], acc[c][4 * g + 2], acc[c][4 * g + 3]};
    }
    __syncthreads();
    const int pcd = NP == 2 ? pass : pass >> 1, pch = NP == 2 ? 0 : pass & 1;
#pragma unroll
    for (int j = 0; j < VPW / 8; ++j) {
      const int v = j * 8 + (lane >> 3);
      // halves: v = (dq·4 + hh)·16 + ww (hh over 4 rows); quarters: v = (dq·2 + hq)·16 + ww,
      // output row hh = 2·hq + ch
      const int dq = NP == 2 ? v >> 6 : v >> 5;
      const int hh = NP == 2 ? (v >> 4) & 3 : 2 * ((v >> 4) & 1) + pch;
      const int ww = v & 15;
      const int od = o0d + 2 * dq + pcd, oh = o0h + 4 * wave + hh, ow = o0w + ww;
      const f32x4 t = *reinterpret_cast<const f32x4*>(ew + v * kRow + 16 * q);
      if (od < a.Do && oh < a.Ho && ow < a.Wo) {
        const float4 r = make_float4(act_fwd(t[0] + bq.x, a.act), act_fwd(t[1] + bq.y, a.act),
                                     act_fwd(t[2] + bq.z, a.act), act_fwd(t[3] + bq.w, a.act));
        float4* dst = reinterpret_cast<float4*>(a.y + ((((int64_t)nb * a.Do + od) * a.Ho + oh) * a.Wo + ow) * a.ny + n0 + 4 * q);
        // non-temporal: the 134 MB output stream otherwise evicts the weight fragments every
        // block re-reads from L2 (measured 165 → 132 µs at 4 × 64³ × 32)
        __builtin_nontemporal_store(f32x4{r.x, r.y, r.z, r.w}, reinterpret_cast<f32x4*>(dst));
        if (a.part && a.sx) {
          const int64_t vo = (((int64_t)nb * a.Do + od) * a.Ho + oh) * a.Wo + ow;
          const float4 xs = *reinterpret_cast<const float4*>(a.sx + vo * a.ny + n0 + 4 * q);
          const float xv[4] = {xs.x, xs.y, xs.z, xs.w}, rv[4] = {r.x, r.y, r.z, r.w};
          const float mv[4] = {smu.x, smu.y, smu.z, smu.w}, sv[4] = {srs.x, srs.y, srs.z, srs.w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float xh = (xv[e] - mv[e]) * sv[e];
            const float gv = (a.sact == kActRelu && !(xh > 0.f)) ? 0.f
                             : (a.sact == kActLrelu && !(xh > 0.f)) ? rv[e] * kLreluSlope : rv[e];
            ps[e] += gv;
            pq[e] += (double)gv * xh;
          }
        } else if (a.part) {
          ps[0] += r.x; ps[1] += r.y; ps[2] += r.z; ps[3] += r.w;
          pq[0] += (double)r.x * r.x; pq[1] += (double)r.y * r.y; pq[2] += (double)r.z * r.z; pq[3] += (double)r.w * r.w;
        }
      }
    }
    if (pass + 1 < NP) __syncthreads();
  }
  // the consumer InstanceNorm's per-(instance, channel) Σy / Σy² of this brick (its separate
  // statistics pass over the 64³ output disappears): the 8 lanes of a channel quad add by
  // shuffles, the 4 waves through LDS past the epilogue rows (4 × 128 rows × kRow)
  if (a.part) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int m = 8; m < 64; m <<= 1) {
        ps[k] += __shfl_xor(ps[k], m);
        pq[k] += __shfl_xor(pq[k], m);
      }
    }
    double* red = reinterpret_cast<double*>(smem + NW * VPW * kRow);  // [NW waves][32 channels][2]
    if (lane < 8) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        red[(wave * 32 + 4 * q + k) * 2] = ps[k];
        red[(wave * 32 + 4 * q + k) * 2 + 1] = pq[k];
      }
    }
    __syncthreads();
    if (tid < 32) {
      double s2 = 0.0, q2 = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        s2 += red[(w * 32 + tid) * 2];
        q2 += red[(w * 32 + tid) * 2 + 1];
      }
      const int chunks = a.nbd * a.nbh * a.nbw, brick = (bd_i * a.nbh + bh_i) * a.nbw + bw_i;
      double* dst = a.part + (((int64_t)nb * chunks + brick) * a.ny + n0 + tid) * 2;
      dst[0] = s2;
      dst[1] = q2;
    }
  }
}

bool brickT_x3_applicable(const IgemmArgs& g) {
  // 32 output channels per block (at 64 per block the 16 class accumulators would take the whole
  // AGPR file and the halo prefetch spill): wider layers (G up1, 128 → 64) run one block per
  // 32-channel group, re-reading the halo per group — on grids of at least 64 four-wave bricks
  // only: the UNet's coarse wide layers (≤ 16³ outputs, up to 512 contraction channels) are a few
  // dozen long blocks there and run faster on the implicit GEMM (r05ab: UNet leg 5.24 ms with them
  // on brickT).  A/B switch MRAGAN_BRICKT_WIDE=<min bricks> (0: ny = 32 only).
  static const int wide_min = [] {
    const char* e = getenv("MRAGAN_BRICKT_WIDE");
    return e ? atoi(e) : 64;
  }();
  const int64_t bricks4 = (int64_t)g.N * ceil_div(g.Do, kOD) * ceil_div(g.Ho, 16) * ceil_div(g.Wo, kOW);
  const bool wide = wide_min > 0 && bricks4 >= wide_min;
  return g.x3 && g.trans && g.s == 2 && g.p == 1 && (g.k == 3 || g.k == 4) && g.cx % kBK == 0 &&
         (g.ny == 32 || (wide && g.ny % 32 == 0 && g.ny > 0)) &&
         (int64_t)g.Di * g.Hi * g.Wi * g.cx * 4 < ((int64_t)1 << 31);
}

// one static per kernel instantiation (the LDS opt-in is per function)
template <int K, int PM, int X16, int NW>
static void launch_brickT_nw(const BrickTArgs& a, unsigned blocks, hipStream_t st) {
  // halos + offsets; the epilogue rows (NW waves × 32·(8/NP) voxels × kRow) and the statistics
  // reduction after them reuse the same bytes
  constexpr int NP = prec::has_lo<PM>() ? 2 : 4;
  const size_t halo = (size_t)2 * hp_t<NW>() * halo_row<PM>() + hp_t<NW>() * sizeof(int);
  const size_t epi = (size_t)NW * 32 * (8 / NP) * kRow + NW * 32 * 2 * sizeof(double);
  const size_t lds = halo > epi ? halo : epi;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(brickT_x3_kernel<K, PM, X16, NW>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((brickT_x3_kernel<K, PM, X16, NW>), dim3(blocks), dim3(64 * NW), lds, st, a);
}

template <int K, int PM, int X16>
static void launch_brickT(const BrickTArgs& a, int nw, unsigned blocks, hipStream_t st) {
  if (nw == 4) {
    launch_brickT_nw<K, PM, X16, 4>(a, blocks, st);
  } else if constexpr (K == 3) {
    // no one-wave form for k3 (fp32 input: its 20 slices per lane spill; and a plane launch must
    // pick the same bricks as the fp32 one — bit-identical outputs and statistics partials)
    launch_brickT_nw<K, PM, X16, 2>(a, blocks, st);
  } else {
    if (nw == 2) launch_brickT_nw<K, PM, X16, 2>(a, blocks, st);
    else launch_brickT_nw<K, PM, X16, 1>(a, blocks, st);
  }
}

size_t brickT_x3_ws_bytes(const IgemmArgs& g) { return (size_t)g.k * g.k * g.k * g.cx * g.ny * sizeof(float); }

static int brickT_cus() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  return ncu;
}

template <int PM>
static int conv_brickT_pm(const IgemmArgs& g, hipStream_t st) {
  const size_t need = brickT_x3_ws_bytes(g);
  if (!g.ws || g.ws_bytes < need) {
    set_error("brickT_x3: workspace %zu < %zu", g.ws_bytes, need);
    return kWorkspace;
  }
  const int T = g.k * g.k * g.k;
  const int64_t groups = (int64_t)T * g.ny * (g.cx / 8);
  hipLaunchKernelGGL(brickT_pack_kernel<PM>, dim3((unsigned)((groups + 255) / 256)), dim3(256), 0, st, g.w, T, g.ny,
                     g.cx, reinterpret_cast<__bf16*>(g.ws));
  int rc = check_launch("brickT_pack");
  if (rc) return rc;
  BrickTArgs a{};
  a.x = g.x; a.N = g.N; a.Di = g.Di; a.Hi = g.Hi; a.Wi = g.Wi; a.C = g.cx;
  a.wx = reinterpret_cast<const __bf16*>(g.ws);
  a.bias = g.bias; a.y = g.y; a.Do = g.Do; a.Ho = g.Ho; a.Wo = g.Wo; a.ny = g.ny;
  a.k = g.k; a.p = g.p; a.act = g.act;
  // waves per block: 4, unless that leaves fewer bricks than CUs (then 2, or 1)
  static const int force_nw = [] {                   // A/B switch: MRAGAN_BRICKT_NW=1|2|4
    const char* e = getenv("MRAGAN_BRICKT_NW");
    return e ? atoi(e) : 0;
  }();
  int nw = 4;
  if (force_nw == 1 || force_nw == 2 || force_nw == 4) {
    nw = force_nw;
  } else {
    while (nw > 1 && (int64_t)g.N * (g.ny / 32) * ceil_div(g.Do, kOD) * ceil_div(g.Ho, 4 * nw) * ceil_div(g.Wo, kOW) < brickT_cus())
      nw >>= 1;
  }
  if (nw == 1 && g.k == 3) nw = 2;
  a.nbd = ceil_div(g.Do, kOD); a.nbh = ceil_div(g.Ho, 4 * nw); a.nbw = ceil_div(g.Wo, kOW);
  a.gn = g.ny / 32;
  const int64_t blocks = (int64_t)g.N * a.nbd * a.nbh * a.nbw * a.gn;
  if (blocks == 0) return kOk;
  static const bool no_stats = getenv("MRAGAN_NO_BRICKT_STATS") != nullptr;   // A/B switch
  if (g.in_part && !no_stats && !g.bs_add) {     // bs_add (ABI 18): brick epilogues only
    // conv3d_in_stats: the following InstanceNorm's partials; conv3d_bwd_stats (a stride-2 data
    // gradient, ABI 12): the backward statistics of the InstanceNorm in front (same grid)
    a.part = g.in_part;
    if (g.bs_x) { a.sx = g.bs_x; a.smean = g.bs_mean; a.srstd = g.bs_rstd; a.sact = g.bs_act; }
    if (g.in_chunks) *g.in_chunks = a.nbd * a.nbh * a.nbw;
  }
  if constexpr (prec::has_lo<PM>()) {
    if (g.x16) {
      set_error("brickT_x3: a 16-bit operand plane needs the bf16 or fp16 mode");
      return kBadArg;
    }
    if (g.k == 3) launch_brickT<3, PM, 0>(a, nw, (unsigned)blocks, st);
    else launch_brickT<4, PM, 0>(a, nw, (unsigned)blocks, st);
  } else if (g.x16) {
    if (g.k == 3) launch_brickT<3, PM, 1>(a, nw, (unsigned)blocks, st);
    else launch_brickT<4, PM, 1>(a, nw, (unsigned)blocks, st);
  } else {
    if (g.k == 3) launch_brickT<3, PM, 0>(a, nw, (unsigned)blocks, st);
    else launch_brickT<4, PM, 0>(a, nw, (unsigned)blocks, st);
  }
  return check_launch(g.x16 ? "brickT_x3(op16)" : "brickT_x3");
}

int conv_brickT_x3(const IgemmArgs& g, hipStream_t st) { MRAGAN_PREC_DISPATCH(g.x3, return conv_brickT_pm<PM>(g, st)) }

}  // namespace mragan
