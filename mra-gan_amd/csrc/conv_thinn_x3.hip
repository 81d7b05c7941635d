// bf16x3 MFMA convolution from 32 input channels to ONE output channel, k = 7, stride 1 (gfx950).
//
//   G head   Conv3d(ngf → 1, k7) + bias + Tanh on the RPad3 input     networks3D.py:211-213
//   G stem   data gradient of Conv3d(1 → ngf, k7)                     networks3D.py:185-186
//            (transposed form s = 1 = forward form, pad 6 − p, taps flipped)
//
//   z[o] = Σ_{kd,kh,kw,c} x[o − pe + (kd,kh,kw)][c] · W[kd,kh,kw][c]
//
// With one output channel the natural GEMM has N = 1.  Here the MFMA's 16 columns are
// (j, kw) — two output depths od = 2q + j and the 8 (padded) w-taps — and its rows are input w
// positions w', so one v_mfma_f32_16x16x32_bf16 produces the partial sums
//
//   P[w'][j, kw] = Σ_{kd',kh,c} x[2q + kd' − pe][oh + kh − pe][w' − pe][c] · W[kd' − j, kh, kw][c]
//
// over K = (input plane kd' = 0..7, kh, c); then z[2q + j][oh][ow] = Σ_kw P[ow + kw][j, kw]
// (an LDS epilogue).  Useful fraction 7/8 (kd' vs kd) × 7/8 (kw) × 64/80 (w halo).
//
// Block = a depth segment of P output-depth pairs × 8 output rows (one per wave, 8 waves) × 74
// output columns (the 80 w' rows less the 6-column halo: one column block covers both 64- and
// 70-wide outputs).  The block streams its 2P + 6 input planes once, in units (plane × 16-channel
// half): each unit's 14 × 80 positions × 16 channels are staged split into bf16 hi/lo (64-B
// swizzled LDS records) and feed every output pair whose 8-plane window contains it — up to 4
// at a time, their accumulators held in a 4-slot ring (slot = pair mod 4), so each staged plane
// is used by 4 pairs instead of being re-staged for each (round 1: 16 units per pair, 4× the
// input through L2).  A fragments are read once per (step, M-tile) and reused across the active
// pairs; the weights come pre-split in fragment order from L1/L2 (thinn_x3_pack).  A pair's
// sums leave through the wave's own LDS scratch (the kw reduction) as soon as its last plane is
// in.  Blocks are dealt to the 8 XCDs in contiguous ranges of the (column, row, segment) order.
#include "kernels.h"
#include "prec.h"

#include <type_traits>

namespace mragan {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

constexpr int kK = 7;
constexpr int kC = 32;                  // input channels
constexpr int kOW = 74;                 // output columns per block (kMW − 6)
constexpr int kMW = 80;                 // w' rows: 64 + 6 halo, 5 M-tiles of 16
constexpr int kBH = 8;                  // output rows per block (one per wave)
constexpr int kRH = kBH + kK - 1;       // staged rows per plane
constexpr int kRec = 64;                // LDS bytes per position: 4 16-B chunks (hi 0-7, hi 8-15,
                                        // lo 0-7, lo 8-15); chunk L sits at slot L ^ rot(pos)
constexpr int kUnitBytes = kRH * kMW * kRec;
constexpr int kNF4 = kRH * kMW * 4;     // float4 per unit (16 channels)
constexpr int kThreads = 512;            // 8 waves, one output row each (2 per SIMD)
constexpr int kF4PT = (kNF4 + kThreads - 1) / kThreads;

// weight fragment table: [kd' 8][half 2][step 4][hi|lo][lane 64][8 bf16]
constexpr int kPackElems = 8 * 2 * 4 * 2 * 64 * 8;
//   lane = 16g + n: column n = 8j + kw, k-group g → kh = 2·step + (g >> 1), channels
//   16·half + 8(g & 1) … +7; zero where kd = kd' − j ∉ [0, 7), kh = 7 or kw = 7
// (ny = 2, one-plane modes: one table per output channel co = blockIdx.y, weights packed
// [343][ny][32])
template <int PM>
__global__ void thinn_x3_pack_kernel(const float* __restrict__ wp, int flip, int ny, __bf16* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, co = blockIdx.y;
  out += (int64_t)co * kPackElems;
  if (i >= 8 * 2 * 4 * 64) return;
  const int lane = i & 63, s = (i >> 6) & 3, half = (i >> 8) & 1, kdp = i >> 9;
  const int n = lane & 15, g = lane >> 4;
  const int j = n >> 3, kw = n & 7, kh = 2 * s + (g >> 1), kd = kdp - j;
  const int c0 = 16 * half + 8 * (g & 1);
  f32x8 v;
  const bool ok = kd >= 0 && kd < kK && kh < kK && kw < kK;
  const int t = ok ? (kd * kK + kh) * kK + kw : 0;
  const int tt = flip ? kK * kK * kK - 1 - t : t;
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = ok ? wp[((int64_t)tt * ny + co) * kC + c0 + e] : 0.f;
  bf16x8 hi, lo;
  prec::split8v<PM>(v, hi, lo);
  const int64_t base = ((int64_t)((kdp * 2 + half) * 4 + s) * 2) * 64 * 8;
  *reinterpret_cast<bf16x8*>(out + base + lane * 8) = hi;
  *reinterpret_cast<bf16x8*>(out + base + 64 * 8 + lane * 8) = lo;
}

}  // namespace

struct ThinnArgs {
  const float* x; int N, Di, Hi, Wi;      // [N][Di][Hi][Wi][32] (fp32, or the 16-bit operand plane: X16)
  const __bf16* wx;
  const float* bias;
  float* y; int Do, Ho, Wo, ny;           // [N][Do][Ho][Wo][ny]
  int pe, act;
  int P, nseg, nr, nw;                    // pairs per segment, segments, row blocks, column blocks
  int total, per;                         // blocks, blocks per XCD range
};

// slot rotation of a position's 16-B chunks: rot = 2·(bit 1 ⊕ bit 3 of pos).  With it the
// ds_read_b128 lane groups of a fragment read ({0–3,12–15,20–27}, … : positions n16, chunk
// g & 1) and the ds_write_b64 groups of the staging stores (16 lanes = 4 positions × 4
// channel quads) both land on distinct banks.
__device__ __forceinline__ int thinn_rot(int pos) { return (pos ^ (pos >> 2)) & 2; }

constexpr int kScratch = kMW * 17;      // floats of a wave's epilogue scratch ([80][16] padded)

// X16 (one-plane modes, round 5): x is the 16-bit operand plane of the input — the bf16 / fp16 words
// the staging below would round it to — so a staged element is one 8-B load stored as it is
// (bit-identical to the fp32-input path, tests/test_kernels_gpu.py::test_k7_planes_bit_identical)
template <int PM, int X16>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2, 2)))
thinn_x3_kernel(ThinnArgs a) {
  static_assert(!X16 || !prec::has_lo<PM>(), "operand planes exist in the one-plane modes only");
  constexpr uint32_t ES = X16 ? 2u : 4u;    // bytes per input element
  extern __shared__ __attribute__((aligned(16))) char smem[];   // [kUnitBytes] | [8][kScratch]
  char* buf = smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* Pw = reinterpret_cast<float*>(smem + kUnitBytes) + wave * kScratch;
  int blk = (blockIdx.x & 7) * a.per + (blockIdx.x >> 3);   // XCD-contiguous logical block
  if (blk >= a.total) return;
  const int cw = blk % a.nw; blk /= a.nw;
  const int r = blk % a.nr; blk /= a.nr;
  const int seg = blk % a.nseg;
  const int nbco = blk / a.nseg;          // (output channel, instance)
  const int nb = nbco % a.N, co = nbco / a.N;
  const int od0 = 2 * a.P * seg, oh0 = r * kBH, ow0 = cw * kOW;
  const int npairs = min(a.P, (a.Do - od0 + 1) / 2);
  const int nunits = 2 * (2 * npairs + kK - 1);
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(reinterpret_cast<const char*>(a.x) + (int64_t)nb * a.Di * a.Hi * a.Wi * kC * ES,
                                              (uint32_t)a.Di * a.Hi * a.Wi * kC * ES);

  // staging of one unit (plane, channel half) into registers / LDS; per-thread element offsets
  // inside an input plane (−1: outside the input), fixed per block
  int poff[kF4PT];
#pragma unroll
  for (int l = 0; l < kF4PT; ++l) {
    const int e = l * kThreads + tid;
    const int pos = e >> 2, cq = e & 3;
    const int h = oh0 - a.pe + pos / kMW, w = ow0 - a.pe + pos % kMW;
    const bool ok = e < kNF4 && (unsigned)h < (unsigned)a.Hi && (unsigned)w < (unsigned)a.Wi;
    poff[l] = ok ? (h * a.Wi + w) * kC + 4 * cq : -1;
  }
  const uint32_t plane = (uint32_t)a.Hi * a.Wi * kC;
  using SV = typename std::conditional<X16 != 0, uint2, float4>::type;
  auto stage_load = [&](int u, SV (&sv)[kF4PT]) __attribute__((always_inline)) {
    const int d = od0 + (u >> 1) - a.pe, half = u & 1;
    const bool dok = (unsigned)d < (unsigned)a.Di;          // planes outside the input read 0
    const uint32_t base = (uint32_t)(dok ? d : 0) * plane + 16u * half;
#pragma unroll
    for (int l = 0; l < kF4PT; ++l) {
      const uint32_t off = (!dok || poff[l] < 0) ? kOobOffset : (base + poff[l]) * ES;
      if constexpr (X16) sv[l] = buf_load_8b(xr, (int)off, 0);
      else sv[l] = buf_load_f32x4(xr, off);
    }
  };
  // element l of this thread sits at position 128l + tid/4 (channels 4(tid&3)…): its chunk
  // rotation depends on tid only, so every store is base + 8192·l
  const int cq = tid & 3, srot = thinn_rot(tid >> 2);
  const int st_hi = (tid >> 2) * kRec + 16 * ((cq >> 1) ^ srot) + 8 * (cq & 1);
  const int st_lo = (tid >> 2) * kRec + 16 * ((2 + (cq >> 1)) ^ srot) + 8 * (cq & 1);
  auto stage_store = [&](const SV (&sv)[kF4PT]) __attribute__((always_inline)) {
#pragma unroll
    for (int l = 0; l < kF4PT; ++l) {
      if (l * kThreads + tid < kNF4) {
        uint2 h, lo;
        if constexpr (X16) h = sv[l];
        else prec::split4<PM>(sv[l], h, lo);
        *reinterpret_cast<uint2*>(buf + l * (kThreads / 4) * kRec + st_hi) = h;
        if constexpr (prec::has_lo<PM>()) *reinterpret_cast<uint2*>(buf + l * (kThreads / 4) * kRec + st_lo) = lo;
      }
    }
  };

  f32x4 acc[4][5];
#pragma unroll
  for (int sl = 0; sl < 4; ++sl)
#pragma unroll
    for (int i = 0; i < 5; ++i) acc[sl][i] = f32x4{};
  const int n16 = lane & 15, g = lane >> 4;
  const int a_hi = 16 * ((g & 1) ^ thinn_rot(n16)), a_lo = 16 * ((2 + (g & 1)) ^ thinn_rot(n16));
  // weight fragments through a buffer descriptor: lane part fixed (VGPR), (plane, half, step)
  // part wave-uniform (SGPR soffset) — no 64-bit address arithmetic per fragment
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.wx + (int64_t)co * kPackElems, kPackElems * 2);
  const int wlane = lane * 16;
  const float bias = a.bias ? a.bias[co] : 0.f;
  const int oh = oh0 + wave;

  // pair j's sums → z[od0 + 2j + jj][oh][ow] = Σ_kw P[ow − ow0 + kw][8jj + kw] through the wave's
  // own scratch (no other wave touches it: no barrier)
  auto epilogue = [&](int j, const f32x4 (&c)[5]) __attribute__((always_inline)) {
#pragma unroll
    for (int mt = 0; mt < 5; ++mt)
#pragma unroll
      for (int e = 0; e < 4; ++e) Pw[(mt * 16 + g * 4 + e) * 17 + n16] = c[mt][e];
    __builtin_amdgcn_s_waitcnt(0xc07f);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int o = k * 64 + lane;               // 148 outputs: jj = o / 74, ow = o % 74
      if (o >= 2 * kOW) break;
      const int jj = o / kOW, owl = o - jj * kOW;
      float sum = 0.f;
#pragma unroll
      for (int kw = 0; kw < kK; ++kw) sum += Pw[(owl + kw) * 17 + 8 * jj + kw];
      const int od = od0 + 2 * j + jj, ow = ow0 + owl;
      if (od < a.Do && oh < a.Ho && ow < a.Wo)
        a.y[((((int64_t)nb * a.Do + od) * a.Ho + oh) * a.Wo + ow) * a.ny + co] = act_fwd(sum + bias, a.act);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
  };

  SV sv[kF4PT];
  stage_load(0, sv);
  for (int u = 0; u < nunits; ++u) {
    __syncthreads();                            // every wave is done with the previous unit
    stage_store(sv);
    __syncthreads();
    if (u + 1 < nunits) stage_load(u + 1, sv);  // in flight during this unit's MFMAs
    const int kk = u >> 1, half = u & 1;
    // active pairs: 2j ≤ kk ≤ 2j + 7 → j ∈ [jlo, jhi], at most 4, slot = j mod 4
    const int jlo = kk >= kK ? (kk - 6) >> 1 : 0;
    const int jhi = min(npairs - 1, kk >> 1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8 bh[4], bl[4];
#pragma unroll
      for (int sl = 0; sl < 4; ++sl) {
        const int j = jlo + ((sl - jlo) & 3);
        const int kdp = j <= jhi ? kk - 2 * j : 0;
        const int wso = __builtin_amdgcn_readfirstlane((((kdp * 2 + half) * 4 + s) * 2) * 64 * 8 * 2);
        bh[sl] = __builtin_bit_cast(bf16x8, buf_load_16b(wr, wlane, wso));
        bl[sl] = prec::has_lo<PM>() ? __builtin_bit_cast(bf16x8, buf_load_16b(wr, wlane, wso + 64 * 8 * 2)) : bh[sl];
      }
      int kh = 2 * s + (g >> 1);
      kh = kh < kK ? kh : kK - 1;               // the padding kh = 7 has zero weights
      const char* rowp = buf + ((wave + kh) * kMW + n16) * kRec;
      bf16x8 ah[5], al[5];
#pragma unroll
      for (int mt = 0; mt < 5; ++mt) {
        ah[mt] = *reinterpret_cast<const bf16x8*>(rowp + mt * 16 * kRec + a_hi);
        al[mt] = prec::has_lo<PM>() ? *reinterpret_cast<const bf16x8*>(rowp + mt * 16 * kRec + a_lo) : ah[mt];
      }
#pragma unroll
      for (int sl = 0; sl < 4; ++sl) {
        const int j = jlo + ((sl - jlo) & 3);
        if (j > jhi) continue;                  // wave-uniform
        if (s == 0 && half == 0 && kk == 2 * j) {
#pragma unroll
          for (int mt = 0; mt < 5; ++mt) acc[sl][mt] = f32x4{};   // the pair's first plane
        }
#pragma unroll
        for (int mt = 0; mt < 5; ++mt) acc[sl][mt] = prec::mma16<PM>(ah[mt], al[mt], bh[sl], bl[sl], acc[sl][mt]);
      }
      __builtin_amdgcn_sched_barrier(0);        // one step per scheduling region (register budget)
    }
    // the pair whose last plane this was (kk = 2j + 7, second half)
    if (half == 1 && kk >= kK && ((kk - kK) & 1) == 0) {
      const int j = (kk - kK) >> 1;
      if (j < npairs) {
        switch (j & 3) {
          case 0: epilogue(j, acc[0]); break;
          case 1: epilogue(j, acc[1]); break;
          case 2: epilogue(j, acc[2]); break;
          default: epilogue(j, acc[3]); break;
        }
      }
    }
  }
}

// ny = 2 (nc = 2 volumes, BASELINE configs[4]) in the one-plane modes
bool thinn_x3_applicable(int cx, int ny, int k, int s, int mode) {
  const bool one_plane = mode == kPrecBf16 || mode == kPrecF16;
  return cx == kC && (ny == 1 || (ny == 2 && one_plane)) && k == kK && s == 1;
}

size_t thinn_x3_ws_bytes(int ny) { return (size_t)ny * kPackElems * sizeof(__bf16); }

template <int PM, int X16>
static int conv_thinn_pm(const ThinArgs& t, void* ws, size_t ws_bytes, hipStream_t st) {
  if (!(t.ny == 1 || (t.ny == 2 && !prec::has_lo<PM>()))) {
    set_error("thinn_x3: %d output channels in precision mode %d", t.ny, PM);
    return kBadArg;
  }
  if (!ws || ws_bytes < thinn_x3_ws_bytes(t.ny)) {
    set_error("thinn_x3: workspace %zu < %zu", ws_bytes, thinn_x3_ws_bytes(t.ny));
    return kWorkspace;
  }
  hipLaunchKernelGGL(thinn_x3_pack_kernel<PM>, dim3(16, t.ny), dim3(256), 0, st, t.w, t.trans ? 1 : 0, t.ny,
                     static_cast<__bf16*>(ws));
  int rc = check_launch("thinn_x3_pack");
  if (rc) return rc;
  ThinnArgs a{};
  a.x = t.x; a.N = t.N; a.Di = t.Di; a.Hi = t.Hi; a.Wi = t.Wi;
  a.wx = static_cast<const __bf16*>(ws);
  a.bias = t.bias; a.y = t.y; a.Do = t.Do; a.Ho = t.Ho; a.Wo = t.Wo; a.ny = t.ny;
  a.pe = t.trans ? kK - 1 - t.p : t.p;
  a.act = t.act;
  a.nr = ceil_div(t.Ho, kBH); a.nw = ceil_div(t.Wo, kOW);
  // pairs per depth segment: rounds of resident blocks (one per CU) × the segment's units
  // (2P + 6 planes)
  const int nq = ceil_div(t.Do, 2);
  const int64_t cols = (int64_t)a.N * a.ny * a.nr * a.nw;
  if (cols == 0 || nq == 0) return kOk;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  double best = 1e30;
  for (int P = 1; P <= 8; ++P) {
    const int nseg = ceil_div(nq, P);
    const int64_t rounds = (cols * nseg + ncu - 1) / ncu;
    const double cost = (double)rounds * (P + 3);
    if (cost < best - 1e-9) { best = cost; a.P = P; a.nseg = nseg; }
    if (P >= nq) break;
  }
  const int64_t blocks = cols * a.nseg;
  MRAGAN_CHECK_ARG((int64_t)t.Di * t.Hi * t.Wi * kC * (X16 ? 2 : 4) < (int64_t)kOobOffset, "thinn_x3: input volume too large");
  a.total = (int)blocks;
  a.per = (int)ceil_div(blocks, 8);
  const size_t lds = (size_t)kUnitBytes + (size_t)kBH * kScratch * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(thinn_x3_kernel<PM, X16>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL((thinn_x3_kernel<PM, X16>), dim3((unsigned)(8 * a.per)), dim3(kThreads), lds, st, a);
  return check_launch(X16 ? "thinn_x3(op16)" : "thinn_x3");
}

int conv_thinn_x3(const ThinArgs& t, int mode, void* ws, size_t ws_bytes, hipStream_t st) {
  if (t.x16) {
    if (mode == kPrecF16) return conv_thinn_pm<kPrecF16, 1>(t, ws, ws_bytes, st);
    MRAGAN_CHECK_ARG(mode == kPrecBf16, "thinn_x3: a 16-bit operand plane needs the bf16 / fp16 mode");
    return conv_thinn_pm<kPrecBf16, 1>(t, ws, ws_bytes, st);
  }
  MRAGAN_PREC_DISPATCH(mode, return conv_thinn_pm<PM, 0>(t, ws, ws_bytes, st))
}

}  // namespace mragan
