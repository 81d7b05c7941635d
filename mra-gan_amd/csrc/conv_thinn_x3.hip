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
// Block = 2 output depths × 8 output rows (one per wave, 8 waves) × 74 output columns (the 80 w' rows
// less the 6-column halo: one column block covers both 64- and 70-wide outputs).  The input is
// streamed in 16 units (plane kd' × 16-channel half): each unit's 14 × 80 positions × 16
// channels are staged split into bf16 hi/lo (64-B swizzled LDS records), double-buffered with
// one barrier per unit and register-prefetched two units ahead; the weights come pre-split in
// fragment order from L2 (thinn_x3_pack).  Blocks are dealt to the 8 XCDs in contiguous
// ranges of the (column, row, depth pair) order, so the blocks resident on one XCD at a time
// are neighbours in depth and re-read their shared input planes from that XCD's L2.
#include "kernels.h"
#include "prec.h"

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
constexpr int kBH = 8;                  // output rows per block (two per wave)
constexpr int kRH = kBH + kK - 1;       // staged rows per plane
constexpr int kRec = 64;                // LDS bytes per position: 4 16-B chunks (hi 0-7, hi 8-15,
                                        // lo 0-7, lo 8-15); chunk L sits at slot L ^ rot(pos)
constexpr int kUnits = 16;              // 8 planes × 2 channel halves
constexpr int kUnitBytes = kRH * kMW * kRec;
constexpr int kNF4 = kRH * kMW * 4;     // float4 per unit (16 channels)
constexpr int kThreads = 512;            // 8 waves, one output row each (2 per SIMD)
constexpr int kF4PT = (kNF4 + kThreads - 1) / kThreads;

// weight fragment table: [kd' 8][half 2][step 4][hi|lo][lane 64][8 bf16]
//   lane = 16g + n: column n = 8j + kw, k-group g → kh = 2·step + (g >> 1), channels
//   16·half + 8(g & 1) … +7; zero where kd = kd' − j ∉ [0, 7), kh = 7 or kw = 7
template <int PM>
__global__ void thinn_x3_pack_kernel(const float* __restrict__ wp, int flip, __bf16* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
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
  for (int e = 0; e < 8; ++e) v[e] = ok ? wp[tt * kC + c0 + e] : 0.f;
  bf16x8 hi, lo;
  prec::split8v<PM>(v, hi, lo);
  const int64_t base = ((int64_t)((kdp * 2 + half) * 4 + s) * 2) * 64 * 8;
  *reinterpret_cast<bf16x8*>(out + base + lane * 8) = hi;
  *reinterpret_cast<bf16x8*>(out + base + 64 * 8 + lane * 8) = lo;
}

}  // namespace

struct ThinnArgs {
  const float* x; int N, Di, Hi, Wi;      // [N][Di][Hi][Wi][32]
  const __bf16* wx;
  const float* bias;
  float* y; int Do, Ho, Wo;               // [N][Do][Ho][Wo]
  int pe, act;
  int nq, nr, nw;                         // depth pairs, row blocks, column blocks
  int total, per;                         // blocks, blocks per XCD range
};

// slot rotation of a position's 16-B chunks: rot = 2·(bit 1 ⊕ bit 3 of pos).  With it the
// ds_read_b128 lane groups of a fragment read ({0–3,12–15,20–27}, … : positions n16, chunk
// g & 1) and the ds_write_b64 groups of the staging stores (16 lanes = 4 positions × 4
// channel quads) both land on distinct banks.
__device__ __forceinline__ int thinn_rot(int pos) { return (pos ^ (pos >> 2)) & 2; }

template <int PM>
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(2, 2)))
thinn_x3_kernel(ThinnArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];   // [2][kUnitBytes]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int blk = (blockIdx.x & 7) * a.per + (blockIdx.x >> 3);   // XCD-contiguous logical block
  if (blk >= a.total) return;
  const int cw = blk % a.nw; blk /= a.nw;
  const int r = blk % a.nr; blk /= a.nr;
  const int q = blk % a.nq;
  const int nb = blk / a.nq;
  const int od0 = 2 * q, oh0 = r * kBH, ow0 = cw * kOW;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x + (int64_t)nb * a.Di * a.Hi * a.Wi * kC, (uint32_t)a.Di * a.Hi * a.Wi * kC * 4u);

  // staging of one unit (plane kd', channel half) into registers / LDS
  // per-thread element offsets inside an input plane (−1: outside the input), fixed per block
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
  auto stage_load = [&](int u, float4 (&sv)[kF4PT]) __attribute__((always_inline)) {
    const int d = od0 + (u >> 1) - a.pe, half = u & 1;     // callers pass valid units only
    const uint32_t base = (uint32_t)d * plane + 16u * half;
#pragma unroll
    for (int l = 0; l < kF4PT; ++l) sv[l] = buf_load_f32x4(xr, poff[l] < 0 ? kOobOffset : (base + poff[l]) * 4u);
  };
  // element l of this thread sits at position 128l + tid/4 (channels 4(tid&3)…): its chunk
  // rotation depends on tid only, so every store is base + 8192·l
  const int cq = tid & 3, srot = thinn_rot(tid >> 2);
  const int st_hi = (tid >> 2) * kRec + 16 * ((cq >> 1) ^ srot) + 8 * (cq & 1);
  const int st_lo = (tid >> 2) * kRec + 16 * ((2 + (cq >> 1)) ^ srot) + 8 * (cq & 1);
  auto stage_store = [&](char* buf, const float4 (&sv)[kF4PT]) __attribute__((always_inline)) {
#pragma unroll
    for (int l = 0; l < kF4PT; ++l) {
      if (l * kThreads + tid < kNF4) {
        uint2 h, lo;
        prec::split4<PM>(sv[l], h, lo);
        *reinterpret_cast<uint2*>(buf + l * (kThreads / 4) * kRec + st_hi) = h;
        if constexpr (prec::has_lo<PM>()) *reinterpret_cast<uint2*>(buf + l * (kThreads / 4) * kRec + st_lo) = lo;
      }
    }
  };

  f32x4 acc[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) acc[i] = f32x4{};
  const int n16 = lane & 15, g = lane >> 4;
  const int a_hi = 16 * ((g & 1) ^ thinn_rot(n16)), a_lo = 16 * ((2 + (g & 1)) ^ thinn_rot(n16));
  const __bf16* wx = a.wx;

  // valid units (input plane inside the input) form a contiguous range [u0, u1)
  int u0 = 0, u1 = kUnits;
  while (u0 < kUnits && (od0 + (u0 >> 1) - a.pe) < 0) ++u0;
  while (u1 > u0 && (od0 + ((u1 - 1) >> 1) - a.pe) >= a.Di) --u1;

  // the unit's weight fragments [step][hi|lo], issued at the top of the unit's iteration BEFORE
  // that iteration's staging loads: the memory counter retires in order, so weights fetched
  // after a staging batch would make the MFMAs wait for the whole batch
  auto w_load = [&](int u, bf16x8 (&w)[4][2]) __attribute__((always_inline)) {
    const int kdp = u >> 1, half = u & 1;
    const __bf16* wt = wx + ((int64_t)(kdp * 2 + half) * 4) * 2 * 64 * 8;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      w[s][0] = *reinterpret_cast<const bf16x8*>(wt + (s * 2 + 0) * 64 * 8 + lane * 8);
      w[s][1] = prec::has_lo<PM>() ? *reinterpret_cast<const bf16x8*>(wt + (s * 2 + 1) * 64 * 8 + lane * 8) : w[s][0];
    }
  };
  auto compute = [&](const char* buf, const bf16x8 (&w)[4][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const bf16x8 bh = w[s][0], bl = w[s][1];
      int kh = 2 * s + (g >> 1);
      kh = kh < kK ? kh : kK - 1;           // the padding kh = 7 has zero weights
      // position (wave + kh)·80 + 16mt + n16: the wave/step part is a multiple of 16
      // positions, so the chunk rotation is the lane's own (of n16) — addresses fold to
      // lane base + immediate
      const char* rowp = buf + ((wave + kh) * kMW + n16) * kRec;
#pragma unroll
      for (int mt = 0; mt < 5; ++mt) {
        const int cofs = (mt * 16) * kRec;
        const bf16x8 ah = *reinterpret_cast<const bf16x8*>(rowp + cofs + a_hi);
        const bf16x8 al = prec::has_lo<PM>() ? *reinterpret_cast<const bf16x8*>(rowp + cofs + a_lo) : ah;
        acc[mt] = prec::mma16<PM>(ah, al, bh, bl, acc[mt]);
      }
      __builtin_amdgcn_sched_barrier(0);    // one step per scheduling region (register budget)
    }
  };

  // pipeline: LDS buffer (u & 1) holds unit u; register set A/B holds the unit after it
  float4 sA[kF4PT], sB[kF4PT];
  bf16x8 w[4][2];
  if (u0 < u1) {
    stage_load(u0, sA);
    stage_store(smem + (u0 & 1) * kUnitBytes, sA);
    if (u0 + 1 < u1) stage_load(u0 + 1, sA);
  }
  __syncthreads();
  for (int u = u0; u < u1; u += 2) {
    // unit u (registers: sA = u + 1); prefetch u + 2 into sB
    w_load(u, w);
    if (u + 2 < u1) stage_load(u + 2, sB);
    compute(smem + (u & 1) * kUnitBytes, w);
    if (u + 1 < u1) stage_store(smem + ((u + 1) & 1) * kUnitBytes, sA);
    __syncthreads();
    if (u + 1 >= u1) break;
    // unit u + 1 (registers: sB = u + 2); prefetch u + 3 into sA
    w_load(u + 1, w);
    if (u + 3 < u1) stage_load(u + 3, sA);
    compute(smem + ((u + 1) & 1) * kUnitBytes, w);
    if (u + 2 < u1) stage_store(smem + (u & 1) * kUnitBytes, sB);
    __syncthreads();
  }

  // epilogue: P[w'][n] (n = 8j + kw) of the wave's row through its LDS slot, then
  // z[od0 + j][oh][ow] = Σ_kw P[ow − ow0 + kw][8j + kw]
  float* P = reinterpret_cast<float*>(smem) + wave * kMW * 17;   // [80][16] padded to 17
  {
#pragma unroll
    for (int mt = 0; mt < 5; ++mt)
#pragma unroll
      for (int e = 0; e < 4; ++e) P[(mt * 16 + g * 4 + e) * 17 + n16] = acc[mt][e];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    const int oh = oh0 + wave;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int o = k * 64 + lane;               // 148 outputs: j = o / 74, ow = o % 74
      if (o >= 2 * kOW) break;
      const int j = o / kOW, owl = o - j * kOW;
      float sum = 0.f;
#pragma unroll
      for (int kw = 0; kw < kK; ++kw) sum += P[(owl + kw) * 17 + 8 * j + kw];
      const int od = od0 + j, ow = ow0 + owl;
      if (od < a.Do && oh < a.Ho && ow < a.Wo)
        a.y[(((int64_t)nb * a.Do + od) * a.Ho + oh) * a.Wo + ow] = act_fwd(sum + (a.bias ? a.bias[0] : 0.f), a.act);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
  }
}

bool thinn_x3_applicable(int cx, int ny, int k, int s) { return cx == kC && ny == 1 && k == kK && s == 1; }

size_t thinn_x3_ws_bytes() { return (size_t)8 * 2 * 4 * 2 * 64 * 8 * sizeof(__bf16); }

template <int PM>
static int conv_thinn_pm(const ThinArgs& t, void* ws, size_t ws_bytes, hipStream_t st) {
  if (!ws || ws_bytes < thinn_x3_ws_bytes()) {
    set_error("thinn_x3: workspace %zu < %zu", ws_bytes, thinn_x3_ws_bytes());
    return kWorkspace;
  }
  hipLaunchKernelGGL(thinn_x3_pack_kernel<PM>, dim3(16), dim3(256), 0, st, t.w, t.trans ? 1 : 0,
                     static_cast<__bf16*>(ws));
  int rc = check_launch("thinn_x3_pack");
  if (rc) return rc;
  ThinnArgs a{};
  a.x = t.x; a.N = t.N; a.Di = t.Di; a.Hi = t.Hi; a.Wi = t.Wi;
  a.wx = static_cast<const __bf16*>(ws);
  a.bias = t.bias; a.y = t.y; a.Do = t.Do; a.Ho = t.Ho; a.Wo = t.Wo;
  a.pe = t.trans ? kK - 1 - t.p : t.p;
  a.act = t.act;
  a.nq = ceil_div(t.Do, 2); a.nr = ceil_div(t.Ho, kBH); a.nw = ceil_div(t.Wo, kOW);
  const int64_t blocks = (int64_t)a.N * a.nq * a.nr * a.nw;
  if (blocks == 0) return kOk;
  MRAGAN_CHECK_ARG((int64_t)t.Di * t.Hi * t.Wi * kC * 4 < (int64_t)kOobOffset, "thinn_x3: input volume too large");
  a.total = (int)blocks;
  a.per = (int)ceil_div(blocks, 8);
  const size_t lds = (size_t)2 * kUnitBytes;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(thinn_x3_kernel<PM>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(thinn_x3_kernel<PM>, dim3((unsigned)(8 * a.per)), dim3(kThreads), lds, st, a);
  return check_launch("thinn_x3");
}

int conv_thinn_x3(const ThinArgs& t, int mode, void* ws, size_t ws_bytes, hipStream_t st) {
  MRAGAN_PREC_DISPATCH(mode, return conv_thinn_pm<PM>(t, ws, ws_bytes, st))
}

}  // namespace mragan
