// bf16x3 MFMA convolution from ONE input channel to 32·TN output channels, k = 7, stride 1 (gfx950).
//
//   G stem   Conv3d(1 → ngf, k7) on the RPad3 input          networks3D.py:185-189 (forward)
//   G head   data gradient of Conv3d(ngf → 1, k7)             networks3D.py:211-212 (transposed
//            form s = 1 = forward form with pad 6 − p and the taps flipped)
//
// As a GEMM: rows = output voxels, cols = output channels, contraction = the 343 taps.  The
// contraction is ordered (kd, kh, kw) with kw padded to 8 (a zero tap), so one MFMA k-group of 8
// is one w-row of taps: A[v][(kd,kh), 0..7] = x[vd+kd][vh+kh][vw+0..7].  That makes the A
// fragment a 16-B read from an "X8" image in LDS, X8[d][h][w] = x[d][h][w..w+7] split into
// planar bf16 hi / lo (16-B rows: a wave's 32 consecutive w hit 32 distinct bank quads).  49 real
// k-groups + 1 zero group = 25 v_mfma_f32_32x32x16_bf16 K-steps, ×3 for the hi/lo split products.
//
// Block: output brick BD × 8 × 32 voxels (BD·8 M-tiles of 32 w-consecutive voxels, TM per
// wave) × all 32·TN channels.  Its (BD+6) × 14 × 39 input halo is staged raw (fp32), expanded
// into X8 once, and the MFMA loop then runs barrier-free; the weights come pre-split and
// fragment-ordered from L2 (thin1_x3_pack), prefetched 5 K-steps ahead.
#include "kernels.h"
#include "prec.h"

namespace mragan {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kK = 7;
constexpr int kGroups = 50;            // 49 (kd, kh) rows + 1 zero group (K = 25 × 16)
constexpr int kKS = kGroups / 2;       // MFMA K-steps
constexpr int kRH = 8 + kK - 1;        // halo rows along h
constexpr int kBW = 32;                // output w per tile
constexpr int kRW = 40;                // raw halo row (39 used), float4-aligned
constexpr int kPFS = 5;                // weight prefetch distance (K-steps), divides kKS

// wp: packed [343][ny] (cin = 1) → out[(g·2 + hl)·ny + co][8] bf16, e = kw (e = 7 and g = 49: 0)
template <int PM>
__global__ void thin1_x3_pack_kernel(const float* __restrict__ wp, int ny, int flip, __bf16* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= kGroups * ny) return;
  const int co = i % ny, g = i / ny;
  f32x8 v;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float w = 0.f;
    if (g < kK * kK && e < kK) {
      const int t = g * kK + e;
      w = wp[(int64_t)(flip ? kK * kK * kK - 1 - t : t) * ny + co];
    }
    v[e] = w;
  }
  bf16x8 hi, lo;
  prec::split8v<PM>(v, hi, lo);
  *reinterpret_cast<bf16x8*>(out + ((int64_t)(g * 2 + 0) * ny + co) * 8) = hi;
  *reinterpret_cast<bf16x8*>(out + ((int64_t)(g * 2 + 1) * ny + co) * 8) = lo;
}

}  // namespace

// diagnostic phase stamps (MRAGAN_STAMPS=1): s_memtime at 5 points per block, read back with
// mragan_debug_stamps(); never written in normal runs
__device__ unsigned long long g_thin1_stamps[8192 * 5];

struct Thin1Args {
  int stamp;
  const float* x; int N, Di, Hi, Wi;
  const __bf16* wx;
  const float* bias;
  float* y; int Do, Ho, Wo, ny;
  int pe, act;
  int nbd, nbh, nbw;
};

template <int BD, int TN, int PM>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) thin1_x3_kernel(Thin1Args a) {
  constexpr int RD = BD + kK - 1;
  constexpr int NRAW = RD * kRH * kRW;                 // raw halo floats
  constexpr int NX8 = RD * kRH * kBW;                  // X8 rows
  constexpr int NL = (NRAW + 255) / 256;               // raw floats per thread
  constexpr int TILES = BD * 8;
  constexpr int TM = TILES / 4;
  static_assert(TILES % 4 == 0, "tiles per wave");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* raw = reinterpret_cast<float*>(smem);                                  // [RD][14][40]
  bf16x8* x8h = reinterpret_cast<bf16x8*>(smem + NRAW * sizeof(float));         // [RD][14][32]
  bf16x8* x8l = x8h + NX8;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int nbricks = a.N * a.nbd * a.nbh * a.nbw;
  auto stampit = [&](int b, int k) __attribute__((always_inline)) {
    if (a.stamp && tid == 0 && b < 8192) g_thin1_stamps[b * 5 + k] = __builtin_amdgcn_s_memtime();
  };
  struct Brick { int nb, od0, oh0, ow0; };
  auto brick_of = [&](int b) -> Brick {
    const int bw_i = b % a.nbw; b /= a.nbw;
    const int bh_i = b % a.nbh; b /= a.nbh;
    const int bd_i = b % a.nbd;
    return Brick{b / a.nbd, bd_i * BD, bh_i * 8, bw_i * kBW};
  };
  // raw halo of a brick into registers (zero outside the input)
  float rv[NL];
  auto raw_load = [&](int b) __attribute__((always_inline)) {
    const Brick k = brick_of(b < nbricks ? b : 0);
    const float* xb = a.x + (int64_t)k.nb * a.Di * a.Hi * a.Wi;
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int e = l * 256 + tid;
      const int rw = e % kRW, rh = (e / kRW) % kRH, rd = e / (kRW * kRH);
      const int id = k.od0 - a.pe + rd, ih = k.oh0 - a.pe + rh, iw = k.ow0 - a.pe + rw;
      const bool ok = e < NRAW && rw < kBW + kK - 1 && (unsigned)id < (unsigned)a.Di && (unsigned)ih < (unsigned)a.Hi &&
                      (unsigned)iw < (unsigned)a.Wi;
      const float t = xb[ok ? ((int64_t)id * a.Hi + ih) * a.Wi + iw : 0];
      rv[l] = ok ? t : 0.f;
    }
  };
  // weights: the same fragments for every brick; the first kPFS K-steps are (re)issued ahead
  const __bf16* wx = a.wx;
  bf16x8 rb[kPFS][TN][2];
  auto b_load = [&](int ks, bf16x8 (&dst)[TN][2]) __attribute__((always_inline)) {
    const int g = 2 * ks + lh;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int co = j * 32 + li;
      dst[j][0] = *reinterpret_cast<const bf16x8*>(wx + ((int64_t)(g * 2 + 0) * a.ny + co) * 8);
      if constexpr (prec::has_lo<PM>()) dst[j][1] = *reinterpret_cast<const bf16x8*>(wx + ((int64_t)(g * 2 + 1) * a.ny + co) * 8);
    }
  };
  // MFMA row m of a tile ↔ voxel w = 4(m mod 8) + m/8 of its 32-voxel row; X8 stores voxel w at
  // position P(w) = 8(w mod 4) + w/4, so the A reads (lane → position li) and the expansion
  // writes (4 consecutive w per thread → positions 8·dw + w0/4) are both bank-conflict free
  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int q = wave * TM + i;
    abase[i] = ((q / 8) * kRH + (q % 8)) * kBW + li;
  }

  int b = blockIdx.x;
#pragma unroll
  for (int ks = 0; ks < kPFS; ++ks) b_load(ks, rb[ks]);
  raw_load(b);
  for (; b < nbricks; b += gridDim.x) {
    const Brick k = brick_of(b);
    stampit(b, 0);
    // 1. raw halo registers → LDS (the previous brick's epilogue used this region: barrier first)
    __syncthreads();
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      const int e = l * 256 + tid;
      if (e < NRAW) raw[e] = rv[l];
    }
    __syncthreads();
    stampit(b, 1);
    // 2. X8 expansion: a thread takes 4 consecutive w of one row (3 aligned float4 reads)
    for (int gq = tid; gq < RD * kRH * (kBW / 4); gq += 256) {
      const int row = gq / (kBW / 4), w0 = (gq % (kBW / 4)) * 4;
      const float4* src = reinterpret_cast<const float4*>(raw + row * kRW + w0);
      const float4 p0 = src[0], p1 = src[1], p2 = src[2];
      const float r[12] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w, p2.x, p2.y, p2.z, p2.w};
#pragma unroll
      for (int dw = 0; dw < 4; ++dw) {
        const f32x8 v = {r[dw], r[dw + 1], r[dw + 2], r[dw + 3], r[dw + 4], r[dw + 5], r[dw + 6], r[dw + 7]};
        bf16x8 hi, lo;
        prec::split8v<PM>(v, hi, lo);
        const int pos = row * kBW + 8 * dw + (w0 >> 2);
        x8h[pos] = hi;
        if constexpr (prec::has_lo<PM>()) x8l[pos] = lo;
      }
    }
    __syncthreads();
    stampit(b, 2);
    // the next brick's raw halo flies while this one computes
    raw_load(b + gridDim.x);

    // 3. MFMA loop: wave owns tiles q = wave·TM + i → (dd, hh) = (q / 8, q % 8)
    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
#pragma unroll
    for (int ks = 0; ks < kKS; ++ks) {
      bf16x8 bh[TN], bl[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = rb[ks % kPFS][j][0];
        bl[j] = prec::has_lo<PM>() ? rb[ks % kPFS][j][1] : bh[j];
      }
      if (ks + kPFS < kKS) b_load(ks + kPFS, rb[ks % kPFS]);
      // this lane's k-group 2ks + lh → (kd, kh); the zero group 49 reads group 48's rows
      const int g0 = 2 * ks, g1 = 2 * ks + 1 < kK * kK ? 2 * ks + 1 : kK * kK - 1;
      const int off = lh ? ((g1 / kK) * kRH + g1 % kK) * kBW : ((g0 / kK) * kRH + g0 % kK) * kBW;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const bf16x8 ah = x8h[abase[i] + off];
        const bf16x8 al = prec::has_lo<PM>() ? x8l[abase[i] + off] : ah;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          // weights as the A operand (rows = channels), voxels as B (cols): each lane ends up
          // holding 4 consecutive channels of one voxel per register quad → 16-B stores
          acc[i][j] = prec::mma<PM>(bh[j], bl[j], ah, al, acc[i][j]);
        }
      }
      // one K-step per scheduling region: left free, the scheduler hoists the unrolled loop's
      // LDS reads far ahead (≈480 registers) and the loop runs 35 % slower (stamped)
      __builtin_amdgcn_sched_barrier(0);
    }
    stampit(b, 3);

    // 4. epilogue straight from the accumulators: register quad g of lane (li, lh) holds
    // channels j·32 + 8g + 4lh … +3 of voxel w = 4(li mod 8) + li/8 (the X8 position order)
    const int wv = 4 * (li & 7) + (li >> 3);
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int q = wave * TM + i;
      const int od = k.od0 + q / 8, oh = k.oh0 + q % 8, ow = k.ow0 + wv;
      if (od >= a.Do || oh >= a.Ho || ow >= a.Wo) continue;
      float* yv = a.y + ((((int64_t)k.nb * a.Do + od) * a.Ho + oh) * a.Wo + ow) * a.ny;
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int co = j * 32 + 8 * g + 4 * lh;
          float4 v = make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
          if (a.bias) {
            const float4 bb = *reinterpret_cast<const float4*>(a.bias + co);
            v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
          }
          v = make_float4(act_fwd(v.x, a.act), act_fwd(v.y, a.act), act_fwd(v.z, a.act), act_fwd(v.w, a.act));
          // non-temporal: the 134 MB output stream (64³ × 32 ch × 4 instances) would otherwise
          // evict the halo and weight lines the persistent blocks re-read from L2
          typedef float f32x4nt __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(f32x4nt{v.x, v.y, v.z, v.w}, reinterpret_cast<f32x4nt*>(yv + co));
        }
    }
    stampit(b, 4);
    // the next brick's first weight steps
#pragma unroll
    for (int ks = 0; ks < kPFS; ++ks) b_load(ks, rb[ks]);
  }
}

int thin1_debug_stamps(unsigned long long* host, int n) {
  if (n > 8192 * 5) n = 8192 * 5;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_thin1_stamps), (size_t)n * 8) == hipSuccess ? kOk : kLaunch;
}

// ny = 32 only: the 64-channel variant (TN = 2) does not fit the register file with the
// persistent prefetch (it falls back to conv_thin's VALU kernel)
bool thin1_x3_applicable(int cx, int ny, int k, int s) { return cx == 1 && k == kK && s == 1 && ny == 32; }

size_t thin1_x3_ws_bytes(int ny) { return (size_t)kGroups * 2 * ny * 8 * sizeof(__bf16); }

template <int BD, int TN, int PM>
static int launch_thin1(const Thin1Args& a, hipStream_t st) {
  constexpr int RD = BD + kK - 1;
  const size_t lds = (size_t)RD * kRH * kRW * sizeof(float) + (size_t)2 * RD * kRH * kBW * 16;
  auto kern = thin1_x3_kernel<BD, TN, PM>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  // persistent: one block per CU (the 133 KB LDS image allows no more), bricks strided by the
  // grid so each block prefetches its next brick's halo during the current MFMA loop
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  const int64_t bricks = (int64_t)a.N * a.nbd * a.nbh * a.nbw;
  hipLaunchKernelGGL(kern, dim3((unsigned)(bricks < ncu ? bricks : ncu)), dim3(256), lds, st, a);
  return check_launch("thin1_x3");
}

template <int PM>
static int conv_thin1_pm(const ThinArgs& t, void* ws, size_t ws_bytes, hipStream_t st) {
  const size_t need = thin1_x3_ws_bytes(t.ny);
  if (!ws || ws_bytes < need) {
    set_error("thin1_x3: workspace %zu < %zu", ws_bytes, need);
    return kWorkspace;
  }
  const int flip = t.trans ? 1 : 0;
  hipLaunchKernelGGL(thin1_x3_pack_kernel<PM>, dim3(ceil_div(kGroups * t.ny, 256)), dim3(256), 0, st, t.w, t.ny, flip,
                     static_cast<__bf16*>(ws));
  int rc = check_launch("thin1_x3_pack");
  if (rc) return rc;
  Thin1Args a{};
  static const int stamps = getenv("MRAGAN_STAMPS") ? 1 : 0;
  a.stamp = stamps;
  a.x = t.x; a.N = t.N; a.Di = t.Di; a.Hi = t.Hi; a.Wi = t.Wi;
  a.wx = static_cast<const __bf16*>(ws);
  a.bias = t.bias; a.y = t.y; a.Do = t.Do; a.Ho = t.Ho; a.Wo = t.Wo; a.ny = t.ny;
  // transposed form with s = 1: forward form with pad k − 1 − p and flipped taps (packed above)
  a.pe = t.trans ? kK - 1 - t.p : t.p;
  a.act = t.act;
  constexpr int BD = 2;
  a.nbd = ceil_div(t.Do, BD); a.nbh = ceil_div(t.Ho, 8); a.nbw = ceil_div(t.Wo, kBW);
  if ((int64_t)a.N * a.nbd * a.nbh * a.nbw == 0) return kOk;
  return launch_thin1<BD, 1, PM>(a, st);
}

int conv_thin1_x3(const ThinArgs& t, int mode, void* ws, size_t ws_bytes, hipStream_t st) {
  MRAGAN_PREC_DISPATCH(mode, return conv_thin1_pm<PM>(t, ws, ws_bytes, st))
}

}  // namespace mragan
