// Conv3d(nc → C, k4, s2, p1) from nc = 1 or 2 image channels on the MFMA units, one-plane modes
// (bf16 / fp16): the PatchGAN's first layer (networks3D.py:389-390, + LeakyReLU), the UNet's
// outermost downconv (networks3D.py:300-303, + LeakyReLU) and the data gradient of the UNet's
// outermost upconv (the forward form of ConvTranspose3d(2·ngf → nc, k4 s2 p1)).
//
// The contraction is one voxel's 4³ taps × nc channels — K = 64·nc — against C = 32 or 64 output
// channels: an MFMA GEMM with M = output voxels, N = C.  The VALU kernel (thin_k: one thread per
// voxel × 32 channels, 2048 FMAs each) took 26–39 µs per launch at 64³.
// A block owns a 2 × 8 × 16 output brick of one instance; its (2·2 + 2) × (2·8 + 2) × (2·16 + 2)
// input region is staged in LDS as 16-bit operands (RNE, as every kernel of the mode rounds), and
// an A fragment — 8 consecutive K of one voxel — is gathered from it:
//   nc = 1: K = (kd·4 + kh)·4 + kw; a lane's 8 K are two kh rows × the 4 kw taps: two runs of 4
//           consecutive inputs (two 4-B reads each: the runs start on even positions);
//   nc = 2: K = ((kd·4 + kh)·4 + kw)·2 + c; a lane's 8 K are one kh row × 4 kw × 2 channels: one
//           run of 8 words in the [w][c] layout (two 8-B reads).
// The weights ([tap][C][nc] packed) are held in registers as B fragments for the whole block.
// Bias and activation in the epilogue; each store instruction writes 32 consecutive channels of
// two voxels.  Products of rounded operands are exact in fp32: results equal the fp64
// convolution of the rounded operands up to fp32 accumulation order (test_down4_mfma).
#include "kernels.h"
#include "prec.h"

#include <cstdlib>
#include <type_traits>

namespace mragan {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// output brick 2 × 8 × 16 (512 blocks for a 4 × 32³ output: two per CU hide each other's
// staging and store phases; 4 × 8 × 16 bricks — 256 blocks, one per CU — took 20 µs)
constexpr int kDD = 2, kDH = 8, kDW = 16;
constexpr int kRD = 2 * kDD + 2, kRH = 2 * kDH + 2, kRW = 2 * kDW + 2;   // input region 6 × 18 × 34
constexpr int kDRT = kDD * kDH * kDW / 32;                    // 8 row tiles of 32 voxels

template <int NC>
constexpr int down4_row_bytes() { return ((kRW * NC * 2 + 15) / 16) * 16 + 8; }   // 72 (nc 1) / 152 (nc 2)

}  // namespace

template <int PM, int NC, int C>
__global__ void __launch_bounds__(256) down4_mfma_kernel(ThinArgs a, int tiles_d, int tiles_h, int tiles_w) {
  static_assert(!prec::has_lo<PM>(), "one-plane modes only");
  constexpr int KS = 4 * NC;                        // K steps of 16
  constexpr int NCT = C / 32;                       // column tiles
  constexpr int ROWB = down4_row_bytes<NC>();
  constexpr int TPW = kDRT / 4;                     // row tiles per wave
  __shared__ __attribute__((aligned(16))) char smem[kRD * kRH * ROWB];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 31, lh = lane >> 5;
  int b = blockIdx.x;
  const int tw_ = b % tiles_w; b /= tiles_w;
  const int th_ = b % tiles_h; b /= tiles_h;
  const int td_ = b % tiles_d;
  const int nb = b / tiles_d;
  const int o0d = td_ * kDD, o0h = th_ * kDH, o0w = tw_ * kDW;
  const int i0d = 2 * o0d - 1, i0h = 2 * o0h - 1, i0w = 2 * o0w - 1;

  // input region → LDS (16-bit, zero outside the volume): one float per element, all loads issued
  // before the first conversion
  constexpr int NEL = kRD * kRH * kRW * NC;
  constexpr int NPT = (NEL + 255) / 256;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x + (int64_t)nb * a.Di * a.Hi * a.Wi * NC,
                                              (uint32_t)a.Di * a.Hi * a.Wi * NC * 4u);
  float xv[NPT];
#pragma unroll
  for (int u = 0; u < NPT; ++u) {
    const int e = tid + 256 * u;
    const int c = e % NC, p = e / NC;
    const int rw = p % kRW, rh = (p / kRW) % kRH, rd = p / (kRW * kRH);
    const int id = i0d + rd, ih = i0h + rh, iw = i0w + rw;
    const bool ok = e < NEL && (unsigned)id < (unsigned)a.Di && (unsigned)ih < (unsigned)a.Hi &&
                    (unsigned)iw < (unsigned)a.Wi;
    xv[u] = buf_load_f32(xr, ok ? (uint32_t)((((id * a.Hi + ih) * a.Wi + iw) * NC + c) * 4) : kOobOffset);
  }
  // B fragments: column = output channel, K as above; packed weights are [tap][C][NC]
  bf16x8 bf[NCT][KS];
#pragma unroll
  for (int j = 0; j < NCT; ++j)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int co = j * 32 + li, k0 = ks * 16 + lh * 8;
      f32x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = k0 + e, t = k / NC, c = k % NC;
        v[e] = a.w[((int64_t)t * C + co) * NC + c];
      }
      bf16x8 lo;
      prec::split8v<PM>(v, bf[j][ks], lo);
    }
#pragma unroll
  for (int u = 0; u < NPT; ++u) {
    const int e = tid + 256 * u;
    if (e < NEL) {
      const int c = e % NC, p = e / NC;
      const int rw = p % kRW, row = p / kRW;
      uint32_t hi, lo;
      prec::split2<PM>(xv[u], 0.f, hi, lo);
      *reinterpret_cast<uint16_t*>(smem + row * ROWB + (rw * NC + c) * 2) = (uint16_t)(hi & 0xffffu);
    }
  }
  __syncthreads();

  f32x16 acc[TPW][NCT];
#pragma unroll
  for (int u = 0; u < TPW; ++u) {
    const int rt = wave * TPW + u;
    // the MFMA row (voxel) of this lane: rows of a tile are 2 × 16 outputs (oh pair, ow)
    const int v = rt * 32 + li;
    const int lw = v % kDW, lhh = (v / kDW) % kDH, ld = v / (kDW * kDH);
#pragma unroll
    for (int j = 0; j < NCT; ++j) acc[u][j] = f32x16{};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8 A;
      if constexpr (NC == 1) {
        // taps kd = ks, kh = 2·lh + {0, 1}, kw = 0..3: input rows (2ld + kd, 2lhh + kh), columns 2lw … +3
        const char* p0 = smem + ((2 * ld + ks) * kRH + 2 * lhh + 2 * lh) * ROWB + 2 * lw * 2;
        const uint32_t r0 = *reinterpret_cast<const uint32_t*>(p0), r1 = *reinterpret_cast<const uint32_t*>(p0 + 4);
        const uint32_t r2 = *reinterpret_cast<const uint32_t*>(p0 + ROWB),
                       r3 = *reinterpret_cast<const uint32_t*>(p0 + ROWB + 4);
        A = __builtin_bit_cast(bf16x8, (uint4){r0, r1, r2, r3});
      } else {
        // taps kd = ks / 2, kh = 2·(ks & 1) + lh, kw = 0..3 × 2 channels: one run of 8 words
        const char* p0 = smem + ((2 * ld + ks / 2) * kRH + 2 * lhh + 2 * (ks & 1) + lh) * ROWB + 2 * lw * NC * 2;
        const uint2 r0 = *reinterpret_cast<const uint2*>(p0), r1 = *reinterpret_cast<const uint2*>(p0 + 8);
        A = __builtin_bit_cast(bf16x8, (uint4){r0.x, r0.y, r1.x, r1.y});
      }
#pragma unroll
      for (int j = 0; j < NCT; ++j) acc[u][j] = prec::mma<PM>(A, A, bf[j][ks], bf[j][ks], acc[u][j]);
    }
  }

  // epilogue: C[row][col] of register r sits at row 8(r/4) + 4lh + r%4, column li
  float bv[NCT];
#pragma unroll
  for (int j = 0; j < NCT; ++j) bv[j] = a.bias ? a.bias[j * 32 + li] : 0.f;
#pragma unroll
  for (int u = 0; u < TPW; ++u) {
    const int rt = wave * TPW + u;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int v = rt * 32 + 8 * (r >> 2) + 4 * lh + (r & 3);
      const int od = o0d + v / (kDW * kDH), oh = o0h + (v / kDW) % kDH, ow = o0w + v % kDW;
      if (od < a.Do && oh < a.Ho && ow < a.Wo) {
        float* dst = a.y + ((((int64_t)nb * a.Do + od) * a.Ho + oh) * a.Wo + ow) * C;
#pragma unroll
        for (int j = 0; j < NCT; ++j) dst[j * 32 + li] = act_fwd(acc[u][j][r] + bv[j], a.act);
      }
    }
  }
}

bool down4_mfma_applicable(const ThinArgs& a) {
  static const bool off = getenv("MRAGAN_NO_DOWN4") != nullptr;   // A/B switch
  return !off && (a.rnd == kPrecBf16 || a.rnd == kPrecF16) && !a.trans && a.k == 4 && a.s == 2 && a.p == 1 &&
         (a.cx == 1 || a.cx == 2) && (a.ny == 32 || a.ny == 64) && !a.x16 &&
         (int64_t)a.Di * a.Hi * a.Wi * a.cx * 4 < ((int64_t)1 << 31);
}

template <int PM, int NC, int C>
static int launch_down4(const ThinArgs& a, hipStream_t st) {
  const int td = ceil_div(a.Do, kDD), th = ceil_div(a.Ho, kDH), tw = ceil_div(a.Wo, kDW);
  const int64_t blocks = (int64_t)a.N * td * th * tw;
  MRAGAN_CHECK_ARG(blocks < ((int64_t)1 << 31), "down4: grid too large");
  hipLaunchKernelGGL((down4_mfma_kernel<PM, NC, C>), dim3((unsigned)blocks), dim3(256), 0, st, a, td, th, tw);
  return check_launch("down4_mfma");
}

int conv_down4_mfma(const ThinArgs& a, hipStream_t st) {
  MRAGAN_CHECK_ARG(down4_mfma_applicable(a), "down4: not a k4 s2 p1 conv from 1-2 to 32 | 64 channels in bf16 / fp16");
  if (a.N == 0) return kOk;
  auto go = [&](auto pm) -> int {
    constexpr int PM = decltype(pm)::value;
    if (a.cx == 1) return a.ny == 32 ? launch_down4<PM, 1, 32>(a, st) : launch_down4<PM, 1, 64>(a, st);
    return a.ny == 32 ? launch_down4<PM, 2, 32>(a, st) : launch_down4<PM, 2, 64>(a, st);
  };
  if (a.rnd == kPrecF16) return go(std::integral_constant<int, kPrecF16>{});
  return go(std::integral_constant<int, kPrecBf16>{});
}

}  // namespace mragan
