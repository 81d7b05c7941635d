// Generic implicit-GEMM 3D convolution on gfx950 fp32 MFMA (v_mfma_f32_32x32x2_f32).
//
// One kernel covers every dense convolution of the hot path (SURVEY §8a A9-A11, A16 and
// all their data-gradients):
//
//   forward form   y[n,o,:] = Σ_{j<k³}  x[n, o*s - p + j, :] · Wp[j]            (zero fill)
//   transposed form y[n,o,:] = Σ_{t : (o+p-t) % s == 0} x[n, (o+p-t)/s, :] · Wp[t]
//
// The transposed form is evaluated per output parity class (o ≡ c mod s, blockIdx.z = class),
// so every tap a block visits is a real one (sub-pixel decomposition; no masked MACs).
// It is used for ConvTranspose3d forward (networks3D.py:203-210) and for the data gradient of
// every forward conv; the forward form also yields the data gradient of ConvTranspose3d.
//
// GEMM view per class: rows = output voxels (M), cols = output channels (N = ny),
// contraction = (tap, input channel) with input channels contiguous (NDHWC) → the A tile is a
// gather of BM voxel rows × BK channels, the B tile is Wp[t][n0:n0+BN][c0:c0+BK].
// Both tiles live in LDS as [row][BK+4] (K contiguous, +16 B row pad → conflict-free
// ds_read_b128), register-staged double buffer, one barrier per K-step.
// MFMA K-order: lane half h supplies k = 4h+s at step s, so each lane reads ONE float4 of
// A and of B per 8-deep chunk and feeds 4 MFMAs from it.
#include "kernels.h"
#include "prec.h"
#include "conv_geo.h"

#include <cstdlib>

namespace mragan {

typedef float f32x16 __attribute__((ext_vector_type(16)));


template <int WM, int WN, int TM, int TN, int BK>
__global__ void __launch_bounds__(256)
conv_igemm_f32_kernel(IgemmArgs a) {
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  constexpr int LDK = BK + 4;               // padded row (floats)
  constexpr int LPR = BK / 4;               // float4 per row
  constexpr int A_LOADS = (BM * LPR + 255) / 256;
  constexpr int B_LOADS = (BN * LPR + 255) / 256;
  constexpr int ROWS_PER_PASS = 256 / LPR;
  static_assert(WM * WN == 4, "4 waves");

  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LDK + BM];
  float* As = smem;                          // [2][BM][LDK]
  float* Bs = smem + 2 * BM * LDK;           // [2][BN][LDK]
  int* out_off = reinterpret_cast<int*>(smem + 2 * (BM + BN) * LDK);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm0 = (wave / WN) * TM * 32;
  const int wn0 = (wave % WN) * TN * 32;

  // class geometry (wave-uniform)
  int cls = blockIdx.z;
  int cw = cls % a.s, ch = (cls / a.s) % a.s, cd = cls / (a.s * a.s);
  if (a.nclass == 1) { cd = ch = cw = 0; }
  const DimGeo gd = dim_geo(cd, a.Do, a.k, a.s, a.p, a.trans);
  const DimGeo gh = dim_geo(ch, a.Ho, a.k, a.s, a.p, a.trans);
  const DimGeo gw = dim_geo(cw, a.Wo, a.k, a.s, a.p, a.trans);
  const int64_t Mc = (int64_t)a.N * gd.Q * gh.Q * gw.Q;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  if (m0 >= Mc) return;
  const int ntaps = gd.ntap * gh.ntap * gw.ntap;

  // output offsets of this tile's rows (for the epilogue)
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

  // loader state: input base coordinates of this thread's A rows
  const int q = tid % LPR;
  int a_nb[A_LOADS], a_bd[A_LOADS], a_bh[A_LOADS], a_bw[A_LOADS];
#pragma unroll
  for (int i = 0; i < A_LOADS; ++i) {
    int r = tid / LPR + i * ROWS_PER_PASS;
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
  const int nK = ntaps * kchunks;

  float4 ra[A_LOADS], rb[B_LOADS];

  auto load_tiles = [&](int ks) {
    int tap = ks / kchunks;
    int c0 = (ks - tap * kchunks) * BK;
    int jw = tap % gw.ntap; int tt = tap / gw.ntap;
    int jh = tt % gh.ntap; int jd = tt / gh.ntap;
    int td = gd.t0 + gd.tstep * jd, th = gh.t0 + gh.tstep * jh, tw = gw.t0 + gw.tstep * jw;
    int wt = (td * a.k + th) * a.k + tw;
    int dd = gd.sign * jd, dh = gh.sign * jh, dw = gw.sign * jw;
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
      int id = a_bd[i] + dd, ih = a_bh[i] + dh, iw = a_bw[i] + dw;
      bool ok = a_nb[i] >= 0 && (unsigned)id < (unsigned)a.Di && (unsigned)ih < (unsigned)a.Hi &&
                (unsigned)iw < (unsigned)a.Wi;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (ok) {
        const float* src = a.x + ((((int64_t)a_nb[i] * a.Di + id) * a.Hi + ih) * a.Wi + iw) * a.cx + c0 + 4 * q;
        v = *reinterpret_cast<const float4*>(src);
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < B_LOADS; ++i) {
      int r = tid / LPR + i * ROWS_PER_PASS;
      int n = n0 + r;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (r < BN && n < a.ny)
        v = *reinterpret_cast<const float4*>(a.w + ((int64_t)wt * a.ny + n) * a.cx + c0 + 4 * q);
      rb[i] = v;
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
      int r = tid / LPR + i * ROWS_PER_PASS;
      if (r < BM) *reinterpret_cast<float4*>(As + (buf * BM + r) * LDK + 4 * q) = op_round4(ra[i], a.x3);
    }
#pragma unroll
    for (int i = 0; i < B_LOADS; ++i) {
      int r = tid / LPR + i * ROWS_PER_PASS;
      if (r < BN) *reinterpret_cast<float4*>(Bs + (buf * BN + r) * LDK + 4 * q) = op_round4(rb[i], a.x3);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};

  if (nK > 0) {
    load_tiles(0);
    store_tiles(0);
  }
  __syncthreads();

  const int li = lane & 31;
  const int lh = lane >> 5;
  for (int ks = 0; ks < nK; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nK) load_tiles(ks + 1);
    const float* Ab = As + buf * BM * LDK;
    const float* Bb = Bs + buf * BN * LDK;
#pragma unroll
    for (int kc = 0; kc < BK / 8; ++kc) {
      float4 av[TM], bv[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        av[i] = *reinterpret_cast<const float4*>(Ab + (wm0 + i * 32 + li) * LDK + kc * 8 + 4 * lh);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bv[j] = *reinterpret_cast<const float4*>(Bb + (wn0 + j * 32 + li) * LDK + kc * 8 + 4 * lh);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].x, bv[j].x, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].y, bv[j].y, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].z, bv[j].z, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i].w, bv[j].w, acc[i][j], 0, 0, 0);
        }
    }
    if (ks + 1 < nK) store_tiles(buf ^ 1);
    __syncthreads();
  }

  // epilogue: C/D map of 32x32 MFMA: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    int col = n0 + wn0 + j * 32 + li;
    if (col >= a.ny) continue;
    float bsum = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        int row = wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        int off = out_off[row];
        if (off >= 0) a.y[(int64_t)off * a.ny + col] = act_fwd(acc[i][j][r] + bsum, a.act);
      }
    }
  }
}

template <int WM, int WN, int TM, int TN, int BK>
static int launch_igemm(const IgemmArgs& a, int64_t max_mc, hipStream_t st) {
  constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  dim3 grid(ceil_div(max_mc, BM), ceil_div(a.ny, BN), a.nclass);
  hipLaunchKernelGGL((conv_igemm_f32_kernel<WM, WN, TM, TN, BK>), grid, dim3(256), 0, st, a);
  return check_launch("conv_igemm_f32");
}

template <int BK>
static int dispatch_tile(const IgemmArgs& a, int64_t max_mc, int64_t total_m, hipStream_t st) {
  // pick the largest tile that still gives ≥ 2 blocks per CU (256 CUs), else the smallest
  auto blocks = [&](int bm, int bn) { return (int64_t)ceil_div(total_m, bm) * ceil_div(a.ny, bn); };
  if (a.ny > 64) {
    if (blocks(128, 128) >= 512) return launch_igemm<2, 2, 2, 2, BK>(a, max_mc, st);
    if (blocks(128, 64) >= 512) return launch_igemm<2, 2, 2, 1, BK>(a, max_mc, st);
    return launch_igemm<2, 2, 1, 1, BK>(a, max_mc, st);
  }
  if (a.ny > 32) {
    if (blocks(128, 64) >= 512) return launch_igemm<2, 2, 2, 1, BK>(a, max_mc, st);
    return launch_igemm<2, 2, 1, 1, BK>(a, max_mc, st);
  }
  if (blocks(256, 32) >= 512) return launch_igemm<4, 1, 2, 1, BK>(a, max_mc, st);
  return launch_igemm<4, 1, 1, 1, BK>(a, max_mc, st);
}

static const bool g_brick_off = getenv("MRAGAN_NO_BRICK") != nullptr;   // A/B switch for benchmarking
static int need_fp32_pack(const IgemmArgs& a) {
  MRAGAN_CHECK_ARG(a.w, "conv: this convolution needs the fp32 weight pack (only a pre-split copy was given)");
  return kOk;
}

// Interior + shell data gradient (below): measured on MI355X (bf16, r03c / r05bb) the interior
// brick plus the shell pass (252 blocks × 36 serial K-steps at 4 × 16³, latency-bound) lose to the
// whole-grid brick on the 64³ configuration's 16³ blocks (N = 4: 42.9 vs 32.7 µs; N = 2: 36.8 vs
// 32.7) and at 1 × 32³ (59.2 vs 55.6), and win from 2 × 32³ on (the 128³ configuration's first
// passes: 92.9 vs 109.6 µs — the 34³ output grid fits no brick shape, the 32³ interior fits the
// forward's), and at the 96³ configuration's 24³ (fp16, r05bj: 2 × 24³ 56.5 vs 61.2, 4 × 24³ 88.5
// vs 117.4 µs; 2 × 28³ loses, 84.4 vs 63.7: no brick fits 28).  On for N ≥ 2 and interior extents
// that are multiples of 8 from 24 on, in the one-plane modes; MRAGAN_DGRAD_SPLIT=1 / 0
// forces it on / off for A/B.  Both passes read the pre-split weights (the shell pass through the
// implicit GEMM's W16 staging), so the fp32 pack — which the engine does not refresh for the
// ResnetBlock convs in these modes and then does not pass at all — is never read here (r05final2's
// garbage 128³ gradients were a stale fp32 pack read by the shell pass).
static const int g_split_env = [] {
  const char* e = getenv("MRAGAN_DGRAD_SPLIT");
  return e ? (atoi(e) ? 1 : 0) : -1;
}();
static int x3_instances_per_launch(const IgemmArgs& a);

// data gradient of a valid k3 s1 conv (transposed form p = 0, output = input + 2): the 16-bit
// modes compute it as interior + shell (the whole-grid brick spent 42 % of its rows on outputs
// whose taps mostly read zero padding and on padded brick rows)
bool full_dgrad_split_applicable(const IgemmArgs& a) {
  const bool big = a.N >= 2 && a.Di >= 24 && a.Di % 8 == 0 && a.Hi % 8 == 0 && a.Wi % 8 == 0;
  const bool on = g_split_env >= 0 ? g_split_env == 1 : (big && (a.x3 == kPrecBf16 || a.x3 == kPrecF16));
  return !g_brick_off && on && !a.bs_x && a.trans && a.s == 1 && a.k == 3 && a.p == 0 && a.Do == a.Di + 2 &&
         a.Ho == a.Hi + 2 && a.Wo == a.Wi + 2 && a.Do == a.Ho && a.Ho == a.Wo && a.Di >= 2 && a.cx % 16 == 0 &&
         conv_brick_x3_active(a) && x3_instances_per_launch(a) >= a.N;
}

// class count and row counts (class 0 is the largest along every dim)
static void igemm_geometry(IgemmArgs& a, int64_t& max_mc, int64_t& total_m) {
  a.nclass = (a.trans && a.s > 1) ? a.s * a.s * a.s : 1;
  auto q = [&](int O, int c) { return a.trans ? (O - c + a.s - 1) / a.s : O; };
  max_mc = (int64_t)a.N * q(a.Do, 0) * q(a.Ho, 0) * q(a.Wo, 0);
  total_m = (int64_t)a.N * a.Do * a.Ho * a.Wo;
}

// conv_igemm_x3 addresses its input through a buffer descriptor with 32-bit byte offsets: the
// instances one launch may cover (0 when a single instance is already too large).  Larger batches
// run as several launches on consecutive instance ranges (exact: every op is per instance).
static int x3_instances_per_launch(const IgemmArgs& a) {
  const int64_t per = (int64_t)a.Di * a.Hi * a.Wi * a.cx * 4;
  const int64_t lim = ((int64_t)1 << 31) - 1;
  if (per > lim) return 0;
  const int64_t nb = lim / per;
  return (int)(nb < a.N ? nb : a.N);
}

size_t conv_igemm_ws_bytes(IgemmArgs a) {
  int64_t max_mc, total_m;
  igemm_geometry(a, max_mc, total_m);
  if (max_mc == 0 || a.ny == 0) return 0;
  if (!g_brick_off && conv_brick_applicable(a))
    return conv_brick_x3_active(a) ? conv_brick_x3_ws_bytes(a.cx, a.ny) : 0;
  if (!g_brick_off && brickT_x3_applicable(a)) return brickT_x3_ws_bytes(a);
  if (a.x3 && a.cx % 16 == 0) {
    const int nb = x3_instances_per_launch(a);
    if (nb > 0 && nb < a.N) {
      a.N = nb;
      igemm_geometry(a, max_mc, total_m);
    }
    return conv_igemm_x3_ws_bytes(a, max_mc, total_m);
  }
  return 0;
}

static int conv_igemm_x3_chunked(const IgemmArgs& a, int64_t max_mc, int64_t total_m, hipStream_t st) {
  const int nb = x3_instances_per_launch(a);
  MRAGAN_CHECK_ARG(nb > 0, "conv (16-bit MFMA modes): one %d×%d×%d×%d instance exceeds 2 GiB", a.Di, a.Hi, a.Wi, a.cx);
  if (nb >= a.N) return conv_igemm_x3(a, max_mc, total_m, st);
  const int64_t in_vol = (int64_t)a.Di * a.Hi * a.Wi * a.cx, out_vol = (int64_t)a.Do * a.Ho * a.Wo * a.ny;
  const int64_t in_bytes = in_vol * (a.x16 ? 2 : 4);
  for (int n0 = 0; n0 < a.N; n0 += nb) {
    IgemmArgs c = a;
    c.in_part = nullptr;                 // instance ranges: no InstanceNorm partials (stats pass instead)
    c.bs_x = nullptr;
    c.N = nb < a.N - n0 ? nb : a.N - n0;
    c.x = reinterpret_cast<const float*>(reinterpret_cast<const char*>(a.x) + n0 * in_bytes);
    c.y = a.y + n0 * out_vol;
    int64_t mc, tm;
    igemm_geometry(c, mc, tm);
    const int rc = conv_igemm_x3(c, mc, tm, st);
    if (rc) return rc;
  }
  return kOk;
}

int conv_igemm(IgemmArgs a, hipStream_t st) {
  MRAGAN_CHECK_ARG(a.cx % 8 == 0, "conv_igemm: contraction channels %d not a multiple of 8", a.cx);
  MRAGAN_CHECK_ARG(a.k >= 1 && a.s >= 1 && a.p >= 0, "conv_igemm: bad k/s/p");
  int64_t max_mc, total_m;
  igemm_geometry(a, max_mc, total_m);
  if (max_mc == 0 || a.ny == 0) return kOk;
  if (a.x16) {
    // 16-bit operand planes: the ResnetBlock convs (forward and whole-grid data gradient) on the
    // brick; the others (the 64³-level stride-2 forward-form convs) on the implicit GEMM
    if (full_dgrad_split_applicable(a)) {
      const int rc = conv_brick(a, st, true);
      return rc ? rc : conv_igemm_x3_shell(a, st);
    }
    if (!g_brick_off && conv_brick_applicable(a)) return conv_brick(a, st);
    // G down1 / down2 (k3 s2 p1 forward) with their pre-split weights: the stride-2 brick (round 6)
    if (!g_brick_off && conv_brick_s2_applicable(a)) return conv_brick_s2(a, st);
    if (int rc = need_fp32_pack(a)) return rc;
    // 32-output-channel stride-2 transposed convs (G up2, G down1's data gradient): brickT (round 4)
    if (!g_brick_off && brickT_x3_applicable(a)) return conv_brickT_x3(a, st);
    MRAGAN_CHECK_ARG(a.x3 && a.cx % 32 == 0, "conv: a 16-bit operand plane input needs the bf16 / fp16 implicit GEMM "
                     "(multiples of 32 input channels)");
    return conv_igemm_x3_chunked(a, max_mc, total_m, st);
  }
  if (full_dgrad_split_applicable(a)) {
    // the 16-bit brick kernel on the interior (no padded rows, no all-zero taps) + the shell pass
    const int rc = conv_brick(a, st, true);
    return rc ? rc : conv_igemm_x3_shell(a, st);
  }
  if (!g_brick_off && conv_brick_applicable(a)) return conv_brick(a, st);
  if (!g_brick_off && conv_brick_s2_applicable(a)) return conv_brick_s2(a, st);
  if (int rc = need_fp32_pack(a)) return rc;
  if (!g_brick_off && brickT_x3_applicable(a)) return conv_brickT_x3(a, st);
  if (a.x3 && a.cx % 16 == 0) return conv_igemm_x3_chunked(a, max_mc, total_m, st);
  if (a.cx % 32 == 0) return dispatch_tile<32>(a, max_mc, total_m, st);
  if (a.cx % 16 == 0) return dispatch_tile<16>(a, max_mc, total_m, st);
  return dispatch_tile<8>(a, max_mc, total_m, st);
}

}  // namespace mragan
