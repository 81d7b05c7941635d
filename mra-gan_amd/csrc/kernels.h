// Internal interface between the C ABI (capi.hip) and the kernel files.
#pragma once
#include "common.h"

namespace mragan {

struct IgemmArgs {
  const float* x;   // [N][Di][Hi][Wi][cx]
  const float* w;   // [k³][ny][cx]
  const float* bias;
  float* y;         // [N][Do][Ho][Wo][ny]
  int N, Di, Hi, Wi, cx;
  int Do, Ho, Wo, ny;
  int k, s, p;
  int trans;
  int act;
  int nclass;       // set by conv_igemm: 1 (forward or s==1) or s³
  int x3;           // precision mode (prec.h): 0 exact f32 MFMA; 1 bf16x3, 2 bf16, 3 fp16 (the *_x3 kernels)
  float* ws;        // split-K partial tiles (conv_igemm_ws_bytes)
  size_t ws_bytes;
  const void* wx3;  // optional: w pre-split in bf16x3 brick fragment order (pack tr 2/3), or null
  double* in_part;  // optional: per-(instance, brick, channel) Σy, Σy² of the output (brick_x3 only)
  int* in_chunks;   // set to the bricks per instance when in_part was filled, else 0
  int shell;        // conv_igemm_x3 only: the 6 shell-face classes of a full (k3 s1 p0) transposed conv
  int x16;          // x is a 16-bit operand plane (bf16 / fp16 words of the precision mode), not fp32
  // with in_part, backward statistics instead (BrickArgs::sx): the producing IN's x, μ, rstd, act
  const float* bs_x; const float* bs_mean; const float* bs_rstd; int bs_act;
  const float* bs_add = nullptr;   // ABI 18, brick kernels only: BrickArgs::sadd
  // optional with in_part (ABI 15): finalize the statistics in the launch where the kernel can
  // (BrickArgs::tick …); *in_finalized = 1 when it did, else left 0 (the caller finalizes)
  unsigned* in_tick = nullptr; float* in_fin0 = nullptr; float* in_fin1 = nullptr; int* in_finalized = nullptr;
  int tmode = 0;    // conv_igemm_x3 timing-only A/B (MRAGAN_IG_TIMING; wrong results by design)
  int sk_slot = -1; // conv_igemm_x3 split-K: first ticket slot of the in-launch reduction (< 0: reduce launch)
};
int conv_igemm(IgemmArgs a, hipStream_t st);
size_t conv_igemm_ws_bytes(IgemmArgs a);
int conv_igemm_x3(IgemmArgs a, int64_t max_mc, int64_t total_m, hipStream_t st);
int conv_igemm_x3_shell(IgemmArgs a, hipStream_t st);
size_t conv_igemm_x3_ws_bytes(const IgemmArgs& a, int64_t max_mc, int64_t total_m);

// k3 s1 convolutions with an LDS-resident input halo (conv_brick.hip)
struct BrickArgs {
  const float* x; int N, Di, Hi, Wi, C;
  const float* w;   // packed [27][ny][C]
  const void* wx3;  // bf16x3 fragment-ordered copy of w (conv_brick_x3.hip), set by the launcher
  const float* bias;
  float* y; int Do, Ho, Wo, ny;
  int p, flip, act;
  short rowvox[128];  // GEMM row → brick voxel (bd·BH + bh)·BW + bw; −v−1: padding row reading voxel v
  int BD, BH, BW;   // output brick
  int HD, HH, HW;   // its input halo
  int nbd, nbh, nbw, gn, ntiles;
  double* part;     // optional InstanceNorm statistics partials [N][nbd·nbh·nbw][ny][2] (Σy, Σy²)
  int ye;           // output embedding: y is [N][Yd][Yh][Yw][ny], output voxel o written at o + ye
  int Yd, Yh, Yw;
  int x16;          // x is a 16-bit operand plane (conv_brick_x3 in the bf16 / fp16 modes)
  // optional (with part): backward-statistics partials instead of forward ones — the output is the
  // padded data gradient dz of a conv whose input was an InstanceNorm(+act) output of sx
  // ([N][Do−2][Ho−2][Wo−2][ny] fp32, statistics smean / srstd [N][ny]): part = Σ_p g, Σ_p g·x̂
  // with g = dz_p·act'(x̂) at the interior voxel p folds into (conv_brick_x3 only)
  const float* sx; const float* smean; const float* srstd; int sact;
  // optional with sx (ABI 18): a gradient added to the fold before act' — the ResnetBlock skip
  // gradient ([N][Do−2][Ho−2][Wo−2][ny] fp32; each interior voxel counted once, at the padded
  // output that maps onto it one to one)
  const float* sadd;
  int stamp;        // diagnostics: record s_memtime phase stamps (conv_brick_ks only)
  // optional with part (ABI 15, conv_brick_ks only): finalize in the launch (in_ticket.h) —
  // tick: N·gn zeroed counters; fin_mode 0: μ → fin0, rstd → fin1 ([N][ny]); 1: the backward
  // coefficients → fin0 ([N][ny][2]); fin_S: voxels per instance of the normalised tensor;
  // finalized (host side): set to 1 when the launch does it
  unsigned* tick; float* fin0; float* fin1; int fin_mode; double fin_S; int* finalized;
};
bool conv_brick_applicable(const IgemmArgs& a);
int conv_brick(const IgemmArgs& a, hipStream_t st, bool interior = false);
// the data gradient of a valid k3 s1 conv (transposed form, output = input + 2 per dim) as the
// interior brick pass plus the shell pass (conv_igemm.hip)
bool full_dgrad_split_applicable(const IgemmArgs& a);
int conv_brick_x3_launch(BrickArgs a, int bm, int bn, void* ws, size_t ws_bytes, const void* wsplit, int mode,
                         hipStream_t st);
size_t conv_brick_x3_ws_bytes(int C, int ny);
int brick_x3_pack(const float* w, int ny, int C, void* out, int mode, hipStream_t st);
// GEMM-row → brick-voxel permutation that makes the brick kernels' A reads bank-conflict free
// (S = 2: the stride-2 brick's halo, voxel (bd, bh, bw) reads row (2bd·HH + 2bh)·HW + bw in tap 0)
void brick_row_perm(int BD, int BH, int BW, int HH, int HW, int BM, short* rowvox, int S = 1);
// the k3 s2 p1 forward conv on the brick kernel's stride-2 form (conv_brick_x3.hip, round 6)
bool conv_brick_s2_applicable(const IgemmArgs& a);
int conv_brick_s2(const IgemmArgs& a, hipStream_t st);
// bf16 / fp16 k3 s1 brick with the contraction split over the block's 4 waves (conv_brick_ks.hip)
bool conv_brick_ks_applicable(const IgemmArgs& a);
int ks_debug_stamps(unsigned long long* host, int n);
int conv_brick_ks(BrickArgs a, int ny, void* ws, size_t ws_bytes, const void* wsplit, int mode, int* in_chunks,
                  hipStream_t st);
bool conv_brick_x3_active(const IgemmArgs& a);
// bf16x3 stride-2 transposed convolutions from an LDS halo (conv_brickT_x3.hip)
bool brickT_x3_applicable(const IgemmArgs& a);
size_t brickT_x3_ws_bytes(const IgemmArgs& a);
int conv_brickT_x3(const IgemmArgs& a, hipStream_t st);

struct ThinArgs {
  const float* x; int N, Di, Hi, Wi, cx;
  const float* w;      // packed [k³][ny][cx]
  const float* bias;
  float* y; int Do, Ho, Wo, ny;
  int k, s, p, trans, act;
  int rnd;             // operand rounding (op_round): the precision mode, set by the C ABI
  double* in_part = nullptr;   // optional (thin1_x3 forward only): the next InstanceNorm's Σy / Σy²
  int* in_chunks = nullptr;    // set to the items per instance when in_part was filled
  // optional, with in_part on the transposed form (thin1_x3): backward statistics of the
  // InstanceNorm(+act) of bs_x whose output, replication-padded by bs_fold, was the conv's input
  const float* bs_x = nullptr; const float* bs_mean = nullptr; const float* bs_rstd = nullptr;
  int bs_act = 0, bs_fold = 0;
  int x16 = 0;                 // x is a 16-bit operand plane (thinn_x3 only, the one-plane modes)
};
int conv_thin(ThinArgs a, hipStream_t st);
// ConvTranspose3d k4 s2 p1 to 1-2 channels on MFMA, one-plane modes (conv_up4.hip)
bool up4_mfma_applicable(const ThinArgs& a);
int conv_up4_mfma(const ThinArgs& a, hipStream_t st);
// Conv3d k4 s2 p1 from 1-2 to 32 | 64 channels on MFMA, one-plane modes (conv_down4.hip)
bool down4_mfma_applicable(const ThinArgs& a);
int conv_down4_mfma(const ThinArgs& a, hipStream_t st);
// MFMA path for 1 → 32-channel k7 s1 convolutions (conv_thin1_ring.hip); 2 → 32 in the one-plane
// modes (mode = the precision code)
bool thin1_x3_applicable(int cx, int ny, int k, int s, int mode);
size_t thin1_x3_ws_bytes(int ny);
int conv_thin1_x3(const ThinArgs& a, int mode, void* ws, size_t ws_bytes, hipStream_t st);
int thin1_debug_stamps(unsigned long long* host, int n);
// bf16x3 MFMA path for 32 → 1-channel k7 s1 convolutions (conv_thinn_x3.hip)
bool thinn_x3_applicable(int cx, int ny, int k, int s, int mode);
size_t thinn_x3_ws_bytes(int ny);
int conv_thinn_x3(const ThinArgs& a, int mode, void* ws, size_t ws_bytes, hipStream_t st);
// bf16x3 MFMA weight gradient of the 1-channel k7 s1 convolutions (conv_thin1_wgrad_x3.hip)
bool thin1_wgrad_x3_applicable(int Cd, int Cg, int k, int s, int mode);
size_t thin1_wgrad_x3_ws_bytes();
// wide16: the 32-channel operand is the 16-bit operand plane of the mode (one-plane modes)
int conv_thin1_wgrad_x3(const float* D, int N, int Dd, int Hd, int Wd, int Cd, const float* G, int Dg, int Hg, int Wg,
                        int Cg, int p, float* out, int accumulate, int mode, void* ws, size_t ws_bytes, hipStream_t st,
                        int wide16 = 0);

struct WgradArgs {
  const float* D; int N, Dd, Hd, Wd, Cd;
  const float* G; int Dg, Hg, Wg, Cg;
  int k, s, p;
  float* ws;       // [splits][k³][Cd][Cg]
  int64_t chunk;   // set by conv_wgrad
  int splits;
  int x3;          // precision mode (prec.h): 0 f32; 1 bf16x3 / 2 bf16 / 3 fp16 MFMA (Cd, Cg multiples of 32)
  int in16;        // D and G are 16-bit operand planes (wgrad3_x3 in the bf16 / fp16 modes only)
  int in16g = 0;   // only G is a 16-bit operand plane (wgrad3s2_x3, the one-plane modes: the fine-grid
                   // operand of the 64³-level stride-2 layers)
  // ABI 19: a second instance set (N2 instances of D2 / G2, same per-instance shape) summed into the
  // same gradient — a generator's first-pass and cycle-pass operands of one ResnetBlock conv in one
  // launch (wgrad3_x3 on operand planes, aligned stages; otherwise two passes)
  const float* D2 = nullptr; const float* G2 = nullptr; int N2 = 0;
};
int conv_wgrad(WgradArgs a, float* out, int accumulate, size_t ws_bytes, hipStream_t st);
// bf16x3 weight gradient of valid k3 s1 convs on padded inputs, 3 kw taps per block (conv_wgrad3_x3.hip)
bool wgrad3_x3_applicable(const WgradArgs& a);
int wgrad3_x3_splits(const WgradArgs& a, int max_splits);
int conv_wgrad3_x3(const WgradArgs& a, int splits, hipStream_t st);   // returns the splits used
// bf16x3 weight gradient of the k3 s2 p1 convs / transposed convs, 3 kw taps per block (conv_wgrad3s2_x3.hip)
bool wgrad3s2_x3_applicable(const WgradArgs& a);
int wgrad3s2_x3_splits(const WgradArgs& a, int max_splits);
int conv_wgrad3s2_x3(const WgradArgs& a, int splits, hipStream_t st);   // returns the splits used
size_t conv_wgrad_ws_bytes(int N, int Dd, int Hd, int Wd, int Cd, int Cg, int k);

struct ThinWgradArgs {
  const float* D; int N, Dd, Hd, Wd, Cd;
  const float* G; int Dg, Hg, Wg, Cg;
  int k, s, p;
  int vec_dn;      // 1: 4-vector over dn (wide side = D), 0: over gn (wide side = G)
  int tiles_d, tiles_h, tiles_w, ntiles;
  int nroles, RS;
  float* slab;     // [gridDim.x][Cd*Cg*k³]
  int rnd;         // operand rounding (op_round): the precision mode, set by the C ABI
};
int conv_thin_wgrad(ThinWgradArgs a, float* out, int accumulate, float* ws, size_t ws_bytes, hipStream_t st);
size_t conv_thin_wgrad_ws_bytes(int N, int Dd, int Hd, int Wd, int Cd, int Cg, int k, int s);

struct InShape {
  int N, D, H, W, C;
  __host__ __device__ int64_t S() const { return (int64_t)D * H * W; }
};
struct InBwdArgs {
  const float* x; const float* mean; const float* rstd;
  const float* dy; int dypad; const float* dy_add; int act;
  float* dx;           // fp32 dx, or null when only dx16 is wanted
  float* g_out;        // optional: g = fold(dy) + dy_add before act' (the ResnetBlock's input gradient)
  void* dx16;          // optional: dx as the 16-bit operand plane of precision mode mode16 (2 bf16, 3 fp16)
  int mode16;
};
// y and / or y16 (the 16-bit operand plane of y in precision mode mode16) are written
int instnorm_fwd(const float* x, InShape s, float* y, int ypad, int act, const float* resid, int rpad, float* mean,
                 float* rstd, void* ws, size_t ws_bytes, hipStream_t st, void* y16 = nullptr, int mode16 = 0);
int instnorm_bwd(const InBwdArgs& a, InShape s, void* ws, size_t ws_bytes, hipStream_t st);
int instnorm_fwd_partials(const float* x, InShape s, float* y, int ypad, int act, const float* resid, int rpad,
                          float* mean, float* rstd, const double* part, int chunks, hipStream_t st, void* y16 = nullptr,
                          int mode16 = 0);
int instnorm_bwd_partials(const InBwdArgs& a, InShape s, const double* part, int chunks, void* ws, size_t ws_bytes,
                          hipStream_t st);
// ABI 15: the apply passes alone (statistics finalized by the producing conv, in_ticket.h)
int instnorm_apply(const float* x, InShape s, float* y, int ypad, int act, const float* resid, int rpad,
                   const float* mean, const float* rstd, hipStream_t st, void* y16, int mode16);
int instnorm_bwd_apply(const InBwdArgs& a, InShape s, const float* coef, hipStream_t st);
size_t instnorm_ws_bytes(int N, int D, int H, int W, int C);
int instnorm_running(const void* table, int nentries, float momentum, hipStream_t st);
size_t instnorm_running_entry_bytes();

int rpad(const float* x, int N, int D, int H, int W, int C, int p, float* y, hipStream_t st);
int rpad_fold(const float* yp, int N, int D, int H, int W, int C, int p, const float* add, float* x, hipStream_t st);
int channel_concat(const float* a, int Ca, int act_a, const float* b, int Cb, int act_b, int64_t M, float* out,
                   hipStream_t st);
int channel_split(const float* g, int Ca, int Cb, int64_t M, const float* ya, int act_a, float* da, const float* yb,
                  int act_b, float* db, hipStream_t st);
int act_bwd(const float* y, const float* g0, const float* g1, const float* g2, int64_t n, int act, float* dx, hipStream_t st);
int l1_loss(const float* a, const float* b, int64_t n, float scale, float gscale, float* loss, int loss_acc, float* grad,
            int grad_acc, float* ws, hipStream_t st);
int gan_loss(const float* p, int64_t n, float target, int lsgan, float scale, float gscale, float* loss, int loss_acc,
             float* dlogit, float* ws, hipStream_t st);
int channel_sum(const float* x, int64_t M, int C, float* out, int acc, void* ws, size_t ws_bytes, hipStream_t st);
size_t channel_sum_ws_bytes(int64_t M, int C);
int adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2, float eps, int step,
         float grad_scale, hipStream_t st);
void adam_hyper(float lr, float beta1, float beta2, float eps, int step, float grad_scale, float* out);
int adam_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper, const int* skip,
             hipStream_t st);
int adam_rebias(const float* base, const int* skipped, float* hyper, hipStream_t st);
int nonfinite_flag(const float* g, int64_t n, int* flag, hipStream_t st);
int skip_count(int* flag, int* counter, hipStream_t st);
int pack_weight(const float* src, int A, int B, int T, int tr, float* dst, hipStream_t st);
struct PackEntry {          // layout shared with include/mragan_hip.h (mragan_pack_entry)
  const float* src;
  float* dst;
  int A, B, T, tr;  // tr 0/1: fp32 [T][A][B] / [T][B][A]; 2/3: same, bf16x3 brick fragment order
};
int pack_weights_batched(const PackEntry* table, int n, int64_t max_elems, hipStream_t st);
int fill(float* p, int64_t n, float v, hipStream_t st);

// sliding-window inference (sliding.hip)
int patch_gather(const float* vol, int X, int Y, int Z, const int* starts, int n, int px, int py, int pz, float* out,
                 hipStream_t st);
int crop_patches(const float* vol, int X, int Y, int Z, const int* starts, int n, int px, int py, int pz, float* out,
                 hipStream_t st);
int patch_combine(const float* pred, int X, int Y, int Z, int px, int py, int pz, int inum, int jnum, int knum, int s_in,
                  int s_lay, float* label, hipStream_t st);

}  // namespace mragan
