/* mragan_hip.h — C ABI of the MI355X (gfx950) kernel library behind the MRA-GAN CycleGAN
 * training step.  Built as mra-gan_amd/lib/libmragan_hip.so.
 *
 * The reference (pedrob37/MRA-GAN) has no FFI: its hot path is PyTorch/ATen called from
 * models/networks3D.py and models/cycle_gan_model.py.  Each entry point below replaces the
 * ATen op(s) those reference lines invoke; the Python layer in mra-gan_amd/ (models/,
 * mragan_hip/) binds them with ctypes.
 *
 * Conventions
 *   - every pointer is a device pointer (hipMalloc / torch caching allocator); kernels never
 *     allocate, callers pass workspaces sized by the *_workspace() queries;
 *   - activations are NDHWC fp32 (channels contiguous); "padded" tensors carry a replication
 *     border of `pad` voxels on every spatial side;
 *   - packed conv weights are [k³][Nout][Kc] fp32 (tap = (td*k + th)*k + tw), produced from the
 *     torch layouts by mragan_pack_weight;
 *   - `stream` is a hipStream_t (NULL = default stream);
 *   - return value 0 = success, otherwise an error code; mragan_last_error() describes it.
 */
#ifndef MRAGAN_HIP_H_
#define MRAGAN_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MRAGAN_ABI_VERSION 19

enum mragan_status { MRAGAN_OK = 0, MRAGAN_EBADARG = 1, MRAGAN_EWORKSPACE = 2, MRAGAN_ELAUNCH = 3, MRAGAN_EUNSUPPORTED = 4 };
enum mragan_act { MRAGAN_ACT_NONE = 0, MRAGAN_ACT_RELU = 1, MRAGAN_ACT_LRELU = 2, MRAGAN_ACT_TANH = 3, MRAGAN_ACT_SIGMOID = 4 };

int mragan_abi_version(void);
const char* mragan_last_error(void);

/* Contraction precision of the MFMA convolutions, process-wide.  The reference computes in fp32
 * (ATen conv); every mode takes and returns fp32 tensors (activations, weights and gradients stay
 * fp32 in HBM; only the MFMA operands are rounded).
 *   MRAGAN_PREC_F32    exact fp32 products (v_mfma_f32_32x32x2_f32 / VALU), 157 TF peak;
 *   MRAGAN_PREC_BF16X3 each operand split into bf16 hi + lo, a·b ≈ lo·hi + hi·lo + hi·hi with fp32
 *                      accumulation (3 × v_mfma_f32_32x32x16_bf16), ≤ 3·2⁻¹⁸ relative error per
 *                      product, up to 5.3× the exact rate;
 *   MRAGAN_PREC_BF16   operands rounded to bf16, one v_mfma_f32_32x32x16_bf16 per product, fp32
 *                      accumulation (BASELINE configs[1]/[2] "bf16"), 2.5 PF peak;     (ABI 7)
 *   MRAGAN_PREC_F16    operands rounded to fp16, one v_mfma_f32_32x32x16_f16 per product, fp32
 *                      accumulation (configs[4] "fp16"); use with a loss scale.          (ABI 7)
 * In the bf16 / fp16 modes EVERY convolution operand is rounded (RNE) to that type — the MFMA
 * kernels' fragments, and the operands the fp32-computing kernels load (the thin VALU convolutions
 * of the image-channel layers: D first / last, the nc > 1 G stem / head; the fp32 fallbacks for
 * channel counts the MFMA kernels do not tile): forward x and W, data-gradient dY and W,
 * weight-gradient X and dY.  Products accumulate in fp32 (the thin D-first data gradient in
 * fp64).  The fp32-grade modes (f32, bf16x3) never round.                              (ABI 10) */
enum mragan_precision { MRAGAN_PREC_F32 = 0, MRAGAN_PREC_BF16X3 = 1, MRAGAN_PREC_BF16 = 2, MRAGAN_PREC_F16 = 3 };
int mragan_set_conv_precision(int mode);
int mragan_get_conv_precision(void);
/* Loss scale (static, process-wide; default 1): mragan_l1_loss / mragan_gan_loss multiply the
 * gradients they write (not the loss values) by it, so every gradient of the backward — and the
 * weight gradients in the flat buffers — carry the factor; the optimizer divides it out through
 * its grad_scale.  The fp16 mode uses it to keep gradients in fp16's normal range.  (ABI 7)    */
int mragan_set_loss_scale(float scale);
float mragan_get_loss_scale(void);

/* ---- convolution --------------------------------------------------------------------------
 * Forward form:     y[n,o,:] = act(bias + Σ_{j<k³} x[n, o*stride − pad + j, :] · Wp[j])  (zero fill)
 * Replaces nn.Conv3d.forward (networks3D.py:186, 192, 241, 257, 212, 389, 397, 406, 414) and the
 * input-gradient of nn.ConvTranspose3d (networks3D.py:203-210).                              */
int mragan_conv3d_fwd(const float* x, int N, int Di, int Hi, int Wi, int cin, const float* wpacked, const float* bias,
                      int cout, int k, int stride, int pad, int act, float* y, int Do, int Ho, int Wo, void* ws,
                      size_t ws_bytes, void* stream);

/* Transposed form:  y[n,o,:] = act(bias + Σ_{t:(o+pad−t)%stride==0} x[n,(o+pad−t)/stride,:] · Wp[t])
 * Replaces nn.ConvTranspose3d.forward (networks3D.py:203-210) and the input-gradient of every
 * nn.Conv3d above (autograd convolution_backward, grad_input branch).                        */
int mragan_conv3d_transposed(const float* x, int N, int Di, int Hi, int Wi, int cin, const float* wpacked,
                             const float* bias, int cout, int k, int stride, int pad, int act, float* y, int Do, int Ho,
                             int Wo, void* ws, size_t ws_bytes, void* stream);
/* Either form (transposed = 0/1) with the weight also given pre-split: `wsplit` is the same packed
 * weight written by mragan_pack_weights with tr = 2 + transpose_ab (bf16x3 brick fragment order).
 * Used by the k3 s1 bf16x3 brick kernel instead of re-splitting `wpacked` on every call (the
 * ResnetBlock convs, networks3D.py:241-257, and their data gradients); ignored by every other
 * kernel.  The caller keeps `wsplit` in step with `wpacked` (same pack launch).  (ABI 6) */
int mragan_conv3d_presplit(const float* x, int N, int Di, int Hi, int Wi, int cin, const float* wpacked,
                           const void* wsplit, const float* bias, int cout, int k, int stride, int pad, int act,
                           float* y, int Do, int Ho, int Wo, int transposed, void* ws, size_t ws_bytes, void* stream);
/* Same, and when the convolution runs on the brick kernel (k3 s1, 16-bit MFMA modes) also the
 * statistics partials of the InstanceNorm that follows it (networks3D.py:241-257: Conv3d →
 * InstanceNorm3d in every ResnetBlock): part[N][chunks][cout][2] = fp64 Σy, Σy² of the written
 * output per brick, *chunks = bricks per instance; *chunks = 0 when another kernel ran (the
 * caller then runs mragan_instnorm_fwd).  part_bytes ≥ 16·N·Do·⌈Ho/4⌉·⌈Wo/6⌉·cout.  ABI 9. */
int mragan_conv3d_presplit_in_stats(const float* x, int N, int Di, int Hi, int Wi, int cin, const float* wpacked,
                                    const void* wsplit, const float* bias, int cout, int k, int stride, int pad, int act,
                                    float* y, int Do, int Ho, int Wo, int transposed, void* ws, size_t ws_bytes,
                                    double* part, size_t part_bytes, int* chunks, void* stream);

/* Workspace (bytes) the two calls above need for these shapes in the current precision mode:
 * split-K partial tiles of small-M / large-K dense convolutions (PatchGAN layers 2-4 and their
 * data gradients), summed in a fixed order by a second kernel; 0 when no split is used. */
size_t mragan_conv3d_workspace(int N, int Di, int Hi, int Wi, int cin, int cout, int k, int stride, int pad,
                               int Do, int Ho, int Wo, int transposed);

/* Weight gradient:  dw[dn][gn][t] (=|+=) Σ_m dense[m][dn] · gathered[m*stride − pad + t][gn]
 * Conv3d:          dense = dY (output grid), gathered = X      → dw = torch [Cout][Cin][k][k][k]
 * ConvTranspose3d: dense = X (input grid),   gathered = dY     → dw = torch [Cin][Cout][k][k][k]
 * Replaces the grad_weight branch of convolution_backward for the same layers.              */
size_t mragan_conv3d_wgrad_workspace(int N, int Dd, int Hd, int Wd, int Cd, int Cg, int k, int stride);
int mragan_conv3d_wgrad(const float* dense, int N, int Dd, int Hd, int Wd, int Cd, const float* gathered, int Dg, int Hg,
                        int Wg, int Cg, int k, int stride, int pad, float* dw, int accumulate, void* ws,
                        size_t ws_bytes, void* stream);

/* src[A][B][k³] (torch layout) → dst[k³][A][B] (transpose_ab = 0) or dst[k³][B][A] (= 1). */
int mragan_pack_weight(const float* src, int A, int B, int T, int transpose_ab, float* dst, void* stream);
/* n packs in one launch (a network's repack after each optimizer step, networks3D.py's conv
 * weights): `table` is a DEVICE array of n entries {const float* src; float* dst; int A, B, T,
 * transpose_ab;} (mragan_pack_entry_size() bytes each), max_elems ≥ every entry's A·B·T.
 * transpose_ab = 2 | 3: the pack of (transpose_ab & 1) written as bf16 hi/lo split fragments
 * for mragan_conv3d_presplit (T = 27 and the contraction side a multiple of 32; dst holds
 * A·B·T·4 bytes).                                                                          */
size_t mragan_pack_entry_size(void);
int mragan_pack_weights(const void* table, int n, int64_t max_elems, void* stream);

/* ---- InstanceNorm3d(affine=False, track_running_stats=True), train mode --------------------
 * y (replication-padded by ypad) = act((x − μ_nc)·rstd_nc) (+ resid interior of an rpad-padded
 * tensor).  mean / rstd: [N][C] outputs saved for the backward.  Replaces nn.InstanceNorm3d +
 * the following nn.ReLU / LeakyReLU / residual add / nn.ReplicationPad3d
 * (networks3D.py:19, 186-189, 191-197, 203-210, 233-263, 396-409).                           */
size_t mragan_instnorm_workspace(int N, int D, int H, int W, int C);
int mragan_instnorm_fwd(const float* x, int N, int D, int H, int W, int C, float* y, int ypad, int act, const float* resid,
                        int rpad, float* mean, float* rstd, void* ws, size_t ws_bytes, void* stream);
/* dx = IN-backward( fold(dy, dypad) + dy_add ) through act; the workspace must hold
 * mragan_instnorm_workspace(...) + 8·N·C bytes.                                              */
int mragan_instnorm_bwd(const float* x, const float* mean, const float* rstd, int N, int D, int H, int W, int C,
                        const float* dy, int dypad, const float* dy_add, int act, float* dx, void* ws, size_t ws_bytes,
                        void* stream);
/* InstanceNorm forward from statistics partials a producer already accumulated (written by
 * mragan_conv3d_presplit_in_stats: [N][chunks][C][2] fp64 Σy, Σy² per brick): finalize + apply
 * only, no statistics pass over x.  ABI 9. */
int mragan_instnorm_fwd_partials(const float* x, int N, int D, int H, int W, int C, float* y, int ypad, int act,
                                 const float* resid, int rpad, float* mean, float* rstd, const double* part, int chunks,
                                 void* stream);
/* Same, and also writes g_out = fold(dy, dypad) + dy_add (before act') — the gradient w.r.t. a
 * ResnetBlock's input, x + conv_block(x) (networks3D.py:262-263), which the block's skip path
 * adds again one block earlier: the ReplicationPad3d backward and the skip-gradient add of the
 * reference's autograd happen in this one pass (no separate mragan_rpad_fold).  ABI 8. */
int mragan_instnorm_bwd_g(const float* x, const float* mean, const float* rstd, int N, int D, int H, int W, int C,
                          const float* dy, int dypad, const float* dy_add, int act, float* dx, float* g_out, void* ws,
                          size_t ws_bytes, void* stream);

/* ---- 16-bit operand planes (bf16 / fp16 modes only; ABI 11) --------------------------------
 * The "operand plane" of an fp32 NDHWC tensor is the same tensor as the 16-bit words (bf16 in
 * MRAGAN_PREC_BF16, fp16 in MRAGAN_PREC_F16, round-to-nearest-even) every MFMA convolution of that
 * mode rounds its fp32 operands to — so a convolution reading the plane computes exactly the
 * products it computes from the fp32 tensor, from half the bytes and with no conversion.  A
 * producer writes the plane of a tensor that is only ever a convolution operand (a ResnetBlock's
 * relu(IN(conv1(x))) and the InstanceNorm-backward outputs that are the dY of its two convs,
 * networks3D.py:241-257) instead of the fp32 tensor, and beside it for a tensor that also feeds
 * fp32 math (a block's output: the next block's skip add, :262-263).  Every entry fails with
 * MRAGAN_EBADARG in the fp32-grade modes.
 *   instnorm_fwd_op16 / _partials_op16: mragan_instnorm_fwd / _fwd_partials writing y (fp32,
 *       nullable) and / or y16 (its plane, nullable, same padded layout);
 *   instnorm_bwd_op16: mragan_instnorm_bwd_g writing dx only as its plane dx16 (g_out nullable);
 *   conv3d_op16: mragan_conv3d_presplit_in_stats (no bias, no activation) on the plane x16 of
 *       the input — the k3 s1 brick kernel (ResnetBlock convs and their whole-grid data
 *       gradients), and (ABI 14) the implicit GEMM for the other forward-form convs with a multiple
 *       of 32 input channels (G down1 / down2 on the stem / down1 InstanceNorm planes);
 *       wsplit nullable (the brick then splits per call); part / chunks nullable (no partials);
 *   conv3d_wgrad_op16: mragan_conv3d_wgrad on the planes of dense and gathered — the k3 s1 valid
 *       weight gradient of the ResnetBlock convs (wgrad3_x3).
 * ABI 19: in mragan_conv3d_presplit(_in_stats), mragan_conv3d_op16(_fin) and the
 * mragan_conv3d_op16_dgrad_in_stats family `wpacked` may be NULL when `wsplit` is given.  The k3 s1
 * bricks and both passes of the interior + shell data gradient read only `wsplit` (the shell pass
 * stages its hi words); every kernel that needs the fp32 pack then fails with MRAGAN_EBADARG
 * instead of reading it.  A caller that refreshes only the pre-split copy after an optimizer step
 * (the fp32 pack stale) passes NULL, so no kernel can read stale weights.
 * mragan_conv3d_dgrad_split: 1 when the whole-grid data gradient of a k3 s1 p0 conv from the plane of
 * dY ([N][Di][Hi][Wi][cin] → [N][Di+2][Hi+2][Wi+2][cout], transposed form) runs as the interior brick
 * plus the shell pass in the current mode, else 0 — the rule the engine schedules by (that form
 * leaves no backward statistics), queried instead of mirrored.                              */
int mragan_conv3d_dgrad_split(int N, int Di, int Hi, int Wi, int cin, int cout);
/* ABI 19: mragan_conv3d_wgrad_op16 over two instance sets of one shape — Na instances of
 * (dense16_a, gathered16_a) and Nb of (dense16_b, gathered16_b) — summed into dw.  The reference
 * accumulates a generator's weight gradient from its first pass and its cycle pass in one
 * loss_G.backward() (cycle_gan_model.py:163-225); here each ResnetBlock conv's weight gradient is
 * one launch (+ its reduce) over both passes' saved planes where the k3 s1 valid kernel's aligned
 * operand-plane path applies, two accumulating passes otherwise.  Workspace:
 * mragan_conv3d_wgrad_workspace(Na + Nb, ...). */
int mragan_conv3d_wgrad_op16_pair(const void* dense16_a, int Na, const void* gathered16_a, const void* dense16_b, int Nb,
                                  const void* gathered16_b, int Dd, int Hd, int Wd, int Cd, int Dg, int Hg, int Wg, int Cg,
                                  int k, int stride, int pad, float* dw, int accumulate, void* ws, size_t ws_bytes,
                                  void* stream);
int mragan_instnorm_fwd_op16(const float* x, int N, int D, int H, int W, int C, float* y, void* y16, int ypad, int act,
                             const float* resid, int rpad, float* mean, float* rstd, void* ws, size_t ws_bytes,
                             void* stream);
int mragan_instnorm_fwd_partials_op16(const float* x, int N, int D, int H, int W, int C, float* y, void* y16, int ypad,
                                      int act, const float* resid, int rpad, float* mean, float* rstd,
                                      const double* part, int chunks, void* stream);
int mragan_instnorm_bwd_op16(const float* x, const float* mean, const float* rstd, int N, int D, int H, int W, int C,
                             const float* dy, int dypad, const float* dy_add, int act, void* dx16, float* g_out, void* ws,
                             size_t ws_bytes, void* stream);
int mragan_conv3d_op16(const void* x16, int N, int Di, int Hi, int Wi, int cin, const float* wpacked, const void* wsplit,
                       int cout, int k, int stride, int pad, float* y, int Do, int Ho, int Wo, int transposed, void* ws,
                       size_t ws_bytes, double* part, size_t part_bytes, int* chunks, void* stream);
int mragan_conv3d_wgrad_op16(const void* dense16, int N, int Dd, int Hd, int Wd, int Cd, const void* gathered16, int Dg,
                             int Hg, int Wg, int Cg, int k, int stride, int pad, float* dw, int accumulate, void* ws,
                             size_t ws_bytes, void* stream);
/* ABI 14: mragan_conv3d_wgrad with only the gathered (fine-grid) operand as its 16-bit plane — the
 * k3 s2 p1 weight gradients of G down1 / down2 (networks3D.py:192-197; the reference's
 * Conv3d.weight.grad via ATen's convolution_backward), whose gathered operand is the stem / down1
 * InstanceNorm output that exists only as a plane in the bf16 / fp16 modes; dense stays fp32. */
int mragan_conv3d_wgrad_g16(const float* dense, int N, int Dd, int Hd, int Wd, int Cd, const void* gathered16, int Dg,
                            int Hg, int Wg, int Cg, int k, int stride, int pad, float* dw, int accumulate, void* ws,
                            size_t ws_bytes, void* stream);
/* InstanceNorm backward statistics in the data-gradient epilogue (ABI 11).  In a
 * ResnetBlock (networks3D.py:241-257) conv2's input is z1 = relu(IN(h1)) padded by 1, so the IN
 * backward of h1 reads g = fold(dz1)·relu'(x̂) with dz1 = conv2's padded data gradient.  Its two
 * statistics are sums over the padded grid: Σ_i g_i = Σ_p dz_p·act'(x̂_c(p)), Σ_i g_i·x̂_i =
 * Σ_p dz_p·act'(x̂_c(p))·x̂_c(p) (c = the fold's clamp).  mragan_conv3d_op16_dgrad_in_stats is the
 * whole-grid data gradient (k3 s1 p0, transposed form, output (Di+2)·(Hi+2)·(Wi+2)) from the
 * plane dy16 that also leaves these per-brick partials, reading x_in (h1, [N][Di][Hi][Wi][cout]
 * fp32) and its IN statistics in the epilogue; mragan_instnorm_bwd_partials_op16 is
 * mragan_instnorm_bwd_op16 from them (finalize + apply: no statistics pass over dy and x). */
int mragan_conv3d_op16_dgrad_in_stats(const void* dy16, int N, int Di, int Hi, int Wi, int cin, const float* wpacked,
                                      const void* wsplit, int cout, float* y, void* ws, size_t ws_bytes, const float* x_in,
                                      const float* mean, const float* rstd, int act, double* part, size_t part_bytes,
                                      int* chunks, void* stream);
int mragan_instnorm_bwd_partials_op16(const float* x, const float* mean, const float* rstd, int N, int D, int H, int W,
                                      int C, const float* dy, int dypad, const float* dy_add, int act, void* dx16,
                                      float* g_out, const double* part, int chunks, void* ws, size_t ws_bytes,
                                      void* stream);
/* ABI 15: InstanceNorm statistics finalized inside the producing conv ("last block done"; VERDICT
 * r03 item 5).  The _fin forms take, besides the partials, `tickets` — N·cout/32 uint32 counters,
 * zero on entry, that no kernel which may run at the same time uses (the launch leaves them zero:
 * hand them out round-robin from one zeroed pool) — and the statistics outputs.  When the kernel
 * that runs the conv finalizes in-launch (the K-split brick, bf16 / fp16, a multiple of 128
 * contraction channels, one round of CU slots), *finalized = 1 and mean / rstd ([N][cout]) — or,
 * for the data gradient, coef ([N][cout][2] = mean(g), mean(g·x̂), the IN backward's two
 * coefficients) — are written; then the apply-only entries below replace
 * mragan_instnorm_fwd_partials_op16 / mragan_instnorm_bwd_partials_op16 (no finalize launch).
 * Otherwise *finalized = 0 and the partials are left as by the non-_fin form.  The in-launch sums
 * run in a different fixed order than the finalize kernel's: deterministic, equal to ~1e-16
 * relative. */
int mragan_conv3d_op16_fin(const void* x16, int N, int Di, int Hi, int Wi, int cin, const float* wpacked, const void* wsplit,
                           int cout, int k, int stride, int pad, float* y, int Do, int Ho, int Wo, int transposed,
                           void* ws, size_t ws_bytes, double* part, size_t part_bytes, int* chunks, unsigned* tickets,
                           float* mean, float* rstd, int* finalized, void* stream);
int mragan_conv3d_op16_dgrad_in_stats_fin(const void* dy16, int N, int Di, int Hi, int Wi, int cin, const float* wpacked,
                                          const void* wsplit, int cout, float* y, void* ws, size_t ws_bytes,
                                          const float* x_in, const float* mean, const float* rstd, int act, double* part,
                                          size_t part_bytes, int* chunks, unsigned* tickets, float* coef, int* finalized,
                                          void* stream);
/* ABI 18: mragan_conv3d_op16_dgrad_in_stats(_fin) with a gradient x_add ([N][Di][Hi][Wi][cout]
 * fp32) that joins the fold before act': the IN backward in front then reads g = fold(dz) + x_add
 * (mragan_instnorm_bwd_partials_op16 with dy_add = x_add).  In the ResnetBlock chain
 * (networks3D.py:241-263, out = x + block(x)) conv1's data gradient dz of block i+1 and the block
 * output gradient G of block i+1 (the skip path) meet at block i's second InstanceNorm, whose
 * backward statistics Σ g, Σ g·x̂ then come from this epilogue (x_add read at the padded outputs
 * that map one to one onto an interior voxel) and its statistics pass goes.  Brick kernels only
 * (bf16 / fp16, whole-grid k3 s1): elsewhere *chunks = 0 (run the statistics pass).  tickets may be
 * null (then as the non-_fin form; coef / finalized unused). */
int mragan_conv3d_op16_dgrad_in_stats_add(const void* dy16, int N, int Di, int Hi, int Wi, int cin, const float* wpacked,
                                          const void* wsplit, int cout, float* y, void* ws, size_t ws_bytes,
                                          const float* x_in, const float* mean, const float* rstd, int act,
                                          const float* x_add, double* part, size_t part_bytes, int* chunks,
                                          unsigned* tickets, float* coef, int* finalized, void* stream);
/* ABI 16: mragan_conv3d_presplit_bwd_stats on the 16-bit operand plane of its input (bf16 / fp16
 * modes; the stride-2 implicit GEMM, a multiple of 32 input channels): the data gradient of G up1 /
 * up2 (ConvTranspose3d k3 s2, networks3D.py:203-209) from the plane of the IN backward's dx, with the
 * backward statistics of the IN in front; results bit-identical to the fp32-input form. */
int mragan_conv3d_op16_bwd_stats(const void* x16, int N, int Di, int Hi, int Wi, int cin, const float* wpacked, int cout,
                                  int k, int stride, int pad, float* y, int Do, int Ho, int Wo, int transposed, void* ws,
                                  size_t ws_bytes, const float* x_in, const float* mean, const float* rstd, int act,
                                  double* part, size_t part_bytes, int* chunks, void* stream);
/* ABI 17: the k7 layers on 16-bit operand planes (bf16 / fp16 modes).
 *   mragan_conv3d_thin_op16: the 32 → nc (1, 2) k7 s1 convolution from the plane of its 32-channel
 *       input — the G head forward on ReplicationPad3d(3)(relu(IN(x))) of the last up-conv
 *       (networks3D.py:211-213) and the G stem's data gradient from the plane of the stem IN
 *       backward's dx (transposed = 1; networks3D.py:185-189).  Same arguments and results as
 *       mragan_conv3d_fwd / _transposed on the fp32 tensor (bit-identical).
 *   mragan_conv3d_wgrad_thin_op16: mragan_conv3d_wgrad of the k7 s1 layers (one side nc = 1 or 2,
 *       the other 32 channels) with the 32-channel operand as its plane, the nc-channel one fp32:
 *       the head's dW (gathered = the head input's plane) and the stem's (dense = the plane of dx). */
int mragan_conv3d_thin_op16(const void* x16, int N, int Di, int Hi, int Wi, int cin, const float* wpacked,
                            const float* bias, int cout, int k, int stride, int pad, int act, float* y, int Do, int Ho,
                            int Wo, int transposed, void* ws, size_t ws_bytes, void* stream);
int mragan_conv3d_wgrad_thin_op16(const void* dense, int N, int Dd, int Hd, int Wd, int Cd, const void* gathered, int Dg,
                                  int Hg, int Wg, int Cg, int k, int stride, int pad, float* dw, int accumulate, void* ws,
                                  size_t ws_bytes, void* stream);
int mragan_instnorm_apply_op16(const float* x, int N, int D, int H, int W, int C, float* y, void* y16, int ypad, int act,
                               const float* resid, int rpad, const float* mean, const float* rstd, void* stream);
int mragan_instnorm_bwd_apply_op16(const float* x, const float* mean, const float* rstd, int N, int D, int H, int W,
                                   int C, const float* dy, int dypad, const float* dy_add, int act, void* dx16,
                                   float* g_out, const float* coef, void* stream);
/* The same for the G head (ABI 12; networks3D.py:211-213): the head conv (ngf → 1, k7 p0) reads
 * ReplicationPad3d(3)(relu(IN(x))) of the last up-conv's output x.  mragan_conv3d_dgrad_in_stats
 * is its data gradient — the transposed form (stride 1, pad 0) of the packed weight, output
 * (Di+k−1)·(Hi+k−1)·(Wi+k−1)·cout fp32 — that also leaves the backward-statistics partials of that
 * InstanceNorm, reading x_in ([N][Di+k−1−2·fold_pad]…[cout]) at the fold's clamp of every padded
 * voxel, when the kernel that runs it has the epilogue (thin1_x3: cin 1, cout 32, k7, 16-bit
 * MFMA modes); otherwise it computes the plain data gradient and *chunks = 0.
 * mragan_instnorm_bwd_partials is mragan_instnorm_bwd (fp32 dx) from such partials. */
int mragan_conv3d_dgrad_in_stats(const float* dy, int N, int Di, int Hi, int Wi, int cin, const float* wpacked, int cout,
                                 int k, float* y, void* ws, size_t ws_bytes, const float* x_in, const float* mean,
                                 const float* rstd, int act, int fold_pad, double* part, size_t part_bytes, int* chunks,
                                 void* stream);
int mragan_instnorm_bwd_partials(const float* x, const float* mean, const float* rstd, int N, int D, int H, int W, int C,
                                 const float* dy, int dypad, const float* dy_add, int act, float* dx, float* g_out,
                                 const double* part, int chunks, void* ws, size_t ws_bytes, void* stream);
/* The same without a fold, for the stride-2 layers (ABI 12): a conv (forward or transposed form,
 * pre-split weights, no bias / act) whose output y is the data gradient of an InstanceNorm(+act)
 * of x_in (same shape as y) — G down1 / up1 norms (networks3D.py:192-210) — leaving that norm's
 * backward-statistics partials when the kernel that runs it has the epilogue (the 16-bit-MFMA
 * implicit GEMM without a K split); otherwise the plain conv and *chunks = 0. */
int mragan_conv3d_presplit_bwd_stats(const float* x, int N, int Di, int Hi, int Wi, int cin, const float* wpacked,
                                     const void* wsplit, int cout, int k, int stride, int pad, float* y, int Do, int Ho,
                                     int Wo, int transposed, void* ws, size_t ws_bytes, const float* x_in,
                                     const float* mean, const float* rstd, int act, double* part, size_t part_bytes,
                                     int* chunks, void* stream);

/* Running-stat update for a table of IN layers (device array of mragan_running_entry), each
 * entry listing the per-instance statistics of the reference's sequential calls in call order. */
typedef struct mragan_running_seg { const float* mean; const float* rstd; int32_t count; int32_t _pad; } mragan_running_seg;
typedef struct mragan_running_entry {
  float* running_mean; float* running_var; const float* bias; int32_t C; int32_t nseg; int64_t S;
  mragan_running_seg seg[8];
} mragan_running_entry;
int mragan_instnorm_running_update(const void* table, int nentries, float momentum, void* stream);
size_t mragan_running_entry_size(void);

/* ---- replication pad (nn.ReplicationPad3d forward / backward) ---------------------------- */
int mragan_rpad(const float* x, int N, int D, int H, int W, int C, int pad, float* y, void* stream);
int mragan_rpad_fold(const float* ypad, int N, int D, int H, int W, int C, int pad, const float* add, float* x, void* stream);

/* ---- element-wise / losses ---------------------------------------------------------------- */
/* dx = (g0 + g1 + g2) · act'(y)   (ReLU/LeakyReLU from their output, Tanh, Sigmoid)         */
int mragan_act_bwd(const float* y, const float* g0, const float* g1, const float* g2, int64_t n, int act, float* dx,
                   void* stream);
/* UnetSkipConnectionBlock skip concatenation (networks3D.py:340-343, torch.cat([x, model(x)], 1)
 * followed by the parent's in-place ReLU, :318-320), NDHWC over M voxels:
 *   concat: out[m] = [act_a(a[m][0:Ca]) | act_b(b[m][0:Cb])]
 *   split (its backward): da[m] = g[m][0:Ca]·act_a'(ya[m]), db[m] = g[m][Ca:]·act_b'(yb[m])
 *   (derivatives from the activation outputs; null ya/yb = identity, null da/db = skipped). */
int mragan_channel_concat(const float* a, int Ca, int act_a, const float* b, int Cb, int act_b, int64_t M, float* out,
                          void* stream);
int mragan_channel_split(const float* g, int Ca, int Cb, int64_t M, const float* ya, int act_a, float* da,
                         const float* yb, int act_b, float* db, void* stream);
/* nn.L1Loss (cycle_gan_model.py:104-105): loss[0] (=|+=) scale·mean|a−b|; grad (=|+=) scale·sign(a−b)/n.
 * ws: ≥ 4096 bytes.                                                                            */
int mragan_l1_loss(const float* a, const float* b, int64_t n, float scale, float* loss, int loss_accumulate, float* grad,
                   int grad_accumulate, void* ws, void* stream);
/* GANLoss (networks3D.py:130-150) on D's output p: BCE (lsgan = 0, p = sigmoid output) or MSE.
 * loss[0] (=|+=) scale·loss; dp = d(scale·loss)/dp (the Sigmoid backward belongs to D's last
 * layer, see mragan_act_bwd).                                                                 */
int mragan_gan_loss(const float* p, int64_t n, float target, int lsgan, float scale, float* loss, int loss_accumulate,
                    float* dp, void* ws, void* stream);
/* bias gradient: out[c] (=|+=) Σ_m x[m][c]  (deterministic two-pass reduction) */
size_t mragan_channel_sum_workspace(int64_t M, int C);
int mragan_channel_sum(const float* x, int64_t M, int C, float* out, int accumulate, void* ws, size_t ws_bytes,
                       void* stream);
/* torch.optim.Adam step (amsgrad=False, weight_decay=0) on flat buffers (cycle_gan_model.py:107-110);
 * the gradient is multiplied by grad_scale first (1/world_size after a SUM all-reduce).      */
int mragan_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2, float eps,
                int step, float grad_scale, void* stream);
/* The same Adam step with its per-step scalars in device memory (CUDA-graph replay: the graph
 * holds the pointer, the host refreshes the six floats before each replay).  mragan_adam_hyper
 * (host only) writes {lr/bc1, beta1, beta2, eps, sqrt(bc2), grad_scale} for step `step` exactly
 * as mragan_adam derives them, so both entry points produce identical parameters.            */
int mragan_adam_hyper(float lr, float beta1, float beta2, float eps, int step, float grad_scale, float* out6);
int mragan_adam_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper, void* stream);
/* fp16 loss scaling without silent divergence (what torch.cuda.amp.GradScaler.step does for the
 * reference's Adam, cycle_gan_model.py:107-110): mragan_nonfinite_flag ORs 1 into the DEVICE int
 * *flag when g[0:n] holds an inf or NaN (call it on every flat gradient buffer of an optimizer);
 * mragan_adam_dev_checked is mragan_adam_dev that leaves p, m and v untouched when *flag != 0;
 * mragan_skip_count then adds (*flag != 0) to the DEVICE int *counter and clears *flag for the
 * next step.  All graph-replayable.  (ABI 10)                                                   */
int mragan_nonfinite_flag(const float* g, int64_t n, int* flag, void* stream);
int mragan_adam_dev_checked(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper, const int* flag,
                            void* stream);
int mragan_skip_count(int* flag, int* counter, void* stream);
/* The step count net of skipped updates (torch's GradScaler does not advance the optimizer on a
 * skipped step): writes into hyper[6] the mragan_adam_hyper scalars for step base[4] − *skipped,
 * base = {lr, beta1, beta2, eps, step, grad_scale} in DEVICE memory (host-refreshed before each
 * replay, like hyper), *skipped the DEVICE counter of mragan_skip_count.  Run it before the step's
 * mragan_adam_dev_checked calls.  (ABI 13)                                                        */
int mragan_adam_rebias(const float* base, const int* skipped, float* hyper, void* stream);
int mragan_fill(float* p, int64_t n, float value, void* stream);
/* ---- sliding-window inference (test.py:38-207 + TestModel, models/test_model.py) -------------
 * The normalised volume vol[X][Y][Z] (fp32, resident) is cut into the reference's patches and the
 * generator's predictions are overlap-averaged back, both on the device.  (ABI 7)
 *   gather:  out[p][a][b][c] = (vol[s_p + (a,b,c)] − 127.5) / 127.5   (test.py:150; numpy rounding)
 *            starts: DEVICE int32 array of n (x, y, z) corners (test.py:111-143 order);
 *   combine: pred[p][px][py][pz] for every patch p of the full grid, p = (i·jnum + j)·knum + k with
 *            inum = ⌈(X−px)/stride_inplane⌉ + 1 etc.; per voxel, label = Σ_p (pred·127.5 + 127.5)
 *            accumulated in fp32 in patch order from 0, divided by the cover count, + 0.01
 *            (test.py:160-173) — bit-identical to the host loop for the same predictions.     */
int mragan_patch_gather(const float* vol, int X, int Y, int Z, const int* starts, int n, int px, int py, int pz,
                        float* out, void* stream);
int mragan_patch_combine(const float* pred, int X, int Y, int Z, int px, int py, int pz, int stride_inplane,
                         int stride_layer, float* label, void* stream);

/* Training patch sampler (train.py:35-52, MONAI RandCropByPosNegLabeld crops, done on the device):
 * out[p][a][b][c] = vol[s_p + (a,b,c)] for n corners s_p (DEVICE int32 [n][3]); every corner must
 * keep the patch inside the volume (the sampler clamps the centers as MONAI does).  (ABI 7)      */
int mragan_crop_patches(const float* vol, int X, int Y, int Z, const int* starts, int n, int px, int py, int pz,
                        float* out, void* stream);

/* diagnostics: the kernel families launched by this thread since the last reset, ';'-joined
 * (e.g. "conv_wgrad3_x3;wgrad_reduce"); reset = 1 clears the log after copying it.  (ABI 7) */
const char* mragan_launch_log(int reset);

/* diagnostics: copy the per-block phase timestamps (s_memtime) the 1-channel bf16x3 convolution
 * records when MRAGAN_STAMPS is set; n ≤ 40960 values, 5 per block.  n < 0: the K-split brick's
 * (conv_brick_ks.hip) −n values, 8 per wave, 32 per block, ≤ 1024 blocks. */
int mragan_debug_stamps(unsigned long long* host, int n);

#ifdef __cplusplus
}
#endif
#endif /* MRAGAN_HIP_H_ */
