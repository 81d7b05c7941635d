// extern "C" entry points of libmragan_hip.so (declared in include/mragan_hip.h).
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "../../include/mragan_hip.h"
#include "kernels.h"

namespace mragan {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// launch log (diagnostics): the names passed to check_launch since the last reset, ';'-joined,
// so a caller can name the kernels one C-ABI call launched (bench.py's roofline label)
static thread_local char g_log[1024] = "";
static thread_local size_t g_log_len = 0;

int check_launch(const char* what) {
  const size_t n = strlen(what);
  if (g_log_len + n + 2 < sizeof(g_log)) {
    if (g_log_len) g_log[g_log_len++] = ';';
    memcpy(g_log + g_log_len, what, n);
    g_log_len += n;
    g_log[g_log_len] = 0;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return kLaunch;
  }
  return kOk;
}

// contraction precision of the MFMA convolutions (prec.h): f32, bf16x3, bf16 or fp16
static int g_conv_precision = MRAGAN_PREC_F32;
// loss scale applied to the gradients the loss kernels emit (fp16 mode; 1 otherwise)
static float g_loss_scale = 1.0f;

static bool thin_side(int kc, int ny) { return kc <= 4 || ny <= 4 || kc % 8 != 0; }

static int conv_common(const float* x, int N, int Di, int Hi, int Wi, int cin, const float* w, const float* bias, int cout,
                       int k, int stride, int pad, int act, float* y, int Do, int Ho, int Wo, int trans, void* ws,
                       size_t ws_bytes, void* stream, const void* wx3 = nullptr, double* in_part = nullptr,
                       int* in_chunks = nullptr) {
  // w may be null when the pre-split copy wx3 is given (a stale fp32 pack is not passed): only the
  // kernels that read wx3 alone accept that (conv_brick, the shell pass); the others refuse it
  MRAGAN_CHECK_ARG(x && (w || wx3) && y, "conv: null pointer");
  MRAGAN_CHECK_ARG(N >= 0 && Di > 0 && Hi > 0 && Wi > 0 && cin > 0 && cout > 0, "conv: bad input shape");
  MRAGAN_CHECK_ARG(Do > 0 && Ho > 0 && Wo > 0, "conv: bad output shape");
  MRAGAN_CHECK_ARG(k >= 1 && stride >= 1 && pad >= 0, "conv: bad k/stride/pad");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (thin_side(cin, cout)) {
    MRAGAN_CHECK_ARG(w, "conv: the thin convolutions need the fp32 weight pack");
    ThinArgs a{x, N, Di, Hi, Wi, cin, w, bias, y, Do, Ho, Wo, cout, k, stride, pad, trans, act, g_conv_precision};
    if (g_conv_precision != MRAGAN_PREC_F32 && thin1_x3_applicable(cin, cout, k, stride, g_conv_precision)) {
      a.in_part = in_part;
      a.in_chunks = in_chunks;
      return conv_thin1_x3(a, g_conv_precision, ws, ws_bytes, st);
    }
    if (g_conv_precision != MRAGAN_PREC_F32 && thinn_x3_applicable(cin, cout, k, stride, g_conv_precision))
      return conv_thinn_x3(a, g_conv_precision, ws, ws_bytes, st);
    return conv_thin(a, st);
  }
  IgemmArgs a{x, w, bias, y, N, Di, Hi, Wi, cin, Do, Ho, Wo, cout, k, stride, pad, trans, act, 1,
              g_conv_precision, static_cast<float*>(ws), ws_bytes, wx3, in_part, in_chunks};
  return conv_igemm(a, st);
}

static bool thin_wgrad_side(int Cd, int Cg) { return Cd < 8 || Cg < 8; }

}  // namespace mragan

using namespace mragan;

extern "C" {

int mragan_abi_version(void) { return MRAGAN_ABI_VERSION; }
const char* mragan_last_error(void) { return g_err; }

int mragan_set_conv_precision(int mode) {
  MRAGAN_CHECK_ARG(mode >= MRAGAN_PREC_F32 && mode <= MRAGAN_PREC_F16, "set_conv_precision: unknown mode %d", mode);
  g_conv_precision = mode;
  return kOk;
}
int mragan_get_conv_precision(void) { return g_conv_precision; }

int mragan_set_loss_scale(float s) {
  MRAGAN_CHECK_ARG(s > 0.f && s < 1e30f, "set_loss_scale: bad scale");
  g_loss_scale = s;
  return kOk;
}
float mragan_get_loss_scale(void) { return g_loss_scale; }

int mragan_conv3d_fwd(const float* x, int N, int Di, int Hi, int Wi, int cin, const float* w, const float* bias, int cout,
                      int k, int stride, int pad, int act, float* y, int Do, int Ho, int Wo, void* ws, size_t ws_bytes,
                      void* stream) {
  return conv_common(x, N, Di, Hi, Wi, cin, w, bias, cout, k, stride, pad, act, y, Do, Ho, Wo, 0, ws, ws_bytes, stream);
}

int mragan_conv3d_transposed(const float* x, int N, int Di, int Hi, int Wi, int cin, const float* w, const float* bias,
                             int cout, int k, int stride, int pad, int act, float* y, int Do, int Ho, int Wo, void* ws,
                             size_t ws_bytes, void* stream) {
  return conv_common(x, N, Di, Hi, Wi, cin, w, bias, cout, k, stride, pad, act, y, Do, Ho, Wo, 1, ws, ws_bytes, stream);
}

int mragan_conv3d_presplit(const float* x, int N, int Di, int Hi, int Wi, int cin, const float* w, const void* wsplit,
                           const float* bias, int cout, int k, int stride, int pad, int act, float* y, int Do, int Ho,
                           int Wo, int transposed, void* ws, size_t ws_bytes, void* stream) {
  MRAGAN_CHECK_ARG(transposed == 0 || transposed == 1, "conv3d_presplit: transposed must be 0/1");
  return conv_common(x, N, Di, Hi, Wi, cin, w, bias, cout, k, stride, pad, act, y, Do, Ho, Wo, transposed, ws, ws_bytes,
                     stream, wsplit);
}

int mragan_conv3d_presplit_in_stats(const float* x, int N, int Di, int Hi, int Wi, int cin, const float* w,
                                    const void* wsplit, const float* bias, int cout, int k, int stride, int pad, int act,
                                    float* y, int Do, int Ho, int Wo, int transposed, void* ws, size_t ws_bytes,
                                    double* part, size_t part_bytes, int* chunks, void* stream) {
  MRAGAN_CHECK_ARG(transposed == 0 || transposed == 1, "conv3d_presplit_in_stats: transposed must be 0/1");
  MRAGAN_CHECK_ARG(part && chunks, "conv3d_presplit_in_stats: null partials");
  // every brick shape has bd ≥ 1, bh ≥ 4, bw ≥ 6 (conv_brick.hip choose_brick)
  const size_t bound = (size_t)N * Do * ceil_div(Ho, 4) * ceil_div(Wo, 6) * cout * 2 * sizeof(double);
  MRAGAN_CHECK_ARG(part_bytes >= bound, "conv3d_presplit_in_stats: partials %zu < %zu bytes", part_bytes, bound);
  *chunks = 0;
  return conv_common(x, N, Di, Hi, Wi, cin, w, bias, cout, k, stride, pad, act, y, Do, Ho, Wo, transposed, ws, ws_bytes,
                     stream, wsplit, part, chunks);
}

int mragan_instnorm_fwd_partials(const float* x, int N, int D, int H, int W, int C, float* y, int ypad, int act,
                                 const float* resid, int rpad, float* mean, float* rstd, const double* part, int chunks,
                                 void* stream) {
  MRAGAN_CHECK_ARG(x && y && mean && rstd && part, "instnorm_fwd_partials: null pointer");
  return instnorm_fwd_partials(x, InShape{N, D, H, W, C}, y, ypad, act, resid, rpad, mean, rstd, part, chunks,
                               static_cast<hipStream_t>(stream));
}

static int op16_mode_ok() {
  MRAGAN_CHECK_ARG(g_conv_precision == MRAGAN_PREC_BF16 || g_conv_precision == MRAGAN_PREC_F16,
                   "16-bit operand planes need the bf16 or fp16 precision mode (current: %d)", g_conv_precision);
  return kOk;
}

static int conv3d_op16_impl(const void* x16, int N, int Di, int Hi, int Wi, int cin, const float* w, const void* wsplit,
                            int cout, int k, int stride, int pad, float* y, int Do, int Ho, int Wo, int transposed,
                            void* ws, size_t ws_bytes, double* part, size_t part_bytes, int* chunks, unsigned* tickets,
                            float* mean, float* rstd, int* finalized, void* stream);

int mragan_conv3d_op16(const void* x16, int N, int Di, int Hi, int Wi, int cin, const float* w, const void* wsplit, int cout,
                       int k, int stride, int pad, float* y, int Do, int Ho, int Wo, int transposed, void* ws,
                       size_t ws_bytes, double* part, size_t part_bytes, int* chunks, void* stream) {
  return conv3d_op16_impl(x16, N, Di, Hi, Wi, cin, w, wsplit, cout, k, stride, pad, y, Do, Ho, Wo, transposed, ws,
                          ws_bytes, part, part_bytes, chunks, nullptr, nullptr, nullptr, nullptr, stream);
}

int mragan_conv3d_op16_fin(const void* x16, int N, int Di, int Hi, int Wi, int cin, const float* w, const void* wsplit,
                           int cout, int k, int stride, int pad, float* y, int Do, int Ho, int Wo, int transposed,
                           void* ws, size_t ws_bytes, double* part, size_t part_bytes, int* chunks, unsigned* tickets,
                           float* mean, float* rstd, int* finalized, void* stream) {
  MRAGAN_CHECK_ARG(part && chunks && tickets && mean && rstd && finalized, "conv3d_op16_fin: null pointer");
  return conv3d_op16_impl(x16, N, Di, Hi, Wi, cin, w, wsplit, cout, k, stride, pad, y, Do, Ho, Wo, transposed, ws,
                          ws_bytes, part, part_bytes, chunks, tickets, mean, rstd, finalized, stream);
}

static int conv3d_op16_impl(const void* x16, int N, int Di, int Hi, int Wi, int cin, const float* w, const void* wsplit,
                            int cout, int k, int stride, int pad, float* y, int Do, int Ho, int Wo, int transposed,
                            void* ws, size_t ws_bytes, double* part, size_t part_bytes, int* chunks, unsigned* tickets,
                            float* mean, float* rstd, int* finalized, void* stream) {
  if (int rc = op16_mode_ok()) return rc;
  if (finalized) *finalized = 0;
  // wsplit: optional (the brick packs per call); w: optional when wsplit is given (conv_common)
  MRAGAN_CHECK_ARG(x16 && (w || wsplit) && y, "conv3d_op16: null pointer");
  MRAGAN_CHECK_ARG(transposed == 0 || transposed == 1, "conv3d_op16: transposed must be 0/1");
  MRAGAN_CHECK_ARG(N >= 0 && Di > 0 && Hi > 0 && Wi > 0 && cin > 0 && cout > 0 && Do > 0 && Ho > 0 && Wo > 0,
                   "conv3d_op16: bad shape");
  MRAGAN_CHECK_ARG(!thin_side(cin, cout), "conv3d_op16: channel counts %d -> %d are not a brick convolution", cin, cout);
  if (part) {
    MRAGAN_CHECK_ARG(chunks, "conv3d_op16: null chunks");
    const size_t bound = (size_t)N * Do * ceil_div(Ho, 4) * ceil_div(Wo, 6) * cout * 2 * sizeof(double);
    MRAGAN_CHECK_ARG(part_bytes >= bound, "conv3d_op16: partials %zu < %zu bytes", part_bytes, bound);
    *chunks = 0;
  }
  IgemmArgs a{static_cast<const float*>(x16), w, nullptr, y, N, Di, Hi, Wi, cin, Do, Ho, Wo, cout, k, stride, pad,
              transposed, kActNone, 1, g_conv_precision, static_cast<float*>(ws), ws_bytes, wsplit, part, chunks};
  a.x16 = 1;
  if (part && tickets) { a.in_tick = tickets; a.in_fin0 = mean; a.in_fin1 = rstd; a.in_finalized = finalized; }
  return conv_igemm(a, static_cast<hipStream_t>(stream));
}

static int op16_dgrad_in_stats_impl(const void* dy16, int N, int Di, int Hi, int Wi, int cin, const float* w,
                                    const void* wsplit, int cout, float* y, void* ws, size_t ws_bytes, const float* x_in,
                                    const float* mean, const float* rstd, int act, double* part, size_t part_bytes,
                                    int* chunks, unsigned* tickets, float* coef, int* finalized, void* stream,
                                    const float* x_add = nullptr);

int mragan_conv3d_op16_dgrad_in_stats(const void* dy16, int N, int Di, int Hi, int Wi, int cin, const float* w,
                                      const void* wsplit, int cout, float* y, void* ws, size_t ws_bytes, const float* x_in,
                                      const float* mean, const float* rstd, int act, double* part, size_t part_bytes,
                                      int* chunks, void* stream) {
  return op16_dgrad_in_stats_impl(dy16, N, Di, Hi, Wi, cin, w, wsplit, cout, y, ws, ws_bytes, x_in, mean, rstd, act,
                                  part, part_bytes, chunks, nullptr, nullptr, nullptr, stream);
}

int mragan_conv3d_op16_dgrad_in_stats_fin(const void* dy16, int N, int Di, int Hi, int Wi, int cin, const float* w,
                                          const void* wsplit, int cout, float* y, void* ws, size_t ws_bytes,
                                          const float* x_in, const float* mean, const float* rstd, int act, double* part,
                                          size_t part_bytes, int* chunks, unsigned* tickets, float* coef, int* finalized,
                                          void* stream) {
  MRAGAN_CHECK_ARG(tickets && coef && finalized, "conv3d_op16_dgrad_in_stats_fin: null pointer");
  return op16_dgrad_in_stats_impl(dy16, N, Di, Hi, Wi, cin, w, wsplit, cout, y, ws, ws_bytes, x_in, mean, rstd, act,
                                  part, part_bytes, chunks, tickets, coef, finalized, stream);
}

int mragan_conv3d_op16_dgrad_in_stats_add(const void* dy16, int N, int Di, int Hi, int Wi, int cin, const float* w,
                                          const void* wsplit, int cout, float* y, void* ws, size_t ws_bytes,
                                          const float* x_in, const float* mean, const float* rstd, int act,
                                          const float* x_add, double* part, size_t part_bytes, int* chunks,
                                          unsigned* tickets, float* coef, int* finalized, void* stream) {
  MRAGAN_CHECK_ARG(x_add, "conv3d_op16_dgrad_in_stats_add: null x_add");
  MRAGAN_CHECK_ARG(!tickets || (coef && finalized), "conv3d_op16_dgrad_in_stats_add: tickets need coef and finalized");
  return op16_dgrad_in_stats_impl(dy16, N, Di, Hi, Wi, cin, w, wsplit, cout, y, ws, ws_bytes, x_in, mean, rstd, act,
                                  part, part_bytes, chunks, tickets, coef, finalized, stream, x_add);
}

static int op16_dgrad_in_stats_impl(const void* dy16, int N, int Di, int Hi, int Wi, int cin, const float* w,
                                    const void* wsplit, int cout, float* y, void* ws, size_t ws_bytes, const float* x_in,
                                    const float* mean, const float* rstd, int act, double* part, size_t part_bytes,
                                    int* chunks, unsigned* tickets, float* coef, int* finalized, void* stream,
                                    const float* x_add) {
  if (int rc = op16_mode_ok()) return rc;
  if (finalized) *finalized = 0;
  MRAGAN_CHECK_ARG(dy16 && wsplit && y && x_in && mean && rstd && part && chunks,     // w: optional (conv_common)
                   "conv3d_op16_dgrad_in_stats: null pointer");
  MRAGAN_CHECK_ARG(N >= 0 && Di > 0 && Hi > 0 && Wi > 0 && cin > 0 && cout > 0 && !thin_side(cin, cout),
                   "conv3d_op16_dgrad_in_stats: bad shape");
  MRAGAN_CHECK_ARG(act == kActNone || act == kActRelu || act == kActLrelu, "conv3d_op16_dgrad_in_stats: act %d", act);
  const int Do = Di + 2, Ho = Hi + 2, Wo = Wi + 2;
  const size_t bound = (size_t)N * Do * ceil_div(Ho, 4) * ceil_div(Wo, 6) * cout * 2 * sizeof(double);
  MRAGAN_CHECK_ARG(part_bytes >= bound, "conv3d_op16_dgrad_in_stats: partials %zu < %zu bytes", part_bytes, bound);
  *chunks = 0;
  IgemmArgs a{static_cast<const float*>(dy16), w, nullptr, y, N, Di, Hi, Wi, cin, Do, Ho, Wo, cout, 3, 1, 0, 1, kActNone,
              1, g_conv_precision, static_cast<float*>(ws), ws_bytes, wsplit, part, chunks};
  a.x16 = 1;
  a.bs_x = x_in; a.bs_mean = mean; a.bs_rstd = rstd; a.bs_act = act; a.bs_add = x_add;
  if (tickets) { a.in_tick = tickets; a.in_fin0 = coef; a.in_fin1 = nullptr; a.in_finalized = finalized; }
  return conv_igemm(a, static_cast<hipStream_t>(stream));
}

int mragan_conv3d_dgrad_split(int N, int Di, int Hi, int Wi, int cin, int cout) {
  // the whole-grid data gradient of a k3 s1 p0 conv from the plane of dY ([N][Di][Hi][Wi][cin]) to
  // the padded grid of cout channels, as mragan_conv3d_op16(transposed = 1) dispatches it (ABI 19)
  if (N <= 0 || Di <= 0 || Hi <= 0 || Wi <= 0 || cin <= 0 || cout <= 0) return 0;
  if (g_conv_precision != MRAGAN_PREC_BF16 && g_conv_precision != MRAGAN_PREC_F16) return 0;
  IgemmArgs a{nullptr, nullptr, nullptr, nullptr, N, Di, Hi, Wi, cin, Di + 2, Hi + 2, Wi + 2, cout, 3, 1, 0, 1,
              kActNone, 1, g_conv_precision, nullptr, 0, nullptr, nullptr, nullptr};
  a.x16 = 1;
  return full_dgrad_split_applicable(a) ? 1 : 0;
}

int mragan_conv3d_thin_op16(const void* x16, int N, int Di, int Hi, int Wi, int cin, const float* w, const float* bias,
                            int cout, int k, int stride, int pad, int act, float* y, int Do, int Ho, int Wo, int transposed,
                            void* ws, size_t ws_bytes, void* stream) {
  if (int rc = op16_mode_ok()) return rc;
  MRAGAN_CHECK_ARG(x16 && w && y, "conv3d_thin_op16: null pointer");
  MRAGAN_CHECK_ARG(transposed == 0 || transposed == 1, "conv3d_thin_op16: transposed must be 0/1");
  MRAGAN_CHECK_ARG(N >= 0 && Di > 0 && Hi > 0 && Wi > 0 && Do > 0 && Ho > 0 && Wo > 0 && pad >= 0,
                   "conv3d_thin_op16: bad shape");
  MRAGAN_CHECK_ARG(thinn_x3_applicable(cin, cout, k, stride, g_conv_precision),
                   "conv3d_thin_op16: only the 32 -> 1|2-channel k7 s1 convolutions (got %d -> %d, k%d s%d)", cin,
                   cout, k, stride);
  ThinArgs a{static_cast<const float*>(x16), N, Di, Hi, Wi, cin, w, bias, y, Do, Ho, Wo, cout, k, stride, pad,
             transposed, act, g_conv_precision};
  a.x16 = 1;
  return conv_thinn_x3(a, g_conv_precision, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

int mragan_conv3d_wgrad_thin_op16(const void* dense, int N, int Dd, int Hd, int Wd, int Cd, const void* gathered, int Dg,
                                  int Hg, int Wg, int Cg, int k, int stride, int pad, float* dw, int accumulate, void* ws,
                                  size_t ws_bytes, void* stream) {
  if (int rc = op16_mode_ok()) return rc;
  MRAGAN_CHECK_ARG(dense && gathered && dw && ws, "wgrad_thin_op16: null pointer");
  MRAGAN_CHECK_ARG(thin1_wgrad_x3_applicable(Cd, Cg, k, stride, g_conv_precision) && pad >= 0,
                   "wgrad_thin_op16: only the k7 s1 layers between nc and 32 channels (got %d, %d, k%d s%d)", Cd, Cg, k,
                   stride);
  return conv_thin1_wgrad_x3(static_cast<const float*>(dense), N, Dd, Hd, Wd, Cd, static_cast<const float*>(gathered), Dg,
                             Hg, Wg, Cg, pad, dw, accumulate, g_conv_precision, ws, ws_bytes,
                             static_cast<hipStream_t>(stream), 1);
}

int mragan_instnorm_apply_op16(const float* x, int N, int D, int H, int W, int C, float* y, void* y16, int ypad, int act,
                               const float* resid, int rpad, const float* mean, const float* rstd, void* stream) {
  if (int rc = op16_mode_ok()) return rc;
  MRAGAN_CHECK_ARG(x && (y || y16) && mean && rstd, "instnorm_apply_op16: null pointer");
  return instnorm_apply(x, InShape{N, D, H, W, C}, y, ypad, act, resid, rpad, mean, rstd,
                        static_cast<hipStream_t>(stream), y16, g_conv_precision);
}

int mragan_instnorm_bwd_apply_op16(const float* x, const float* mean, const float* rstd, int N, int D, int H, int W,
                                   int C, const float* dy, int dypad, const float* dy_add, int act, void* dx16,
                                   float* g_out, const float* coef, void* stream) {
  if (int rc = op16_mode_ok()) return rc;
  MRAGAN_CHECK_ARG(x && mean && rstd && dy && dx16 && coef, "instnorm_bwd_apply_op16: null pointer");
  MRAGAN_CHECK_ARG(!g_out || (g_out != dy && g_out != dy_add), "instnorm_bwd_apply_op16: g_out aliases an operand");
  InBwdArgs a{x, mean, rstd, dy, dypad, dy_add, act, nullptr, g_out, dx16, g_conv_precision};
  return instnorm_bwd_apply(a, InShape{N, D, H, W, C}, coef, static_cast<hipStream_t>(stream));
}

int mragan_instnorm_bwd_partials_op16(const float* x, const float* mean, const float* rstd, int N, int D, int H, int W,
                                      int C, const float* dy, int dypad, const float* dy_add, int act, void* dx16,
                                      float* g_out, const double* part, int chunks, void* ws, size_t ws_bytes,
                                      void* stream) {
  if (int rc = op16_mode_ok()) return rc;
  MRAGAN_CHECK_ARG(x && mean && rstd && dy && dx16 && part && ws, "instnorm_bwd_partials_op16: null pointer");
  MRAGAN_CHECK_ARG(!g_out || (g_out != dy && g_out != dy_add), "instnorm_bwd_partials_op16: g_out aliases an operand");
  InBwdArgs a{x, mean, rstd, dy, dypad, dy_add, act, nullptr, g_out, dx16, g_conv_precision};
  return instnorm_bwd_partials(a, InShape{N, D, H, W, C}, part, chunks, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

int mragan_conv3d_dgrad_in_stats(const float* dy, int N, int Di, int Hi, int Wi, int cin, const float* w, int cout, int k,
                                 float* y, void* ws, size_t ws_bytes, const float* x_in, const float* mean,
                                 const float* rstd, int act, int fold_pad, double* part, size_t part_bytes, int* chunks,
                                 void* stream) {
  MRAGAN_CHECK_ARG(dy && w && y && x_in && mean && rstd && part && chunks, "conv3d_dgrad_in_stats: null pointer");
  MRAGAN_CHECK_ARG(N >= 0 && Di > 0 && Hi > 0 && Wi > 0 && cin > 0 && cout > 0 && k >= 1, "conv3d_dgrad_in_stats: bad shape");
  MRAGAN_CHECK_ARG(act == kActNone || act == kActRelu || act == kActLrelu, "conv3d_dgrad_in_stats: act %d", act);
  const int Do = Di + k - 1, Ho = Hi + k - 1, Wo = Wi + k - 1;
  MRAGAN_CHECK_ARG(fold_pad >= 0 && Do > 2 * fold_pad && Ho > 2 * fold_pad && Wo > 2 * fold_pad,
                   "conv3d_dgrad_in_stats: fold %d does not fit the %d×%d×%d gradient", fold_pad, Do, Ho, Wo);
  const size_t bound = (size_t)N * Do * ceil_div(Ho, 4) * ceil_div(Wo, 6) * cout * 2 * sizeof(double);
  MRAGAN_CHECK_ARG(part_bytes >= bound, "conv3d_dgrad_in_stats: partials %zu < %zu bytes", part_bytes, bound);
  *chunks = 0;
  if (g_conv_precision != MRAGAN_PREC_F32 && thin_side(cin, cout) && thin1_x3_applicable(cin, cout, k, 1, g_conv_precision)) {
    ThinArgs a{dy, N, Di, Hi, Wi, cin, w, nullptr, y, Do, Ho, Wo, cout, k, 1, 0, 1, kActNone, g_conv_precision};
    a.in_part = part; a.in_chunks = chunks;
    a.bs_x = x_in; a.bs_mean = mean; a.bs_rstd = rstd; a.bs_act = act; a.bs_fold = fold_pad;
    return conv_thin1_x3(a, g_conv_precision, ws, ws_bytes, static_cast<hipStream_t>(stream));
  }
  // no kernel with the statistics epilogue for this shape / mode: the plain data gradient, chunks = 0
  return conv_common(dy, N, Di, Hi, Wi, cin, w, nullptr, cout, k, 1, 0, kActNone, y, Do, Ho, Wo, 1, ws, ws_bytes, stream);
}

int mragan_conv3d_presplit_bwd_stats(const float* x, int N, int Di, int Hi, int Wi, int cin, const float* w,
                                     const void* wsplit, int cout, int k, int stride, int pad, float* y, int Do, int Ho,
                                     int Wo, int transposed, void* ws, size_t ws_bytes, const float* x_in,
                                     const float* mean, const float* rstd, int act, double* part, size_t part_bytes,
                                     int* chunks, void* stream) {
  MRAGAN_CHECK_ARG(x && w && y && x_in && mean && rstd && part && chunks, "conv3d_presplit_bwd_stats: null pointer");
  MRAGAN_CHECK_ARG(transposed == 0 || transposed == 1, "conv3d_presplit_bwd_stats: transposed must be 0/1");
  MRAGAN_CHECK_ARG(act == kActNone || act == kActRelu || act == kActLrelu, "conv3d_presplit_bwd_stats: act %d", act);
  // the shape checks conv_common makes, before the partials bound is computed from these ints
  MRAGAN_CHECK_ARG(N >= 0 && Di > 0 && Hi > 0 && Wi > 0 && cin > 0 && cout > 0, "conv3d_presplit_bwd_stats: bad input shape");
  MRAGAN_CHECK_ARG(Do > 0 && Ho > 0 && Wo > 0, "conv3d_presplit_bwd_stats: bad output shape");
  MRAGAN_CHECK_ARG(k >= 1 && stride >= 1 && pad >= 0, "conv3d_presplit_bwd_stats: bad k/stride/pad");
  const size_t bound = (size_t)N * Do * ceil_div(Ho, 4) * ceil_div(Wo, 6) * cout * 2 * sizeof(double);
  MRAGAN_CHECK_ARG(part_bytes >= bound, "conv3d_presplit_bwd_stats: partials %zu < %zu bytes", part_bytes, bound);
  *chunks = 0;
  // the epilogue exists in the 16-bit-MFMA implicit GEMM (stride-2 layers); elsewhere the plain conv
  if (stride < 2 || g_conv_precision == MRAGAN_PREC_F32)
    return conv_common(x, N, Di, Hi, Wi, cin, w, nullptr, cout, k, stride, pad, kActNone, y, Do, Ho, Wo, transposed, ws,
                       ws_bytes, stream, wsplit);
  if (thin_side(cin, cout))
    return conv_common(x, N, Di, Hi, Wi, cin, w, nullptr, cout, k, stride, pad, kActNone, y, Do, Ho, Wo, transposed, ws,
                       ws_bytes, stream, wsplit);
  IgemmArgs a{x, w, nullptr, y, N, Di, Hi, Wi, cin, Do, Ho, Wo, cout, k, stride, pad, transposed, kActNone, 1,
              g_conv_precision, static_cast<float*>(ws), ws_bytes, wsplit, part, chunks};
  a.bs_x = x_in; a.bs_mean = mean; a.bs_rstd = rstd; a.bs_act = act;
  return conv_igemm(a, static_cast<hipStream_t>(stream));
}

int mragan_conv3d_op16_bwd_stats(const void* x16, int N, int Di, int Hi, int Wi, int cin, const float* w, int cout,
                                  int k, int stride, int pad, float* y, int Do, int Ho, int Wo, int transposed, void* ws,
                                  size_t ws_bytes, const float* x_in, const float* mean, const float* rstd, int act,
                                  double* part, size_t part_bytes, int* chunks, void* stream) {
  if (int rc = op16_mode_ok()) return rc;
  MRAGAN_CHECK_ARG(x16 && w && y && x_in && mean && rstd && part && chunks, "conv3d_op16_bwd_stats: null pointer");
  MRAGAN_CHECK_ARG(transposed == 0 || transposed == 1, "conv3d_op16_bwd_stats: transposed must be 0/1");
  MRAGAN_CHECK_ARG(act == kActNone || act == kActRelu || act == kActLrelu, "conv3d_op16_bwd_stats: act %d", act);
  MRAGAN_CHECK_ARG(N >= 0 && Di > 0 && Hi > 0 && Wi > 0 && cin > 0 && cout > 0, "conv3d_op16_bwd_stats: bad input shape");
  MRAGAN_CHECK_ARG(Do > 0 && Ho > 0 && Wo > 0, "conv3d_op16_bwd_stats: bad output shape");
  MRAGAN_CHECK_ARG(k >= 1 && stride >= 2 && pad >= 0 && !thin_side(cin, cout) && cin % 32 == 0,
                   "conv3d_op16_bwd_stats: the stride-2 implicit GEMM (a multiple of 32 input channels) only");
  const size_t bound = (size_t)N * Do * ceil_div(Ho, 4) * ceil_div(Wo, 6) * cout * 2 * sizeof(double);
  MRAGAN_CHECK_ARG(part_bytes >= bound, "conv3d_op16_bwd_stats: partials %zu < %zu bytes", part_bytes, bound);
  *chunks = 0;
  IgemmArgs a{static_cast<const float*>(x16), w, nullptr, y, N, Di, Hi, Wi, cin, Do, Ho, Wo, cout, k, stride, pad,
              transposed, kActNone, 1, g_conv_precision, static_cast<float*>(ws), ws_bytes, nullptr, part, chunks};
  a.x16 = 1;
  a.bs_x = x_in; a.bs_mean = mean; a.bs_rstd = rstd; a.bs_act = act;
  return conv_igemm(a, static_cast<hipStream_t>(stream));
}

int mragan_instnorm_bwd_partials(const float* x, const float* mean, const float* rstd, int N, int D, int H, int W, int C,
                                 const float* dy, int dypad, const float* dy_add, int act, float* dx, float* g_out,
                                 const double* part, int chunks, void* ws, size_t ws_bytes, void* stream) {
  MRAGAN_CHECK_ARG(x && mean && rstd && dy && dx && part && ws, "instnorm_bwd_partials: null pointer");
  MRAGAN_CHECK_ARG(!g_out || (g_out != dy && g_out != dy_add), "instnorm_bwd_partials: g_out aliases an operand");
  InBwdArgs a{x, mean, rstd, dy, dypad, dy_add, act, dx, g_out, nullptr, 0};
  return instnorm_bwd_partials(a, InShape{N, D, H, W, C}, part, chunks, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

int mragan_conv3d_wgrad_op16(const void* dense16, int N, int Dd, int Hd, int Wd, int Cd, const void* gathered16, int Dg,
                             int Hg, int Wg, int Cg, int k, int stride, int pad, float* dw, int accumulate, void* ws,
                             size_t ws_bytes, void* stream) {
  if (int rc = op16_mode_ok()) return rc;
  MRAGAN_CHECK_ARG(dense16 && gathered16 && dw && ws, "wgrad_op16: null pointer");
  MRAGAN_CHECK_ARG(!thin_wgrad_side(Cd, Cg) && k >= 1 && stride >= 1 && pad >= 0, "wgrad_op16: bad args");
  WgradArgs a{static_cast<const float*>(dense16), N, Dd, Hd, Wd, Cd, static_cast<const float*>(gathered16), Dg, Hg, Wg,
              Cg, k, stride, pad, static_cast<float*>(ws), 0, 0, g_conv_precision, 1};
  return conv_wgrad(a, dw, accumulate, ws_bytes, static_cast<hipStream_t>(stream));
}

int mragan_conv3d_wgrad_op16_pair(const void* dense16_a, int Na, const void* gathered16_a, const void* dense16_b, int Nb,
                                  const void* gathered16_b, int Dd, int Hd, int Wd, int Cd, int Dg, int Hg, int Wg, int Cg,
                                  int k, int stride, int pad, float* dw, int accumulate, void* ws, size_t ws_bytes,
                                  void* stream) {
  if (int rc = op16_mode_ok()) return rc;
  MRAGAN_CHECK_ARG(dense16_a && gathered16_a && dw && ws, "wgrad_op16_pair: null pointer");
  MRAGAN_CHECK_ARG(Na >= 0 && Nb >= 0 && (Nb == 0 || (dense16_b && gathered16_b)), "wgrad_op16_pair: bad second set");
  MRAGAN_CHECK_ARG(!thin_wgrad_side(Cd, Cg) && k >= 1 && stride >= 1 && pad >= 0, "wgrad_op16_pair: bad args");
  WgradArgs a{static_cast<const float*>(dense16_a), Na, Dd, Hd, Wd, Cd, static_cast<const float*>(gathered16_a), Dg, Hg,
              Wg, Cg, k, stride, pad, static_cast<float*>(ws), 0, 0, g_conv_precision, 1};
  if (Nb > 0) {
    a.D2 = static_cast<const float*>(dense16_b); a.G2 = static_cast<const float*>(gathered16_b); a.N2 = Nb;
  }
  return conv_wgrad(a, dw, accumulate, ws_bytes, static_cast<hipStream_t>(stream));
}

int mragan_conv3d_wgrad_g16(const float* dense, int N, int Dd, int Hd, int Wd, int Cd, const void* gathered16, int Dg,
                            int Hg, int Wg, int Cg, int k, int stride, int pad, float* dw, int accumulate, void* ws,
                            size_t ws_bytes, void* stream) {
  if (int rc = op16_mode_ok()) return rc;
  MRAGAN_CHECK_ARG(dense && gathered16 && dw && ws, "wgrad_g16: null pointer");
  MRAGAN_CHECK_ARG(!thin_wgrad_side(Cd, Cg) && k == 3 && stride == 2 && pad == 1, "wgrad_g16: the k3 s2 p1 weight "
                   "gradients only");
  WgradArgs a{dense, N, Dd, Hd, Wd, Cd, static_cast<const float*>(gathered16), Dg, Hg, Wg, Cg, k, stride, pad,
              static_cast<float*>(ws), 0, 0, g_conv_precision, 0};
  a.in16g = 1;
  return conv_wgrad(a, dw, accumulate, ws_bytes, static_cast<hipStream_t>(stream));
}

int mragan_instnorm_fwd_op16(const float* x, int N, int D, int H, int W, int C, float* y, void* y16, int ypad, int act,
                             const float* resid, int rpad, float* mean, float* rstd, void* ws, size_t ws_bytes,
                             void* stream) {
  if (int rc = op16_mode_ok()) return rc;
  MRAGAN_CHECK_ARG(x && (y || y16) && mean && rstd && ws, "instnorm_fwd_op16: null pointer");
  return instnorm_fwd(x, InShape{N, D, H, W, C}, y, ypad, act, resid, rpad, mean, rstd, ws, ws_bytes,
                      static_cast<hipStream_t>(stream), y16, g_conv_precision);
}

int mragan_instnorm_fwd_partials_op16(const float* x, int N, int D, int H, int W, int C, float* y, void* y16, int ypad,
                                      int act, const float* resid, int rpad, float* mean, float* rstd,
                                      const double* part, int chunks, void* stream) {
  if (int rc = op16_mode_ok()) return rc;
  MRAGAN_CHECK_ARG(x && (y || y16) && mean && rstd && part, "instnorm_fwd_partials_op16: null pointer");
  return instnorm_fwd_partials(x, InShape{N, D, H, W, C}, y, ypad, act, resid, rpad, mean, rstd, part, chunks,
                               static_cast<hipStream_t>(stream), y16, g_conv_precision);
}

int mragan_instnorm_bwd_op16(const float* x, const float* mean, const float* rstd, int N, int D, int H, int W, int C,
                             const float* dy, int dypad, const float* dy_add, int act, void* dx16, float* g_out, void* ws,
                             size_t ws_bytes, void* stream) {
  if (int rc = op16_mode_ok()) return rc;
  MRAGAN_CHECK_ARG(x && mean && rstd && dy && dx16 && ws, "instnorm_bwd_op16: null pointer");
  MRAGAN_CHECK_ARG(!g_out || (g_out != dy && g_out != dy_add), "instnorm_bwd_op16: g_out aliases an operand");
  InBwdArgs a{x, mean, rstd, dy, dypad, dy_add, act, nullptr, g_out, dx16, g_conv_precision};
  return instnorm_bwd(a, InShape{N, D, H, W, C}, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

size_t mragan_conv3d_workspace(int N, int Di, int Hi, int Wi, int cin, int cout, int k, int stride, int pad, int Do,
                               int Ho, int Wo, int transposed) {
  if (thin_side(cin, cout)) {
    if (g_conv_precision == MRAGAN_PREC_F32) return 0;
    if (thin1_x3_applicable(cin, cout, k, stride, g_conv_precision)) return thin1_x3_ws_bytes(cout);
    if (thinn_x3_applicable(cin, cout, k, stride, g_conv_precision)) return thinn_x3_ws_bytes(cout);
    return 0;
  }
  IgemmArgs a{nullptr, nullptr, nullptr, nullptr, N, Di, Hi, Wi, cin, Do, Ho, Wo, cout, k, stride, pad, transposed, 0, 1,
              g_conv_precision, nullptr, 0};
  return conv_igemm_ws_bytes(a);
}

size_t mragan_conv3d_wgrad_workspace(int N, int Dd, int Hd, int Wd, int Cd, int Cg, int k, int stride) {
  if (thin_wgrad_side(Cd, Cg)) {
    if (g_conv_precision != MRAGAN_PREC_F32 && thin1_wgrad_x3_applicable(Cd, Cg, k, stride, g_conv_precision))
      return thin1_wgrad_x3_ws_bytes();
    return conv_thin_wgrad_ws_bytes(N, Dd, Hd, Wd, Cd, Cg, k, stride);
  }
  return conv_wgrad_ws_bytes(N, Dd, Hd, Wd, Cd, Cg, k);
}

int mragan_conv3d_wgrad(const float* dense, int N, int Dd, int Hd, int Wd, int Cd, const float* gathered, int Dg, int Hg,
                        int Wg, int Cg, int k, int stride, int pad, float* dw, int accumulate, void* ws, size_t ws_bytes,
                        void* stream) {
  MRAGAN_CHECK_ARG(dense && gathered && dw && ws, "wgrad: null pointer");
  MRAGAN_CHECK_ARG(Cd > 0 && Cg > 0 && k >= 1 && stride >= 1 && pad >= 0, "wgrad: bad args");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (thin_wgrad_side(Cd, Cg) && g_conv_precision != MRAGAN_PREC_F32 && thin1_wgrad_x3_applicable(Cd, Cg, k, stride, g_conv_precision))
    return conv_thin1_wgrad_x3(dense, N, Dd, Hd, Wd, Cd, gathered, Dg, Hg, Wg, Cg, pad, dw, accumulate, g_conv_precision,
                               ws, ws_bytes, st);
  if (thin_wgrad_side(Cd, Cg)) {
    ThinWgradArgs a{};
    a.D = dense; a.N = N; a.Dd = Dd; a.Hd = Hd; a.Wd = Wd; a.Cd = Cd;
    a.G = gathered; a.Dg = Dg; a.Hg = Hg; a.Wg = Wg; a.Cg = Cg; a.k = k; a.s = stride; a.p = pad;
    a.rnd = g_conv_precision;
    return conv_thin_wgrad(a, dw, accumulate, static_cast<float*>(ws), ws_bytes, st);
  }
  WgradArgs a{dense, N, Dd, Hd, Wd, Cd, gathered, Dg, Hg, Wg, Cg, k, stride, pad, static_cast<float*>(ws), 0, 0,
              g_conv_precision};
  return conv_wgrad(a, dw, accumulate, ws_bytes, st);
}

size_t mragan_pack_entry_size(void) { return sizeof(PackEntry); }

int mragan_pack_weights(const void* table, int n, int64_t max_elems, void* stream) {
  MRAGAN_CHECK_ARG(table && n >= 0 && n <= 65535 && max_elems >= 0, "pack_weights: bad args");
  return pack_weights_batched(static_cast<const PackEntry*>(table), n, max_elems, static_cast<hipStream_t>(stream));
}

int mragan_pack_weight(const float* src, int A, int B, int T, int tr, float* dst, void* stream) {
  MRAGAN_CHECK_ARG(src && dst && A > 0 && B > 0 && T > 0, "pack_weight: bad args");
  return pack_weight(src, A, B, T, tr, dst, static_cast<hipStream_t>(stream));
}

size_t mragan_instnorm_workspace(int N, int D, int H, int W, int C) {
  return instnorm_ws_bytes(N, D, H, W, C) + (size_t)N * C * 2 * sizeof(float) + 256;
}

int mragan_instnorm_fwd(const float* x, int N, int D, int H, int W, int C, float* y, int ypad, int act, const float* resid,
                        int rpad_, float* mean, float* rstd, void* ws, size_t ws_bytes, void* stream) {
  MRAGAN_CHECK_ARG(x && y && mean && rstd && ws, "instnorm_fwd: null pointer");
  return instnorm_fwd(x, InShape{N, D, H, W, C}, y, ypad, act, resid, rpad_, mean, rstd, ws, ws_bytes,
                      static_cast<hipStream_t>(stream));
}

int mragan_instnorm_bwd(const float* x, const float* mean, const float* rstd, int N, int D, int H, int W, int C,
                        const float* dy, int dypad, const float* dy_add, int act, float* dx, void* ws, size_t ws_bytes,
                        void* stream) {
  MRAGAN_CHECK_ARG(x && mean && rstd && dy && dx && ws, "instnorm_bwd: null pointer");
  InBwdArgs a{x, mean, rstd, dy, dypad, dy_add, act, dx, nullptr};
  return instnorm_bwd(a, InShape{N, D, H, W, C}, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

int mragan_instnorm_bwd_g(const float* x, const float* mean, const float* rstd, int N, int D, int H, int W, int C,
                          const float* dy, int dypad, const float* dy_add, int act, float* dx, float* g_out, void* ws,
                          size_t ws_bytes, void* stream) {
  MRAGAN_CHECK_ARG(x && mean && rstd && dy && dx && g_out && ws, "instnorm_bwd_g: null pointer");
  MRAGAN_CHECK_ARG(g_out != dx && g_out != dy && g_out != dy_add, "instnorm_bwd_g: g_out aliases an operand");
  InBwdArgs a{x, mean, rstd, dy, dypad, dy_add, act, dx, g_out};
  return instnorm_bwd(a, InShape{N, D, H, W, C}, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

int mragan_instnorm_running_update(const void* table, int nentries, float momentum, void* stream) {
  return instnorm_running(table, nentries, momentum, static_cast<hipStream_t>(stream));
}

size_t mragan_running_entry_size(void) { return instnorm_running_entry_bytes(); }

int mragan_rpad(const float* x, int N, int D, int H, int W, int C, int pad, float* y, void* stream) {
  MRAGAN_CHECK_ARG(x && y && pad >= 0, "rpad: bad args");
  return rpad(x, N, D, H, W, C, pad, y, static_cast<hipStream_t>(stream));
}

int mragan_rpad_fold(const float* yp, int N, int D, int H, int W, int C, int pad, const float* add, float* x, void* stream) {
  MRAGAN_CHECK_ARG(yp && x && pad >= 0, "rpad_fold: bad args");
  return rpad_fold(yp, N, D, H, W, C, pad, add, x, static_cast<hipStream_t>(stream));
}

int mragan_act_bwd(const float* y, const float* g0, const float* g1, const float* g2, int64_t n, int act, float* dx,
                   void* stream) {
  MRAGAN_CHECK_ARG(dx && n >= 0, "act_bwd: bad args");
  return act_bwd(y, g0, g1, g2, n, act, dx, static_cast<hipStream_t>(stream));
}

int mragan_channel_concat(const float* a, int Ca, int act_a, const float* b, int Cb, int act_b, int64_t M, float* out,
                          void* stream) {
  MRAGAN_CHECK_ARG(a && b && out && Ca > 0 && Cb > 0 && M >= 0, "channel_concat: bad args");
  return channel_concat(a, Ca, act_a, b, Cb, act_b, M, out, static_cast<hipStream_t>(stream));
}

int mragan_channel_split(const float* g, int Ca, int Cb, int64_t M, const float* ya, int act_a, float* da,
                         const float* yb, int act_b, float* db, void* stream) {
  MRAGAN_CHECK_ARG(g && Ca > 0 && Cb > 0 && M >= 0 && (da || db), "channel_split: bad args");
  return channel_split(g, Ca, Cb, M, ya, act_a, da, yb, act_b, db, static_cast<hipStream_t>(stream));
}

int mragan_l1_loss(const float* a, const float* b, int64_t n, float scale, float* loss, int loss_acc, float* grad,
                   int grad_acc, void* ws, void* stream) {
  MRAGAN_CHECK_ARG(a && b && loss && ws && n > 0, "l1_loss: bad args");
  return l1_loss(a, b, n, scale, g_loss_scale, loss, loss_acc, grad, grad_acc, static_cast<float*>(ws),
                 static_cast<hipStream_t>(stream));
}

int mragan_gan_loss(const float* p, int64_t n, float target, int lsgan, float scale, float* loss, int loss_acc,
                    float* dlogit, void* ws, void* stream) {
  MRAGAN_CHECK_ARG(p && loss && ws && n > 0, "gan_loss: bad args");
  return gan_loss(p, n, target, lsgan, scale, g_loss_scale, loss, loss_acc, dlogit, static_cast<float*>(ws),
                  static_cast<hipStream_t>(stream));
}

size_t mragan_channel_sum_workspace(int64_t M, int C) { return channel_sum_ws_bytes(M, C); }
int mragan_channel_sum(const float* x, int64_t M, int C, float* out, int acc, void* ws, size_t ws_bytes, void* stream) {
  MRAGAN_CHECK_ARG(x && out && ws, "channel_sum: bad args");
  return channel_sum(x, M, C, out, acc, ws, ws_bytes, static_cast<hipStream_t>(stream));
}

int mragan_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2, float eps,
                int step, float grad_scale, void* stream) {
  MRAGAN_CHECK_ARG(p && g && m && v && step >= 1, "adam: bad args");
  return adam(p, g, m, v, n, lr, beta1, beta2, eps, step, grad_scale, static_cast<hipStream_t>(stream));
}

int mragan_adam_hyper(float lr, float beta1, float beta2, float eps, int step, float grad_scale, float* out6) {
  MRAGAN_CHECK_ARG(out6 && step >= 1, "adam_hyper: bad args");
  adam_hyper(lr, beta1, beta2, eps, step, grad_scale, out6);
  return kOk;
}

int mragan_adam_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper, void* stream) {
  MRAGAN_CHECK_ARG(p && g && m && v && hyper, "adam_dev: bad args");
  return adam_dev(p, g, m, v, n, hyper, nullptr, static_cast<hipStream_t>(stream));
}

int mragan_adam_dev_checked(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper, const int* flag,
                            void* stream) {
  MRAGAN_CHECK_ARG(p && g && m && v && hyper && flag, "adam_dev_checked: bad args");
  return adam_dev(p, g, m, v, n, hyper, flag, static_cast<hipStream_t>(stream));
}

int mragan_adam_rebias(const float* base, const int* skipped, float* hyper, void* stream) {
  MRAGAN_CHECK_ARG(base && skipped && hyper && base != hyper, "adam_rebias: bad args");
  return adam_rebias(base, skipped, hyper, static_cast<hipStream_t>(stream));
}

int mragan_nonfinite_flag(const float* g, int64_t n, int* flag, void* stream) {
  MRAGAN_CHECK_ARG(g && flag && n >= 0, "nonfinite_flag: bad args");
  return nonfinite_flag(g, n, flag, static_cast<hipStream_t>(stream));
}

int mragan_skip_count(int* flag, int* counter, void* stream) {
  MRAGAN_CHECK_ARG(flag && counter, "skip_count: bad args");
  return skip_count(flag, counter, static_cast<hipStream_t>(stream));
}

int mragan_debug_stamps(unsigned long long* host, int n) {
  return n < 0 ? ks_debug_stamps(host, -n) : thin1_debug_stamps(host, n);
}

int mragan_fill(float* p, int64_t n, float value, void* stream) {
  MRAGAN_CHECK_ARG(p, "fill: null");
  return fill(p, n, value, static_cast<hipStream_t>(stream));
}

int mragan_patch_gather(const float* vol, int X, int Y, int Z, const int* starts, int n, int px, int py, int pz,
                        float* out, void* stream) {
  MRAGAN_CHECK_ARG(vol && starts && out && n >= 0, "patch_gather: bad args");
  MRAGAN_CHECK_ARG(px > 0 && py > 0 && pz > 0 && px <= X && py <= Y && pz <= Z, "patch_gather: patch larger than volume");
  return patch_gather(vol, X, Y, Z, starts, n, px, py, pz, out, static_cast<hipStream_t>(stream));
}

int mragan_patch_combine(const float* pred, int X, int Y, int Z, int px, int py, int pz, int stride_inplane,
                         int stride_layer, float* label, void* stream) {
  MRAGAN_CHECK_ARG(pred && label, "patch_combine: null pointer");
  MRAGAN_CHECK_ARG(px > 0 && py > 0 && pz > 0 && px <= X && py <= Y && pz <= Z, "patch_combine: patch larger than volume");
  MRAGAN_CHECK_ARG(stride_inplane > 0 && stride_layer > 0, "patch_combine: bad stride");
  const int inum = (X - px + stride_inplane - 1) / stride_inplane + 1;
  const int jnum = (Y - py + stride_inplane - 1) / stride_inplane + 1;
  const int knum = (Z - pz + stride_layer - 1) / stride_layer + 1;
  return patch_combine(pred, X, Y, Z, px, py, pz, inum, jnum, knum, stride_inplane, stride_layer, label,
                       static_cast<hipStream_t>(stream));
}

const char* mragan_launch_log(int reset) {
  static thread_local char copy[1024];
  memcpy(copy, g_log, sizeof(copy));
  if (reset) {
    g_log_len = 0;
    g_log[0] = 0;
  }
  return copy;
}

int mragan_crop_patches(const float* vol, int X, int Y, int Z, const int* starts, int n, int px, int py, int pz,
                        float* out, void* stream) {
  MRAGAN_CHECK_ARG(vol && starts && out && n >= 0, "crop_patches: bad args");
  MRAGAN_CHECK_ARG(px > 0 && py > 0 && pz > 0 && px <= X && py <= Y && pz <= Z, "crop_patches: patch larger than volume");
  return crop_patches(vol, X, Y, Z, starts, n, px, py, pz, out, static_cast<hipStream_t>(stream));
}

}  // extern "C"
