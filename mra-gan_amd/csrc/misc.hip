// Element-wise / reduction kernels of the CycleGAN step:
//   ReplicationPad3d forward + backward fold   (networks3D.py:185, 211, 233, 249)
//   activation backward (ReLU/LeakyReLU from the output, Tanh, Sigmoid)
//   L1Loss (cycle_gan_model.py:104-105), GANLoss BCE-on-sigmoid / MSE (networks3D.py:130-150)
//   bias gradients (channel sums), torch.optim.Adam (cycle_gan_model.py:107-110),
//   weight packing torch layout → [tap][Nout][Kc].
#include "kernels.h"

namespace mragan {

static int grid_cap(int64_t work, int cap = 8192) {
  int64_t b = (work + 255) / 256;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

#define GRID_STRIDE(i, n) \
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)

// ---- replication pad ---------------------------------------------------------------------
__global__ void rpad_kernel(const float* __restrict__ x, int N, int D, int H, int W, int C, int p, float* __restrict__ y) {
  const int Dp = D + 2 * p, Hp = H + 2 * p, Wp = W + 2 * p;
  const int64_t total = (int64_t)N * Dp * Hp * Wp * C;
  GRID_STRIDE(e, total) {
    const int c = (int)(e % C); int64_t u = e / C;
    const int w = (int)(u % Wp); u /= Wp;
    const int h = (int)(u % Hp); u /= Hp;
    const int d = (int)(u % Dp); const int n = (int)(u / Dp);
    const int sd = min(max(d - p, 0), D - 1), sh = min(max(h - p, 0), H - 1), sw = min(max(w - p, 0), W - 1);
    y[e] = x[((((int64_t)n * D + sd) * H + sh) * W + sw) * C + c];
  }
}

// `add` may alias `x` (in-place accumulate): each element is read before it is written by the
// same thread, so neither carries __restrict__.
__global__ void rpad_fold_kernel(const float* __restrict__ yp, int N, int D, int H, int W, int C, int p,
                                 const float* add, float* x) {
  const int Dp = D + 2 * p, Hp = H + 2 * p, Wp = W + 2 * p;
  const int64_t total = (int64_t)N * D * H * W * C;
  GRID_STRIDE(e, total) {
    const int c = (int)(e % C); int64_t u = e / C;
    const int w = (int)(u % W); u /= W;
    const int h = (int)(u % H); u /= H;
    const int d = (int)(u % D); const int n = (int)(u / D);
    const int d0 = d == 0 ? 0 : d + p, d1 = d == D - 1 ? D - 1 + 2 * p : d + p;
    const int h0 = h == 0 ? 0 : h + p, h1 = h == H - 1 ? H - 1 + 2 * p : h + p;
    const int w0 = w == 0 ? 0 : w + p, w1 = w == W - 1 ? W - 1 + 2 * p : w + p;
    float s = add ? add[e] : 0.f;
    for (int a = d0; a <= d1; ++a)
      for (int b = h0; b <= h1; ++b)
        for (int cc = w0; cc <= w1; ++cc) s += yp[((((int64_t)n * Dp + a) * Hp + b) * Wp + cc) * C + c];
    x[e] = s;
  }
}

// ---- activation backward: dx = (dy0 + dy1 + dy2) · act'(y) --------------------------------
__global__ void act_bwd_kernel(const float* __restrict__ y, const float* __restrict__ g0, const float* __restrict__ g1,
                               const float* __restrict__ g2, int64_t n, int act, float* __restrict__ dx) {
  GRID_STRIDE(i, n) {
    float g = g0 ? g0[i] : 0.f;
    if (g1) g += g1[i];
    if (g2) g += g2[i];
    const float v = y ? y[i] : 0.f;
    float d;
    switch (act) {
      case kActRelu: d = v > 0.f ? 1.f : 0.f; break;
      case kActLrelu: d = v > 0.f ? 1.f : kLreluSlope; break;
      case kActTanh: d = 1.f - v * v; break;
      case kActSigmoid: d = v * (1.f - v); break;
      default: d = 1.f;
    }
    dx[i] = g * d;
  }
}

// ---- channel concatenation (UnetSkipConnectionBlock, networks3D.py:340-343) ----------------
// out[m] = [act_a(a[m][0:Ca]) | act_b(b[m][0:Cb])]: torch.cat([x, model(x)], 1) followed by the
// parent's in-place uprelu, in NDHWC (m = voxel).  Channel-pair granularity keeps the loads and
// stores of a wave contiguous.
__global__ void concat_kernel(const float* __restrict__ a, int Ca, int act_a, const float* __restrict__ b, int Cb,
                              int act_b, int64_t M, float* __restrict__ out) {
  const int Co = Ca + Cb;
  GRID_STRIDE(e, M * Co) {
    const int64_t m = e / Co;
    const int c = (int)(e - m * Co);
    out[e] = c < Ca ? act_fwd(a[m * Ca + c], act_a) : act_fwd(b[m * Cb + (c - Ca)], act_b);
  }
}

// backward of concat: da = g[:, :Ca]·act_a'(ya), db = g[:, Ca:]·act_b'(yb) (derivatives from the
// activation outputs, as act_bwd; a null y means identity).  da may accumulate into itself.
__device__ __forceinline__ float act_deriv_from_y(float v, int act) {
  switch (act) {
    case kActRelu: return v > 0.f ? 1.f : 0.f;
    case kActLrelu: return v > 0.f ? 1.f : kLreluSlope;
    case kActTanh: return 1.f - v * v;
    case kActSigmoid: return v * (1.f - v);
    default: return 1.f;
  }
}

__global__ void split_kernel(const float* __restrict__ g, int Ca, int Cb, int64_t M, const float* __restrict__ ya,
                             int act_a, float* __restrict__ da, const float* __restrict__ yb, int act_b,
                             float* __restrict__ db) {
  const int Co = Ca + Cb;
  GRID_STRIDE(e, M * Co) {
    const int64_t m = e / Co;
    const int c = (int)(e - m * Co);
    const float v = g[e];
    if (c < Ca) {
      const int64_t i = m * Ca + c;
      if (da) da[i] = ya ? v * act_deriv_from_y(ya[i], act_a) : v;
    } else {
      const int64_t i = m * Cb + (c - Ca);
      if (db) db[i] = yb ? v * act_deriv_from_y(yb[i], act_b) : v;
    }
  }
}

int channel_concat(const float* a, int Ca, int act_a, const float* b, int Cb, int act_b, int64_t M, float* out,
                   hipStream_t st) {
  if (M == 0) return kOk;
  hipLaunchKernelGGL(concat_kernel, dim3(grid_cap(M * (Ca + Cb))), dim3(256), 0, st, a, Ca, act_a, b, Cb, act_b, M, out);
  return check_launch("concat");
}

int channel_split(const float* g, int Ca, int Cb, int64_t M, const float* ya, int act_a, float* da, const float* yb,
                  int act_b, float* db, hipStream_t st) {
  if (M == 0) return kOk;
  hipLaunchKernelGGL(split_kernel, dim3(grid_cap(M * (Ca + Cb))), dim3(256), 0, st, g, Ca, Cb, M, ya, act_a, da, yb,
                     act_b, db);
  return check_launch("split");
}

// ---- block reduction helper --------------------------------------------------------------
__device__ __forceinline__ double block_sum(double v) {
  __shared__ double sh[4];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  double t = 0;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += sh[i];
  return t;
}

// ---- L1 loss: loss += scale·mean|a−b| ; grad (=|+=) gscale·scale·sign(a−b)/n -------------
// (gscale: the library's loss scale, mragan_set_loss_scale; 1 unless the fp16 mode scales the
// backward — the loss value itself is never scaled)
__global__ void __launch_bounds__(256) l1_kernel(const float* __restrict__ a, const float* __restrict__ b, int64_t n,
                                                 float scale, float gscale, float* loss_partial, float* __restrict__ grad,
                                                 int acc) {
  double s = 0;
  const float gs = scale * gscale / (float)n;
  GRID_STRIDE(i, n) {
    const float d = a[i] - b[i];
    s += fabsf(d);
    if (grad) {
      const float g = d > 0.f ? gs : (d < 0.f ? -gs : 0.f);
      grad[i] = acc ? grad[i] + g : g;
    }
  }
  const double t = block_sum(s);
  if (threadIdx.x == 0) loss_partial[blockIdx.x] = (float)(t * (double)scale / (double)n);
}

// ---- GAN loss on D's output map ------------------------------------------------------------
// BCE (default, pred = sigmoid output p): loss = −mean(t·max(ln p,−100) + (1−t)·max(ln(1−p),−100));
//   dp = scale/n · (p−t)/max(p(1−p),1e-12)     (ATen binary_cross_entropy_backward; the sigmoid
//   backward is applied by the discriminator's last stage)
// MSE (--no_lsgan given → LSGAN): loss = mean((x−t)²); dp = scale/n · 2(x−t)
__global__ void __launch_bounds__(256) gan_kernel(const float* __restrict__ p, int64_t n, float t, int lsgan, float scale,
                                                  float gscale, float* loss_partial, float* __restrict__ dlogit) {
  double s = 0;
  GRID_STRIDE(i, n) {
    const float v = p[i];
    float g;
    if (lsgan) {
      const float d = v - t;
      s += (double)d * d;
      g = 2.f * d;
    } else {
      const float lp = fmaxf(logf(v), -100.f), l1p = fmaxf(logf(1.f - v), -100.f);
      s += -(t * lp + (1.f - t) * l1p);
      g = (v - t) / fmaxf((1.f - v) * v, 1e-12f);
    }
    if (dlogit) dlogit[i] = g * (scale * gscale / (float)n);
  }
  const double tt = block_sum(s);
  if (threadIdx.x == 0) loss_partial[blockIdx.x] = (float)(tt * (double)scale / (double)n);
}

__global__ void partial_sum_kernel(const float* __restrict__ part, int nb, float* __restrict__ out, int acc) {
  double s = 0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += part[i];
  const double t = block_sum(s);
  if (threadIdx.x == 0) out[0] = acc ? out[0] + (float)t : (float)t;
}

// ---- channel sums (bias gradients): out[c] (=|+=) Σ_m x[m][c] ------------------------------
// pass 1: grid (chunks, C); each block sums a contiguous chunk of rows of one channel
__global__ void __launch_bounds__(256) channel_sum_kernel(const float* __restrict__ x, int64_t M, int C, int chunks,
                                                          double* __restrict__ part) {
  const int c = blockIdx.y;
  const int64_t per = (M + chunks - 1) / chunks;
  const int64_t m0 = blockIdx.x * per, m1 = min(M, m0 + per);
  double s = 0;
  for (int64_t m = m0 + threadIdx.x; m < m1; m += blockDim.x) s += x[m * C + c];
  const double t = block_sum(s);
  if (threadIdx.x == 0) part[(int64_t)c * chunks + blockIdx.x] = t;
}

// pass 2: one block per channel adds the chunk partials in a fixed order (deterministic)
__global__ void channel_sum_final_kernel(const double* __restrict__ part, int chunks, float* __restrict__ out, int acc) {
  const int c = blockIdx.x;
  double s = 0;
  for (int i = threadIdx.x; i < chunks; i += blockDim.x) s += part[(int64_t)c * chunks + i];
  const double t = block_sum(s);
  if (threadIdx.x == 0) out[c] = acc ? out[c] + (float)t : (float)t;
}

// ---- Adam (torch.optim.Adam, amsgrad=False, weight_decay=0, single-tensor formula) ---------
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m, float* __restrict__ v,
                            int64_t n, float step_size, float beta1, float beta2, float eps, float bc2_sqrt,
                            float grad_scale) {
  const float w1 = 1.f - beta1;
  GRID_STRIDE(i, n) {
    const float gi = g[i] * grad_scale;
    float mi = m[i];
    // torch lerp: weight < 0.5 ? self + w·(end−self) : end − (end−self)·(1−w)
    mi = (w1 < 0.5f) ? mi + w1 * (gi - mi) : gi - (gi - mi) * (1.f - w1);
    float vi = v[i] * beta2 + (1.f - beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] - step_size * (mi / denom);
  }
}

// Graph-replayable variant: the per-step scalars come from device memory, hyper =
// {step_size, beta1, beta2, eps, sqrt(bc2), grad_scale} (adam_hyper computes them exactly as
// adam() does, so both paths produce identical bits)
__global__ void adam_dev_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                float* __restrict__ v, int64_t n, const float* __restrict__ hyper,
                                const int* __restrict__ skip) {
  if (skip && *skip) return;        // a non-finite gradient this step: no update (GradScaler's skip)
  const float step_size = hyper[0], beta1 = hyper[1], beta2 = hyper[2], eps = hyper[3], bc2_sqrt = hyper[4],
              grad_scale = hyper[5];
  const float w1 = 1.f - beta1;
  GRID_STRIDE(i, n) {
    const float gi = g[i] * grad_scale;
    float mi = m[i];
    mi = (w1 < 0.5f) ? mi + w1 * (gi - mi) : gi - (gi - mi) * (1.f - w1);
    float vi = v[i] * beta2 + (1.f - beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] - step_size * (mi / denom);
  }
}

// ---- weight packing: src[A][B][T] → dst[T][A][B] (transpose_ab=0) or dst[T][B][A] (=1) ----
__global__ void pack_kernel(const float* __restrict__ src, int A, int B, int T, int tr, float* __restrict__ dst) {
  const int64_t total = (int64_t)A * B * T;
  GRID_STRIDE(e, total) {
    // e enumerates dst
    const int t = (int)(e / ((int64_t)A * B));
    const int r = (int)(e % ((int64_t)A * B));
    int a, b;
    if (!tr) { a = r / B; b = r % B; } else { b = r / A; a = r % A; }
    dst[e] = src[((int64_t)a * B + b) * T + t];
  }
}

// Many packs in one launch (a network's repack after an optimizer step): blockIdx.y = entry,
// the x blocks stride over its elements.  Same element mapping as pack_kernel.
//
// tr = 2 | 3 (transpose_ab = tr & 1): the same [T][ny][C] packed weight, but written straight in
// the bf16x3 brick kernel's fragment order (conv_brick_x3.hip: [tap][chunk][16-ch half][hi|lo]
// [n][8-ch group][8] bf16, hi = rne(w), lo = rne(w − hi)), so the k3 s1 convs of a step skip
// their per-call split.  Requires T = 27, C % 32 == 0 (entries that do not fit are skipped).
// tr = 4 | 5: the same with fp16 hi / lo (the kPrecF16 mode, prec.h).
typedef float pk_f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 pk_bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 pk_f16x8 __attribute__((ext_vector_type(8)));

__device__ void pack_split_entry(const PackEntry& e) {
  const int tr = e.tr & 1;
  const int ny = tr ? e.B : e.A, C = tr ? e.A : e.B;
  if (e.T != 27 || C % 32 != 0) return;
  const int G = C / 8, nch = C / 32;
  const int total = e.T * ny * G;
  __bf16* out = reinterpret_cast<__bf16*>(e.dst);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int g = i % G, tn = i / G;
    const int n = tn % ny, tap = tn / ny;
    pk_f32x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = g * 8 + j;
      const int a = tr ? c : n, b = tr ? n : c;
      v[j] = e.src[(a * e.B + b) * e.T + tap];
    }
    pk_bf16x8 hi, lo;
    if (e.tr >= 4) {          // fp16 fragments (kPrecF16), bit patterns in the same 16-bit slots
      const pk_f16x8 h = __builtin_convertvector(v, pk_f16x8);
      hi = __builtin_bit_cast(pk_bf16x8, h);
      lo = __builtin_bit_cast(pk_bf16x8, __builtin_convertvector(v - __builtin_convertvector(h, pk_f32x8), pk_f16x8));
    } else {
      hi = __builtin_convertvector(v, pk_bf16x8);
      lo = __builtin_convertvector(v - __builtin_convertvector(hi, pk_f32x8), pk_bf16x8);
    }
    const int chunk = g >> 2, kk = (g >> 1) & 1, lh = g & 1;
    const int base = (((tap * nch + chunk) * 2 + kk) * 2) * ny * 16 + n * 16 + lh * 8;
    *reinterpret_cast<pk_bf16x8*>(out + base) = hi;
    *reinterpret_cast<pk_bf16x8*>(out + base + ny * 16) = lo;
  }
}

__global__ void pack_split_kernel(PackEntry e) { pack_split_entry(e); }

// Tiled form of one entry (A % 8 == 0, B % 16 == 0, T ≤ 64): a block stages src[a0 .. a0+8)
// [b0 .. b0+16)[0 .. T) — 8 contiguous runs of 16·T floats — in LDS, then writes every output
// it feeds with contiguous runs (fp32: 16 or 8 floats; split: one 16-B hi / lo fragment per
// (tap, n, 8 channels)).  The element-wise form reads src with a stride of T floats and re-reads
// each line T times through L2 (86 µs for a generator's repack).  Same conversions, so the
// output is bit-identical.
constexpr int kPkA = 8, kPkB = 16, kPkTMax = 64;
__device__ __forceinline__ bool pack_tiled_ok(const PackEntry& e) {
  if (e.A % kPkA || e.B % kPkB || e.T > kPkTMax) return false;
  if (e.tr >= 2) {
    const int C = (e.tr & 1) ? e.A : e.B;
    return e.T == 27 && C % 32 == 0;
  }
  return true;
}

__device__ void pack_tiled_entry(const PackEntry& e, float* S) {
  const int T = e.T, TP = T + 1;
  const int nbt = e.B / kPkB, tiles = (e.A / kPkA) * nbt;
  const int tid = threadIdx.x;
  for (int tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
    const int a0 = (tile / nbt) * kPkA, b0 = (tile % nbt) * kPkB;
    __syncthreads();                                   // the previous tile's reads of S are done
    for (int i = tid; i < kPkA * kPkB * T; i += blockDim.x) {
      const int la = i / (kPkB * T), rem = i - la * (kPkB * T);
      const int lb = rem / T, t = rem - lb * T;
      S[(la * kPkB + lb) * TP + t] = e.src[((a0 + la) * e.B + b0) * T + rem];
    }
    __syncthreads();
    if (e.tr == 0) {                                   // dst[t][a][b]
      for (int i = tid; i < T * kPkA * kPkB; i += blockDim.x) {
        const int t = i / (kPkA * kPkB), la = (i / kPkB) % kPkA, lb = i % kPkB;
        e.dst[(t * e.A + a0 + la) * e.B + b0 + lb] = S[(la * kPkB + lb) * TP + t];
      }
    } else if (e.tr == 1) {                            // dst[t][b][a]
      for (int i = tid; i < T * kPkA * kPkB; i += blockDim.x) {
        const int t = i / (kPkA * kPkB), lb = (i / kPkA) % kPkB, la = i % kPkA;
        e.dst[(t * e.B + b0 + lb) * e.A + a0 + la] = S[(la * kPkB + lb) * TP + t];
      }
    } else {                                           // split fragments, as pack_split_entry
      const int trs = e.tr & 1;
      const int ny = trs ? e.B : e.A, C = trs ? e.A : e.B, nch = C / 32;
      __bf16* out = reinterpret_cast<__bf16*>(e.dst);
      // fragments in this tile: tr 2 — (tap, n = a0 + la, g = (b0 + 8h) / 8): 27 × 8 × 2;
      //                         tr 3 — (tap, n = b0 + lb, g = a0 / 8):      27 × 16 × 1
      for (int i = tid; i < T * 16; i += blockDim.x) {
        const int tap = i / 16, f = i % 16;
        pk_f32x8 v;
        int n, g;
        if (!trs) {
          const int la = f >> 1, h = f & 1;
          n = a0 + la;
          g = (b0 + 8 * h) >> 3;
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = S[(la * kPkB + 8 * h + j) * TP + tap];
        } else {
          const int lb = f;
          n = b0 + lb;
          g = a0 >> 3;
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = S[(j * kPkB + lb) * TP + tap];
        }
        pk_bf16x8 hi, lo;
        if (e.tr >= 4) {
          const pk_f16x8 h16 = __builtin_convertvector(v, pk_f16x8);
          hi = __builtin_bit_cast(pk_bf16x8, h16);
          lo = __builtin_bit_cast(pk_bf16x8, __builtin_convertvector(v - __builtin_convertvector(h16, pk_f32x8), pk_f16x8));
        } else {
          hi = __builtin_convertvector(v, pk_bf16x8);
          lo = __builtin_convertvector(v - __builtin_convertvector(hi, pk_f32x8), pk_bf16x8);
        }
        const int chunk = g >> 2, kk = (g >> 1) & 1, lh = g & 1;
        const int base = (((tap * nch + chunk) * 2 + kk) * 2) * ny * 16 + n * 16 + lh * 8;
        *reinterpret_cast<pk_bf16x8*>(out + base) = hi;
        *reinterpret_cast<pk_bf16x8*>(out + base + ny * 16) = lo;
      }
    }
  }
}

__global__ void pack_batched_kernel(const PackEntry* __restrict__ tab) {
  __shared__ float S[kPkA * kPkB * (kPkTMax + 1)];
  const PackEntry e = tab[blockIdx.y];
  if (pack_tiled_ok(e)) {
    pack_tiled_entry(e, S);
    return;
  }
  if (e.tr >= 2) {
    pack_split_entry(e);
    return;
  }
  const int AB = e.A * e.B, total = AB * e.T;          // < 2^31 (checked by the caller)
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int t = i / AB, r = i - t * AB;
    int a, b;
    if (!e.tr) { a = r / e.B; b = r - a * e.B; } else { b = r / e.A; a = r - b * e.A; }
    e.dst[i] = e.src[(a * e.B + b) * e.T + t];
  }
}

__global__ void fill_kernel(float* __restrict__ p, int64_t n, float v) {
  GRID_STRIDE(i, n) p[i] = v;
}

// ---- host wrappers -------------------------------------------------------------------------
int rpad(const float* x, int N, int D, int H, int W, int C, int p, float* y, hipStream_t st) {
  const int64_t total = (int64_t)N * (D + 2 * p) * (H + 2 * p) * (W + 2 * p) * C;
  hipLaunchKernelGGL(rpad_kernel, dim3(grid_cap(total)), dim3(256), 0, st, x, N, D, H, W, C, p, y);
  return check_launch("rpad");
}
int rpad_fold(const float* yp, int N, int D, int H, int W, int C, int p, const float* add, float* x, hipStream_t st) {
  const int64_t total = (int64_t)N * D * H * W * C;
  hipLaunchKernelGGL(rpad_fold_kernel, dim3(grid_cap(total)), dim3(256), 0, st, yp, N, D, H, W, C, p, add, x);
  return check_launch("rpad_fold");
}
int act_bwd(const float* y, const float* g0, const float* g1, const float* g2, int64_t n, int act, float* dx, hipStream_t st) {
  hipLaunchKernelGGL(act_bwd_kernel, dim3(grid_cap(n)), dim3(256), 0, st, y, g0, g1, g2, n, act, dx);
  return check_launch("act_bwd");
}
int l1_loss(const float* a, const float* b, int64_t n, float scale, float gscale, float* loss, int loss_acc, float* grad,
            int grad_acc, float* ws, hipStream_t st) {
  const int nb = grid_cap(n, 1024);
  hipLaunchKernelGGL(l1_kernel, dim3(nb), dim3(256), 0, st, a, b, n, scale, gscale, ws, grad, grad_acc);
  int rc = check_launch("l1_loss");
  if (rc) return rc;
  hipLaunchKernelGGL(partial_sum_kernel, dim3(1), dim3(256), 0, st, ws, nb, loss, loss_acc);
  return check_launch("l1_loss_sum");
}
int gan_loss(const float* p, int64_t n, float target, int lsgan, float scale, float gscale, float* loss, int loss_acc,
             float* dlogit, float* ws, hipStream_t st) {
  const int nb = grid_cap(n, 1024);
  hipLaunchKernelGGL(gan_kernel, dim3(nb), dim3(256), 0, st, p, n, target, lsgan, scale, gscale, ws, dlogit);
  int rc = check_launch("gan_loss");
  if (rc) return rc;
  hipLaunchKernelGGL(partial_sum_kernel, dim3(1), dim3(256), 0, st, ws, nb, loss, loss_acc);
  return check_launch("gan_loss_sum");
}
static int channel_sum_chunks(int64_t M, int C) {
  int64_t ch = (M + 4095) / 4096;
  int64_t cap = (2048 + C - 1) / C;
  if (ch > cap) ch = cap;
  return ch < 1 ? 1 : (int)ch;
}
size_t channel_sum_ws_bytes(int64_t M, int C) { return (size_t)channel_sum_chunks(M, C) * C * sizeof(double); }
int channel_sum(const float* x, int64_t M, int C, float* out, int acc, void* ws, size_t ws_bytes, hipStream_t st) {
  if (C <= 0) return kOk;
  const int chunks = channel_sum_chunks(M, C);
  if (channel_sum_ws_bytes(M, C) > ws_bytes) { set_error("channel_sum: workspace too small"); return kWorkspace; }
  double* part = static_cast<double*>(ws);
  hipLaunchKernelGGL(channel_sum_kernel, dim3(chunks, C), dim3(256), 0, st, x, M, C, chunks, part);
  int rc = check_launch("channel_sum");
  if (rc) return rc;
  hipLaunchKernelGGL(channel_sum_final_kernel, dim3(C), dim3(256), 0, st, part, chunks, out, acc);
  return check_launch("channel_sum_final");
}
int adam(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2, float eps, int step,
         float grad_scale, hipStream_t st) {
  // bias corrections and step size in double on the host, as torch does with python floats
  const double bc1 = 1.0 - pow((double)beta1, step);
  const double bc2 = 1.0 - pow((double)beta2, step);
  const float step_size = (float)((double)lr / bc1);
  hipLaunchKernelGGL(adam_kernel, dim3(grid_cap(n)), dim3(256), 0, st, p, g, m, v, n, step_size, beta1, beta2, eps,
                     (float)sqrt(bc2), grad_scale);
  return check_launch("adam");
}
void adam_hyper(float lr, float beta1, float beta2, float eps, int step, float grad_scale, float* out) {
  const double bc1 = 1.0 - pow((double)beta1, step);
  const double bc2 = 1.0 - pow((double)beta2, step);
  out[0] = (float)((double)lr / bc1);
  out[1] = beta1;
  out[2] = beta2;
  out[3] = eps;
  out[4] = (float)sqrt(bc2);
  out[5] = grad_scale;
}
// loss-scaled training: the six scalars of adam_hyper for t = base[4] − *skipped (the step count
// net of the updates skipped for a non-finite gradient, as GradScaler leaves the optimizer's step
// alone): base = {lr, beta1, beta2, eps, step, grad_scale}, written by the host; same formulas
__global__ void adam_rebias_kernel(const float* __restrict__ base, const int* __restrict__ skipped,
                                   float* __restrict__ hyper) {
  if (threadIdx.x != 0) return;
  const double t = (double)base[4] - (double)*skipped;
  const double bc1 = 1.0 - pow((double)base[1], t);
  const double bc2 = 1.0 - pow((double)base[2], t);
  hyper[0] = (float)((double)base[0] / bc1);
  hyper[1] = base[1];
  hyper[2] = base[2];
  hyper[3] = base[3];
  hyper[4] = (float)sqrt(bc2);
  hyper[5] = base[5];
}
int adam_rebias(const float* base, const int* skipped, float* hyper, hipStream_t st) {
  hipLaunchKernelGGL(adam_rebias_kernel, dim3(1), dim3(64), 0, st, base, skipped, hyper);
  return check_launch("adam_rebias");
}
int adam_dev(float* p, const float* g, float* m, float* v, int64_t n, const float* hyper, const int* skip,
             hipStream_t st) {
  hipLaunchKernelGGL(adam_dev_kernel, dim3(grid_cap(n)), dim3(256), 0, st, p, g, m, v, n, hyper, skip);
  return check_launch("adam_dev");
}

// ---- found-inf (fp16 loss scaling) ----------------------------------------------------------
// flag |= 1 when any of g[0:n] is inf / NaN: one vector atomic per wave that saw one
__global__ void nonfinite_kernel(const float* __restrict__ g, int64_t n, int* flag) {
  bool bad = false;
  GRID_STRIDE(i, n) bad |= !isfinite(g[i]);
  if (__builtin_amdgcn_ballot_w64(bad) != 0 && (threadIdx.x & 63) == __builtin_ctzll(__builtin_amdgcn_ballot_w64(bad)))
    atomicOr(flag, 1);
}
int nonfinite_flag(const float* g, int64_t n, int* flag, hipStream_t st) {
  hipLaunchKernelGGL(nonfinite_kernel, dim3(grid_cap(n, 2048)), dim3(256), 0, st, g, n, flag);
  return check_launch("nonfinite");
}
// after the step's updates: counter += (flag != 0); flag = 0
__global__ void skip_count_kernel(int* flag, int* counter) {
  if (threadIdx.x == 0) {
    const int f = *flag;
    *counter += f != 0;
    *flag = 0;
  }
}
int skip_count(int* flag, int* counter, hipStream_t st) {
  hipLaunchKernelGGL(skip_count_kernel, dim3(1), dim3(64), 0, st, flag, counter);
  return check_launch("skip_count");
}
int pack_weights_batched(const PackEntry* table, int n, int64_t max_elems, hipStream_t st) {
  if (n <= 0) return kOk;
  if (max_elems >= ((int64_t)1 << 31)) { set_error("pack_weights: entry too large"); return kBadArg; }
  // ≤ 256 blocks per entry: the tiled entries have ≤ 128 tiles at these shapes and the
  // element-wise ones grid-stride; every extra (empty) block still reserves the tile's LDS
  int gx = (int)((max_elems + 2047) / 2048);
  if (gx > 256) gx = 256;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(pack_batched_kernel, dim3(gx, n), dim3(256), 0, st, table);
  return check_launch("pack_batched");
}
int pack_weight(const float* src, int A, int B, int T, int tr, float* dst, hipStream_t st) {
  if (tr >= 2) {
    const int C = (tr & 1) ? A : B;
    MRAGAN_CHECK_ARG(T == 27 && C % 32 == 0, "pack_weight: split pack needs T = 27, contraction %% 32 (T=%d C=%d)", T, C);
    const PackEntry e{src, dst, A, B, T, tr};
    hipLaunchKernelGGL(pack_split_kernel, dim3(grid_cap((int64_t)A * B * T / 8)), dim3(256), 0, st, e);
    return check_launch("pack_split");
  }
  hipLaunchKernelGGL(pack_kernel, dim3(grid_cap((int64_t)A * B * T)), dim3(256), 0, st, src, A, B, T, tr, dst);
  return check_launch("pack_weight");
}
int fill(float* p, int64_t n, float v, hipStream_t st) {
  hipLaunchKernelGGL(fill_kernel, dim3(grid_cap(n)), dim3(256), 0, st, p, n, v);
  return check_launch("fill");
}

}  // namespace mragan
