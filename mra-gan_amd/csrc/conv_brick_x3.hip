// bf16x3 3×3×3 stride-1 convolution: LDS-resident input halo, weights streamed from L2 straight
// into registers (gfx950).
//
// Same problem as conv_brick.hip (ResnetBlock convs networks3D.py:241-243, 256-257 and their
// data gradients), re-organised around one measurement: the staged kernel spends ~1,500 cycles
// per (tap × 32-channel) K-step of which the MFMAs are ~400 — it is bound by the per-step
// barrier + staging round trip, not by the matrix pipe (rocprofv3: SQ_WAIT_ANY 42 % of wave
// cycles, MFMA busy 25 %).  Here:
//
//   * the A operand (input voxels) comes from an LDS halo of the output brick, (BD+2)(BH+2)(BW+2)
//     positions × 32 channels, split once into [hi 32 × bf16][lo 32 × bf16] 144-B rows; the next
//     channel chunk's halo is streamed into the second buffer while the current chunk runs;
//   * the B operand is NOT staged: the weights are pre-split once per call (brick_x3_pack) into
//     bf16 hi/lo fragment order [tap][chunk][16-ch half][hi|lo][n][8-ch group][8], so each lane's
//     MFMA fragment is one 16-B load and the 64 lanes of a wave read 1 KB contiguous; fragments
//     are loaded kPF K-steps ahead into a register ring;
//   * so the only barrier is one per 32-channel chunk (4 per 128-channel conv instead of 108),
//     and every wave runs its 54 (tap, 16-channel) steps independently.
//
// Products: a·b ≈ a_hi·b_hi + a_hi·b_lo + a_lo·b_hi (three v_mfma_f32_32x32x16_bf16, fp32
// accumulate; see conv_igemm_x3.hip for the error bound).
//
// Precision modes (prec.h): bf16x3 as above; bf16 / fp16 run one MFMA per block product and
// neither store nor load the lo planes (halo rows keep their layout, the lo half stays unused).
#include "conv_geo.h"
#include "in_ticket.h"
#include "kernels.h"
#include "prec.h"

// build-time A/B knobs of the one-plane modes (tools/gpu_libs_ab.sh): weight prefetch distance
// (one n-tile) and A-fragment read distance, in steps
#ifndef MRAGAN_BRICK_KPF1
#define MRAGAN_BRICK_KPF1 9
#endif
#ifndef MRAGAN_BRICK_KAD1
#define MRAGAN_BRICK_KAD1 2
#endif
#ifndef MRAGAN_BRICK_S2_KPF
#define MRAGAN_BRICK_S2_KPF 18
#endif

namespace mragan {

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kBK = 32;                 // channels per chunk
// LDS row bytes of one halo position (32 channels): bf16x3 hi 64 B | lo 64 B | 16 B pad; the
// one-plane modes (bf16, fp16) hi 64 B | 16 B pad — half the halo, so two blocks fit a CU.  Both
// strides are an odd number of 16-B slots (9, 5): rows distinct mod 16 land on distinct slots, so
// brick_row_perm's conflict-free assignment holds for either.
template <int PM>
constexpr int row_bytes() { return prec::has_lo<PM>() ? 144 : 80; }
constexpr int kTaps = 27;
constexpr int kSteps = 2 * kTaps;       // (tap, 16-channel half) steps per chunk

// packed weights [27][ny][C] fp32 → fragment order (see the file comment); one thread per 8
// channels of one (tap, n)
template <int PM>
__global__ void brick_x3_pack_kernel(const float* __restrict__ wp, int ny, int C, __bf16* __restrict__ out) {
  const int nch = C / kBK;
  const int64_t total = (int64_t)kTaps * ny * (C / 8);
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
    *reinterpret_cast<bf16x8*>(out + base + (int64_t)ny * 16) = lo;
  }
}

template <int PM>
__device__ __forceinline__ void split4_store(char* row, int q, const float4& v) {
  uint2 h, l;
  prec::split4<PM>(v, h, l);
  *reinterpret_cast<uint2*>(row + 8 * q) = h;
  if constexpr (prec::has_lo<PM>()) *reinterpret_cast<uint2*>(row + 64 + 8 * q) = l;
}

// one 16-B slice q of a halo position: fp32 input → 4 channels split into the row; a 16-bit
// operand plane (X16) → 8 channels already in MFMA format, copied as they are
template <int PM, int X16>
__device__ __forceinline__ void halo_store(char* row, int q, const float4& v) {
  if constexpr (X16) *reinterpret_cast<float4*>(row + 16 * q) = v;
  else split4_store<PM>(row, q, v);
}

}  // namespace

// S = 2 (round 6): the stride-2 forward convs k3 s2 p1 (G down1 / down2,
// networks3D.py:191-197) on the same kernel.  The output brick's input halo is (2BD+1)(2BH+1)(2BW+1)
// positions; each halo row of HW = 2BW + 1 positions is stored as its even-w positions then its
// odd-w ones, so the 32 output voxels of an A fragment (consecutive bw) read consecutive LDS rows in
// every tap (tap kw = 0 / 2: the even half at sw = bw / bw + 1, kw = 1: the odd half at sw = bw) —
// the stride-1 kernel's 80-B row stride and brick_row_perm_s's conflict-free GEMM-row assignment
// hold, and the implicit GEMM's per-K-step tap addressing, bounds checks, LDS stores and barrier
// (≈ 15 VALU + 17 SALU per MFMA, PMC r05) are gone: one barrier per 32-channel chunk.
// STREAM = 0: one halo buffer (the 128-row bricks' 1377-position halo fills 110 KB); a further
// chunk is loaded after the previous one's MFMAs behind a barrier instead of streamed.
template <int WM, int WN, int TM, int TN, int HMAX, int PM, int X16, int S = 1, int STREAM = 1>
__global__ void __launch_bounds__(WM * WN * 64)
conv_brick_x3_kernel(BrickArgs a) {
  static_assert(!X16 || !prec::has_lo<PM>(), "16-bit operand planes exist in the one-plane modes only");
  constexpr int NT = WM * WN * 64;
  constexpr int BM = WM * TM * 32;
  constexpr int BN = WN * TN * 32;
  // input: fp32 NDHWC, or (X16) the producer's 16-bit operand plane of it (bf16 / fp16 words,
  // already rounded as this kernel would round them): half the halo bytes, no conversion
  constexpr int ES = X16 ? 2 : 4;                    // bytes per input element
  constexpr int SPP = X16 ? 4 : 8;                   // 16-B slices per halo position (32 channels)
  constexpr int CPS = kBK / SPP;                     // channels per slice
  constexpr int NSL = (HMAX * SPP + NT - 1) / NT;    // halo slices per thread per chunk
  // next-chunk halo: slice s is loaded at step 3s and split + stored kHD steps later (a ring of
  // 3 float4); vmcnt drains in issue order, so a load's real deadline is the next weight wait
  // kPF steps on — kHD < kPF keeps the store inside that window
  constexpr int kHD = 8;
  static_assert(!STREAM || 3 * (NSL - 1) + kHD < kSteps, "halo slices do not fit the chunk's steps");
  static_assert(S == 1 || (S == 2 && !prec::has_lo<PM>()), "stride 2: the one-plane modes only");
  static_assert(BN % 32 == 0 && BM % 32 == 0, "tile");
  // weight prefetch distance in steps; divides kSteps so a ring slot maps to the same step
  // residue in every chunk
  // (S = 2: 18 — one block per CU leaves one wave per SIMD, and 9 steps of 2 MFMAs do not cover the
  // weight loads' latency under the whole chip's halo traffic)
  constexpr int kPF = S == 2 ? MRAGAN_BRICK_S2_KPF : (!prec::has_lo<PM>() && TN == 1) ? MRAGAN_BRICK_KPF1 : 9;
  constexpr int kP = 18;                             // unrolled period: ring slots compile-time
  constexpr int kAD = prec::has_lo<PM>() ? 1 : MRAGAN_BRICK_KAD1;    // A-fragment read distance (steps)
  static_assert(kP % (kAD + 1) == 0, "A ring period");
  static_assert(kSteps % kP == 0 && kP % kPF == 0 && kP % 9 == 0 && kHD < kPF, "step period");

  constexpr int kRow = row_bytes<PM>();
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NBUF = STREAM ? 2 : 1;
  char* halo_buf = smem;                                                // [NBUF][HMAX][kRow]
  int* out_off = reinterpret_cast<int*>(smem + NBUF * HMAX * kRow);    // [BM]
  int* hoff = out_off + BM;                                            // [HMAX]
  int* xoff = hoff + HMAX;                                             // [BM] (backward statistics)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm0 = (wave / WN) * TM * 32, wn0 = (wave % WN) * TN * 32;
  const int li = lane & 31, lh = lane >> 5;

  // tile → (instance, brick, n-block); XCD-aware order (n fastest, then bricks)
  int L = blockIdx.x, tile = L;
  if ((a.ntiles & 7) == 0) tile = (L & 7) * (a.ntiles >> 3) + (L >> 3);
  const int nbk = tile % a.gn;
  int rest = tile / a.gn;
  const int bw_i = rest % a.nbw; rest /= a.nbw;
  const int bh_i = rest % a.nbh; rest /= a.nbh;
  const int bd_i = rest % a.nbd;
  const int nb = rest / a.nbd;
  const int od0 = bd_i * a.BD, oh0 = bh_i * a.BH, ow0 = bw_i * a.BW;
  const int n0 = nbk * BN;
  const int HP = a.HD * a.HH * a.HW;

  for (int r = tid; r < BM; r += NT) {
    int off = -1;
    const int v = a.rowvox[r];
    if (v >= 0) {
      const int bd = v / (a.BH * a.BW), bh = (v / a.BW) % a.BH, bw = v % a.BW;
      const int od = od0 + bd, oh = oh0 + bh, ow = ow0 + bw;
      if (od < a.Do && oh < a.Ho && ow < a.Wo) {
        off = (int)((((int64_t)nb * a.Yd + od + a.ye) * a.Yh + oh + a.ye) * a.Yw + ow + a.ye);
        // backward statistics: the interior voxel this padded output folds into (clamp of o − 1)
        if (a.sx) {
          const int cd = min(max(od - 1, 0), a.Do - 3), ch = min(max(oh - 1, 0), a.Ho - 3),
                    cw = min(max(ow - 1, 0), a.Wo - 3);
          xoff[r] = (int)((((int64_t)nb * (a.Do - 2) + cd) * (a.Ho - 2) + ch) * (a.Wo - 2) + cw);
          // bit 30: the padded output is the interior voxel's own (no clamp) — where sadd joins
          if (od >= 1 && od <= a.Do - 2 && oh >= 1 && oh <= a.Ho - 2 && ow >= 1 && ow <= a.Wo - 2) xoff[r] |= 1 << 30;
        }
      }
    }
    out_off[r] = off;
  }
  for (int pos = tid; pos < HP; pos += NT) {
    const int hw = pos % a.HW, hh = (pos / a.HW) % a.HH, hd = pos / (a.HW * a.HH);
    // S = 2: halo row position hw < BW + 1 is even w 2·hw, the rest odd w 2·(hw − BW − 1) + 1
    const int iwl = S == 1 ? hw : (hw <= a.BW ? 2 * hw : 2 * (hw - a.BW - 1) + 1);
    const int id = S * od0 - a.p + hd, ih = S * oh0 - a.p + hh, iw = S * ow0 - a.p + iwl;
    const bool ok = (unsigned)id < (unsigned)a.Di && (unsigned)ih < (unsigned)a.Hi && (unsigned)iw < (unsigned)a.Wi;
    hoff[pos] = ok ? ((id * a.Hi + ih) * a.Wi + iw) * a.C : -1;
  }
  // A: byte offset of each fragment row in a halo buffer (tap 0, this lane's 16-B half)
  int abase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    int v = a.rowvox[wm0 + i * 32 + li];
    if (v < 0) v = -v - 1;
    const int bd = v / (a.BH * a.BW), bh = (v / a.BW) % a.BH, bw = v % a.BW;
    abase[i] = ((S * bd * a.HH + S * bh) * a.HW + bw) * kRow + lh * 16;
  }
  // S = 2: LDS position of tap kw = 1 (the odd half of a halo row)
  const int wodd = __builtin_amdgcn_readfirstlane(a.BW + 1);
  // B: this lane's 16-B fragment inside each (tap, chunk, half, hi|lo) block of the packed weights,
  // read through a buffer descriptor: the lane part of the offset is fixed (VGPR), the step part
  // is wave-uniform (SGPR soffset) — no per-step 64-bit address arithmetic in VALU (the flat-
  // pointer form spent ~5 VALU instructions per weight load)
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.wx3, __builtin_amdgcn_readfirstlane(kTaps * a.C * a.ny * 4));
  int boff[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) boff[j] = ((n0 + wn0 + j * 32 + li) * 16 + lh * 8) * 2;
  // uniform scalars (readfirstlane: the compiler otherwise keeps the chunk loop's bound in a VGPR
  // and every offset derived from the chunk index with it)
  const int nch_ = __builtin_amdgcn_readfirstlane(a.C / kBK);
  const int flip = __builtin_amdgcn_readfirstlane(a.flip);
  const int blkb = a.ny * 16 * 2;               // bytes of one (hi|lo) block
  // halo loads through the instance's range-checked descriptor: an out-of-volume position gets
  // an offset past the end and reads 0, with no select on the loaded value (a conditional
  // overwrite made hipcc drain the memory counter — the 9-step weight prefetch included — at
  // every halo load)
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(reinterpret_cast<const char*>(a.x) + (int64_t)nb * a.Di * a.Hi * a.Wi * a.C * ES,
                                              (uint32_t)a.Di * a.Hi * a.Wi * a.C * (uint32_t)ES);
  const int nchunks = nch_;
  __syncthreads();

  // whole halo of chunk c into buffer 0: all loads in flight before the first store, in batches of
  // ≤ kWB slices (the stride-2 halos run to 44 slices per thread)
  constexpr int kWB = NSL < 24 ? NSL : 24;
  auto halo_whole = [&](int c) __attribute__((always_inline)) {
#pragma unroll
    for (int s0 = 0; s0 < NSL; s0 += kWB) {
      float4 pv[kWB];
#pragma unroll
      for (int q = 0; q < kWB; ++q) {
        const int sl = s0 + q, e = sl * NT + tid, pos = e / SPP;
        const int o = (sl < NSL && pos < HP) ? hoff[pos] : -1;
        pv[q] = buf_load_f32x4(xr, o < 0 ? kOobOffset : (uint32_t)(o + c * kBK + CPS * (e % SPP)) * (uint32_t)ES);
      }
#pragma unroll
      for (int q = 0; q < kWB; ++q) {
        const int sl = s0 + q, e = sl * NT + tid, pos = e / SPP;
        if (sl < NSL && pos < HP) halo_store<PM, X16>(halo_buf + pos * kRow, e % SPP, pv[q]);
      }
    }
  };
  halo_whole(0);

  // weight prefetch ring: slot s holds the two float4 of every n-tile for some step ≡ s (mod kPF)
  bf16x8 rb[kPF][TN][2];
  auto b_load = [&](int chunk, int u, bf16x8 (&dst)[TN][2]) __attribute__((always_inline)) {
    const int t = u >> 1, kk = u & 1;
    const int tap = flip ? kTaps - 1 - t : t;
    const int sb = __builtin_amdgcn_readfirstlane(((tap * nch_ + chunk) * 2 + kk) * 2 * blkb);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      dst[j][0] = __builtin_bit_cast(bf16x8, buf_load_16b(wr, boff[j], sb));
      if constexpr (prec::has_lo<PM>()) dst[j][1] = __builtin_bit_cast(bf16x8, buf_load_16b(wr, boff[j], sb + blkb));
    }
  };
#pragma unroll
  for (int u = 0; u < kPF; ++u) b_load(0, u, rb[u]);

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{};
  __syncthreads();

  for (int c = 0; c < nchunks; ++c) {
    const char* H = halo_buf + (STREAM ? (c & 1) * HMAX * kRow : 0);
    char* Hn = halo_buf + ((c + 1) & 1) * HMAX * kRow;
    const bool stream = STREAM && c + 1 < nchunks;
    float4 rh[3];
    // A fragments kAD steps ahead (ring of kAD + 1): one LDS round trip (~120 cycles under load)
    // outlasts a one-plane mode's step (1–2 MFMAs), so those read two steps ahead
    bf16x8 af[kAD + 1][2][TM];   // [step mod kAD+1][hi|lo][fragment]
    auto a_read = [&](int u, bf16x8 (&dst)[2][TM]) __attribute__((always_inline)) {
      const int t = u >> 1, kk = u & 1;
      const int tw = t % 3;
      const int tap_off = (((t / 9) * a.HH + (t / 3) % 3) * a.HW + (S == 1 ? tw : tw == 1 ? wodd : tw >> 1)) * kRow +
                          kk * 32;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        dst[0][i] = *reinterpret_cast<const bf16x8*>(H + abase[i] + tap_off);
        if constexpr (prec::has_lo<PM>()) dst[1][i] = *reinterpret_cast<const bf16x8*>(H + abase[i] + tap_off + 64);
      }
    };
#pragma unroll
    for (int v = 0; v < kAD; ++v) a_read(v, af[v]);
    for (int u0 = 0; u0 < kSteps; u0 += kP) {
#pragma unroll
    for (int du = 0; du < kP; ++du) {
      const int u = u0 + du;
      // one scheduling region per step, loads first: left free, the scheduler sinks the next
      // step's A reads next to their MFMAs and every step waits out a full LDS round trip
      __builtin_amdgcn_sched_barrier(0);
      // next chunk's halo: slice s = u/3 loaded into ring slot s mod 3 (u0/3 ≡ 0 mod 3) …
      if (STREAM && du % 3 == 0 && u / 3 < NSL) {
        const int e = (u / 3) * NT + tid, hpos = e / SPP;
        const int o = (stream && hpos < HP) ? hoff[hpos] : -1;
        rh[(du / 3) % 3] = buf_load_f32x4(
            xr, o < 0 ? kOobOffset
                      : (uint32_t)(o + (c + 1 < nchunks ? c + 1 : c) * kBK + CPS * (e % SPP)) * (uint32_t)ES);
      }
      // … and split + stored kHD steps later
      if (STREAM && (du + kP - kHD) % 3 == 0 && u >= kHD && (u - kHD) / 3 < NSL) {
        const int e = ((u - kHD) / 3) * NT + tid, hpos = e / SPP;
        if (stream && hpos < HP) halo_store<PM, X16>(Hn + hpos * kRow, e % SPP, rh[((du + kP - kHD) / 3) % 3]);
      }
      // B fragments of this step (loaded kPF steps ago), then refill the slot with step u + kPF
      bf16x8 bh[TN], bl[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        bh[j] = rb[du % kPF][j][0];
        bl[j] = prec::has_lo<PM>() ? rb[du % kPF][j][1] : bh[j];
      }
      {
        const int un = u + kPF;
        if (un < kSteps) b_load(c, un, rb[du % kPF]);
        else b_load(c + 1 < nchunks ? c + 1 : c, un - kSteps, rb[du % kPF]);
      }
      // A fragments of the NEXT step from the halo (software pipelined: the LDS latency hides
      // under this step's MFMAs; the chunk's first step is read after its barrier)
      if (u + kAD < kSteps) a_read(u + kAD, af[(du + kAD) % (kAD + 1)]);
      __builtin_amdgcn_sched_barrier(0);
      const bf16x8 (&ah)[TM] = af[du % (kAD + 1)][0];
      const bf16x8 (&al)[TM] = af[du % (kAD + 1)][1];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          acc[i][j] = prec::mma<PM>(ah[i], prec::has_lo<PM>() ? al[i] : ah[i], bh[j], bl[j], acc[i][j]);
        }
    }
    }
    __syncthreads();
    if (!STREAM && c + 1 < nchunks) {
      // one buffer: the next chunk's whole halo after every wave's last reads of this one
      halo_whole(c + 1);
      __syncthreads();
    }
  }

  double ps[TN], pq[TN];                 // InstanceNorm statistics of the written values
  if (!a.sx) {
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = n0 + wn0 + j * 32 + li;
    const float bsum = a.bias ? a.bias[col] : 0.f;
    ps[j] = 0.0;
    pq[j] = 0.0;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const int off = out_off[row];
        if (off >= 0) {
          const float v = act_fwd(acc[i][j][r] + bsum, a.act);
          a.y[(int64_t)off * a.ny + col] = v;
          ps[j] += v;
          pq[j] += (double)v * v;
        }
      }
    }
  }
  } else {
    // backward statistics of the InstanceNorm in front of this conv (the data gradient of a
    // ResnetBlock conv is the padded dz; IN-backward reads g = fold(dz)·act'(x̂)): Σ_i g_i =
    // Σ_p dz_p·act'(x̂_c(p)) and Σ_i g_i·x̂_i = Σ_p dz_p·act'(x̂_c(p))·x̂_c(p), c = the fold's clamp
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn0 + j * 32 + li;
      const float mu = a.smean[nb * a.ny + col], rs = a.srstd[nb * a.ny + col];
      ps[j] = 0.0;
      pq[j] = 0.0;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = wm0 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
          const int off = out_off[row];
          if (off >= 0) {
            const float v = acc[i][j][r];
            a.y[(int64_t)off * a.ny + col] = v;
            const int xo = xoff[row];
            const int64_t xi = (int64_t)(xo & ((1 << 30) - 1)) * a.ny + col;
            const float xh = (a.sx[xi] - mu) * rs;
            const float gin = (a.sadd && (xo >> 30)) ? v + a.sadd[xi] : v;
            const float gv = (a.sact == kActRelu && !(xh > 0.f)) ? 0.f : (a.sact == kActLrelu && !(xh > 0.f)) ? gin * kLreluSlope : gin;
            ps[j] += gv;
            pq[j] += (double)gv * xh;
          }
        }
      }
    }
  }
  // the consumer InstanceNorm's per-(instance, channel) Σy / Σy² partial of this brick (the
  // separate statistics pass over y disappears): lanes li / li + 32 share a column, the WM waves
  // of a column group add through LDS (the halo buffers are idle), one double2 per column
  if (a.part) {
    __syncthreads();
    double* red = reinterpret_cast<double*>(halo_buf);        // [WM][BN][2]
    const int wmi = wave / WN;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const double s2 = ps[j] + __shfl_xor(ps[j], 32);
      const double q2 = pq[j] + __shfl_xor(pq[j], 32);
      if (lh == 0) {
        red[(wmi * BN + wn0 + j * 32 + li) * 2] = s2;
        red[(wmi * BN + wn0 + j * 32 + li) * 2 + 1] = q2;
      }
    }
    __syncthreads();
    const int chunks = a.nbd * a.nbh * a.nbw;
    const int brick = (bd_i * a.nbh + bh_i) * a.nbw + bw_i;
    for (int c = tid; c < BN; c += NT) {
      double s2 = 0.0, q2 = 0.0;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        s2 += red[(w * BN + c) * 2];
        q2 += red[(w * BN + c) * 2 + 1];
      }
      double* dst = a.part + (((int64_t)nb * chunks + brick) * a.ny + n0 + c) * 2;
      if (a.tick) {                     // write-through: the tile's reducer reads them (in_ticket.h)
        st_sc1(dst, s2);
        st_sc1(dst + 1, q2);
      } else {
        dst[0] = s2;
        dst[1] = q2;
      }
    }
    // ABI 15 (round 6 for this kernel): the last block of this (instance, column tile) finalizes
    // its statistics — μ / rstd, or the IN backward's coefficients — in the launch, as the K-split
    // brick does: the 18³ data gradient at N = 4 (this kernel) no longer leaves a finalize launch
    if (a.tick && in_ticket_draw(a.tick + nb * a.gn + nbk, chunks, reinterpret_cast<int*>(halo_buf))) {
      if (tid < 256) in_ticket_reduce<BN>(a.part, chunks, a.ny, nb, n0, a.fin_mode, a.fin_S, a.fin0, a.fin1);
    }
  }
}

template <int WM, int WN, int TM, int TN, int HMAX, int PM, int X16, int S = 1, int STREAM = 1>
static int launch_brick_x3_as(const BrickArgs& a, hipStream_t st) {
  constexpr int BM = WM * TM * 32;
  const size_t lds = (size_t)(STREAM ? 2 : 1) * HMAX * row_bytes<PM>() + (size_t)(2 * BM + HMAX) * sizeof(int);
  static_assert((STREAM ? 2 : 1) * HMAX * row_bytes<PM>() + (2 * BM + HMAX) * 4 <= 160 * 1024, "LDS");
  auto kern = conv_brick_x3_kernel<WM, WN, TM, TN, HMAX, PM, X16, S, STREAM>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(a.ntiles), dim3(WM * WN * 64), lds, st, a);
  return check_launch(X16 ? "conv_brick_x3(op16)" : "conv_brick_x3");
}

template <int WM, int WN, int TM, int TN, int HMAX, int PM>
static int launch_brick_x3(const BrickArgs& a, hipStream_t st) {
  if (!a.x16) return launch_brick_x3_as<WM, WN, TM, TN, HMAX, PM, 0>(a, st);
  if constexpr (prec::has_lo<PM>()) {
    set_error("conv_brick_x3: a 16-bit operand plane needs the bf16 or fp16 mode");
    return kBadArg;
  } else {
    return launch_brick_x3_as<WM, WN, TM, TN, HMAX, PM, 1>(a, st);
  }
}

// bm ∈ {64, 128}, bn ∈ {64, 128}: 4 waves (one per SIMD), wave tile (bm/2)×(bn/2) — the
// 117 KB LDS halo allows one block per CU, and two-per-SIMD (8-wave) variants spill at kPF = 9
size_t conv_brick_x3_ws_bytes(int C, int ny) { return (size_t)kTaps * C * ny * sizeof(float); }

// packed fp32 weights [27][ny][C] → the fragment-order copy in `out` (conv_brick_x3_ws_bytes)
int brick_x3_pack(const float* w, int ny, int C, void* out, int mode, hipStream_t st) {
  const int64_t groups = (int64_t)kTaps * ny * (C / 8);
  const dim3 grid((unsigned)((groups + 255) / 256));
  MRAGAN_PREC_DISPATCH(mode, hipLaunchKernelGGL(brick_x3_pack_kernel<PM>, grid, dim3(256), 0, st, w, ny, C,
                                                static_cast<__bf16*>(out));
                       return check_launch("brick_x3_pack"))
}

template <int PM>
static int brick_x3_launch_pm(BrickArgs a, int bm, int bn, void* ws, size_t ws_bytes, const void* wsplit, hipStream_t st) {
  if (wsplit) {
    a.wx3 = wsplit;                     // pre-split by mragan_pack_weights (tr 2/3) with the fp32 pack
  } else {
    const size_t need = conv_brick_x3_ws_bytes(a.C, a.ny);
    if (!ws || ws_bytes < need) {
      set_error("conv_brick_x3: workspace %zu < %zu", ws_bytes, need);
      return kWorkspace;
    }
    const int rc = brick_x3_pack(a.w, a.ny, a.C, ws, PM, st);
    if (rc) return rc;
    a.wx3 = ws;
  }
  // 128-row bricks on 8 waves (two per SIMD): one wave's halo staging and LDS waits overlap the
  // other's MFMAs (the LDS-resident halo allows only one block per CU)
  static const int var = [] {
    const char* e = getenv("MRAGAN_BRICK_VAR");
    return e ? atoi(e) : 0;
  }();
  // one-plane modes (bf16 / fp16): one MFMA per 32×32 tile and step, so the 8-wave tiles' weight
  // loads (1 KB per wave per MFMA, each fragment loaded by 2–4 waves) outrun the L1 → SIMD return
  // rate (≈ 64 B per clock per CU) and pace the MFMAs.  These tiles run one wave per SIMD with 64
  // GEMM rows × 32 columns per wave: half the weight bytes per MFMA (128×64: 24.7 vs 26.1 µs,
  // res dgrad [2×18³] 22.5 vs 26.2 µs, profiles/r03q/ – r03s/).  var 5 = the 8-wave tiles (A/B).
  // The 128×128 tile keeps its 8 waves: with 64×32 per wave its weight loads per MFMA already
  // match these, and the 18³ data gradient at N = 4 runs it in one round (30.2 µs against 32.7 /
  // 33.0 µs for 432 blocks of 128×64 / 64×128).
  const bool onep = !prec::has_lo<PM>() && var != 5;
  if (bm == 128 && bn == 128 && var == 1) return launch_brick_x3<1, 4, 4, 1, 400, PM>(a, st);
  if (bm == 128 && bn == 128 && var == 2) return launch_brick_x3<2, 2, 2, 2, 400, PM>(a, st);
  if (bm == 128 && bn == 128) return launch_brick_x3<2, 4, 2, 1, 400, PM>(a, st);
  if (bm == 128 && (onep || var == 4)) return launch_brick_x3<2, 2, 2, 1, 400, PM>(a, st);
  if (bm == 128) return launch_brick_x3<4, 2, 1, 1, 400, PM>(a, st);
  if (bn == 128 && (onep || var == 3)) return launch_brick_x3<1, 4, 2, 1, 300, PM>(a, st);
  if (bn == 128) return launch_brick_x3<2, 2, 1, 2, 300, PM>(a, st);
  return launch_brick_x3<2, 2, 1, 1, 300, PM>(a, st);
}

int conv_brick_x3_launch(BrickArgs a, int bm, int bn, void* ws, size_t ws_bytes, const void* wsplit, int mode,
                         hipStream_t st) {
  MRAGAN_PREC_DISPATCH(mode, return brick_x3_launch_pm<PM>(a, bm, bn, ws, ws_bytes, wsplit, st))
}

// ---- k3 s2 p1 forward on the brick (S = 2) -------------------------------------------------------
// Variants (A/B switch MRAGAN_BRICK_S2_VAR):
//   1: 128-row bricks 4×8×4 (halo 9×17×9 = 1377 positions, 110 KB: one buffer), 128×64 tiles on 4
//      waves of 64×32;
//   2: 64-row bricks 2×8×4 (halo 5×17×9 = 765, two buffers streamed), 64×64 tiles on 4 waves of 32×32;
//   3: 64-row bricks, 64×128 tiles on 4 waves of 64×32;
//   4: as 2 with one halo buffer (61 KB: two blocks per CU, the next chunk loaded behind a barrier);
//   5: as 1 on 8 waves of 32×32 (two per SIMD).
// Both shapes' tap-0 halo rows have at most BM / 16 voxels per residue mod 16 (brick_row_perm: every
// A read conflict-free).
// The fp32-input form (the kernel rounds the staged values to the very words of the operand plane)
// runs the same kernel with one halo buffer: a plane input and an fp32 input give the same bits
// (tests/test_graph_gpu.py::test_stride2_planes_bit_identical).
// G down1 (32 input channels) stays on the implicit GEMM: its 64³ / 128³ input is HBM-bound either way
// (r06u: [4×64³] 54.2 vs 56.4 µs, [2×64³] 29.4 vs 29.9) and the 128³ step ran 0.08 ms slower with the
// brick on it (r06v: 28.24-28.28 vs 28.16-28.17 ms); MRAGAN_BRICK_S2_VAR set forces the brick on it too
bool conv_brick_s2_applicable(const IgemmArgs& g) {
  static const bool off = getenv("MRAGAN_NO_BRICK_S2") != nullptr;
  static const bool forced = getenv("MRAGAN_BRICK_S2_VAR") != nullptr;
  return !off && (forced || g.cx >= 2 * kBK) && (g.x3 == kPrecBf16 || g.x3 == kPrecF16) && g.wx3 && g.k == 3 &&
         g.s == 2 && g.p == 1 &&
         !g.trans && !g.bs_x && g.act == kActNone && g.cx % kBK == 0 && g.ny % 64 == 0 && g.Di > 0 &&
         (int64_t)g.Di * g.Hi * g.Wi * g.cx * 4 < ((int64_t)1 << 31);
}

int conv_brick_s2(const IgemmArgs& g, hipStream_t st) {
  MRAGAN_CHECK_ARG(conv_brick_s2_applicable(g), "conv_brick_s2: not a k3 s2 p1 operand-plane forward conv");
  static const int var_env = [] {
    const char* e = getenv("MRAGAN_BRICK_S2_VAR");
    return e ? atoi(e) : 0;
  }();
  // default 4 (rocprof kernel traces, bf16, r06u: G down2 [4×32³] 21.6 vs the implicit GEMM's 26.4 µs,
  // [2×32³] 15.7 vs 21.7; G down1 [4×64³] 54.2 vs 56.4, [2×64³] 29.4 vs 29.9 — down1's 64³ input is
  // streamed once either way, its HBM bytes bound both; variants 1 / 2 / 5 lost on down1, 65.6 /
  // 82.9 / 59.0 µs: one block per CU leaves one wave per SIMD to wait out its own loads)
  int var = var_env ? var_env : 4;
  if (var == 3 && g.ny % 128) var = 2;                 // 64×128 tiles: whole column tiles only
  BrickArgs a{};
  a.x = g.x; a.N = g.N; a.Di = g.Di; a.Hi = g.Hi; a.Wi = g.Wi; a.C = g.cx;
  a.w = g.w; a.wx3 = g.wx3; a.bias = g.bias; a.y = g.y; a.Do = g.Do; a.Ho = g.Ho; a.Wo = g.Wo; a.ny = g.ny;
  a.act = g.act; a.p = g.p; a.flip = 0;
  a.ye = 0; a.Yd = g.Do; a.Yh = g.Ho; a.Yw = g.Wo;
  a.x16 = g.x16;
  const int bm = (var == 1 || var == 5) ? 128 : 64, bn = var == 3 ? 128 : 64;
  MRAGAN_CHECK_ARG(g.ny % bn == 0, "conv_brick_s2: %d output channels are not a multiple of the %d-column tile", g.ny, bn);
  a.BD = (var == 1 || var == 5) ? 4 : 2; a.BH = 8; a.BW = 4;
  a.HD = 2 * a.BD + 1; a.HH = 2 * a.BH + 1; a.HW = 2 * a.BW + 1;
  a.nbd = ceil_div(a.Do, a.BD); a.nbh = ceil_div(a.Ho, a.BH); a.nbw = ceil_div(a.Wo, a.BW);
  a.gn = ceil_div(g.ny, bn);
  const int64_t ntiles = (int64_t)a.N * a.nbd * a.nbh * a.nbw * a.gn;
  MRAGAN_CHECK_ARG(ntiles < ((int64_t)1 << 31), "conv_brick_s2: grid too large");
  a.ntiles = (int)ntiles;
  if (a.ntiles == 0) return kOk;
  if (g.in_part) {
    a.part = g.in_part;
    if (g.in_chunks) *g.in_chunks = a.nbd * a.nbh * a.nbw;
    static const bool no_fin = getenv("MRAGAN_NO_X3_FIN") != nullptr;   // A/B switch, as conv_brick's
    if (g.in_tick && bn <= 128 && !no_fin) {
      a.tick = g.in_tick; a.fin0 = g.in_fin0; a.fin1 = g.in_fin1;
      a.fin_mode = 0;
      a.fin_S = (double)a.Do * a.Ho * a.Wo;
      if (g.in_finalized) *g.in_finalized = 1;
    }
  }
  brick_row_perm(a.BD, a.BH, a.BW, a.HH, a.HW, bm, a.rowvox, 2);
  MRAGAN_PREC_DISPATCH(g.x3, {
    if constexpr (prec::has_lo<PM>()) {
      set_error("conv_brick_s2: the one-plane modes only");
      return kBadArg;
    } else {
      if (g.x16) {
        if (var == 1) return launch_brick_x3_as<2, 2, 2, 1, 1380, PM, 1, 2, 0>(a, st);
        if (var == 3) return launch_brick_x3_as<1, 4, 2, 1, 768, PM, 1, 2, 1>(a, st);
        if (var == 4) return launch_brick_x3_as<2, 2, 1, 1, 768, PM, 1, 2, 0>(a, st);
        if (var == 5) return launch_brick_x3_as<4, 2, 1, 1, 1380, PM, 1, 2, 0>(a, st);
        return launch_brick_x3_as<2, 2, 1, 1, 768, PM, 1, 2, 1>(a, st);
      }
      if (var == 1) return launch_brick_x3_as<2, 2, 2, 1, 1380, PM, 0, 2, 0>(a, st);
      if (var == 3) return launch_brick_x3_as<1, 4, 2, 1, 768, PM, 0, 2, 0>(a, st);
      if (var == 5) return launch_brick_x3_as<4, 2, 1, 1, 1380, PM, 0, 2, 0>(a, st);
      return launch_brick_x3_as<2, 2, 1, 1, 768, PM, 0, 2, 0>(a, st);
    }
  })
}

}  // namespace mragan
