// Contraction precision of the MFMA convolutions (include/mragan_hip.h, mragan_precision).
//
// Every MFMA kernel stages its fp32 operands into 16-bit MFMA fragments.  The mode decides what
// those fragments hold and how many MFMAs one product costs:
//
//   kPrecBf16x3  hi = bf16(x), lo = bf16(x − hi); a·b ≈ lo_a·hi_b + hi_a·lo_b + hi_a·hi_b
//                (three v_mfma_f32_32x32x16_bf16, ≤ 3·2⁻¹⁸ relative error per product): the
//                reference's fp32 arithmetic at a third of the bf16 MFMA rate;
//   kPrecBf16    hi = bf16(x) only: one v_mfma_f32_32x32x16_bf16 per product (2⁻⁸ relative
//                rounding per operand), fp32 accumulation — BASELINE configs[1]/[2] "bf16";
//   kPrecF16     hi = fp16(x) only: one v_mfma_f32_32x32x16_f16 (2⁻¹¹ per operand), fp32
//                accumulation — BASELINE configs[4] "fp16".  Gradients enter the backward
//                scaled by the library's loss scale (mragan_set_grad_scale) so that they stay in
//                fp16's normal range; the optimizer divides it out.
//
// The fragments always travel as 16-bit words (typed bf16x8 in the kernels); in kPrecF16 mode
// they hold fp16 bit patterns and are re-typed for the f16 MFMA.  kPrecF32 kernels are separate
// (exact fp32 v_mfma_f32_32x32x2_f32 / VALU).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mragan {

enum Prec : int { kPrecF32 = 0, kPrecBf16x3 = 1, kPrecBf16 = 2, kPrecF16 = 3 };

namespace prec {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// does the mode carry a lo plane?
template <int PM> constexpr bool has_lo() { return PM == kPrecBf16x3; }

// two floats → packed 16-bit hi (and, for bf16x3, lo) words
template <int PM>
__device__ __forceinline__ void split2(float a, float b, uint32_t& hi, uint32_t& lo) {
  if constexpr (PM == kPrecF16) {
    hi = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, f16x2));
    lo = 0;
  } else {
    const bf16x2 h = __builtin_convertvector((f32x2){a, b}, bf16x2);
    hi = __builtin_bit_cast(uint32_t, h);
    if constexpr (PM == kPrecBf16x3) {
      const f32x2 f = __builtin_convertvector(h, f32x2);
      lo = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a - f.x, b - f.y}, bf16x2));
    } else {
      lo = 0;
    }
  }
}

// four floats → 8-byte hi / lo quads
template <int PM>
__device__ __forceinline__ void split4(const float4& v, uint2& hi, uint2& lo) {
  split2<PM>(v.x, v.y, hi.x, lo.x);
  split2<PM>(v.z, v.w, hi.y, lo.y);
}

// eight floats → 16-byte hi / lo fragments
template <int PM>
__device__ __forceinline__ void split8(const float4& a, const float4& b, bf16x8& hi, bf16x8& lo) {
  uint4 h, l;
  split2<PM>(a.x, a.y, h.x, l.x);
  split2<PM>(a.z, a.w, h.y, l.y);
  split2<PM>(b.x, b.y, h.z, l.z);
  split2<PM>(b.z, b.w, h.w, l.w);
  hi = __builtin_bit_cast(bf16x8, h);
  lo = __builtin_bit_cast(bf16x8, l);
}

// an 8-float vector → 16-byte hi / lo fragments
template <int PM>
__device__ __forceinline__ void split8v(const f32x8& v, bf16x8& hi, bf16x8& lo) {
  if constexpr (PM == kPrecF16) {
    const f16x8 h = __builtin_convertvector(v, f16x8);
    hi = __builtin_bit_cast(bf16x8, h);
    lo = hi;
  } else {
    hi = __builtin_convertvector(v, bf16x8);
    if constexpr (PM == kPrecBf16x3) lo = __builtin_convertvector(v - __builtin_convertvector(hi, f32x8), bf16x8);
    else lo = hi;
  }
}

// one 32×32×16 block product into acc: 3 MFMAs (bf16x3) or 1 (bf16 / fp16)
template <int PM>
__device__ __forceinline__ f32x16 mma(const bf16x8& ah, const bf16x8& al, const bf16x8& bh, const bf16x8& bl,
                                      f32x16 acc) {
  if constexpr (PM == kPrecBf16x3) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
  } else if constexpr (PM == kPrecF16) {
    (void)al;
    (void)bl;
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, ah), __builtin_bit_cast(f16x8, bh), acc, 0,
                                                  0, 0);
  } else {
    (void)al;
    (void)bl;
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
  }
}

// the 16×16×32 form (f32x4 accumulator)
template <int PM>
__device__ __forceinline__ f32x4 mma16(const bf16x8& ah, const bf16x8& al, const bf16x8& bh, const bf16x8& bl,
                                       f32x4 acc) {
  if constexpr (PM == kPrecBf16x3) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
  } else if constexpr (PM == kPrecF16) {
    (void)al;
    (void)bl;
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, ah), __builtin_bit_cast(f16x8, bh), acc, 0,
                                                  0, 0);
  } else {
    (void)al;
    (void)bl;
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
  }
}

}  // namespace prec

// run the statement block with `constexpr int PM` set to the run-time mode (1..3)
#define MRAGAN_PREC_DISPATCH(mode, ...)         \
  switch (mode) {                               \
    case ::mragan::kPrecBf16: {                 \
      constexpr int PM = ::mragan::kPrecBf16;   \
      __VA_ARGS__;                              \
    }                                           \
    case ::mragan::kPrecF16: {                  \
      constexpr int PM = ::mragan::kPrecF16;    \
      __VA_ARGS__;                              \
    }                                           \
    default: {                                  \
      constexpr int PM = ::mragan::kPrecBf16x3; \
      __VA_ARGS__;                              \
    }                                           \
  }

}  // namespace mragan
