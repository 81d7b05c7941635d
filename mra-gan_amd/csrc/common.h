// Shared helpers for the MRA-GAN MI355X (gfx950) kernel library.
//
// Layout conventions:
//   * activations are NDHWC fp32: element (n, d, h, w, c) at ((((n*D + d)*H + h)*W + w)*C + c)
//   * packed conv weights are [tap][Nout][Kc] (contraction channels contiguous), tap = (td*k + th)*k + tw
//   * master weights / gradients keep the reference's torch layouts
//       Conv3d [Cout][Cin][k][k][k], ConvTranspose3d [Cin][Cout][k][k][k]
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

namespace mragan {

// status codes returned through the C ABI
enum Status : int {
  kOk = 0,
  kBadArg = 1,
  kWorkspace = 2,
  kLaunch = 3,
  kUnsupported = 4,
};

// activation codes shared with include/mragan_hip.h
enum Act : int { kActNone = 0, kActRelu = 1, kActLrelu = 2, kActTanh = 3, kActSigmoid = 4 };

constexpr float kLreluSlope = 0.2f;   // reference networks3D.py:393

void set_error(const char* fmt, ...);
int check_launch(const char* what);

__device__ __forceinline__ float act_fwd(float v, int act) {
  switch (act) {
    case kActRelu: return v > 0.f ? v : 0.f;
    case kActLrelu: return v > 0.f ? v : v * kLreluSlope;
    case kActTanh: return tanhf(v);
    case kActSigmoid: return 1.f / (1.f + expf(-v));
    default: return v;
  }
}

// Operand rounding of the 16-bit contraction modes in the kernels that compute in fp32 (the
// thin VALU convolutions and the fp32 implicit-GEMM / weight-gradient fallbacks), so that a
// bf16 / fp16 mode rounds EVERY convolution operand exactly as the MFMA kernels' fragment
// conversion does (RNE): `mode` is the precision code (prec.h, kPrecBf16 = 2, kPrecF16 = 3);
// the fp32-grade modes (f32, bf16x3 = 1) keep the value.
__device__ __forceinline__ float op_round(float v, int mode) {
  if (mode == 2) return (float)(__bf16)v;
  if (mode == 3) return (float)(_Float16)v;
  return v;
}
__device__ __forceinline__ float4 op_round4(float4 v, int mode) {
  if (mode != 2 && mode != 3) return v;
  return make_float4(op_round(v.x, mode), op_round(v.y, mode), op_round(v.z, mode), op_round(v.w, mode));
}

struct Vol {   // batch + spatial extents of an NDHWC tensor
  int n, d, h, w;
  __host__ __device__ int64_t spatial() const { return (int64_t)d * h * w; }
  __host__ __device__ int64_t voxels() const { return (int64_t)n * d * h * w; }
};

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Range-checked loads through a buffer descriptor: a byte offset at or beyond `bytes` reads 0
// (the hardware bounds check), so a halo load needs no select after it — a select on the
// loaded value makes the compiler wait for each load before issuing the next one.
// Build the descriptor from wave-uniform values only (cdna_hip_programming.md T8 / T20).
constexpr uint32_t kOobOffset = 0x80000000u;
// The base and size go through readfirstlane: a descriptor the compiler cannot prove uniform
// (e.g. a base offset by an instance index derived from blockIdx through divisions) lands in
// VGPRs, and every load through it becomes a waterfall loop (4 readfirstlane + 64-bit compares +
// exec juggling per load — found in conv_brick_x3's halo loads).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
#ifdef MRAGAN_RSRC_NO_RFL   // A/B baseline (tools/gpu_libs_ab.sh)
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
#endif
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p), hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
  void* ub = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(ub, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ float buf_load_f32(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)byte_off, 0, 0));
}
// (the clang builtin __builtin_amdgcn_raw_buffer_load_b128 of ROCm 7.2 emits a single
// buffer_load_dword: the 16-byte form goes through the LLVM intrinsic directly)
typedef float buf_f32x4 __attribute__((ext_vector_type(4)));
__device__ buf_f32x4 llvm_raw_buffer_load_f32x4(__amdgpu_buffer_rsrc_t r, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.ptr.buffer.load.v4f32");
__device__ __forceinline__ float4 buf_load_f32x4(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  const buf_f32x4 v = llvm_raw_buffer_load_f32x4(r, (int)byte_off, 0, 0);
  return make_float4(v.x, v.y, v.z, v.w);
}
// 16 bytes at voffset (per lane, VGPR) + soffset (wave-uniform, SGPR): a streamed operand whose
// per-step offset is uniform costs no VALU address arithmetic
__device__ __forceinline__ buf_f32x4 buf_load_16b(__amdgpu_buffer_rsrc_t r, int voffset, int soffset) {
  return llvm_raw_buffer_load_f32x4(r, voffset, soffset, 0);
}
// 8 bytes (four 16-bit operand words of a 16-bit operand plane), same addressing
typedef float buf_f32x2 __attribute__((ext_vector_type(2)));
__device__ buf_f32x2 llvm_raw_buffer_load_f32x2(__amdgpu_buffer_rsrc_t r, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.ptr.buffer.load.v2f32");
__device__ __forceinline__ uint2 buf_load_8b(__amdgpu_buffer_rsrc_t r, int voffset, int soffset) {
  return __builtin_bit_cast(uint2, llvm_raw_buffer_load_f32x2(r, voffset, soffset, 0));
}

}  // namespace mragan

#define MRAGAN_CHECK_ARG(cond, ...)           \
  do {                                        \
    if (!(cond)) {                            \
      ::mragan::set_error(__VA_ARGS__);       \
      return ::mragan::kBadArg;               \
    }                                         \
  } while (0)
