// Lane-permutation helpers shared by the MFMA kernels' epilogues (DPP, no LDS).
#pragma once
#include <hip/hip_runtime.h>

namespace mragan {

typedef float f32x4v __attribute__((ext_vector_type(4)));

// 4×4 transpose inside each quad of lanes (lane 4m + k holds row k of the block as v[0..3] → it
// ends up holding column k): two DPP bit-swap stages
__device__ __forceinline__ f32x4v quad_transpose(f32x4v v, int k) {
  const bool k0 = k & 1, k1 = k & 2;
  // stage 1, lanes k ↔ k ^ 1: the components whose bit 0 differs from the lane's
  {
    const float s01 = k0 ? v[0] : v[1], s23 = k0 ? v[2] : v[3];
    const float r01 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s01), 0xB1, 0xF, 0xF, false));
    const float r23 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s23), 0xB1, 0xF, 0xF, false));
    if (k0) { v[0] = r01; v[2] = r23; } else { v[1] = r01; v[3] = r23; }
  }
  // stage 2, lanes k ↔ k ^ 2: the components whose bit 1 differs from the lane's
  {
    const float s02 = k1 ? v[0] : v[2], s13 = k1 ? v[1] : v[3];
    const float r02 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s02), 0x4E, 0xF, 0xF, false));
    const float r13 = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s13), 0x4E, 0xF, 0xF, false));
    if (k1) { v[0] = r02; v[1] = r13; } else { v[2] = r02; v[3] = r13; }
  }
  return v;
}

}  // namespace mragan
