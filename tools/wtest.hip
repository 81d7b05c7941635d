// Store-throughput probe (diagnostic, GPU box): 1024 blocks × 256 threads each write 128 KB of
// a 134 MB fp32 volume [4][64][64][64][32], in the brickT epilogue pattern (4 × 16 × 16 voxel
// bricks, 2 KB w-rows) or linearly, with one block per CU (117 KB LDS) or unconstrained.
//   hipcc --offload-arch=gfx950 -O3 tools/wtest.hip -o /tmp/wtest && /tmp/wtest
#include <hip/hip_runtime.h>
#include <cstdio>

template <bool BRICK>
__global__ void __launch_bounds__(256) wkern(float* y) {
  extern __shared__ char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 999) smem[0] = 0;
  const int q = lane & 7;
  int blk = blockIdx.x;
  const int bw = blk % 4; blk /= 4;
  const int bh = blk % 4; blk /= 4;
  const int bd = blk % 16;
  const int nb = blk / 16;
  const float4 r = make_float4(1.f, 2.f, 3.f, 4.f);
  for (int half = 0; half < 2; ++half)
    for (int j = 0; j < 16; ++j) {
      const int v = j * 8 + (lane >> 3);
      const int dq = v >> 6, hh = (v >> 4) & 3, ww = v & 15;
      int64_t off;
      if (BRICK) {
        const int od = bd * 4 + 2 * dq + half, oh = bh * 16 + 4 * wave + hh, ow = bw * 16 + ww;
        off = ((((int64_t)nb * 64 + od) * 64 + oh) * 64 + ow) * 32 + 4 * q;
      } else {
        off = (int64_t)blockIdx.x * 32768 + ((half * 16 + j) * 4 + wave) * 256 + lane * 4;
      }
      *reinterpret_cast<float4*>(y + off) = r;
    }
}

int main() {
  float* y;
  const size_t n = (size_t)4 * 64 * 64 * 64 * 32;
  hipMalloc(&y, n * 4);
  hipMemset(y, 0, n * 4);
  const int lds_big = 116800;
  hipFuncSetAttribute((const void*)wkern<true>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_big);
  hipFuncSetAttribute((const void*)wkern<false>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_big);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int brick = 0; brick < 2; ++brick)
    for (int lds = 0; lds < 2; ++lds) {
      auto k = brick ? wkern<true> : wkern<false>;
      const int sh = lds ? lds_big : 0;
      for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k, dim3(1024), dim3(256), sh, 0, y);
      hipEventRecord(a);
      for (int it = 0; it < 20; ++it) hipLaunchKernelGGL(k, dim3(1024), dim3(256), sh, 0, y);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      printf("pattern %-6s lds %-3s : %7.1f us  %5.2f TB/s\n", brick ? "brick" : "linear", lds ? "117K" : "0", ms / 20 * 1e3,
             n * 4 / (ms / 20 * 1e-3) / 1e12);
    }
  return 0;
}
