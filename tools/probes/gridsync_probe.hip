// Cost of an in-kernel grid barrier on MI355X (one atomic counter vs per-XCD counters), with a
// bounded spin (s_memrealtime, 100 MHz) so a non-resident block cannot hang the GPU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ unsigned ld_acq(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void flat_barrier(unsigned* ctr, int iters, int* err) {
  const unsigned G = gridDim.x;
  for (int i = 0; i < iters; ++i) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)(i + 1) * G;
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (ld_acq(ctr) < target) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) { atomicAdd(err, 1); break; }  // 20 ms
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
  }
}

// blocks with the same blockIdx % 8 (same XCD under round-robin dispatch) meet on a local
// counter; the last of each group bumps the global one
__global__ void xcd_barrier(unsigned* ctr, int iters, int* err) {
  const unsigned G = gridDim.x, g = blockIdx.x & 7, per = G / 8;
  unsigned* loc = ctr + 64 + 64 * g;
  for (int i = 0; i < iters; ++i) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned o = __hip_atomic_fetch_add(loc, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      if (o + 1 == (unsigned)(i + 1) * per) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)(i + 1) * 8;
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (ld_acq(ctr) < target) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) { atomicAdd(err, 1); break; }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
  }
}

__global__ void empty_kernel(int) {}

int main() {
  unsigned* ctr; int* err;
  hipMalloc(&ctr, 4096); hipMalloc(&err, 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int kind = 0; kind < 2; ++kind)
    for (int G : {64, 128, 256, 512}) {
      float ms[2];
      int its[2] = {1, 201};
      for (int k = 0; k < 2; ++k) {
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
          hipMemset(ctr, 0, 4096); hipMemset(err, 0, 4);
          hipEventRecord(a);
          if (kind == 0) hipLaunchKernelGGL(flat_barrier, dim3(G), dim3(256), 0, 0, ctr, its[k], err);
          else hipLaunchKernelGGL(xcd_barrier, dim3(G), dim3(256), 0, 0, ctr, its[k], err);
          hipEventRecord(b); hipEventSynchronize(b);
          float t; hipEventElapsedTime(&t, a, b); if (t < best) best = t;
          int e; hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost);
          if (e) { printf("timeout kind %d G %d\n", kind, G); return 1; }
        }
        ms[k] = best;
      }
      printf("%s G=%4d : 1 barrier kernel %.2f us, per barrier %.3f us\n", kind ? "xcd " : "flat", G, ms[0] * 1e3,
             (ms[1] - ms[0]) * 1e3 / 200);
    }
  // back-to-back empty kernels: launch-to-launch floor
  hipEventRecord(a);
  for (int i = 0; i < 1000; ++i) hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, 0, i);
  hipEventRecord(b); hipEventSynchronize(b);
  float t; hipEventElapsedTime(&t, a, b);
  printf("empty kernel back-to-back: %.2f us each\n", t);
  return 0;
}
