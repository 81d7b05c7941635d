// Sliding-window inference (reference test.py:38-207, TestModel models/test_model.py:7-48).
//
// The reference cuts a normalised volume into overlapping patches on the host (prepare_batch,
// test.py:22-34), runs the generator on one patch at a time, and averages the overlaps into a
// float32 volume on the host (test.py:160-173).  Here the volume stays resident in HBM:
//
//   patch_gather   volume [X][Y][Z] → a batch of patches [n][px][py][pz] (NDHWC with C = 1),
//                  scaled like test.py:150, (v − 127.5) / 127.5, rounded op by op as numpy does;
//   patch_combine  per output voxel, the patches that cover it, IN THE REFERENCE'S VISIT ORDER
//                  (i over x, j over y, k over z), accumulated in fp32 exactly like
//                  `label_np[...] += pred * 127.5 + 127.5` (test.py:161-168) starting from 0,
//                  then label / count + 0.01 (test.py:173).  Output-centric, so no atomics and
//                  the same bits as the sequential host loop for the same predictions.
//
// Both are HBM-bound byte movers: gather reads the covered volume once per patch and writes the
// patch (8 B per patch voxel); combine reads every prediction once and writes the volume
// (4 B per prediction voxel + 4 B per volume voxel).
#include "kernels.h"

namespace mragan {

namespace {

__global__ void patch_gather_kernel(const float* __restrict__ vol, int Y, int Z, const int* __restrict__ starts, int n,
                                    int px, int py, int pz, float* __restrict__ out) {
#pragma clang fp contract(off)
  const int64_t per = (int64_t)px * py * pz;
  const int64_t total = per * n;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(e / per);
    const int64_t r = e - p * per;
    const int c = (int)(r % pz);
    const int b = (int)((r / pz) % py);
    const int a = (int)(r / ((int64_t)pz * py));
    const int x = starts[3 * p] + a, y = starts[3 * p + 1] + b, z = starts[3 * p + 2] + c;
    const float v = vol[((int64_t)x * Y + y) * Z + z];
    const float d = v - 127.5f;
    out[e] = d / 127.5f;
  }
}

// covering patch range on one axis: starts s_i = min(i * stride, N − P), i < num; voxel x is
// covered by patch i iff s_i ≤ x < s_i + P.  The starts are non-decreasing, so the covering i
// form one contiguous run.
__device__ __forceinline__ void cover(int x, int num, int stride, int N, int P, int& lo, int& hi) {
  lo = num;
  hi = -1;
  for (int i = 0; i < num; ++i) {
    int s = i * stride;
    if (s + P > N) s = N - P;
    if (s <= x && x < s + P) {
      lo = i < lo ? i : lo;
      hi = i;
    }
  }
}

__device__ __forceinline__ int axis_start(int i, int stride, int N, int P) {
  const int s = i * stride;
  return s + P > N ? N - P : s;
}

__global__ void patch_combine_kernel(const float* __restrict__ pred, int X, int Y, int Z, int px, int py, int pz,
                                     int inum, int jnum, int knum, int s_in, int s_lay, float* __restrict__ label) {
  // numpy rounds every operation: no mul+add → fma contraction here (hipcc contracts by default;
  // the pragma covers only operators written in this scope — HIP's __fmul_rn / __fadd_rn are
  // header functions whose operators stay contractible after inlining)
#pragma clang fp contract(off)
  const int64_t total = (int64_t)X * Y * Z;
  const int64_t per = (int64_t)px * py * pz;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int z = (int)(e % Z);
    const int y = (int)((e / Z) % Y);
    const int x = (int)(e / ((int64_t)Z * Y));
    int i0, i1, j0, j1, k0, k1;
    cover(x, inum, s_in, X, px, i0, i1);
    cover(y, jnum, s_in, Y, py, j0, j1);
    cover(z, knum, s_lay, Z, pz, k0, k1);
    float acc = 0.f;
    float cnt = 0.f;
    for (int i = i0; i <= i1; ++i) {
      const int a = x - axis_start(i, s_in, X, px);
      for (int j = j0; j <= j1; ++j) {
        const int b = y - axis_start(j, s_in, Y, py);
        for (int k = k0; k <= k1; ++k) {
          const int c = z - axis_start(k, s_lay, Z, pz);
          const int64_t p = ((int64_t)i * jnum + j) * knum + k;
          const float v = pred[p * per + ((int64_t)a * py + b) * pz + c];
          const float sv = v * 127.5f;
          acc = acc + (sv + 127.5f);
          cnt += 1.f;
        }
      }
    }
    const float q = acc / cnt;          // IEEE division (hipcc's default for fp32 '/')
    label[e] = q + 0.01f;
  }
}

// plain crop of n patches (no scaling): the training patch sampler (train.py:42's
// RandCropByPosNegLabeld crops, mragan_hip/patch_sampler.py)
__global__ void crop_patches_kernel(const float* __restrict__ vol, int Y, int Z, const int* __restrict__ starts, int n,
                                    int px, int py, int pz, float* __restrict__ out) {
  const int64_t per = (int64_t)px * py * pz;
  const int64_t total = per * n;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(e / per);
    const int64_t r = e - p * per;
    const int c = (int)(r % pz);
    const int b = (int)((r / pz) % py);
    const int a = (int)(r / ((int64_t)pz * py));
    out[e] = vol[((int64_t)(starts[3 * p] + a) * Y + starts[3 * p + 1] + b) * Z + starts[3 * p + 2] + c];
  }
}

int grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  return (int)(g < 65536 ? (g < 1 ? 1 : g) : 65536);
}

}  // namespace

int crop_patches(const float* vol, int X, int Y, int Z, const int* starts, int n, int px, int py, int pz, float* out,
                 hipStream_t st) {
  (void)X;
  const int64_t total = (int64_t)n * px * py * pz;
  hipLaunchKernelGGL(crop_patches_kernel, dim3(grid_for(total)), dim3(256), 0, st, vol, Y, Z, starts, n, px, py, pz, out);
  return check_launch("crop_patches");
}

int patch_gather(const float* vol, int X, int Y, int Z, const int* starts, int n, int px, int py, int pz, float* out,
                 hipStream_t st) {
  const int64_t total = (int64_t)n * px * py * pz;
  hipLaunchKernelGGL(patch_gather_kernel, dim3(grid_for(total)), dim3(256), 0, st, vol, Y, Z, starts, n, px, py, pz, out);
  return check_launch("patch_gather");
}

int patch_combine(const float* pred, int X, int Y, int Z, int px, int py, int pz, int inum, int jnum, int knum, int s_in,
                  int s_lay, float* label, hipStream_t st) {
  const int64_t total = (int64_t)X * Y * Z;
  hipLaunchKernelGGL(patch_combine_kernel, dim3(grid_for(total)), dim3(256), 0, st, pred, X, Y, Z, px, py, pz, inum, jnum,
                     knum, s_in, s_lay, label);
  return check_launch("patch_combine");
}

}  // namespace mragan
