// FETCH_SIZE / WRITE_SIZE calibration for the env kernel's access widths (MI355X_MICROARCH.md
// 'HBM': only 16-B-per-lane streams are calibrated there). Reads and writes a known byte count
// with 4-B-per-lane coalesced accesses (one dword per lane, consecutive lanes on consecutive
// words, 64 lanes per workgroup as in env_step_kernel) and with 16-B-per-lane accesses, one
// kernel each, so that rocprofv3 --pmc FETCH_SIZE (or WRITE_SIZE) per kernel can be divided by
// the byte count. The buffer (512 MiB) is larger than the Infinity Cache.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(64) void read_dword(const float* __restrict__ x, float* __restrict__ out, size_t n) {
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * 64 + threadIdx.x; i < n; i += (size_t)gridDim.x * 64) acc += x[i];
  if (acc == 12345.678f) out[blockIdx.x] = acc;  // keeps the loads; never true for the zero input
}
__global__ __launch_bounds__(64) void read_dwordx4(const float4* __restrict__ x, float* __restrict__ out, size_t n4) {
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * 64 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 64) {
    const float4 v = x[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.678f) out[blockIdx.x] = acc;
}
__global__ __launch_bounds__(64) void write_dword(float* __restrict__ y, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 64 + threadIdx.x; i < n; i += (size_t)gridDim.x * 64) y[i] = 1.0f;
}

int main() {
  const size_t bytes = (size_t)512 << 20, n = bytes / 4;
  float *x, *y, *out;
  if (hipMalloc(&x, bytes) != hipSuccess || hipMalloc(&y, bytes) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess)
    return 1;
  (void)hipMemset(x, 0, bytes);
  (void)hipDeviceSynchronize();
  const int grid = 16384;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(read_dword, dim3(grid), dim3(64), 0, 0, x, out, n);
    hipLaunchKernelGGL(read_dwordx4, dim3(grid), dim3(64), 0, 0, (const float4*)x, out, n / 4);
    hipLaunchKernelGGL(write_dword, dim3(grid), dim3(64), 0, 0, y, n);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("bytes per kernel: %zu\n", bytes);
  return 0;
}
