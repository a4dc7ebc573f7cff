// Block -> CU placement probe (dev tool): a persistent-shaped launch of `n` 256-thread blocks with
// `lds` bytes of dynamic LDS each; every block records its XCC_ID and HW_ID (CU, SH, SE) and the
// wall clock at start, so the host can see which blocks share a CU.
#include <hip/hip_runtime.h>
#include <stdint.h>
__global__ void probe(uint32_t* out, int spin) {
  extern __shared__ char lds[];
  if (threadIdx.x == 0) {
    out[blockIdx.x * 4 + 0] = __builtin_amdgcn_s_getreg(20 | (31 << 11)) & 15;  // XCC_ID
    out[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_getreg(4 | (31 << 11));          // HW_ID
    out[blockIdx.x * 4 + 2] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    lds[0] = 1;
  }
  // keep the block resident a while so the launch is placed as a full residency round
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)spin) __builtin_amdgcn_s_sleep(10);
  if (threadIdx.x == 0) out[blockIdx.x * 4 + 3] = (uint32_t)__builtin_amdgcn_s_memrealtime();
}
extern "C" int run_probe(uint32_t* out, int n, int lds, int spin) {
  hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipLaunchKernelGGL(probe, dim3(n), dim3(256), lds, 0, out, spin);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
