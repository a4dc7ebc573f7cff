// EXPERIMENT (dev only, not built into the product): forward-kind learner GEMM
//   C[M][N] = ELU(A[M][K] · B[N][K]ᵀ + bias)
// from operands stored pre-split as bf16 planes (A = Ah + Al, B = Bh + Bl; k contiguous;
// row stride ld, K padded with zeros to a multiple of 32), staged global -> LDS by
// global_load_lds (16 B per lane, no VALU split, no LDS stores by the waves), products
// lo·hi + hi·lo + hi·hi on v_mfma_f32_16x16x32_bf16 as lgx_mlp.hip's gemm_tile.
// Question it answers: how fast is the same 128x128 / 4-wave / BK-32 tile when the split is
// moved out of the staging path.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace gx {
constexpr int BM = 128, BN = 128, BK = 32, NT = 256;
constexpr int PLANE = BM * BK * 2;   // bytes of one plane tile (128 rows x 64 B)
constexpr int STAGE = 4 * PLANE;     // Ah, Al, Bh, Bl
// LDS byte offset of 16-B chunk c of row r: linear rows of 64 B, chunk XOR (bit 2 of r) << 1
// (conflict-free ds_read_b128 fragment reads; glds writes whole 1-KB runs)
__device__ __forceinline__ int off(int r, int c) { return r * 64 + 16 * (c ^ (((r >> 2) & 1) << 1)); }

__device__ __forceinline__ void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// one plane tile (rows row0.., k0..k0+31) into LDS: wave w issues rows 16(2w+t)..+15, lane i
// lands at byte 16 i of that 1-KB run = row 16(2w+t) + i/4, physical chunk i%4, i.e. it loads
// the logical chunk (i%4) ^ swz(row) of that row (the source carries the swizzle)
__device__ __forceinline__ void stage_plane(const __bf16* __restrict__ p, int64_t ld, int row0, int rows, int k0,
                                            char* lds_plane, int wave, int lane) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int run = 2 * wave + t;
    const int r = run * 16 + (lane >> 2);
    const int c = (lane & 3) ^ (((r >> 2) & 1) << 1);
    const int gr = min(row0 + r, rows - 1);
    glds16(p + (int64_t)gr * ld + k0 + 8 * c, lds_plane + run * 1024);
  }
}

__device__ __forceinline__ float elu(float v) { return v > 0.f ? v : __expf(v) - 1.f; }

__global__ __launch_bounds__(NT, 2) void fwd_planes(const __bf16* __restrict__ Ah, const __bf16* __restrict__ Al,
                                                    int64_t lda, const __bf16* __restrict__ Bh,
                                                    const __bf16* __restrict__ Bl, int64_t ldb,
                                                    const float* __restrict__ bias, float* __restrict__ C, int64_t ldc,
                                                    int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tiles_n = (N + BN - 1) / BN;
  const int nb = gridDim.x, per = (nb + 7) / 8;
  const int L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);  // XCD-contiguous tiles
  if (L >= ((M + BM - 1) / BM) * tiles_n) return;
  const int m0 = (L / tiles_n) * BM, n0 = (L % tiles_n) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave & 1) * 64, wn = (wave >> 1) * 64;
  const int nsteps = K / BK;
  auto stage = [&](int s, int buf) {
    char* b = lds + buf * STAGE;
    const int k0 = s * BK;
    stage_plane(Ah, lda, m0, M, k0, b, wave, lane);
    stage_plane(Al, lda, m0, M, k0, b + PLANE, wave, lane);
    stage_plane(Bh, ldb, n0, N, k0, b + 2 * PLANE, wave, lane);
    stage_plane(Bl, ldb, n0, N, k0, b + 3 * PLANE, wave, lane);
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fc = lane >> 4;
  stage(0, 0);
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    if (s + 1 < nsteps) stage(s + 1, (s + 1) & 1);
    const char* b = lds + (s & 1) * STAGE;
    bf16x8 bh[4], bl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = off(wn + j * 16 + fr, fc);
      bh[j] = *reinterpret_cast<const bf16x8*>(b + 2 * PLANE + o);
      bl[j] = *reinterpret_cast<const bf16x8*>(b + 3 * PLANE + o);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = off(wm + i * 16 + fr, fc);
      const bf16x8 ah = *reinterpret_cast<const bf16x8*>(b + o);
      const bf16x8 al = *reinterpret_cast<const bf16x8*>(b + PLANE + o);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[j], acc[i][j], 0, 0, 0);
      }
    }
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next stage has landed
    __syncthreads();
  }
  // epilogue straight from the accumulators: col = lane & 15, rows (lane >> 4) * 4 + r
  const int ec = lane & 15, er = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn + j * 16 + ec;
      if (n >= N) continue;
      const float bb = bias[n];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + er + r;
        if (m < M) C[(int64_t)m * ldc + n] = elu(acc[i][j][r] + bb);
      }
    }
}

// single LDS buffer, two barriers per K step: 32 KB per block, 3 blocks per CU
__global__ __launch_bounds__(NT, 3) void fwd_planes1(const __bf16* __restrict__ Ah, const __bf16* __restrict__ Al,
                                                    int64_t lda, const __bf16* __restrict__ Bh,
                                                    const __bf16* __restrict__ Bl, int64_t ldb,
                                                    const float* __restrict__ bias, float* __restrict__ C, int64_t ldc,
                                                    int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tiles_n = (N + BN - 1) / BN;
  const int nb = gridDim.x, per = (nb + 7) / 8;
  const int L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);  // XCD-contiguous tiles
  if (L >= ((M + BM - 1) / BM) * tiles_n) return;
  const int m0 = (L / tiles_n) * BM, n0 = (L % tiles_n) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave & 1) * 64, wn = (wave >> 1) * 64;
  const int nsteps = K / BK;
  auto stage = [&](int s, int buf) {
    char* b = lds + buf * STAGE;
    const int k0 = s * BK;
    stage_plane(Ah, lda, m0, M, k0, b, wave, lane);
    stage_plane(Al, lda, m0, M, k0, b + PLANE, wave, lane);
    stage_plane(Bh, ldb, n0, N, k0, b + 2 * PLANE, wave, lane);
    stage_plane(Bl, ldb, n0, N, k0, b + 3 * PLANE, wave, lane);
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fc = lane >> 4;
  for (int s = 0; s < nsteps; ++s) {
    if (s) __syncthreads();  // every wave is done reading the previous step
    stage(s, 0);
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const char* b = lds;
    bf16x8 bh[4], bl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int o = off(wn + j * 16 + fr, fc);
      bh[j] = *reinterpret_cast<const bf16x8*>(b + 2 * PLANE + o);
      bl[j] = *reinterpret_cast<const bf16x8*>(b + 3 * PLANE + o);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = off(wm + i * 16 + fr, fc);
      const bf16x8 ah = *reinterpret_cast<const bf16x8*>(b + o);
      const bf16x8 al = *reinterpret_cast<const bf16x8*>(b + PLANE + o);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  // epilogue straight from the accumulators: col = lane & 15, rows (lane >> 4) * 4 + r
  const int ec = lane & 15, er = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn + j * 16 + ec;
      if (n >= N) continue;
      const float bb = bias[n];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + er + r;
        if (m < M) C[(int64_t)m * ldc + n] = elu(acc[i][j][r] + bb);
      }
    }
}

// Exact-fp32 variant ("time an exact v_mfma_f32 variant"): fp32 operands
// staged by global_load_lds as they are (128 rows x 128 B per operand and K step), products
// on v_mfma_f32_16x16x4_f32. The k order inside a step is permuted identically for A and B:
// lane group g = lane >> 4 reads logical chunks 2g, 2g+1 (k = 8g .. 8g+7) once per step, and
// sub-step e feeds k = 8g + e to the instruction's k slot g.
constexpr int PLANE32 = BM * BK * 4;  // 16 KB
constexpr int STAGE32 = 2 * PLANE32;
__device__ __forceinline__ int off32(int r, int c) { return r * 128 + 16 * (c ^ (r & 7)); }

__device__ __forceinline__ void stage32(const float* __restrict__ p, int64_t ld, int row0, int rows, int k0,
                                        char* lds_plane, int wave, int lane) {
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int run = 4 * wave + t;  // 16 runs of 8 rows
    const int r = run * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    const int gr = min(row0 + r, rows - 1);
    glds16(p + (int64_t)gr * ld + k0 + 4 * c, lds_plane + run * 1024);
  }
}

__global__ __launch_bounds__(NT, 2) void fwd_f32(const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
                                                 int64_t ldb, const float* __restrict__ bias, float* __restrict__ C,
                                                 int64_t ldc, int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tiles_n = (N + BN - 1) / BN;
  const int nb = gridDim.x, per = (nb + 7) / 8;
  const int L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
  if (L >= ((M + BM - 1) / BM) * tiles_n) return;
  const int m0 = (L / tiles_n) * BM, n0 = (L % tiles_n) * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave & 1) * 64, wn = (wave >> 1) * 64;
  const int nsteps = K / BK;
  auto stage = [&](int s, int buf) {
    char* b = lds + buf * STAGE32;
    stage32(A, lda, m0, M, s * BK, b, wave, lane);
    stage32(B, ldb, n0, N, s * BK, b + PLANE32, wave, lane);
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, g = lane >> 4;
  stage(0, 0);
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    if (s + 1 < nsteps) stage(s + 1, (s + 1) & 1);
    const char* b = lds + (s & 1) * STAGE32;
    f32x4 bv[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = wn + j * 16 + fr;
      bv[j][0] = *reinterpret_cast<const f32x4*>(b + PLANE32 + off32(r, 2 * g));
      bv[j][1] = *reinterpret_cast<const f32x4*>(b + PLANE32 + off32(r, 2 * g + 1));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wm + i * 16 + fr;
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(b + off32(r, 2 * g));
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(b + off32(r, 2 * g + 1));
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(e < 4 ? a0[e & 3] : a1[e & 3],
                                                           e < 4 ? bv[j][0][e & 3] : bv[j][1][e & 3], acc[i][j], 0, 0,
                                                           0);
    }
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const int ec = lane & 15, er = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn + j * 16 + ec;
      if (n >= N) continue;
      const float bb = bias[n];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + er + r;
        if (m < M) C[(int64_t)m * ldc + n] = elu(acc[i][j][r] + bb);
      }
    }
}
}  // namespace gx

extern "C" int gx_fwd_f32(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias, float* C,
                          int64_t ldc, int M, int N, int K, void* stream) {
  if (K % gx::BK || lda % 4 || ldb % 4) return -1;
  const int tiles = ((M + gx::BM - 1) / gx::BM) * ((N + gx::BN - 1) / gx::BN);
  const int grid = 8 * ((tiles + 7) / 8);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gx::fwd_f32), hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * gx::STAGE32);
    attr = true;
  }
  hipLaunchKernelGGL(gx::fwd_f32, dim3(grid), dim3(gx::NT), 2 * gx::STAGE32, (hipStream_t)stream, A, lda, B, ldb, bias,
                     C, ldc, M, N, K);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int gx_fwd_planes1(const void* Ah, const void* Al, int64_t lda, const void* Bh, const void* Bl,
                              int64_t ldb, const float* bias, float* C, int64_t ldc, int M, int N, int K, void* stream) {
  if (K % gx::BK || lda % 8 || ldb % 8) return -1;
  const int tiles = ((M + gx::BM - 1) / gx::BM) * ((N + gx::BN - 1) / gx::BN);
  const int grid = 8 * ((tiles + 7) / 8);
  hipLaunchKernelGGL(gx::fwd_planes1, dim3(grid), dim3(gx::NT), gx::STAGE, (hipStream_t)stream, (const __bf16*)Ah,
                     (const __bf16*)Al, lda, (const __bf16*)Bh, (const __bf16*)Bl, ldb, bias, C, ldc, M, N, K);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int gx_fwd_planes(const void* Ah, const void* Al, int64_t lda, const void* Bh, const void* Bl, int64_t ldb,
                             const float* bias, float* C, int64_t ldc, int M, int N, int K, void* stream) {
  if (K % gx::BK || lda % 8 || ldb % 8) return -1;
  const int tiles = ((M + gx::BM - 1) / gx::BM) * ((N + gx::BN - 1) / gx::BN);
  const int grid = 8 * ((tiles + 7) / 8);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gx::fwd_planes), hipFuncAttributeMaxDynamicSharedMemorySize,
                              2 * gx::STAGE);
    attr = true;
  }
  hipLaunchKernelGGL(gx::fwd_planes, dim3(grid), dim3(gx::NT), 2 * gx::STAGE, (hipStream_t)stream,
                     (const __bf16*)Ah, (const __bf16*)Al, lda, (const __bf16*)Bh, (const __bf16*)Bl, ldb, bias, C, ldc,
                     M, N, K);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
