// EXPERIMENT (dev only, not built into the product): forward-kind learner GEMM
//   C[M][N] = ELU(A[M][K] · B[N][K]ᵀ + bias), fp32 operands as the product keeps them,
// staged global -> LDS by global_load_lds into an NS-slot ring (fp32 images, 16 KB per
// operand and K step of 32), with counted vmcnt waits and a raw s_barrier per step (no
// __syncthreads: its vmcnt(0) would drain the ring); the 3xbf16 split (x = hi + lo) happens
// on the fragments after their LDS read. One 128 x 128 tile per block, 4 waves (2 x 2 of 64 x
// 64), one block per CU. Question: does a pipelined LDS-DMA ring beat the product's
// register-staged 2-block-per-CU structure on the update's shapes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace gr {
constexpr int BN = 128, BK = 32;
constexpr int IMGB = BN * BK * 4;       // B's fp32 image per step: 16 KB (A: BM / 128 times that)

// physical 16-B chunk of logical chunk c (0..7) in row r: conflict-free ds_read_b128 of the
// fragment pattern (rows r & 15 = lane & 15, chunks 2 (lane >> 4) + {0, 1}); found by search
__device__ __forceinline__ int swz(int r) { return ((r >> 1) & 1) | (r & 4); }

__device__ __forceinline__ void glds16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}

// one operand image (rows row0.., k k0..k0+31): 16 runs of 8 rows x 128 B; wave w issues runs
// w, w+4, w+8, w+12. Lane i of a run lands at byte 16 i = row run*8 + i/8, physical chunk i%8,
// and loads the logical chunk (i%8) ^ swz(row). Chunks past K load a valid chunk (masked later).
template <int RUNS, int WAVES>
__device__ __forceinline__ void stage_img(const float* __restrict__ p, int64_t ld, int row0, int rows, int k0, int K,
                                          char* img, int wave, int lane) {
#pragma unroll
  for (int t = 0; t < RUNS / WAVES; ++t) {
    const int run = wave + WAVES * t;
    const int r = run * 8 + (lane >> 3);
    const int c = (lane & 7) ^ swz(r);
    int k = k0 + 4 * c;
    k = k < K ? k : 0;
    const int g = min(row0 + r, rows - 1);
    glds16(p + (int64_t)g * ld + k, img + run * 1024);
  }
}

__device__ __forceinline__ bf16x8 split8(const f32x4& x0, const f32x4& x1, bf16x8& lo) {
  bf16x8 hi;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const __bf16 a = (__bf16)x0[j], b = (__bf16)x1[j];
    hi[j] = a;
    hi[4 + j] = b;
    lo[j] = (__bf16)(x0[j] - (float)a);
    lo[4 + j] = (__bf16)(x1[j] - (float)b);
  }
  return hi;
}

__device__ __forceinline__ float elu(float v) { return v > 0.f ? v : __expf(v) - 1.f; }

// vmcnt = glds per stage per wave (PER) x stages still allowed in flight
template <int PER>
__device__ __forceinline__ void wait_ahead(int ahead) {
  if (PER == 8) {
    if (ahead >= 2) __asm__ volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (ahead >= 1) __asm__ volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {  // PER == 6
    if (ahead >= 2) __asm__ volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (ahead >= 1) __asm__ volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

template <int BM, int NS>
__global__ __launch_bounds__(BM * 2, 1) void ring_fwd(const float* __restrict__ A, int64_t lda, const float* __restrict__ B,
                                                  int64_t ldb, const float* __restrict__ bias, float* __restrict__ C,
                                                  int64_t ldc, int M, int N, int K) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tiles_n = (N + BN - 1) / BN, tiles = ((M + BM - 1) / BM) * tiles_n;
  const int per = (tiles + 7) / 8;
  const int L = (blockIdx.x & 7) * per + (blockIdx.x >> 3);  // XCD-contiguous tiles
  if (L >= tiles) return;
  const int m0 = (L / tiles_n) * BM, n0 = (L % tiles_n) * BN;
  constexpr int WAVES = BM / 32, WM = BM / 64;  // waves WM (rows) x 2 (cols) of 64 x 64
  constexpr int IMGA = BM * BK * 4, SLOT = IMGA + IMGB, PER = BM / 8 / WAVES + 16 / WAVES;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave % WM) * 64, wn = (wave / WM) * 64;
  const int nsteps = (K + BK - 1) / BK;
  auto stage = [&](int s) {
    char* slot = lds + (s % NS) * SLOT;
    stage_img<BM / 8, WAVES>(A, lda, m0, M, s * BK, K, slot, wave, lane);
    stage_img<16, WAVES>(B, ldb, n0, N, s * BK, K, slot + IMGA, wave, lane);
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nsteps) stage(s);
  for (int s = 0; s < nsteps; ++s) {
    wait_ahead<PER>(min(nsteps - 1, s + NS - 2) - s);
    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + NS - 1 < nsteps) stage(s + NS - 1);  // the slot everyone finished reading last step
    const char* slot = lds + (s % NS) * SLOT;
    const bool tail = (s + 1) * BK > K;
    const int kq = s * BK + 8 * fq;  // this lane's first k
    auto frag = [&](const char* img, int row, bf16x8& lo) {
      const int sw = swz(row);
      f32x4 x0 = *reinterpret_cast<const f32x4*>(img + row * 128 + 16 * ((2 * fq) ^ sw));
      f32x4 x1 = *reinterpret_cast<const f32x4*>(img + row * 128 + 16 * ((2 * fq + 1) ^ sw));
      if (tail) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          x0[j] = kq + j < K ? x0[j] : 0.f;
          x1[j] = kq + 4 + j < K ? x1[j] : 0.f;
        }
      }
      return split8(x0, x1, lo);
    };
    bf16x8 bh[4], bl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bh[j] = frag(slot + IMGA, wn + 16 * j + fr, bl[j]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bf16x8 al;
      const bf16x8 ah = frag(slot, wm + 16 * i + fr, al);
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
}  // namespace gr

template <int BM, int NS>
static int launch(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias, float* C, int64_t ldc,
                  int M, int N, int K, hipStream_t s) {
  const int tiles = ((M + BM - 1) / BM) * ((N + gr::BN - 1) / gr::BN);
  const int grid = (tiles + 7) / 8 * 8;
  const size_t lds = (size_t)NS * (BM * gr::BK * 4 + gr::IMGB);
  static bool a = false;
  if (!a) {
    (void)hipFuncSetAttribute((const void*)&gr::ring_fwd<BM, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    a = true;
  }
  hipLaunchKernelGGL((gr::ring_fwd<BM, NS>), dim3(grid), dim3(BM * 2), lds, s, A, lda, B, ldb, bias, C, ldc, M, N, K);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// variant: 0 = 128x128 tile NS 3, 1 = 128x128 NS 4, 2 = 256x128 (8 waves) NS 3
extern "C" int gr_ring_fwd(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias, float* C,
                           int64_t ldc, int M, int N, int K, int variant, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (variant == 0) return launch<128, 3>(A, lda, B, ldb, bias, C, ldc, M, N, K, s);
  if (variant == 1) return launch<128, 4>(A, lda, B, ldb, bias, C, ldc, M, N, K, s);
  if (variant == 2) return launch<256, 3>(A, lda, B, ldb, bias, C, ldc, M, N, K, s);
  return -1;
}
