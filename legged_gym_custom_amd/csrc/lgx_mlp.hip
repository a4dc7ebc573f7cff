// lgx_mlp.hip — fused MLP-layer GEMMs for the rsl_rl learner on gfx950 (include/lgx_mlp.h).
//
// Block: 256 threads = 4 waves, output tile 128 x 64, K step 32. Each wave owns a 64 x 32
// sub-tile = 4 x 2 MFMA tiles of v_mfma_f32_16x16x32_bf16. fp32 operands are split on
// the way into LDS, x = hi + lo (hi = bf16(x), lo = bf16(x - hi)), and every product is
// lo*hi + hi*lo + hi*hi accumulated in fp32 (3 x bf16 MFMA, ~2^-16 relative per product).
//
// Staging goes through registers (the split needs them anyway), so both global layouts
// land in the same LDS image: [row = m or n][k], k contiguous, 80-B row pitch
// (conflict-free ds_read_b128 fragment reads: row r of a 16-lane group hits banks
// 20r mod 64 .. +3). K-contiguous operands: 4 lanes cover one row's 32 k (128 B, float4
// loads when aligned); MN-contiguous operands: consecutive lanes take consecutive rows,
// 8 k each (coalesced 256-B rows per load instruction). Double-buffered LDS, one
// barrier per K step, next tile's global loads in flight during the MFMAs.
//
// Epilogues fuse what the torch graph runs as separate kernels: bias + ELU (forward),
// ELU'(y) of the previous layer (input gradient), split-K partials + the bias gradient
// (column sums of dY) in the weight-gradient pass; a small deterministic reduce adds
// the split-K partials (fixed order, no atomics).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/lgx_mlp.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace lgxm {

constexpr int BM = 128, BKS = 32, NT = 256;
constexpr int PITCH = BKS + 8;           // bf16 per LDS row (80 B)
constexpr int A_ELEMS = BM * PITCH;      // one A image (hi or lo)

struct Params {
  const float* A; int64_t lda;
  const float* B; int64_t ldb;
  float* C; int64_t ldc;
  int M, N, K;
  int epi;
  const float* bias;
  const float* act; int64_t ld_act;
  int split, kchunk;
  int tiles_m, tiles_n, tiles;           // logical tile grid (per split) and total incl. splits
  float* ws;
  float* colsum_ws;
};

// 8 consecutive-k values of one tile row; GUARD = tile crosses an M/N/K edge.
template <bool KCONTIG, bool VEC, bool GUARD>
__device__ __forceinline__ void load8(const float* __restrict__ p, int64_t ld, int row, int rows, int k, int kend,
                                      float v[8]) {
  if (KCONTIG) {
    const float* q = p + (int64_t)row * ld + k;
    if (!GUARD && VEC) {
      const float4 x0 = *reinterpret_cast<const float4*>(q);
      const float4 x1 = *reinterpret_cast<const float4*>(q + 4);
      v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w;
      v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
    } else if (!GUARD) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = q[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (row < rows && k + j < kend) ? q[j] : 0.f;
    }
  } else {
    const float* q = p + (int64_t)k * ld + row;
    if (!GUARD) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = q[(int64_t)j * ld];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (row < rows && k + j < kend) ? q[(int64_t)j * ld] : 0.f;
    }
  }
}

__device__ __forceinline__ void split_store(__bf16* hi, __bf16* lo, int off, const float v[8]) {
  bf16x8 h, l;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 b = (__bf16)v[j];
    h[j] = b;
    l[j] = (__bf16)(v[j] - (float)b);
  }
  *reinterpret_cast<bf16x8*>(hi + off) = h;
  *reinterpret_cast<bf16x8*>(lo + off) = l;
}

// task -> (row, kgroup) of a tile with ROWS rows and 4 k-groups of 8
template <bool KCONTIG, int ROWS>
__device__ __forceinline__ void task_rc(int task, int& r, int& g) {
  if (KCONTIG) { r = task >> 2; g = task & 3; }
  else { r = task % ROWS; g = task / ROWS; }
}

// Block tile BM x BN_ (BN_ = 64: waves 2x2 of 64x32; BN_ = 128: waves 2x2 of 64x64).
template <bool AK, bool BKC, bool VA, bool VB, bool COLSUM, int BN_>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(Params p) {
  constexpr int NJ = BN_ / 32;             // 16-wide MFMA column tiles per wave
  constexpr int BT = BN_ * 32 / 8 / NT;    // B staging tasks per thread
  constexpr int B_ELEMS = BN_ * PITCH;
  constexpr int STAGE = 2 * A_ELEMS + 2 * B_ELEMS;
  extern __shared__ __align__(16) __bf16 lds[];
  // XCD-aware logical tile: hardware spreads consecutive block ids over the 8 XCDs, so
  // give each XCD a contiguous run of logical tiles (n fastest, then m, then split):
  // blocks sharing an A row-block run together on one XCD and hit its L2.
  const int per_xcd = (p.tiles + 7) >> 3;
  const int L = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (L >= p.tiles) return;
  const int tn = L % p.tiles_n;
  const int tm = (L / p.tiles_n) % p.tiles_m;
  const int z = L / (p.tiles_n * p.tiles_m);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = tm * BM, n0 = tn * BN_;
  const int kbeg = z * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nsteps = kend > kbeg ? (kend - kbeg + BKS - 1) / BKS : 0;
  const int wm = (wave & 1) * 64, wn = (wave >> 1) * (BN_ / 2);
  const bool mn_in = (m0 + BM <= p.M) && (n0 + BN_ <= p.N);

  float va[2][8], vb[BT][8];
  float csum = 0.f;
  auto gload = [&](int k0) {
    if (mn_in && k0 + BKS <= kend) {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        int r, g;
        task_rc<AK, BM>(tid + t * NT, r, g);
        load8<AK, VA, false>(p.A, p.lda, m0 + r, p.M, k0 + g * 8, kend, va[t]);
      }
#pragma unroll
      for (int t = 0; t < BT; ++t) {
        int r, g;
        task_rc<BKC, BN_>(tid + t * NT, r, g);
        load8<BKC, VB, false>(p.B, p.ldb, n0 + r, p.N, k0 + g * 8, kend, vb[t]);
      }
    } else {
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        int r, g;
        task_rc<AK, BM>(tid + t * NT, r, g);
        load8<AK, VA, true>(p.A, p.lda, m0 + r, p.M, k0 + g * 8, kend, va[t]);
      }
#pragma unroll
      for (int t = 0; t < BT; ++t) {
        int r, g;
        task_rc<BKC, BN_>(tid + t * NT, r, g);
        load8<BKC, VB, true>(p.B, p.ldb, n0 + r, p.N, k0 + g * 8, kend, vb[t]);
      }
    }
  };
  auto sstore = [&](int buf) {
    __bf16* base = lds + buf * STAGE;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      int r, g;
      task_rc<AK, BM>(tid + t * NT, r, g);
      split_store(base, base + A_ELEMS, r * PITCH + g * 8, va[t]);
      if (COLSUM) {
#pragma unroll
        for (int j = 0; j < 8; ++j) csum += va[t][j];
      }
    }
#pragma unroll
    for (int t = 0; t < BT; ++t) {
      int r, g;
      task_rc<BKC, BN_>(tid + t * NT, r, g);
      split_store(base + 2 * A_ELEMS, base + 2 * A_ELEMS + B_ELEMS, r * PITCH + g * 8, vb[t]);
    }
  };

  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nsteps > 0) {
    gload(kbeg);
    sstore(0);
  }
  __syncthreads();
  const int fr = lane & 15, fk = (lane >> 4) * 8;
  for (int s = 0; s < nsteps; ++s) {
    const int buf = s & 1;
    if (s + 1 < nsteps) gload(kbeg + (s + 1) * BKS);
    const __bf16* base = lds + buf * STAGE;
    const __bf16* ahi = base;
    const __bf16* alo = base + A_ELEMS;
    const __bf16* bhi = base + 2 * A_ELEMS;
    const __bf16* blo = base + 2 * A_ELEMS + B_ELEMS;
    bf16x8 bh[NJ], bl[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int off = (wn + j * 16 + fr) * PITCH + fk;
      bh[j] = *reinterpret_cast<const bf16x8*>(bhi + off);
      bl[j] = *reinterpret_cast<const bf16x8*>(blo + off);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int off = (wm + i * 16 + fr) * PITCH + fk;
      const bf16x8 ah = *reinterpret_cast<const bf16x8*>(ahi + off);
      const bf16x8 al = *reinterpret_cast<const bf16x8*>(alo + off);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[j], acc[i][j], 0, 0, 0);
      }
    }
    if (s + 1 < nsteps) sstore(buf ^ 1);
    __syncthreads();
  }

  // bias gradient partial: this block's A rows summed over its K range (n-tile 0 only)
  if (COLSUM && tn == 0) {
    float* red = reinterpret_cast<float*>(lds);
    red[tid] = csum;
    __syncthreads();
    if (tid < BM) {
      const float v = red[tid] + red[tid + BM];
      if (m0 + tid < p.M) p.colsum_ws[(int64_t)z * p.M + m0 + tid] = v;
    }
  }

  // epilogue: C/D map of 16x16 MFMA tiles: col = lane & 15, row = (lane >> 4) * 4 + r
  const int ec = lane & 15, er = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int n = n0 + wn + j * 16 + ec;
      if (n >= p.N) continue;
      float bn = 0.f;
      if (p.split == 1 && (p.epi & LGX_EPI_BIAS)) bn = p.bias[n];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + i * 16 + er + r;
        if (m >= p.M) continue;
        float v = acc[i][j][r];
        if (p.split > 1) {
          p.ws[((int64_t)z * p.M + m) * p.N + n] = v;
          continue;
        }
        v += bn;
        if (p.epi & LGX_EPI_ELU) v = v > 0.f ? v : expm1f(v);
        if (p.epi & LGX_EPI_DELU) {
          const float y = p.act[(int64_t)m * p.ld_act + n];
          v *= y > 0.f ? 1.f : y + 1.f;
        }
        float* c = p.C + (int64_t)m * p.ldc + n;
        *c = (p.epi & LGX_EPI_ACCUM) ? *c + v : v;
      }
    }
}

// C (=|+=) epilogue(sum_z ws[z]) and colsum[m] = sum_z colsum_ws[z][m], fixed z order.
__global__ void splitk_reduce(Params p, float* colsum) {
  const int64_t mn = (int64_t)p.M * p.N;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < mn) {
    float v = 0.f;
    for (int z = 0; z < p.split; ++z) v += p.ws[z * mn + i];
    const int m = (int)(i / p.N), n = (int)(i % p.N);
    if (p.epi & LGX_EPI_BIAS) v += p.bias[n];
    if (p.epi & LGX_EPI_ELU) v = v > 0.f ? v : expm1f(v);
    if (p.epi & LGX_EPI_DELU) {
      const float y = p.act[(int64_t)m * p.ld_act + n];
      v *= y > 0.f ? 1.f : y + 1.f;
    }
    float* c = p.C + (int64_t)m * p.ldc + n;
    *c = (p.epi & LGX_EPI_ACCUM) ? *c + v : v;
  } else if (colsum != nullptr && i < mn + p.M) {
    const int m = (int)(i - mn);
    float v = 0.f;
    for (int z = 0; z < p.split; ++z) v += p.colsum_ws[(int64_t)z * p.M + m];
    colsum[m] = (p.epi & LGX_EPI_ACCUM) ? colsum[m] + v : v;
  }
}

template <bool AK, bool BKC, bool VA, bool VB, bool CS>
void launch(Params p, int bn, hipStream_t s) {
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (p.N + bn - 1) / bn;
  p.tiles = p.tiles_m * p.tiles_n * p.split;
  const int grid = (p.tiles + 7) / 8 * 8;
  if (bn == 128) {
    const size_t lds = 2 * (2 * A_ELEMS + 2 * 128 * PITCH) * sizeof(__bf16);
    hipLaunchKernelGGL((gemm_kernel<AK, BKC, VA, VB, CS, 128>), dim3(grid), dim3(NT), lds, s, p);
  } else {
    const size_t lds = 2 * (2 * A_ELEMS + 2 * 64 * PITCH) * sizeof(__bf16);
    hipLaunchKernelGGL((gemm_kernel<AK, BKC, VA, VB, CS, 64>), dim3(grid), dim3(NT), lds, s, p);
  }
}

static bool g_attr_set = false;

template <bool AK, bool BKC, bool VA, bool VB, bool CS>
void allow_big_lds() {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_kernel<AK, BKC, VA, VB, CS, 128>),
                      hipFuncAttributeMaxDynamicSharedMemorySize, 2 * (2 * A_ELEMS + 2 * 128 * PITCH) * 2);
}

}  // namespace lgxm

static thread_local char g_err[256] = "";

static int fail(const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return -1;
}

static bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

extern "C" {

int32_t lgx_mlp_abi_version(void) { return LGX_MLP_ABI_VERSION; }

const char* lgx_mlp_last_error(void) { return g_err; }

int32_t lgx_mlp_pick_split(int32_t M, int32_t N, int32_t K) {
  const int bn = N >= 128 ? 128 : 64;
  const int tiles = ((M + lgxm::BM - 1) / lgxm::BM) * ((N + bn - 1) / bn);
  int s = (1024 + tiles - 1) / tiles;           // ~4 blocks per CU over 256 CUs
  const int kmax = (K + 255) / 256;             // keep >= 256 rows of K per split
  if (s > kmax) s = kmax;
  if (s < 1) s = 1;
  if (s > 64) s = 64;
  return s;
}

int32_t lgx_gemm(const lgx_gemm_args* a, void* stream) {
  using namespace lgxm;
  if (!a) return fail("lgx_gemm: null args");
  if (a->M < 0 || a->N < 0 || a->K < 0) return fail("lgx_gemm: negative size");
  if (a->M == 0 || a->N == 0) return 0;
  if (!a->A || !a->B || !a->C) return fail("lgx_gemm: null operand");
  if ((a->epilogue & LGX_EPI_BIAS) && !a->bias) return fail("lgx_gemm: EPI_BIAS without bias");
  if ((a->epilogue & LGX_EPI_DELU) && !a->act) return fail("lgx_gemm: EPI_DELU without act");
  const int split = a->split_k < 1 ? 1 : a->split_k;
  if (split > 1 && !a->workspace) return fail("lgx_gemm: split_k > 1 needs a workspace");
  const bool cs = a->colsum != nullptr;
  if (cs && (a->a_kcontig || !a->colsum_ws)) return fail("lgx_gemm: colsum needs a_kcontig = 0 and colsum_ws");
  if (cs && split == 1) return fail("lgx_gemm: colsum requires split_k > 1");
  if (!g_attr_set) {
    allow_big_lds<true, true, true, true, false>();
    allow_big_lds<true, true, true, false, false>();
    allow_big_lds<true, true, false, true, false>();
    allow_big_lds<true, true, false, false, false>();
    allow_big_lds<true, false, true, false, false>();
    allow_big_lds<true, false, false, false, false>();
    allow_big_lds<false, false, false, false, true>();
    allow_big_lds<false, false, false, false, false>();
    g_attr_set = true;
  }
  Params p;
  p.A = a->A; p.lda = a->lda; p.B = a->B; p.ldb = a->ldb; p.C = a->C; p.ldc = a->ldc;
  p.M = a->M; p.N = a->N; p.K = a->K; p.epi = a->epilogue; p.bias = a->bias; p.act = a->act;
  p.ld_act = a->ld_act; p.split = split;
  p.kchunk = ((a->K + split - 1) / split + BKS - 1) / BKS * BKS;
  if (p.kchunk == 0) p.kchunk = BKS;
  p.ws = a->workspace;
  p.colsum_ws = a->colsum_ws;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int bn = a->N >= 128 ? 128 : 64;
  const bool va = a->a_kcontig && (a->lda % 4 == 0) && aligned16(a->A);
  const bool vb = a->b_kcontig && (a->ldb % 4 == 0) && aligned16(a->B);
  if (a->a_kcontig && a->b_kcontig) {
    if (va && vb) launch<true, true, true, true, false>(p, bn, s);
    else if (va) launch<true, true, true, false, false>(p, bn, s);
    else if (vb) launch<true, true, false, true, false>(p, bn, s);
    else launch<true, true, false, false, false>(p, bn, s);
  } else if (a->a_kcontig && !a->b_kcontig) {
    if (va) launch<true, false, true, false, false>(p, bn, s);
    else launch<true, false, false, false, false>(p, bn, s);
  } else if (!a->a_kcontig && !a->b_kcontig) {
    if (cs) launch<false, false, false, false, true>(p, bn, s);
    else launch<false, false, false, false, false>(p, bn, s);
  } else {
    return fail("lgx_gemm: a_kcontig = 0 with b_kcontig = 1 is not built");
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(hipGetErrorString(e));
  if (split > 1) {
    const int64_t n = (int64_t)a->M * a->N + (cs ? a->M : 0);
    hipLaunchKernelGGL(splitk_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, a->colsum);
    e = hipGetLastError();
    if (e != hipSuccess) return fail(hipGetErrorString(e));
  }
  return 0;
}

}  // extern "C"
