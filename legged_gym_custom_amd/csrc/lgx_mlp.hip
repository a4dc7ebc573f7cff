// lgx_mlp.hip — fused MLP-layer GEMMs for the rsl_rl learner on gfx950 (include/lgx_mlp.h).
//
// Block: 256 threads = 4 waves; output tile 128 x BN (BN = 128: waves 2 x 2 of 64 x 64;
// BN = 64: waves 2 x 2 of 64 x 32); K step 32. Products run on v_mfma_f32_16x16x32_bf16:
// fp32 operands are split on the way into LDS, x = hi + lo (hi = bf16(x), lo = bf16(x - hi)),
// and every product is lo*hi + hi*lo + hi*hi accumulated in fp32 (~2^-16 relative).
//
// Operand staging ("stager" modes) goes through registers — the split needs them anyway —
// so every global layout lands in the same LDS image [row = m or n][k] (k contiguous):
//   KV  k-contiguous rows, 8 consecutive k per lane (two float4 loads)
//   MV  m/n-contiguous, float4 along m/n: a lane loads a 4-row x (ROWS/32)-k block
// Vector loads need only 4-B alignment (global_load_dwordx4 on gfx950), so odd leading
// dimensions (the actor's 627-wide input) stay vectorised. The LDS image has 64-B rows
// (32 bf16) with rows and 16-B chunks swizzled (lds_off) so that the fragment reads
// (ds_read_b128), the KV stores (ds_write_b128) and the MV stores (ds_write_b64/_b32) are
// all conflict-free under the gfx950 bank rules (MI355X_MICROARCH.md §LDS).
// Pipeline: double-buffered LDS; two register sets, so a K step's global loads are
// issued two steps before they are staged; one barrier per step.
// Grid: 1-D, XCD-aware — each XCD gets a contiguous run of logical tiles (n fastest),
// so blocks sharing an A row-block run together on one XCD's L2.
// Epilogue through an fp32 LDS image of the tile, then row-contiguous float4 traffic:
//   forward   + bias, ELU                    input grad  * ELU'(y_prev) (y_prev prefetched)
//   weight grad split-K partials to a workspace + the bias gradient (column sums of dY,
//   taken from the unsplit fp32 values), reduced in fixed order by splitk_reduce.
#include <hip/hip_runtime.h>
#include "lgx_knobs.h"
#include <algorithm>
#include <limits.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../include/lgx_mlp.h"
#include "lgx_device.h"  // philox4x32_10 / u01: the env's counter RNG (the act head's noise)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace lgxm {

constexpr int BM = 128, BKS = 32, NT = 256;
#ifndef LGX_PF
#define LGX_PF 2
#endif
#ifndef LGX_PF_DW  // the weight-gradient kind's prefetch depth (dev knob)
#define LGX_PF_DW LGX_PF
#endif
// LGX_PF: global-load register sets (prefetch depth in K steps), gemm_tile's PF (3 measured
// slower for every launch: 246 VGPRs in the weight-gradient tile)
constexpr int PITCH = BKS;               // bf16 per LDS row (64 B, swizzled: lds_off)
enum Mode { KV = 1, MV = 3, MVE = 4 };  // MVE: MV for a row count that is not a multiple of 4

typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));  // 4-B aligned float4

// bf16 offset of 16-B chunk c (0..3) of row r in an LDS image: adjacent rows swap when
// bit 2 of r is set, and the chunk index is XORed with (b3, b3 ^ b4) of the physical row.
// Found by exhaustive search over XOR swizzles (bank model of MI355X_MICROARCH.md §LDS):
// the fragment reads (ds_read_b128) and the k-contiguous stores (ds_write_b128) are
// conflict-free, the m/n-contiguous stores (ds_write_b64 / _b32, lane-contiguous rows)
// 2-way (the old swizzle: 4-way).
__device__ __forceinline__ int lds_off(int r, int c) {
  const int pr = r ^ ((r >> 2) & 1);
  const int b3 = (pr >> 3) & 1, b4 = (pr >> 4) & 1;
  return pr * PITCH + 8 * (c ^ (b3 | ((b3 ^ b4) << 1)));
}

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
  int ws_vec;                            // N % 4 == 0 (float4 runs of the flat workspace)
};

__device__ __forceinline__ void split8(const float* v, bf16x8& h, bf16x8& l) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 b = (__bf16)v[j];
    h[j] = b;
    l[j] = (__bf16)(v[j] - (float)b);
  }
}

// Staging of one operand tile [ROWS][BKS] by NTH threads — R = ROWS * BKS / NTH floats per thread
// (256 threads: ROWS / 8).
template <int MODE, int ROWS, int NTH = NT>
struct Stager {
  static constexpr int R = ROWS * BKS / NTH;
  static constexpr int T = 4 * ROWS / NTH;     // 8-k tasks per thread (KV)
  static constexpr int KG = ROWS * BKS / (4 * NTH);  // k per thread (MV)
  static constexpr int NKQ = BKS / KG;         // k groups per step (MV): 8 or 16
  static_assert(T >= 1 && KG >= 2, "tile too small for the thread count");
  // MV thread map: rg = tid % NRG (4-row group), kq = tid / NRG (k group): consecutive lanes
  // read consecutive 16 B of one source row (k), so a wave's load is 2 (ROWS 128) or 4 (ROWS 64)
  // fully contiguous row segments — the texture path coalesces it (round 1's kq-fastest map
  // covered NKQ source rows x 64 B per load: 4x the L1 accesses, measured).
  static constexpr int NRG = ROWS / 4;
  __device__ __forceinline__ static int mv_kq(int tid) { return tid / NRG; }
  __device__ __forceinline__ static int mv_rg(int tid) { return tid % NRG; }

  // Rows past the M/N edge are clamped to a valid row (their products only reach outputs
  // that are never stored), so loads stay vectorised at the edges; KGUARD (the last,
  // partial K step of a split) zero-fills k >= kend, which does reach valid outputs.
  template <bool KGUARD>
  __device__ __forceinline__ static void load(const float* __restrict__ p, int64_t ld, int row0, int rows, int k0,
                                              int kend, int tid, float (&v)[R]) {
    if (MODE == KV) {
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const int idx = tid + t * NTH, r = idx >> 2, g = idx & 3;
        const int row = min(row0 + r, rows - 1), k = k0 + g * 8;
        const float* q = p + (int64_t)row * ld + k;
        float* o = v + t * 8;
        if (!KGUARD || k + 8 <= kend) {  // whole 8-k chunk inside the K range: vector loads
          const f32x4u x0 = *reinterpret_cast<const f32x4u*>(q);
          const f32x4u x1 = *reinterpret_cast<const f32x4u*>(q + 4);
          o[0] = x0.x; o[1] = x0.y; o[2] = x0.z; o[3] = x0.w;
          o[4] = x1.x; o[5] = x1.y; o[6] = x1.z; o[7] = x1.w;
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = k + j < kend ? q[j] : 0.f;
        }
      }
    } else {  // MV / MVE
      const int kq = mv_kq(tid), rg = mv_rg(tid);
      const int k = k0 + kq * KG;
      if (MODE == MV) {
        // rows % 4 == 0 (host), or an interior tile (interior_bits), so a 4-row group is
        // all valid or all past the edge
        const int row = min(row0 + rg * 4, rows - 4);
#pragma unroll
        for (int kk = 0; kk < KG; ++kk) {
          if (!KGUARD || k + kk < kend) {
            const f32x4u x = *reinterpret_cast<const f32x4u*>(p + (int64_t)(k + kk) * ld + row);
            v[kk * 4 + 0] = x.x; v[kk * 4 + 1] = x.y; v[kk * 4 + 2] = x.z; v[kk * 4 + 3] = x.w;
          } else {
            v[kk * 4 + 0] = v[kk * 4 + 1] = v[kk * 4 + 2] = v[kk * 4 + 3] = 0.f;
          }
        }
      } else {  // MVE edge tile: per-row loads, clamped
        const int row = row0 + rg * 4;
#pragma unroll
        for (int kk = 0; kk < KG; ++kk) {
          const float* q = p + (int64_t)(k + kk) * ld;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[kk * 4 + e] = (!KGUARD || k + kk < kend) ? q[min(row + e, rows - 1)] : 0.f;
        }
      }
    }
  }

  // The staging store in PARTS independent pieces (KV: one 8-k task; MV: one of the 4 rows
  // of the thread's 4-row group), so they can be spread between the MFMAs of a K step.
  static constexpr int PARTS = MODE == KV ? T : 4;
  __device__ __forceinline__ static void store_part(__bf16* hi, __bf16* lo, int tid, const float (&v)[R], int q) {
    if (MODE == KV) {
      const int t = q;
      const int idx = tid + t * NTH, r = idx >> 2, g = idx & 3;
      bf16x8 h, l;
      split8(v + t * 8, h, l);
      const int off = lds_off(r, g);
      *reinterpret_cast<bf16x8*>(hi + off) = h;
      *reinterpret_cast<bf16x8*>(lo + off) = l;
    } else {
      const int kq = mv_kq(tid), rg = mv_rg(tid);
      const int kb = kq * KG;  // first k of this thread inside the step
      const int e = q;
      const int off = lds_off(rg * 4 + e, kb >> 3) + (kb & 7);
      if (KG == 4) {
        bf16x4 h, l;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const float x = v[kk * 4 + e];
          const __bf16 b = (__bf16)x;
          h[kk] = b;
          l[kk] = (__bf16)(x - (float)b);
        }
        *reinterpret_cast<bf16x4*>(hi + off) = h;
        *reinterpret_cast<bf16x4*>(lo + off) = l;
      } else {
        bf16x2 h, l;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const float x = v[kk * 4 + e];
          const __bf16 b = (__bf16)x;
          h[kk] = b;
          l[kk] = (__bf16)(x - (float)b);
        }
        *reinterpret_cast<bf16x2*>(hi + off) = h;
        *reinterpret_cast<bf16x2*>(lo + off) = l;
      }
    }
  }

  __device__ __forceinline__ static void store(__bf16* hi, __bf16* lo, int tid, const float (&v)[R]) {
#pragma unroll
    for (int q = 0; q < PARTS; ++q) store_part(hi, lo, tid, v, q);
  }

  // Row sums of the A tile (bias gradient), MV/MVE only: rows 4*rg + e, slot kq.
  __device__ __forceinline__ static void colsum(const float (&v)[R], float (&cs)[4]) {
#pragma unroll
    for (int kk = 0; kk < KG; ++kk)
#pragma unroll
      for (int e = 0; e < 4; ++e) cs[e] += v[kk * 4 + e];
  }
};

// ELU(alpha = 1): v > 0 ? v : expm1(v), branch-free. expm1 on v <= 0: a degree-8 Taylor
// polynomial for v > -0.5 (truncation < 1.2e-8 relative), exp(v) - 1 below (v_exp_f32;
// within ~3 ulp of expm1f at the switch, < 1 ulp past v = -1).
__device__ __forceinline__ float elu(float v) {
  float q = fmaf(v, 1.f / 40320.f, 1.f / 5040.f);
  q = fmaf(v, q, 1.f / 720.f);
  q = fmaf(v, q, 1.f / 120.f);
  q = fmaf(v, q, 1.f / 24.f);
  q = fmaf(v, q, 1.f / 6.f);
  q = fmaf(v, q, 0.5f);
  q = fmaf(v, q, 1.f);
  const float small = v * q;
  const float big = __expf(v) - 1.f;
  return v > 0.f ? v : (v > -0.5f ? small : big);
}

// One output tile (logical index L: n fastest, then m, then the K split) of one GEMM.
// BM_ rows x BN_ columns; NW = 4 waves as 2 (rows) x 2 (columns), each BM_/2 x BN_/2, or NW = 8
// as 2 x 4, each BM_/2 x BN_/4 (half the MFMAs and staging per wave: twice the waves in flight
// on the same LDS). BM_ = 64 serves the rollout's 4096-row forward launches (twice the blocks,
// half the work per K step).
template <int AM, int BMODE, bool COLSUM, int BN_, int BM_ = BM, int PF = LGX_PF, int NW = 4>
__device__ __forceinline__ void gemm_tile(const Params& p, const int L) {
  constexpr int NTH = 64 * NW;
  using SA = Stager<AM, BM_, NTH>;
  using SB = Stager<BMODE, BN_, NTH>;
  constexpr int MI = BM_ / 32;             // 16-row MFMA tiles per wave
  constexpr int A_ELEMS = BM_ * PITCH;     // one A image (hi or lo)
  constexpr int NJ = BN_ / (8 * NW);       // 16-wide MFMA column tiles per wave
  constexpr int B_ELEMS = BN_ * PITCH;
  constexpr int STAGE = 2 * A_ELEMS + 2 * B_ELEMS;
  extern __shared__ __align__(16) __bf16 lds[];
  const int tn = L % p.tiles_n;
  const int tm = (L / p.tiles_n) % p.tiles_m;
  const int z = L / (p.tiles_n * p.tiles_m);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = tm * BM_, n0 = tn * BN_;
  const int kbeg = z * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nsteps = kend > kbeg ? (kend - kbeg + BKS - 1) / BKS : 0;
  const int wm = (wave & 1) * (BM_ / 2), wn = (wave >> 1) * (BN_ / (NW / 2));

  float va[PF][SA::R], vb[PF][SB::R];  // PF register sets: loads run PF steps ahead
  float csum[4] = {0.f, 0.f, 0.f, 0.f};
  // The chunk's full K steps run in a straight-line pipeline: their loads are unconditional
  // (a prefetch past the last full step re-reads that step; it is staged into a buffer that is
  // never computed) and unguarded, so hipcc's wait counting sees the same pending loads on
  // every trip and waits only for the older register set (vmcnt(N)) before staging it. With
  // the loads behind `if (step exists)` and guarded/unguarded branches (round 2-3), every
  // staging drained ALL pending loads (vmcnt(0)): one step of latency hiding instead of PF.
  // A partial last step (K chunk % 32 != 0) is loaded guarded (zero-filled k >= kend) and
  // computed once after the loop — the same products in the same order.
  const int nfull = kend > kbeg ? (kend - kbeg) / BKS : 0;
  auto gloadU = [&](float (&va)[SA::R], float (&vb)[SB::R], int t) {
    const int k0 = kbeg + min(t, nfull - 1) * BKS;
    SA::template load<false>(p.A, p.lda, m0, p.M, k0, kend, tid, va);
    SB::template load<false>(p.B, p.ldb, n0, p.N, k0, kend, tid, vb);
  };
  auto sstore = [&](const float (&va)[SA::R], const float (&vb)[SB::R], int buf, bool cs_on) {
    __bf16* base = lds + buf * STAGE;
    SA::store(base, base + A_ELEMS, tid, va);
    SB::store(base + 2 * A_ELEMS, base + 2 * A_ELEMS + B_ELEMS, tid, vb);
    if constexpr (COLSUM) {
      if (cs_on) SA::colsum(va, csum);
    }
  };

  f32x4 acc[MI][NJ];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fc = lane >> 4;
  // MFMAs of one K step on LDS[buf]. (Spreading the next step's staging stores between the
  // MFMA groups, with or without sched_group_barrier / s_setprio, measured the same:
  // tools/gemm_variants.py.)
  auto compute = [&](int buf) {
    const __bf16* base = lds + buf * STAGE;
    const __bf16* ahi = base;
    const __bf16* alo = base + A_ELEMS;
    const __bf16* bhi = base + 2 * A_ELEMS;
    const __bf16* blo = base + 2 * A_ELEMS + B_ELEMS;
    bf16x8 bh[NJ], bl[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int off = lds_off(wn + j * 16 + fr, fc);
      bh[j] = *reinterpret_cast<const bf16x8*>(bhi + off);
      bl[j] = *reinterpret_cast<const bf16x8*>(blo + off);
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int off = lds_off(wm + i * 16 + fr, fc);
      const bf16x8 ah = *reinterpret_cast<const bf16x8*>(ahi + off);
      const bf16x8 al = *reinterpret_cast<const bf16x8*>(alo + off);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[j], acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[j], acc[i][j], 0, 0, 0);
      }
    }
  };
  // full step s: MFMAs on LDS[s&1], then step s+1 (registers loaded PF steps ago) staged into
  // LDS[(s+1)&1] (garbage after the last full step: never computed, kept out of the bias
  // gradient), those registers refilled with step s+1+PF; one barrier.
  auto stepU = [&](int s, float (&ra)[SA::R], float (&rb)[SB::R]) {
    compute(s & 1);
    sstore(ra, rb, (s + 1) & 1, s + 1 < nfull);
    gloadU(ra, rb, s + 1 + PF);
    __syncthreads();
  };

  if (nfull > 0) {
    gloadU(va[0], vb[0], 0);
    sstore(va[0], vb[0], 0, true);
#pragma unroll
    for (int j = 1; j <= PF; ++j) gloadU(va[j % PF], vb[j % PF], j);
  }
  __syncthreads();
  // step s stages register set (s + 1) % PF (step s + 1, loaded PF steps earlier) and refills
  // it with step s + 1 + PF
  int s = 0;
  for (; s + PF <= nfull; s += PF) {
#pragma unroll
    for (int j = 0; j < PF; ++j) stepU(s + j, va[(j + 1) % PF], vb[(j + 1) % PF]);
  }
#pragma unroll
  for (int j = 0; j + 1 < PF; ++j)
    if (s + j < nfull) stepU(s + j, va[(j + 1) % PF], vb[(j + 1) % PF]);
  if (nsteps > nfull) {  // the partial last step, zero-filled past kend
    const int k0 = kbeg + nfull * BKS;
    SA::template load<true>(p.A, p.lda, m0, p.M, k0, kend, tid, va[0]);
    SB::template load<true>(p.B, p.ldb, n0, p.N, k0, kend, tid, vb[0]);
    sstore(va[0], vb[0], nfull & 1, true);
    __syncthreads();
    compute(nfull & 1);
    __syncthreads();
  }

  float* cs = reinterpret_cast<float*>(lds);
  // bias gradient partial: this block's A rows summed over its K range (n-tile 0 only)
  if constexpr (COLSUM) {
    if (tn == 0) {
      static_assert(AM == MV || AM == MVE, "colsum needs the m-contiguous A stager");
      constexpr int SLOTS = SA::NKQ;
      const int kq = SA::mv_kq(tid), rg = SA::mv_rg(tid);
#pragma unroll
      for (int e = 0; e < 4; ++e) cs[kq * BM_ + rg * 4 + e] = csum[e];
      __syncthreads();
      if (tid < BM_) {
        float v = 0.f;
#pragma unroll
        for (int sl = 0; sl < SLOTS; ++sl) v += cs[sl * BM_ + tid];
        if (m0 + tid < p.M) p.colsum_ws[(int64_t)z * p.M + m0 + tid] = v;
      }
    }
    __syncthreads();
  }

  // epilogue through LDS: MFMA C/D map (col = lane & 15, row = (lane >> 4) * 4 + r) into a
  // [BM_][BN_ + 4] fp32 image, then row-contiguous float4 reads/writes of C (and act).
  constexpr int CP = BN_ + 4;
  constexpr int CH = BN_ / 4;              // float4 chunks per row
  constexpr int IT = BM_ * CH / NTH;        // chunks per thread
  const bool part = p.split > 1;
  const bool delu = !part && (p.epi & LGX_EPI_DELU);
  // ELU outputs of the previous layer: issue every load before the tile is even staged
  float4 yv[IT];
  if (delu) {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int idx = tid + it * NTH;
      const int m = m0 + idx / CH, n = n0 + (idx % CH) * 4;
      const float* ap = p.act + (int64_t)m * p.ld_act + n;
      if (m < p.M && n + 4 <= p.N) {
        const f32x4u y = *reinterpret_cast<const f32x4u*>(ap);
        yv[it] = make_float4(y.x, y.y, y.z, y.w);
      } else {
        float y[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) y[e] = (m < p.M && n + e < p.N) ? ap[e] : 0.f;
        yv[it] = make_float4(y[0], y[1], y[2], y[3]);
      }
    }
  }
  const int ec = lane & 15, er = (lane >> 4) * 4;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) cs[(wm + i * 16 + er + r) * CP + wn + j * 16 + ec] = acc[i][j][r];
  __syncthreads();
  float* dst = part ? p.ws + (int64_t)z * p.M * p.N : p.C;
  const int64_t ldd = part ? p.N : p.ldc;

  const bool accum = !part && (p.epi & LGX_EPI_ACCUM);
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = tid + it * NTH;
    const int row = idx / CH, c = (idx % CH) * 4;
    const int m = m0 + row, n = n0 + c;
    if (m >= p.M || n >= p.N) continue;
    const float4 t = *reinterpret_cast<const float4*>(cs + row * CP + c);
    float v[4] = {t.x, t.y, t.z, t.w};
    const bool full = n + 4 <= p.N;
    if (!part) {
      if (p.epi & LGX_EPI_BIAS) {
        if (full) {
          const f32x4u bb = *reinterpret_cast<const f32x4u*>(p.bias + n);
          v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += n + e < p.N ? p.bias[n + e] : 0.f;
        }
      }
      if (p.epi & LGX_EPI_ELU) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = elu(v[e]);
      }
      if (delu) {
        const float y[4] = {yv[it].x, yv[it].y, yv[it].z, yv[it].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] *= y[e] > 0.f ? 1.f : y[e] + 1.f;
      }
    }
    float* d = dst + (int64_t)m * ldd + n;
    if (full) {
      f32x4u o = {v[0], v[1], v[2], v[3]};
      if (accum) o += *reinterpret_cast<const f32x4u*>(d);
      *reinterpret_cast<f32x4u*>(d) = o;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (n + e < p.N) d[e] = accum ? d[e] + v[e] : v[e];
    }
  }
}

// Grid: 1-D, XCD-aware (each XCD gets a contiguous run of logical tiles).
__device__ __forceinline__ int xcd_tile(int tiles) {
  const int per_xcd = (tiles + 7) >> 3;
  return (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
}

// An MVE operand (row count not a multiple of 4) on a tile whose rows all lie inside it takes
// the MV stager (same loads, values and stores): MVE's interior/edge branch would otherwise
// sit inside the K loop's loads, where it breaks hipcc's wait counting (gemm_tile). Bit 0:
// the tile's N rows (B of the input gradient) are interior, bit 1: its M rows.
template <int BM_, int BN_>
__device__ __forceinline__ int interior_bits(const Params& p, int L) {
  const int tn = L % p.tiles_n, tm = (L / p.tiles_n) % p.tiles_m;
  return (tn * BN_ + BN_ <= p.N ? 1 : 0) | (tm * BM_ + BM_ <= p.M ? 2 : 0);
}

template <int AM, int BMODE, bool COLSUM, int BN_>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(Params p) {
  const int L = xcd_tile(p.tiles);
  if (L >= p.tiles) return;
  constexpr int AI = AM == MVE ? MV : AM, BI = BMODE == MVE ? MV : BMODE;  // interior-tile stagers
  const int ib = interior_bits<BM, BN_>(p, L);
  const bool a_in = AM != MVE || (ib & 2), b_in = BMODE != MVE || (ib & 1);
  if (a_in && b_in) gemm_tile<AI, BI, COLSUM, BN_>(p, L);
  else if (a_in) gemm_tile<AI, BMODE, COLSUM, BN_>(p, L);
  else if (b_in) gemm_tile<AM, BI, COLSUM, BN_>(p, L);
  else gemm_tile<AM, BMODE, COLSUM, BN_>(p, L);
}

// ---------------------------------------------------------------- grouped launch
// Independent GEMMs of one kind in ONE launch (lgx_gemm_group). Every problem's logical
// tiles are spread evenly over the 8 XCDs (XCD x runs a contiguous 1/8 of each problem,
// problems in the host's order — longest K chunk first), so the per-XCD work stays
// balanced when the problems' tile costs differ; each block dispatches on its problem's
// stager modes (block-uniform). Kinds: forward (KV, KV), input grad (KV, MV|MVE), weight
// grad with the bias gradient (MV|MVE, MV|MVE, colsum).
constexpr int GMAX = LGX_GEMM_GROUP_MAX;
enum GroupKind { G_FWD = 0, G_DX = 1, G_DW = 2 };
struct GroupParams {
  int n, per_xcd;    // per_xcd: sum over problems of ceil(tiles_i / 8)
  int start[GMAX + 1];  // prefix sums of ceil(tiles_i / 8)
  int mode[GMAX];   // G_DX: B is MVE; G_DW: bit 0 A is MVE, bit 1 B is MVE
  Params p[GMAX];
};
static_assert(sizeof(GroupParams) <= 4096, "kernel argument segment");

// NW = 8 (512-thread blocks, 128 x 128 tiles only): two blocks per CU are 4 waves per SIMD,
// so at most 128 VGPRs (launch bound)
template <int KIND, int BN_, int BM_ = BM, int NW = 4>
__global__ __launch_bounds__(64 * NW, NW == 8 ? 4 : 2) void gemm_group_kernel(GroupParams g) {
  const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
  if (j >= g.per_xcd) return;
  int i = 0;
  while (i + 1 < g.n && j >= g.start[i + 1]) ++i;
  const int l = x * (g.start[i + 1] - g.start[i]) + (j - g.start[i]);
  const int m = g.mode[i];
  // Forward kinds take a register copy of their problem's parameters (the tile loop then
  // reads them from SGPRs, not by a scalar load from the argument segment every K step:
  // forward launches 3-5 % shorter); the weight-gradient tile measured 14 % slower with
  // the copy (more SGPRs live across its loop), so it keeps the reference.
  if constexpr (KIND == G_FWD) {
    const Params p = g.p[i];
    if (l >= p.tiles) return;
    gemm_tile<KV, KV, false, BN_, BM_, LGX_PF, NW>(p, l);
  } else if constexpr (KIND == G_DX) {
    const Params p = g.p[i];
    if (l >= p.tiles) return;
    if (m & ~interior_bits<BM_, BN_>(p, l)) gemm_tile<KV, MVE, false, BN_, BM_, LGX_PF, NW>(p, l);
    else gemm_tile<KV, MV, false, BN_, BM_, LGX_PF, NW>(p, l);
  } else {
    const Params& p = g.p[i];
    if (l >= p.tiles) return;
    const int ib = interior_bits<BM, BN_>(p, l);
    const int e = m & ~((ib >> 1) | ((ib & 1) << 1));  // mode bit 0: A (M rows), bit 1: B (N rows)
    if (e == 0) gemm_tile<MV, MV, true, BN_, BM, LGX_PF_DW, NW>(p, l);
    else if (e == 1) gemm_tile<MVE, MV, true, BN_, BM, LGX_PF_DW, NW>(p, l);
    else if (e == 2) gemm_tile<MV, MVE, true, BN_, BM, LGX_PF_DW, NW>(p, l);
    else gemm_tile<MVE, MVE, true, BN_, BM, LGX_PF_DW, NW>(p, l);
  }
}

// ---------------------------------------------------------------- chain launch (lgx_chain)
// The narrow tail layers of up to LGX_CHAIN_MAX chains in one launch. A block owns BR rows of
// one chain and 4 waves; the activations between layers never leave the CU: the chain input's
// rows are split once into an LDS image (bf16 hi | lo planes, [BR][IP], zero past K, pitch
// IP = width + 8 bf16: fragment reads conflict-free); every layer reads its A fragments from
// the image and, after a barrier, overwrites it with its own output, split (fp32 copies go to
// HBM: the backward pass and the next launch read them). B fragments (weight rows,
// k-contiguous, L2-resident) go straight from global memory into registers, two K steps
// ahead; the next layer's first two steps and the input-gradient epilogue's ELU outputs are
// requested before the current layer's results are written, so their latency overlaps it.
// Wave w owns the 16-wide output column tiles w, w + 4, ... (NJW of them) for all BR/16 row
// tiles. Per output the MFMA sequence is gemm_tile's (32-deep K steps in order, lo*hi +
// hi*lo + hi*hi, partial last step zero-filled in both operands) and so are the epilogues:
// bit-identical to lgx_gemm.
constexpr int CHMAX = LGX_CHAIN_MAX, CHMAXL = LGX_CHAIN_MAXL;
struct ChainParams {
  int n, ip;
  int start[CHMAX + 1];  // prefix sums of the chains' row blocks
  lgx_chain_desc c[CHMAX];
};
static_assert(sizeof(ChainParams) <= 4096, "kernel argument segment");

// B fragment of tile t at K step s of layer L: W row n = 16 j + fr (clamped: a tile past N
// computes nothing that is stored), k = 32 s + 8 fc .. + 8; past K (a partial step): zero,
// from clamped addresses
template <int NJW>
__device__ __forceinline__ void chain_bload(const lgx_chain_layer& L, int s, int wave, int fr, int fc,
                                            float (&b)[NJW][8]) {
  const int k = s * BKS + fc * 8;
#pragma unroll
  for (int t = 0; t < NJW; ++t) {
    const int n = min((wave + 4 * t) * 16 + fr, L.N - 1);
    const float* row = L.B + n * (int)L.ldb;  // 32-bit lane offsets from a uniform base
    if ((s + 1) * BKS <= L.K) {  // wave-uniform
      const f32x4u x0 = *reinterpret_cast<const f32x4u*>(row + k);
      const f32x4u x1 = *reinterpret_cast<const f32x4u*>(row + k + 4);
      b[t][0] = x0.x; b[t][1] = x0.y; b[t][2] = x0.z; b[t][3] = x0.w;
      b[t][4] = x1.x; b[t][5] = x1.y; b[t][6] = x1.z; b[t][7] = x1.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = row[min(k + j, L.K - 1)];
        b[t][j] = k + j < L.K ? x : 0.f;
      }
    }
  }
}

template <int BR, int NJW>
__global__ __launch_bounds__(NT, 2) void chain_kernel(ChainParams P) {
  constexpr int MI = BR / 16;
  extern __shared__ __align__(16) __bf16 lds[];
  const int ip = P.ip;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fc = lane >> 4;
  const int blk = blockIdx.x;
  if (blk >= P.start[P.n]) return;
  int ci = 0;
  while (ci + 1 < P.n && blk >= P.start[ci + 1]) ++ci;
  const lgx_chain_desc& c = P.c[ci];
  const int rows = c.rows, r0 = (blk - P.start[ci]) * BR;
  __bf16* ih = lds;            // image planes [BR][ip]
  __bf16* il = lds + BR * ip;

  float b0[NJW][8], b1[NJW][8];  // B register sets: K steps s (b0) and s + 1 (b1)
  {
    const lgx_chain_layer& L0 = c.layers[0];
    const int ns = (L0.K + BKS - 1) / BKS;
    chain_bload<NJW>(L0, 0, wave, fr, fc, b0);
    chain_bload<NJW>(L0, min(1, ns - 1), wave, fr, fc, b1);
    // the chain input's rows (clamped at the edge, as gemm_tile) -> the image, zero past K
    const int K = L0.K, c8 = ns * 4;
    const float* a0 = c.A + (int64_t)r0 * c.lda;
    for (int idx = tid; idx < BR * c8; idx += NT) {
      const int r = idx / c8, k = (idx % c8) * 8;
      const float* q = a0 + (min(r0 + r, rows - 1) - r0) * (int)c.lda + k;
      float v[8];
      if (k + 8 <= K) {
        const f32x4u x0 = *reinterpret_cast<const f32x4u*>(q);
        const f32x4u x1 = *reinterpret_cast<const f32x4u*>(q + 4);
        v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = k + j < K ? q[j] : 0.f;
      }
      bf16x8 h, l;
      split8(v, h, l);
      *reinterpret_cast<bf16x8*>(ih + r * ip + k) = h;
      *reinterpret_cast<bf16x8*>(il + r * ip + k) = l;
    }
  }
  __syncthreads();

  for (int li = 0; li < c.nlayers; ++li) {
    const lgx_chain_layer& L = c.layers[li];
    const int K = L.K, N = L.N, ntile = (N + 15) / 16;
    const int nsteps = (K + BKS - 1) / BKS;
    // the input-gradient epilogue's ELU outputs, requested before the K loop
    float yv[MI][NJW][4];
    const int mlast = rows - 1 - r0;  // last valid row of the block (local)
    if (L.epilogue & LGX_EPI_DELU) {
      const float* y0 = L.act + (int64_t)r0 * L.ld_act;
#pragma unroll
      for (int t = 0; t < NJW; ++t) {
        const int n = min((wave + 4 * t) * 16 + fr, N - 1);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) yv[i][t][r] = y0[min(i * 16 + fc * 4 + r, mlast) * (int)L.ld_act + n];
      }
    }
    f32x4 acc[MI][NJW];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int t = 0; t < NJW; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto mma = [&](const float (&b)[NJW][8], int s) {
      bf16x8 bh[NJW], bl[NJW];
#pragma unroll
      for (int t = 0; t < NJW; ++t) split8(b[t], bh[t], bl[t]);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int off = (i * 16 + fr) * ip + s * BKS + fc * 8;
        const bf16x8 ah = *reinterpret_cast<const bf16x8*>(ih + off);
        const bf16x8 al = *reinterpret_cast<const bf16x8*>(il + off);
#pragma unroll
        for (int t = 0; t < NJW; ++t) {
          if (wave + 4 * t < ntile) {  // wave-uniform
            acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[t], acc[i][t], 0, 0, 0);
            acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[t], acc[i][t], 0, 0, 0);
            acc[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[t], acc[i][t], 0, 0, 0);
          }
        }
      }
    };
    // steps s, s + 1 are in b0, b1; each refill requests s + 2 (clamped to the last step)
    int s = 0;
    for (; s + 2 <= nsteps; s += 2) {
      mma(b0, s);
      if (s + 2 < nsteps) chain_bload<NJW>(L, s + 2, wave, fr, fc, b0);
      mma(b1, s + 1);
      if (s + 3 < nsteps) chain_bload<NJW>(L, s + 3, wave, fr, fc, b1);
    }
    if (s < nsteps) mma(b0, s);
    const bool next = li + 1 < c.nlayers;
    if (next) {  // the next layer's first two steps
      const lgx_chain_layer& Ln = c.layers[li + 1];
      const int ns = (Ln.K + BKS - 1) / BKS;
      chain_bload<NJW>(Ln, 0, wave, fr, fc, b0);
      chain_bload<NJW>(Ln, min(1, ns - 1), wave, fr, fc, b1);
    }
    __syncthreads();  // every wave is done reading the image

    // epilogue: lane holds rows 4 fc + r (r < 4) of column fr of each tile
    float* c0 = L.C + (int64_t)r0 * L.ldc;
#pragma unroll
    for (int t = 0; t < NJW; ++t) {
      const int j = wave + 4 * t;
      if (j >= ntile) continue;
      const int n = j * 16 + fr;
      const bool nok = n < N;
      const float bn = (L.epilogue & LGX_EPI_BIAS) && nok ? L.bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ml = i * 16 + fc * 4 + r;
          float v = acc[i][t][r];
          if (L.epilogue & LGX_EPI_BIAS) v += bn;
          if (L.epilogue & LGX_EPI_ELU) v = elu(v);
          if (L.epilogue & LGX_EPI_DELU) {
            const float y = yv[i][t][r];
            v *= y > 0.f ? 1.f : y + 1.f;
          }
          if (!nok) v = 0.f;
          if (nok && ml <= mlast) c0[ml * (int)L.ldc + n] = v;
          if (next) {
            const __bf16 h = (__bf16)v;
            ih[ml * ip + n] = h;
            il[ml * ip + n] = (__bf16)(v - (float)h);
          }
        }
      }
    }
    if (next) {  // zero the image's columns [16 ntile, next K padded to 32)
      const int z0 = ntile * 16, z1 = ((N + 31) / 32) * 32;
      for (int idx = tid; idx < BR * (z1 - z0); idx += NT) {
        const int r = idx / (z1 - z0), k = z0 + idx % (z1 - z0);
        ih[r * ip + k] = (__bf16)0.f;
        il[r * ip + k] = (__bf16)0.f;
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------- adaptation encoder (lgx_adaptation_forward)
// The adaptation encoder's forward without gradient (support_networks.py:116-175: per-position
// Linear(P -> C1) + ELU, Conv1d(C1 -> C2, k1, s1) + ELU, Conv1d(C2 -> C3, k2, s2) + ELU, flatten,
// Linear(L2*C3 -> NO) + ELU) for AR rows per block in ONE launch: only the H history positions the
// convolutions read are formed, every intermediate stays in LDS (fp32, channels-last: position
// t's channels at [t*C + c], so a conv window is one contiguous run) and only the latent goes to
// HBM. Each stage is a GEMM over "virtual rows" (row, output position) whose A row is a window of
// the previous stage; per output the MFMA sequence is gemm_tile's (32-deep K steps in order, fp32
// values split hi/lo as they are read, lo*hi + hi*lo + hi*hi, zero past K) and so is the bias +
// ELU epilogue: bit-identical to the per-layer launches of hip_mlp._AdaptationFn.
constexpr int AR = 16;  // rows per block
struct AdaptParams {
  lgx_adapt_args a;
  int L1, L2;
};

// one GEMM stage: vrows virtual rows, A(v, k) = lda_(v)[k] for k < K (a global or LDS row),
// W [N][K] k-contiguous, epilogue bias + ELU, result to st_(v, n) for n < N
template <class ALoad, class Store>
__device__ __forceinline__ void adapt_stage(int vrows, int K, int N, const float* __restrict__ W,
                                            const float* __restrict__ bias, ALoad lda_, Store st_) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fc = lane >> 4;
  const int nrt = (vrows + 15) / 16, nct = (N + 15) / 16, nsteps = (K + BKS - 1) / BKS;
  for (int item = wave; item < nrt * nct; item += NT / 64) {
    const int rt = item / nct, ct = item % nct;
    const int v = min(rt * 16 + fr, vrows - 1);
    const int n = min(ct * 16 + fr, N - 1);
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const float* arow = lda_(v);
    const float* brow = W + n * K;
    for (int s = 0; s < nsteps; ++s) {
      const int k = s * BKS + fc * 8;
      float av[8], bv[8];
      if (k + 8 <= K) {  // vector loads (4-B alignment suffices for global dwordx4)
        const f32x4u a0 = *reinterpret_cast<const f32x4u*>(arow + k), a1 = *reinterpret_cast<const f32x4u*>(arow + k + 4);
        const f32x4u b0 = *reinterpret_cast<const f32x4u*>(brow + k), b1 = *reinterpret_cast<const f32x4u*>(brow + k + 4);
        av[0] = a0.x; av[1] = a0.y; av[2] = a0.z; av[3] = a0.w; av[4] = a1.x; av[5] = a1.y; av[6] = a1.z; av[7] = a1.w;
        bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w; bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          av[j] = k + j < K ? arow[k + j] : 0.f;
          bv[j] = k + j < K ? brow[k + j] : 0.f;
        }
      }
      bf16x8 ah, al, bh, bl;
      split8(av, ah, al);
      split8(bv, bh, bl);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
    }
    // C/D map: column fr of the tile, rows 4 fc + r
    const int nn = ct * 16 + fr;
    if (nn < N) {
      const float bn = bias[nn];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int vv = rt * 16 + fc * 4 + r;
        if (vv < vrows) st_(vv, nn, elu(acc[r] + bn));
      }
    }
  }
}

__global__ __launch_bounds__(NT) void adapt_fwd_kernel(AdaptParams P) {
  const lgx_adapt_args& a = P.a;
  extern __shared__ __align__(16) float alds[];
  const int r0 = blockIdx.x * AR;
  const int H = a.H, C1 = a.C1, C2 = a.C2, C3 = a.C3, L1 = P.L1, L2 = P.L2;
  float* y0 = alds;                  // [AR][H*C1]
  float* y1 = y0 + AR * H * C1;      // [AR][L1*C2]
  float* y2 = y1 + AR * L1 * C2;     // [AR][L2*C3]
  const int last = a.B - 1 - r0;     // last valid local row
  const float* x0 = a.x + (int64_t)r0 * a.ldx;
  const int ldx = (int)a.ldx, Pn = a.P;
  // per-position Linear(P -> C1) over H positions: virtual row v = (r, t)
  adapt_stage(AR * H, Pn, C1, a.w0, a.b0,
              [&](int v) { return x0 + min(v / H, last) * ldx + (v % H) * Pn; },
              [&](int v, int n, float y) { y0[(v / H) * (H * C1) + (v % H) * C1 + n] = y; });
  __syncthreads();
  // Conv1d(C1 -> C2, k1, s1): window t of row r = y0[r][t*s1*C1 .. + k1*C1)
  adapt_stage(AR * L1, a.k1 * C1, C2, a.w1, a.b1,
              [&](int v) { return (const float*)y0 + (v / L1) * (H * C1) + (v % L1) * a.s1 * C1; },
              [&](int v, int n, float y) { y1[(v / L1) * (L1 * C2) + (v % L1) * C2 + n] = y; });
  __syncthreads();
  adapt_stage(AR * L2, a.k2 * C2, C3, a.w2, a.b2,
              [&](int v) { return (const float*)y1 + (v / L2) * (L1 * C2) + (v % L2) * a.s2 * C2; },
              [&](int v, int n, float y) { y2[(v / L2) * (L2 * C3) + (v % L2) * C3 + n] = y; });
  __syncthreads();
  adapt_stage(AR, L2 * C3, a.NO, a.wf, a.bf, [&](int v) { return (const float*)y2 + v * (L2 * C3); },
              [&](int v, int n, float y) {
                if (v <= last) a.out[(int64_t)(r0 + v) * a.ldo + n] = y;
              });
}

// ---- the adaptation encoder's DAgger minibatch (lgx_adaptation_train) on f32-input MFMA
// (v_mfma_f32_16x16x4_f32: exact f32, each output a k-ordered fmaf chain). A block walks `chunks`
// chunks of ATR = 16 rows with everything in LDS: the forward (4 GEMM stages over virtual rows
// (row, position), each A row a window of the previous stage), the loss rows, and the backward:
// each input gradient as a GEMM per output position over the (position, tap) pairs that reach
// it, times ELU'; each weight gradient as a GEMM over the chunk's virtual rows, accumulated in
// registers across the chunks (each wave owns fixed 16 x 16 tiles; a bias gradient is the tile
// column whose B operand is 1). One partial row per block (flat layout, torch's order) and one
// loss partial. The next chunk's rows are loaded into registers while this one computes.
constexpr int ATR = 16;                                     // rows per chunk (one 16-row tile)
constexpr int AT_W0 = 2, AT_W1 = 4, AT_W2 = 1, AT_WF = 1;  // weight-gradient tiles per wave
constexpr int AT_XPT = 36, AT_TPT = 2, AT_K0 = 16;          // prefetch floats per thread; W0 steps
enum { AL_XS, AL_Y0, AL_Y1, AL_Y2, AL_Y3, AL_TG, AL_W1, AL_W2, AL_WF, AL_BIAS, AL_ONE, AL_END };
struct AdaptTrainParams {
  lgx_adapt_train_args t;
  int L1, L2, NP, chunks;
  int off[9];                     // entry ranges in the flat layout: w0 b0 w1 b1 w2 b2 wf bf | NP
  int Y0P, W1P, W2P, Y2P, C2P, C3P, NOP;  // LDS pitches / padded K extents (floats)
  int lds[AL_END + 1];            // LDS region offsets (floats)
};

__device__ __forceinline__ float elu_d(float y) { return y > 0.f ? 1.f : y + 1.f; }

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// acc += sum_{s < n} A_s B_s: this lane's operands of step s are a[s * as], b[s * bs] (LDS); the
// loads of 8 (then 4) steps are issued before their MFMAs
__device__ __forceinline__ f32x4 mma_run(f32x4 acc, const float* a, int as, const float* b, int bs, int n) {
  int s = 0;
  for (; s + 8 <= n; s += 8) {
    float av[8], bv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { av[j] = a[j * as]; bv[j] = b[j * bs]; }
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = mfma4(av[j], bv[j], acc);
    a += 8 * as; b += 8 * bs;
  }
  if (s + 4 <= n) {
    float av[4], bv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) { av[j] = a[j * as]; bv[j] = b[j * bs]; }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc = mfma4(av[j], bv[j], acc);
    a += 4 * as; b += 4 * bs; s += 4;
  }
  for (; s < n; ++s, a += as, b += bs) acc = mfma4(*a, *b, acc);
  return acc;
}

// forward stage: st(v, n, ELU(sum_k A(v, k) w[n * wp + k] + bias[n])) for v < M, n < N; A(v, k) =
// arow(v)[k], K = 4 * K4 (the weight rows zero past the layer's K)
template <class ARow, class St>
__device__ __forceinline__ void at_fwd(int lane, int wave, int M, int N, int K4, ARow arow, const float* w, int wp,
                                       const float* bias, St st) {
  const int i = lane & 15, g = lane >> 4;
  const int ntn = (N + 15) >> 4, ntiles = ((M + 15) >> 4) * ntn;
  for (int tile = wave; tile < ntiles; tile += NT / 64) {
    const int mt = tile / ntn, nt = tile - mt * ntn;
    const int v = min(mt * 16 + i, M - 1), n = min(nt * 16 + i, N - 1);
    const f32x4 acc = mma_run(f32x4{0.f, 0.f, 0.f, 0.f}, arow(v) + g, 4, w + n * wp + g, 4, K4);
    const int nn = nt * 16 + i;  // C/D map: column i, rows 4 g + q
    if (nn < N) {
      const float bn = bias[nn];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int vv = mt * 16 + 4 * g + q;
        if (vv < M) st(vv, nn, elu(acc[q] + bn));
      }
    }
  }
}

// input-gradient stage, per output position p < npos and column n < N of the 16 rows:
// out(r, p, n) *= ... := (sum_{l < Ls, k = p - l s in [0, ktaps)} sum_c src[r srs + l sps + c]
// w[c wp + k tw + n]) * ELU'(out(r, p, n)), c over 4 * K4 (the weight rows zero past the channels)
template <class Out>
__device__ __forceinline__ void at_dx(int lane, int wave, int npos, int N, int Ls, int s, int ktaps, const float* src,
                                      int srs, int sps, int K4, const float* w, int wp, int tw, Out outp) {
  const int i = lane & 15, g = lane >> 4;
  const int ntn = (N + 15) >> 4;
  for (int tile = wave; tile < npos * ntn; tile += NT / 64) {
    const int p = tile / ntn, nt = tile - p * ntn;
    const int n = min(nt * 16 + i, N - 1);
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int l = 0; l < Ls; ++l) {
      const int k = p - l * s;
      if (k < 0 || k >= ktaps) continue;
      acc = mma_run(acc, src + i * srs + l * sps + g, 4, w + g * wp + k * tw + n, 4 * wp, K4);
    }
    const int nn = nt * 16 + i;
    if (nn < N) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float* o = outp(4 * g + q, p, nn);
        *o = acc[q] * elu_d(*o);
      }
    }
  }
}

// weight-gradient stage: tiles wave + 4 j (j < J) of the M x (nvalid + 1) gradient; column nvalid
// is the bias (B = 1). A(m, step s) = a0[m + s as] with a0 = abase (this lane's k slot) or the
// zero word when the slot is invalid; B(step s, n) = bbase[n + s bs], 1 at n == nvalid, else 0.
template <int J>
__device__ __forceinline__ void at_dw(int lane, int wave, f32x4 (&acc)[J], int M, int nvalid, int nsteps, bool kval,
                                      const float* abase, int as, const float* bbase, int bs, const float* one) {
  const int i = lane & 15;
  const int ntn = (nvalid + 16) >> 4, ntiles = ((M + 15) >> 4) * ntn;
  const float* zero = one + 4;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int tile = wave + (NT / 64) * j;
    if (tile >= ntiles) break;
    const int mt = tile / ntn, nt = tile - mt * ntn;
    const int m = min(mt * 16 + i, M - 1), n = nt * 16 + i;
    const float* a = kval ? abase + m : zero;
    const float* b = kval && n < nvalid ? bbase + n : (n == nvalid ? one : zero);
    acc[j] = mma_run(acc[j], a, kval ? as : 0, b, kval && n < nvalid ? bs : 0, nsteps);
  }
}

// the tiles of at_dw to the block's gradient row: idx(m, n) = flat entry or -1
template <int J, class Idx>
__device__ __forceinline__ void at_dw_store(int lane, int wave, const f32x4 (&acc)[J], int M, int nvalid, float* row,
                                            Idx idx) {
  const int i = lane & 15, g = lane >> 4;
  const int ntn = (nvalid + 16) >> 4, ntiles = ((M + 15) >> 4) * ntn;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int tile = wave + (NT / 64) * j;
    if (tile >= ntiles) break;
    const int mt = tile / ntn, nt = tile - mt * ntn, n = nt * 16 + i;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int m = mt * 16 + 4 * g + q;
      if (m < M && n <= nvalid) {
        const int e = idx(m, n);
        if (e >= 0) row[e] = acc[j][q];
      }
    }
  }
}

__device__ __forceinline__ int at_opq_s(int v) {  // a uniform value the compiler must treat as changed here
  __asm__ volatile("" : "+s"(v));
  return v;
}
__device__ __forceinline__ int at_opq_v(int v) {
  __asm__ volatile("" : "+v"(v));
  return v;
}

// a workgroup barrier over LDS only: the chunk's global prefetch stays in flight across it
// (__syncthreads() waits vmcnt(0) first, which exposed the prefetch at the next barrier)
__device__ __forceinline__ void at_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

#ifdef LGX_ADAPT_CLOCK
__device__ uint32_t* g_adclk = nullptr;
#endif
__global__ __launch_bounds__(NT, 2) void adapt_train_kernel(AdaptTrainParams Q) {
  const lgx_adapt_args& a = Q.t.f;
  extern __shared__ __align__(16) float alds[];
  __shared__ float lrow[ATR];
  const int tid = threadIdx.x, wave0 = __builtin_amdgcn_readfirstlane(tid >> 6);
  const float invB = 1.f / (float)a.B;
#ifdef LGX_ADAPT_CLOCK
  uint64_t ckl = clock64();
  uint32_t ck[16] = {0};
#define ACK(q) do { if (tid == 0) { const uint64_t t_ = clock64(); ck[q] += (uint32_t)(t_ - ckl); ckl = t_; } } while (0)
#else
#define ACK(q) do { } while (0)
#endif
  // prologue: LDS zeroed (pads and K tails read zeros), the weights staged in the LDS layouts
  {
    const int C1 = a.C1, C2 = a.C2, C3 = a.C3, NO = a.NO, k1 = a.k1, k2 = a.k2, L2 = Q.L2;
    for (int e = 4 * tid; e < Q.lds[AL_END]; e += 4 * NT)
      *reinterpret_cast<float4*>(alds + e) = float4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    float* w1l = alds + Q.lds[AL_W1];  // [C2P][W1P]: w1[o][k C1 + c] at k Y0P + c, zero pads
    float* w2l = alds + Q.lds[AL_W2];  // [C3P][W2P]
    float* wfl = alds + Q.lds[AL_WF];  // [NOP][Y2P]
    float* bl = alds + Q.lds[AL_BIAS];  // b0 | b1 | b2 | bf
    for (int e = tid; e < C2 * k1 * C1; e += NT) {
      const int o = e / (k1 * C1), j = e - o * (k1 * C1), k = j / C1, c = j - k * C1;
      w1l[o * Q.W1P + k * Q.Y0P + c] = a.w1[e];
    }
    for (int e = tid; e < C3 * k2 * C2; e += NT) w2l[(e / (k2 * C2)) * Q.W2P + e % (k2 * C2)] = a.w2[e];
    for (int e = tid; e < NO * L2 * C3; e += NT) wfl[(e / (L2 * C3)) * Q.Y2P + e % (L2 * C3)] = a.wf[e];
    for (int e = tid; e < C1 + C2 + C3 + NO; e += NT)
      bl[e] = e < C1 ? a.b0[e] : e < C1 + C2 ? a.b1[e - C1] : e < C1 + C2 + C3 ? a.b2[e - C1 - C2] : a.bf[e - C1 - C2 - C3];
    if (tid < 4) alds[Q.lds[AL_ONE] + tid] = 1.f;  // then 4 zero words
  }
  // W0 fragment of the wave's fc_encoder column tile (wave % ntn0; ntn0 divides 4): k = 4 s + g
  float w0r[AT_K0];
  {
    const int ntn0 = (a.C1 + 15) >> 4, K40 = (a.P + 3) >> 2, lane = tid & 63, g = lane >> 4;
    const int n = min((wave0 % ntn0) * 16 + (lane & 15), a.C1 - 1);
#pragma unroll
    for (int s = 0; s < AT_K0; ++s) w0r[s] = s < K40 && 4 * s + g < a.P ? a.w0[n * a.P + 4 * s + g] : 0.f;
  }
  f32x4 g0[AT_W0], g1[AT_W1], g2[AT_W2], gf[AT_WF];
#pragma unroll
  for (int j = 0; j < AT_W0; ++j) g0[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < AT_W1; ++j) g1[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < AT_W2; ++j) g2[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < AT_WF; ++j) gf[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // a chunk's rows in registers: element e = tid + k NT of its [ATR][H P] block
  float xr[AT_XPT], tr[AT_TPT];
  auto fetch = [&](int r0) {
    const int last = a.B - 1 - r0, HP = a.H * a.P, NO = a.NO;
    int r = tid / HP, c = tid - r * HP;
#pragma unroll
    for (int k = 0; k < AT_XPT; ++k) {
      if (r < ATR) xr[k] = a.x[(int64_t)(r0 + min(r, last)) * a.ldx + c];
      c += NT;
      while (c >= HP) { c -= HP; ++r; }
    }
#pragma unroll
    for (int k = 0; k < AT_TPT; ++k) {
      const int e = tid + k * NT, rr = e / NO;
      if (rr < ATR) tr[k] = Q.t.target[(int64_t)(r0 + min(rr, last)) * Q.t.ldt + (e - rr * NO)];
    }
  };
  float lsum = 0.f;  // wave 0, lanes 4 r: row slot r's loss terms, chunks in order
  if (blockIdx.x * Q.chunks * ATR < a.B) fetch(blockIdx.x * Q.chunks * ATR);
  for (int ch = 0; ch < Q.chunks; ++ch) {
    const int r0 = (blockIdx.x * Q.chunks + ch) * ATR;
    if (r0 >= a.B) break;  // uniform
    // per-chunk opaque copies of the shape and the lane: every stage's addresses are derived
    // here, not hoisted out of the chunk loop (which spilled them)
    const int H = at_opq_s(a.H), P = at_opq_s(a.P), C1 = at_opq_s(a.C1), C2 = at_opq_s(a.C2), C3 = at_opq_s(a.C3);
    const int NO = at_opq_s(a.NO), L1 = at_opq_s(Q.L1), L2 = at_opq_s(Q.L2), k1 = at_opq_s(a.k1);
    const int s1 = at_opq_s(a.s1), k2 = at_opq_s(a.k2), s2 = at_opq_s(a.s2);
    const int Y0P = at_opq_s(Q.Y0P), W1P = at_opq_s(Q.W1P), W2P = at_opq_s(Q.W2P), Y2P = at_opq_s(Q.Y2P);
    const int lane = at_opq_v(tid & 63), wave = at_opq_s(wave0), i = lane & 15, g = lane >> 4, HP = H * P;
    float* xs = alds + at_opq_s(Q.lds[AL_XS]);   // [ATR][H][P]
    float* y0 = alds + at_opq_s(Q.lds[AL_Y0]);   // [ATR][H][Y0P]  (then dpre0)
    float* y1 = alds + at_opq_s(Q.lds[AL_Y1]);   // [ATR][L1][C2]  (then dpre1)
    float* y2 = alds + at_opq_s(Q.lds[AL_Y2]);   // [ATR][Y2P]: (t, c) flatten + zero pad (then dpre2)
    float* y3 = alds + at_opq_s(Q.lds[AL_Y3]);   // [ATR][NO]      (then dpre3)
    float* tg = alds + at_opq_s(Q.lds[AL_TG]);   // [ATR][NO] target rows
    const float* w1l = alds + at_opq_s(Q.lds[AL_W1]);
    const float* w2l = alds + at_opq_s(Q.lds[AL_W2]);
    const float* wfl = alds + at_opq_s(Q.lds[AL_WF]);
    const float* bl = alds + at_opq_s(Q.lds[AL_BIAS]);
    const float* one = alds + at_opq_s(Q.lds[AL_ONE]);
    const int last = a.B - 1 - r0;
    at_bar();  // the previous chunk's last readers of xs / y0 are done (and the weights staged)
#pragma unroll
    for (int k = 0; k < AT_XPT; ++k)
      if (tid + k * NT < ATR * HP) xs[tid + k * NT] = xr[k];
#pragma unroll
    for (int k = 0; k < AT_TPT; ++k)
      if (tid + k * NT < ATR * NO) tg[tid + k * NT] = tr[k];
    if (ch + 1 < Q.chunks && r0 + ATR < a.B) fetch(r0 + ATR);
    at_bar(); ACK(0);
    // fc_encoder per position: y0[v][c], v = (r, t) = r H + t, K = P (W0 from registers)
    {
      const int ntn0 = (C1 + 15) >> 4, K40 = (P + 3) >> 2;
      for (int tile = wave; tile < (ATR * H / 16) * ntn0; tile += NT / 64) {
        const int mt = tile / ntn0, nt = tile - mt * ntn0;
        const float* ap = xs + (mt * 16 + i) * P + g;
        float av[AT_K0];
#pragma unroll
        for (int s = 0; s < AT_K0; ++s)
          if (s < K40) av[s] = ap[4 * s];
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < AT_K0; ++s)
          if (s < K40) acc = mfma4(av[s], w0r[s], acc);
        const int nn = nt * 16 + i;
        if (nn < C1) {
          const float bn = bl[nn];
#pragma unroll
          for (int q = 0; q < 4; ++q) y0[(mt * 16 + 4 * g + q) * Y0P + nn] = elu(acc[q] + bn);
        }
      }
    }
    at_bar(); ACK(1);
    // conv1: y1[(r, l)][o], window of y0 at row r, position l s1 (K = k1 Y0P, pads zero)
    at_fwd(lane, wave, ATR * L1, C2, W1P / 4,
           [&](int v) { return (const float*)y0 + ((v / L1) * H + (v % L1) * s1) * Y0P; }, w1l, W1P, bl + C1,
           [&](int v, int n, float y) { y1[v * C2 + n] = y; });
    at_bar(); ACK(2);
    at_fwd(lane, wave, ATR * L2, C3, W2P / 4,
           [&](int v) { return (const float*)y1 + ((v / L2) * L1 + (v % L2) * s2) * C2; }, w2l, W2P, bl + C1 + C2,
           [&](int v, int n, float y) { y2[(v / L2) * Y2P + (v % L2) * C3 + n] = y; });
    at_bar(); ACK(3);
    at_fwd(lane, wave, ATR, NO, Y2P / 4, [&](int v) { return (const float*)y2 + v * Y2P; }, wfl, Y2P,
           bl + C1 + C2 + C3, [&](int v, int n, float y) {
             y3[v * NO + n] = y;
             if (a.out && v <= last) a.out[(int64_t)(r0 + v) * a.ldo + n] = y;
           });
    at_bar(); ACK(4);
    // loss rows and dpre3 = (y3 - t) / (B ||y3 - t||) * ELU'(y3) (wave 0: 4 lanes per row; rows past B: 0)
    if (wave == 0) {
      const int r = lane >> 2, sub = lane & 3;
      float ss = 0.f;
      for (int j = sub; j < NO; j += 4) {
        const float d = y3[r * NO + j] - tg[r * NO + j];
        ss = fmaf(d, d, ss);
      }
      ss += __shfl_xor(ss, 1);
      ss += __shfl_xor(ss, 2);
      const float nrm = sqrtf(ss);
      const bool ok = r <= last;
      if (ok) lsum += nrm * invB;
      const float kk = ok && nrm > 0.f ? invB / nrm : 0.f;
      for (int j = sub; j < NO; j += 4) {
        const float y = y3[r * NO + j];
        y3[r * NO + j] = kk * (y - tg[r * NO + j]) * elu_d(y);
      }
    }
    at_bar(); ACK(5);
    // fc_final: dW[j][f] += sum_r dpre3[r][j] y2[r][f], K = rows
    at_dw(lane, wave, gf, NO, L2 * C3, ATR / 4, true, y3 + g * NO, 4 * NO, y2 + g * Y2P, 4 * Y2P, one);
    at_bar(); ACK(6);
    at_dx(lane, wave, 1, L2 * C3, 1, 1, 1, y3, NO, 0, at_opq_s(Q.NOP) / 4, wfl, Y2P, 0,
          [&](int r, int, int n) { return y2 + r * Y2P + n; });
    at_bar(); ACK(7);
    // conv2: dW[o][k C2 + c] += sum_{r, l} dpre2[r][l][o] y1[r][l s2 + k][c]; K = (row, l = k slot)
    at_dw(lane, wave, g2, C3, k2 * C2, ATR, g < L2, y2 + g * C3, Y2P, y1 + g * s2 * C2, L1 * C2, one);
    at_bar(); ACK(8);
    at_dx(lane, wave, L1, C2, L2, s2, k2, y2, Y2P, C3, at_opq_s(Q.C3P) / 4, w2l, W2P, C2,
          [&](int r, int p, int n) { return y1 + (r * L1 + p) * C2 + n; });
    at_bar(); ACK(9);
    // conv1: dW[o][k Y0P + c] += sum_{r, l} dpre1[r][l][o] y0[r][l s1 + k][c]
    at_dw(lane, wave, g1, C2, k1 * Y0P, ATR, g < L1, y1 + g * C2, L1 * C2, y0 + g * s1 * Y0P, H * Y0P, one);
    at_bar(); ACK(10);
    at_dx(lane, wave, H, C1, L1, s1, k1, y1, L1 * C2, C2, at_opq_s(Q.C2P) / 4, w1l, W1P, Y0P,
          [&](int r, int p, int n) { return y0 + (r * H + p) * Y0P + n; });
    at_bar(); ACK(11);
    // fc_encoder: dW[c][p] += sum_v dpre0[v][c] x[v][p], K = virtual rows
    at_dw(lane, wave, g0, C1, P, ATR * H / 4, true, y0 + g * Y0P, 4 * Y0P, xs + g * P, 4 * P, one);
    ACK(12);
  }
  {
    const int C1 = a.C1, C2 = a.C2, C3 = a.C3, NO = a.NO, P = a.P, k1 = a.k1, k2 = a.k2, L2 = Q.L2, Y0P = Q.Y0P;
    const int lane = tid & 63;
    float* row = Q.t.gws + (int64_t)blockIdx.x * Q.NP;
    const int* off = Q.off;
    at_dw_store(lane, wave0, g0, C1, P, row, [&](int m, int n) { return n < P ? off[0] + m * P + n : off[1] + m; });
    at_dw_store(lane, wave0, g1, C2, k1 * Y0P, row, [&](int m, int n) {
      if (n == k1 * Y0P) return off[3] + m;
      const int k = n / Y0P, c = n - k * Y0P;
      return c < C1 ? off[2] + m * (C1 * k1) + c * k1 + k : -1;
    });
    at_dw_store(lane, wave0, g2, C3, k2 * C2, row, [&](int m, int n) {
      if (n == k2 * C2) return off[5] + m;
      const int k = n / C2, c = n - k * C2;
      return off[4] + m * (C2 * k2) + c * k2 + k;
    });
    at_dw_store(lane, wave0, gf, NO, L2 * C3, row, [&](int m, int n) {
      if (n == L2 * C3) return off[7] + m;
      const int t = n / C3, c = n - t * C3;
      return off[6] + m * (C3 * L2) + c * L2 + t;
    });
    if (wave0 == 0 && (lane & 3) == 0) lrow[lane >> 2] = lsum;
  }
#ifdef LGX_ADAPT_CLOCK
  if (tid == 0 && g_adclk)
    for (int q = 0; q < 16; ++q) g_adclk[(size_t)blockIdx.x * 16 + q] = ck[q];
#endif
  __syncthreads();
  if (tid == 0) {
    float l = 0.f;
    for (int r = 0; r < ATR; ++r) l += lrow[r];
    Q.t.loss_ws[blockIdx.x] = l;
  }
}

// C (=|+=) epilogue(sum_z ws[z]) and colsum[m] (=|+=) sum_z colsum_ws[z][m]. Each thread owns
// 4 consecutive outputs (float4 when N % 4 == 0) and walks the splits with 4 independent
// accumulators (z mod 4) combined in a fixed order: deterministic, memory-level parallel.
__device__ __forceinline__ float sum_splits(const float* ws, int64_t stride, int split, int64_t i) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int z = 0;
  for (; z + 4 <= split; z += 4) {
    a0 += ws[(z + 0) * stride + i]; a1 += ws[(z + 1) * stride + i];
    a2 += ws[(z + 2) * stride + i]; a3 += ws[(z + 3) * stride + i];
  }
  for (; z < split; ++z) a0 += ws[z * stride + i];
  return (a0 + a1) + (a2 + a3);
}

// One split-K reduction: item t < ceil(M*N/4) sums 4 consecutive outputs (float4 when
// N % 4 == 0) and applies the epilogue; items past that sum one bias-gradient row each.
__device__ __forceinline__ void splitk_item(const float* __restrict__ ws, const float* __restrict__ colsum_ws,
                                            float* C, int64_t ldc, float* colsum, int M, int N, int split, int epi,
                                            const float* bias, const float* act, int64_t ld_act, int64_t t) {
  const int64_t mn = (int64_t)M * N;
  const int64_t nq = (mn + 3) / 4;
  if (t < nq) {
    const int64_t q = t * 4;
    float v[4];
    if (N % 4 == 0) {
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f), b = a, c = a, d = a;
      int z = 0;
      for (; z + 4 <= split; z += 4) {
        const float4 x0 = *reinterpret_cast<const float4*>(ws + (z + 0) * mn + q);
        const float4 x1 = *reinterpret_cast<const float4*>(ws + (z + 1) * mn + q);
        const float4 x2 = *reinterpret_cast<const float4*>(ws + (z + 2) * mn + q);
        const float4 x3 = *reinterpret_cast<const float4*>(ws + (z + 3) * mn + q);
        a.x += x0.x; a.y += x0.y; a.z += x0.z; a.w += x0.w;
        b.x += x1.x; b.y += x1.y; b.z += x1.z; b.w += x1.w;
        c.x += x2.x; c.y += x2.y; c.z += x2.z; c.w += x2.w;
        d.x += x3.x; d.y += x3.y; d.z += x3.z; d.w += x3.w;
      }
      for (; z < split; ++z) {
        const float4 x = *reinterpret_cast<const float4*>(ws + z * mn + q);
        a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
      }
      v[0] = (a.x + b.x) + (c.x + d.x); v[1] = (a.y + b.y) + (c.y + d.y);
      v[2] = (a.z + b.z) + (c.z + d.z); v[3] = (a.w + b.w) + (c.w + d.w);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = q + e < mn ? sum_splits(ws, mn, split, q + e) : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int64_t i = q + e;
      if (i >= mn) break;
      const int m = (int)(i / N), n = (int)(i % N);
      float x = v[e];
      if (epi & LGX_EPI_BIAS) x += bias[n];
      if (epi & LGX_EPI_ELU) x = x > 0.f ? x : expm1f(x);
      if (epi & LGX_EPI_DELU) {
        const float y = act[(int64_t)m * ld_act + n];
        x *= y > 0.f ? 1.f : y + 1.f;
      }
      float* c = C + (int64_t)m * ldc + n;
      *c = (epi & LGX_EPI_ACCUM) ? *c + x : x;
    }
    return;
  }
  const int64_t r = t - nq;  // bias gradient: one row of A
  if (colsum != nullptr && r < M) {
    const float x = sum_splits(colsum_ws, M, split, r);
    colsum[r] = (epi & LGX_EPI_ACCUM) ? colsum[r] + x : x;
  }
}

__global__ void splitk_reduce(Params p, float* colsum) {
  splitk_item(p.ws, p.colsum_ws, p.C, p.ldc, colsum, p.M, p.N, p.split, p.epi, p.bias, p.act, p.ld_act,
              (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

struct SplitkBatch {
  lgx_splitk_desc d[LGX_SPLITK_MAX];
};

// blockIdx.y = entry; blocks stride over the entry's items
__global__ __launch_bounds__(256) void splitk_reduce_batch(SplitkBatch b) {
  const lgx_splitk_desc& d = b.d[blockIdx.y];
  const int64_t items = ((int64_t)d.M * d.N + 3) / 4 + (d.colsum ? d.M : 0);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < items; t += stride)
    splitk_item(d.ws, d.colsum_ws, d.C, d.ldc, d.colsum, d.M, d.N, d.split, d.epilogue & LGX_EPI_ACCUM, nullptr,
                nullptr, 0, t);
}

__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, float b1, float b2, float eps,
                                      float step_size, float bc2s) {
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  p -= step_size * m / (sqrtf(v) / bc2s + eps);
}

struct TransposeBatch {
  lgx_transpose_desc d[LGX_TRANSPOSE_MAX];
};

// blockIdx.z = entry; 32 x 32 tiles through LDS (padded rows), blocks stride over the tiles
__global__ __launch_bounds__(256) void transpose_batch_kernel(TransposeBatch b) {
  __shared__ float tile[32][33];
  const lgx_transpose_desc& d = b.d[blockIdx.z];
  const int tiles_c = (d.cols + 31) / 32, tiles = ((d.rows + 31) / 32) * tiles_c;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int r0 = (t / tiles_c) * 32, c0 = (t % tiles_c) * 32;
#pragma unroll
    for (int k = 0; k < 32; k += 8) {
      const int r = r0 + ty + k, c = c0 + tx;
      tile[ty + k][tx] = (r < d.rows && c < d.cols) ? d.src[(int64_t)r * d.ld + c] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 32; k += 8) {
      const int c = c0 + ty + k, r = r0 + tx;
      if (c < d.cols && r < d.rows) d.dst[(int64_t)c * d.rows + r] = tile[tx][ty + k];
    }
    __syncthreads();
  }
}

// clip_grad_norm_ + Adam over one small flat segment in ONE block (the DAgger step of the
// adaptation encoder, rsl_rl ppo.py:336-345): ||g||_2 in a fixed order (thread partials over a
// stride, then a tree), coef = min(max_norm / (||g|| + 1e-6), 1), g *= coef in place (torch keeps
// the clipped gradient), step += 1, and lgx_adam_step's arithmetic with the clipped gradient.
constexpr int CLIP_ADAM_NT = 1024;
__global__ __launch_bounds__(CLIP_ADAM_NT) void clip_adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                                  float* __restrict__ m, float* __restrict__ v, int n,
                                                                  const float* __restrict__ lr_dev, float lr, float b1,
                                                                  float b2, float eps, float* __restrict__ step,
                                                                  float max_norm, float* __restrict__ coef_out) {
  __shared__ float red[CLIP_ADAM_NT];
  const int tid = threadIdx.x;
  // the step counter and the learning rate are read before the reduction's barriers: thread 0
  // writes *step after its own Adam loop, which a late wave could otherwise already see
  const float t = *step + 1.f;
  const float lr_ = lr_dev ? *lr_dev : lr;
  float ss = 0.f;
  for (int i = tid; i < n; i += CLIP_ADAM_NT) ss = fmaf(g[i], g[i], ss);
  red[tid] = ss;
  __syncthreads();
  for (int w = CLIP_ADAM_NT / 2; w > 0; w >>= 1) {
    if (tid < w) red[tid] += red[tid + w];
    __syncthreads();
  }
  const float coef = fminf(max_norm / (sqrtf(red[0]) + 1e-6f), 1.f);
  const float step_size = lr_ / (1.f - powf(b1, t)), bc2s = sqrtf(1.f - powf(b2, t));
  for (int i = tid; i < n; i += CLIP_ADAM_NT) {
    const float gc = g[i] * coef;
    g[i] = gc;
    float P = p[i], M = m[i], V = v[i];
    adam1(P, gc, M, V, b1, b2, eps, step_size, bc2s);
    p[i] = P;
    m[i] = M;
    v[i] = V;
  }
  if (tid == 0) {
    *step = t;
    if (coef_out) *coef_out = coef;
  }
}

// Adam over a flat fp32 segment: float4 lanes, grid-stride.
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, int64_t n, const float* __restrict__ lr_dev, float lr, float b1,
                            float b2, float eps, const float* __restrict__ step, const float* __restrict__ gscale) {
  const float t = *step;
  const float lr_ = lr_dev ? *lr_dev : lr;
  const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
  const float step_size = lr_ / bc1, bc2s = sqrtf(bc2);
  const float sc = gscale ? *gscale : 1.f;
  const int64_t n4 = n / 4;
  const bool vec = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(m) |
                     reinterpret_cast<uintptr_t>(v)) & 15) == 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (vec) {
    for (int64_t i = i0; i < n4; i += stride) {
      float4 P = reinterpret_cast<float4*>(p)[i], G = reinterpret_cast<const float4*>(g)[i];
      float4 M = reinterpret_cast<float4*>(m)[i], V = reinterpret_cast<float4*>(v)[i];
      adam1(P.x, G.x * sc, M.x, V.x, b1, b2, eps, step_size, bc2s);
      adam1(P.y, G.y * sc, M.y, V.y, b1, b2, eps, step_size, bc2s);
      adam1(P.z, G.z * sc, M.z, V.z, b1, b2, eps, step_size, bc2s);
      adam1(P.w, G.w * sc, M.w, V.w, b1, b2, eps, step_size, bc2s);
      reinterpret_cast<float4*>(p)[i] = P;
      reinterpret_cast<float4*>(m)[i] = M;
      reinterpret_cast<float4*>(v)[i] = V;
    }
    for (int64_t i = n4 * 4 + i0; i < n; i += stride) adam1(p[i], g[i] * sc, m[i], v[i], b1, b2, eps, step_size, bc2s);
  } else {
    for (int64_t i = i0; i < n; i += stride) adam1(p[i], g[i] * sc, m[i], v[i], b1, b2, eps, step_size, bc2s);
  }
}

// ---------------------------------------------------------------- PPO loss head
#ifndef LGX_HT
#define LGX_HT 256
#endif
constexpr int HT = LGX_HT;  // threads per block (rows per block and grid-stride pass)
// the loss heads' cross-wave scratch (red[4 * ...]) holds at most 4 waves
static_assert(HT % 64 == 0 && HT >= 64 && HT <= 256, "LGX_HT: 64..256 threads, whole waves");
// one row per thread (grid-stride loops, so any grid is correct; fewer blocks measured slower)
__host__ __device__ inline unsigned head_grid(int B) { return (unsigned)((B + HT - 1) / HT); }
constexpr int HMAXA = 16;   // max actions

// block-wide sum of NV values per thread into red[NV] (thread 0 holds the result)
template <int NV>
__device__ void block_sum(float (&v)[NV], float* red) {
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float x = v[k];
    for (int o = 32; o > 0; o >>= 1) x += __shfl_down(x, o, 64);
    v[k] = x;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) red[wv * NV + k] = v[k];
  __syncthreads();
  if (threadIdx.x == 0)
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      float t = red[k];
      for (int w = 1; w < (int)(blockDim.x >> 6); ++w) t += red[w * NV + k];  // waves in order
      v[k] = t;
    }
}

// The last block to finish reduces the per-block partials. Thread 0 wrote this block's
// partials: it alone releases them (agent scope) before the counter — an agent-scope fence
// by every thread of every block costs microseconds per block — and the last block's
// threads acquire before they read the other blocks' partials.
__device__ bool last_block(uint32_t* counter, unsigned nblk = 0) {
  __shared__ bool last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(counter, 1u) == (nblk ? nblk : gridDim.x) - 1;
  }
  __syncthreads();
  if (last) __threadfence();
  return last;
}

// Sum of the NV-wide partial rows ws[b * stride + k] over b < nblk, by the whole block: a
// fixed assignment (thread t takes rows t, t + 256, ...) and the fixed block_sum tree, so
// the result is deterministic for a given grid. Thread 0 holds the totals.
template <int NV>
__device__ void final_sum(const float* ws, int stride, int nblk, float (&v)[NV], float* red) {
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = 0.f;
  for (int b = threadIdx.x; b < nblk; b += blockDim.x)
#pragma unroll
    for (int k = 0; k < NV; ++k) v[k] += ws[b * stride + k];
  __syncthreads();  // red is reused
  block_sum<NV>(v, red);
}

struct HeadRow {
  float logp, ratio;
};

// One row's action-wide inputs, loaded up front at clamped columns (columns past A repeat the
// last one and are discarded by selects): no branch around a load, so all of a row's loads
// are in flight together (a guarded or late load is a round trip of its own, ~0.3 us).
template <int NA>
__device__ __forceinline__ void load_cols(const float* __restrict__ x, int i, int A, float (&v)[NA]) {
#pragma unroll
  for (int j = 0; j < NA; ++j) v[j] = x[(int64_t)i * A + min(j, A - 1)];
}

template <int NA>
__device__ __forceinline__ HeadRow head_row(const lgx_ppo_head_args& p, int i, const float* stdv, const float* lstd,
                                            const float (&act)[NA], const float (&mu)[NA]) {
  const float l2pi = 0.9189385332046727f;  // log(sqrt(2 pi))
  float lp = 0.f;
#pragma unroll
  for (int j = 0; j < NA; ++j) {  // same summation order as the reference's sum over actions
    const float d = act[j] - mu[j];
    const float t = -(d * d) / (2.f * stdv[j] * stdv[j]) - lstd[j] - l2pi;
    lp = j < p.A ? lp + t : lp;
  }
  HeadRow r;
  r.logp = lp;
  r.ratio = expf(lp - p.old_logp[i]);
  return r;
}

template <int NA>
__device__ __forceinline__ void ppo_head_fwd_body(const lgx_ppo_head_args& p) {
  __shared__ float red[4 * 4];
  __shared__ float stdv[HMAXA], lstd[HMAXA];
  if (threadIdx.x < HMAXA) {  // columns past A repeat the last one (read by the clamped, discarded terms)
    const float sd = p.std[min((int)threadIdx.x, p.A - 1)];
    stdv[threadIdx.x] = sd;
    lstd[threadIdx.x] = logf(sd);
  }
  __syncthreads();
  float v[3] = {0.f, 0.f, 0.f};
  for (int i = blockIdx.x * HT + threadIdx.x; i < p.B; i += gridDim.x * HT) {
    float act[NA], mu[NA], os[NA], om[NA];
    load_cols(p.actions, i, p.A, act);
    load_cols(p.mu, i, p.A, mu);
    load_cols(p.old_sigma, i, p.A, os);
    load_cols(p.old_mu, i, p.A, om);
    const HeadRow h = head_row<NA>(p, i, stdv, lstd, act, mu);
    const float a = p.adv[i];
    const float s1 = -a * h.ratio, s2 = -a * fminf(fmaxf(h.ratio, 1.f - p.clip), 1.f + p.clip);
    v[0] += fmaxf(s1, s2);
    const float val = p.value[i], R = p.returns[i];
    const float tv = (p.clipped_value ? p.target_values : p.value)[i];  // unconditional load
    if (p.clipped_value) {
      const float vc = tv + fminf(fmaxf(val - tv, -p.clip), p.clip);
      v[1] += fmaxf((val - R) * (val - R), (vc - R) * (vc - R));
    } else {
      v[1] += (R - val) * (R - val);
    }
    float kl = 0.f;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const float dm = om[j] - mu[j];
      const float t = logf(stdv[j] / os[j] + 1.0e-5f) + (os[j] * os[j] + dm * dm) / (2.f * (stdv[j] * stdv[j])) - 0.5f;
      kl = j < p.A ? kl + t : kl;
    }
    v[2] += kl;
  }
  block_sum<3>(v, red);
  if (threadIdx.x == 0)
    for (int k = 0; k < 3; ++k) p.ws[blockIdx.x * 3 + k] = v[k];
  if (last_block(p.counter)) {
    float t[3];
    final_sum<3>(p.ws, 3, gridDim.x, t, red);
    if (threadIdx.x == 0) {
      p.out[0] = t[0] / p.B;
      p.out[1] = t[1] / p.B;
      p.out[3] = t[2] / p.B;
      if (p.kl_dst) *p.kl_dst = t[2] / p.B;
      float ent = 0.f;
      for (int j = 0; j < p.A; ++j) ent += 0.5f + 0.9189385332046727f + lstd[j];
      p.out[2] = ent;
      *p.counter = 0u;
    }
  }
}

template <int NA>
__device__ __forceinline__ void ppo_head_bwd_body(const lgx_ppo_head_args& p) {
  __shared__ float red[4 * HMAXA];
  __shared__ float stdv[HMAXA], lstd[HMAXA];
  if (threadIdx.x < HMAXA) {  // columns past A repeat the last one (read by the clamped, discarded terms)
    const float sd = p.std[min((int)threadIdx.x, p.A - 1)];
    stdv[threadIdx.x] = sd;
    lstd[threadIdx.x] = logf(sd);
  }
  __syncthreads();
  const float gs = p.g[0] / p.B, gv = p.g[1] / p.B, ge = p.g[2];
  float ds[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) ds[j] = 0.f;
  for (int i = blockIdx.x * HT + threadIdx.x; i < p.B; i += gridDim.x * HT) {
    float act[NA], mu[NA];
    load_cols(p.actions, i, p.A, act);
    load_cols(p.mu, i, p.A, mu);
    const HeadRow h = head_row<NA>(p, i, stdv, lstd, act, mu);
    const float a = p.adv[i];
    const float lo = 1.f - p.clip, hi = 1.f + p.clip;
    const float s1 = -a * h.ratio, s2 = -a * fminf(fmaxf(h.ratio, lo), hi);
    // torch.max(s1, s2): ties split evenly; clamp passes on [lo, hi]
    const float w1 = s1 > s2 ? 1.f : (s1 == s2 ? 0.5f : 0.f);
    const float w2 = 1.f - w1;
    const float in = (h.ratio >= lo && h.ratio <= hi) ? 1.f : 0.f;
    const float dratio = gs * (w1 * -a + w2 * -a * in);
    const float dlogp = dratio * h.ratio;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const float d = act[j] - mu[j];
      const float var = stdv[j] * stdv[j];
      if (j < p.A) {
        p.dmu[(int64_t)i * p.A + j] = dlogp * d / var;
        ds[j] += dlogp * (d * d / (var * stdv[j]) - 1.f / stdv[j]);
      }
    }
    const float val = p.value[i], R = p.returns[i];
    const float tv = (p.clipped_value ? p.target_values : p.value)[i];
    float dv;
    if (p.clipped_value) {
      const float vc = tv + fminf(fmaxf(val - tv, -p.clip), p.clip);
      const float l1 = (val - R) * (val - R), l2 = (vc - R) * (vc - R);
      const float u1 = l1 > l2 ? 1.f : (l1 == l2 ? 0.5f : 0.f);
      const float inv = (val - tv >= -p.clip && val - tv <= p.clip) ? 1.f : 0.f;
      dv = gv * (u1 * 2.f * (val - R) + (1.f - u1) * 2.f * (vc - R) * inv);
    } else {
      dv = gv * 2.f * (val - R);
    }
    p.dvalue[i] = dv;
  }
  block_sum<NA>(ds, red);
  if (threadIdx.x == 0)
    for (int j = 0; j < p.A; ++j) p.ws[blockIdx.x * HMAXA + j] = ds[j];
  if (last_block(p.counter)) {
    float t[NA];
    final_sum<NA>(p.ws, HMAXA, gridDim.x, t, red);
    if (threadIdx.x == 0) {
      for (int j = 0; j < p.A; ++j) {  // entropy: d(sum_j log std_j)/d std_j
        const float d = t[j] + ge / stdv[j];
        p.dstd[j] = p.accumulate_dstd ? p.dstd[j] + d : d;
      }
      *p.counter = 0u;
    }
  }
}

// ---------------------------------------------------------------- ROA + estimator losses
// p rows i0 .. i0 + HT - 1, columns [j0, j0 + w) (w <= AUX_CW) staged into st[row][AUX_CW + 1]
// with coalesced loads: p is usually a column span of the actor-input buffer (row stride
// ld_p), where one row per thread would touch a separate cache line per lane and load.
constexpr int AUX_CW = 16;
constexpr int AUX_EU = 8;  // estimator columns per unrolled group
// Every load below is unconditional (row and column clamped into range, the extra values
// discarded by selects or by guarded stores): a load under a branch is a round trip of its
// own, and these kernels are a few dependent round trips long.
__device__ __forceinline__ void aux_stage_p(const lgx_aux_loss_args& p, int64_t ldp, int i0, int j0, int w,
                                            float* st) {
  __syncthreads();
  const int n = HT * w;
  // k / w through a float reciprocal (k < 4096, w <= 16: the product is within 1e-3 of the
  // quotient and 1/32 of the next integer, so floor is exact) — an integer division by a
  // run-time w is ~40 instructions, and one wave per SIMD pays every one of them
  const float rw = 1.f / (float)w;
  float x[AUX_CW];
#pragma unroll
  for (int u = 0; u < AUX_CW; ++u) {
    const int k = min((int)threadIdx.x + HT * u, n - 1);
    const int r = (int)(((float)k + 0.5f) * rw), j = k - r * w;
    x[u] = p.p[(int64_t)min(i0 + r, p.B - 1) * ldp + j0 + j];
  }
#pragma unroll
  for (int u = 0; u < AUX_CW; ++u) {
    const int k = (int)threadIdx.x + HT * u;
    const int r = (int)(((float)k + 0.5f) * rw), j = k - r * w;
    if (k < n) st[r * (AUX_CW + 1) + j] = x[u];
  }
  __syncthreads();
}

// sum_j (p[i, j] - a[i, j])^2 in column order for row i = i0 + threadIdx.x (block-uniform call;
// rows past B return a value of a clamped row, unused)
__device__ __forceinline__ float aux_row_sq(const lgx_aux_loss_args& p, int64_t ldp, int i0, float* st) {
  const int64_t ic = min(i0 + (int)threadIdx.x, p.B - 1);
  float s = 0.f;
  for (int j0 = 0; j0 < p.L; j0 += AUX_CW) {
    const int w = min(AUX_CW, p.L - j0);
    float a[AUX_CW];
#pragma unroll
    for (int j = 0; j < AUX_CW; ++j) a[j] = p.a[ic * p.L + j0 + min(j, w - 1)];
    aux_stage_p(p, ldp, i0, j0, w, st);
#pragma unroll
    for (int j = 0; j < AUX_CW; ++j) {
      const float d = st[threadIdx.x * (AUX_CW + 1) + j] - a[j];
      s = j < w ? s + d * d : s;
    }
  }
  return s;
}

// sum_j (e[i, j] - t[i, j])^2 in column order
__device__ __forceinline__ float aux_est_sq(const lgx_aux_loss_args& p, int64_t i) {
  float q = 0.f;
  for (int j0 = 0; j0 < p.E; j0 += AUX_EU) {
    float e[AUX_EU], t[AUX_EU];
#pragma unroll
    for (int u = 0; u < AUX_EU; ++u) {
      const int64_t c = i * p.E + min(j0 + u, p.E - 1);
      e[u] = p.e[c];
      t[u] = p.t[c];
    }
#pragma unroll
    for (int u = 0; u < AUX_EU; ++u) {
      const float d = e[u] - t[u];
      q = j0 + u < p.E ? q + d * d : q;
    }
  }
  return q;
}

__device__ __forceinline__ void aux_loss_fwd_body(const lgx_aux_loss_args& p) {
  __shared__ float red[4 * 2];
  __shared__ float st[HT * (AUX_CW + 1)];
  float v[2] = {0.f, 0.f};
  const int64_t ldp = p.ld_p > 0 ? p.ld_p : p.L;
  for (int i0 = blockIdx.x * HT; i0 < p.B; i0 += gridDim.x * HT) {
    const float s = aux_row_sq(p, ldp, i0, st);
    const int i = i0 + threadIdx.x;
    const float q = aux_est_sq(p, min(i, p.B - 1));
    if (i >= p.B) continue;
    v[0] += sqrtf(s);
    const float nq = sqrtf(q);  // torch: norm(dim=1).pow(2)
    v[1] += nq * nq;
  }
  block_sum<2>(v, red);
  if (threadIdx.x == 0) { p.ws[blockIdx.x * 2] = v[0]; p.ws[blockIdx.x * 2 + 1] = v[1]; }
  if (last_block(p.counter)) {
    float t[2];
    final_sum<2>(p.ws, 2, gridDim.x, t, red);
    if (threadIdx.x == 0) {
      p.out[0] = t[0] / p.B;
      p.out[1] = t[1] / p.B;
      *p.counter = 0u;
    }
  }
}

__device__ __forceinline__ void aux_loss_bwd_body(const lgx_aux_loss_args& p) {
  __shared__ float st[HT * (AUX_CW + 1)];
  const int i0 = blockIdx.x * HT, i = i0 + threadIdx.x;
  const int64_t ic = min(i, p.B - 1);
  const float gr = p.g[0] / p.B, ge = p.g[1] / p.B;
  const int64_t ldp = p.ld_p > 0 ? p.ld_p : p.L;
  const float n = sqrtf(aux_row_sq(p, ldp, i0, st));
  const float k = n > 0.f ? gr / n : 0.f;
  for (int j0 = 0; j0 < p.L; j0 += AUX_CW) {
    const int w = min(AUX_CW, p.L - j0);
    float a[AUX_CW];
#pragma unroll
    for (int j = 0; j < AUX_CW; ++j) a[j] = p.a[ic * p.L + j0 + min(j, w - 1)];
    aux_stage_p(p, ldp, i0, j0, w, st);
#pragma unroll
    for (int j = 0; j < AUX_CW; ++j)
      if (i < p.B && j < w) p.dp[ic * p.L + j0 + j] = k * (st[threadIdx.x * (AUX_CW + 1) + j] - a[j]);
  }
  for (int j0 = 0; j0 < p.E; j0 += AUX_EU) {
#pragma unroll
    for (int u = 0; u < AUX_EU; ++u) {
      const int64_t c = ic * p.E + min(j0 + u, p.E - 1);
      const float d = ge * 2.f * (p.e[c] - p.t[c]);
      if (i < p.B && j0 + u < p.E) p.de[c] = d;
    }
  }
}

// NA: action columns unrolled (A <= NA; the go2/anymal heads have 12)
template <int NA>
__global__ __launch_bounds__(HT) void ppo_head_fwd(lgx_ppo_head_args p) { ppo_head_fwd_body<NA>(p); }
template <int NA>
__global__ __launch_bounds__(HT) void ppo_head_bwd(lgx_ppo_head_args p) { ppo_head_bwd_body<NA>(p); }
__global__ __launch_bounds__(HT) void aux_loss_fwd(lgx_aux_loss_args p) { aux_loss_fwd_body(p); }
__global__ __launch_bounds__(HT) void aux_loss_bwd(lgx_aux_loss_args p) { aux_loss_bwd_body(p); }
// both heads in one launch: blockIdx.y = 0 the PPO head, 1 the ROA/estimator losses (each
// y-slice is the single-head grid, with its own counter)
template <int NA>
__global__ __launch_bounds__(HT) void loss_heads_fwd(lgx_ppo_head_args h, lgx_aux_loss_args a) {
  if (blockIdx.y == 0) ppo_head_fwd_body<NA>(h);
  else aux_loss_fwd_body(a);
}
template <int NA>
__global__ __launch_bounds__(HT) void loss_heads_bwd(lgx_ppo_head_args h, lgx_aux_loss_args a) {
  if (blockIdx.y == 0) ppo_head_bwd_body<NA>(h);
  else aux_loss_bwd_body(a);
}

// ---- both heads' forward sums AND input gradients in ONE launch (the S8 update): the
// gradients need none of the forward's sums, so one pass over the rows serves both. The
// narrow output gradients (dmu, dvalue, de) are also written in S8 (bf16 hi / lo interleaved
// per 8 columns, lgx_s8.h) with one column-sum partial per block of HT = 256 rows — the
// operands and bias-gradient partials of the update's GEMMs (replaces an lgx_s8_split launch).
__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
  const __bf16 x = (__bf16)a, y = (__bf16)b;
  return (unsigned)__builtin_bit_cast(unsigned short, x) | ((unsigned)__builtin_bit_cast(unsigned short, y) << 16);
}
// 8 fp32 -> one S8 group (32 B: the 8 bf16 hi values, then the 8 bf16 lo = bf16(x - hi))
__device__ __forceinline__ void store_s8_group(char* dst, const float (&v)[8]) {
  float lo[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) lo[e] = v[e] - (float)(__bf16)v[e];
  typedef unsigned u32x4_ __attribute__((ext_vector_type(4)));
  const u32x4_ H = {pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7])};
  const u32x4_ L = {pack_bf16x2(lo[0], lo[1]), pack_bf16x2(lo[2], lo[3]), pack_bf16x2(lo[4], lo[5]),
                    pack_bf16x2(lo[6], lo[7])};
  reinterpret_cast<u32x4_*>(dst)[0] = H;
  reinterpret_cast<u32x4_*>(dst)[1] = L;
}

// One row of the fused PPO head (forward sums into v, input gradients dmu / dv, the S8 / fp32
// gradient rows and the decisions): mu and the value come from the caller (global rows, or the
// fused last layers of lgx_loss_heads_tail).
// A row's inputs of the PPO head besides mu and the value (columns past A repeat the last one)
template <int NA>
struct HeadIn {
  float act[NA], os[NA], om[NA];
  float old_logp, adv, tv, R;
  __device__ __forceinline__ void load(const lgx_ppo_head_args& p, int i) {
    load_cols(p.actions, i, p.A, act);
    load_cols(p.old_sigma, i, p.A, os);
    load_cols(p.old_mu, i, p.A, om);
    old_logp = p.old_logp[i];
    adv = p.adv[i];
    tv = p.clipped_value ? p.target_values[i] : 0.f;
    R = p.returns[i];
  }
};

template <int NA>
__device__ __forceinline__ void head_fused_row(const lgx_ppo_head_args& p, const lgx_heads_s8_args& s, int i,
                                               const float* stdv, const float* lstd, const float (&mu)[NA], float val,
                                               const HeadIn<NA>& x, float gs, float gv, float (&v)[3 + 2 * NA + 1],
                                               float (&dmu)[NA], float& dv) {
  const float(&act)[NA] = x.act;
  const float(&os)[NA] = x.os;
  const float(&om)[NA] = x.om;
  HeadRow h;
  {
    const float l2pi = 0.9189385332046727f;  // log(sqrt(2 pi)); head_row's arithmetic
    float lp = 0.f;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const float d = act[j] - mu[j];
      const float t = -(d * d) / (2.f * stdv[j] * stdv[j]) - lstd[j] - l2pi;
      lp = j < p.A ? lp + t : lp;
    }
    h.logp = lp;
    h.ratio = expf(lp - x.old_logp);
  }
  const float a = x.adv;
  const float lo = 1.f - p.clip, hi = 1.f + p.clip;
  // forward (ppo_head_fwd_body)
  const float s1 = -a * h.ratio, s2 = -a * fminf(fmaxf(h.ratio, lo), hi);
  const float R = x.R;
  const float tv = p.clipped_value ? x.tv : val;
  const float vc = p.clipped_value ? tv + fminf(fmaxf(val - tv, -p.clip), p.clip) : 0.f;
  const float l1 = (val - R) * (val - R), l2 = (vc - R) * (vc - R);
  // the discrete decisions (torch's gradient rules: max splits ties, clamp passes on [lo, hi])
  float w1 = s1 > s2 ? 1.f : (s1 == s2 ? 0.5f : 0.f);
  float in = (h.ratio >= lo && h.ratio <= hi) ? 1.f : 0.f;
  float u1 = l1 > l2 ? 1.f : (l1 == l2 ? 0.5f : 0.f);
  float inv = (val - tv >= -p.clip && val - tv <= p.clip) ? 1.f : 0.f;
  if (s.decisions_out)
    s.decisions_out[i] = (uint8_t)((unsigned)(2.f * w1) | ((unsigned)in << 2) | ((unsigned)(2.f * u1) << 3) |
                                   ((unsigned)inv << 5));
  // a decisions_in byte with bit 6 set leaves the row its own decisions (near-tie-only replays)
  const bool forced = s.decisions_in != nullptr && !(s.decisions_in[i] & 0x40u);
  if (forced) {
    const unsigned d = s.decisions_in[i];
    w1 = 0.5f * (float)(d & 3u);
    in = (float)((d >> 2) & 1u);
    u1 = 0.5f * (float)((d >> 3) & 3u);
    inv = (float)((d >> 5) & 1u);
  }
  if (!forced) {
    v[0] += fmaxf(s1, s2);
    v[1] += p.clipped_value ? fmaxf(l1, l2) : (R - val) * (R - val);
  } else {  // the forced branch's value (a tie: either)
    v[0] += w1 > 0.75f ? s1 : (w1 < 0.25f ? s2 : fmaxf(s1, s2));
    v[1] += p.clipped_value ? (u1 > 0.75f ? l1 : (u1 < 0.25f ? l2 : fmaxf(l1, l2))) : (R - val) * (R - val);
  }
  float kl = 0.f;
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const float dm = om[j] - mu[j];
    const float t = logf(stdv[j] / os[j] + 1.0e-5f) + (os[j] * os[j] + dm * dm) / (2.f * (stdv[j] * stdv[j])) - 0.5f;
    kl = j < p.A ? kl + t : kl;
  }
  v[2] += kl;
  // backward (ppo_head_bwd_body)
  const float w2 = 1.f - w1;
  const float dratio = gs * (w1 * -a + w2 * -a * in);
  const float dlogp = dratio * h.ratio;
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const float d = act[j] - mu[j];
    const float var = stdv[j] * stdv[j];
    dmu[j] = j < p.A ? dlogp * d / var : 0.f;
    if (j < p.A) {
      if (p.dmu) p.dmu[(int64_t)i * p.A + j] = dmu[j];
      v[3 + j] += dlogp * (d * d / (var * stdv[j]) - 1.f / stdv[j]);
      v[3 + NA + j] += dmu[j];
    }
  }
  if (p.clipped_value) {
    dv = gv * (u1 * 2.f * (val - R) + (1.f - u1) * 2.f * (vc - R) * inv);
  } else {
    dv = gv * 2.f * (val - R);
  }
  if (p.dvalue) p.dvalue[i] = dv;
  v[3 + 2 * NA] += dv;
  if (s.dmu_s8) {
#pragma unroll
    for (int g0 = 0; g0 < NA; g0 += 8) {
      if (g0 >= p.A) break;
      float q[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) q[e] = g0 + e < NA ? dmu[g0 + e] : 0.f;
      store_s8_group(static_cast<char*>(s.dmu_s8) + ((int64_t)i * s.ld_dmu + g0) * 4, q);
    }
  }
  if (s.dvalue_s8) {
    const float q[8] = {dv, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    store_s8_group(static_cast<char*>(s.dvalue_s8) + (int64_t)i * s.ld_dvalue * 4, q);
  }
}

// The fused PPO head's block partials (ws, the gradient column sums) and the last block's
// totals: the losses, the KL, the entropy, dstd (one block per grid x-index)
template <int NA>
__device__ __forceinline__ void head_block_finish(const lgx_ppo_head_args& p, const lgx_heads_s8_args& s,
                                                  float (&v)[3 + 2 * NA + 1], float* red, const float* stdv,
                                                  const float* lstd, float ge) {
  constexpr int NV = 3 + 2 * NA + 1;
  block_sum<NV>(v, red);
  if (threadIdx.x == 0) {
    for (int k = 0; k < 3; ++k) p.ws[blockIdx.x * (3 + HMAXA) + k] = v[k];
    for (int j = 0; j < p.A; ++j) p.ws[blockIdx.x * (3 + HMAXA) + 3 + j] = v[3 + j];
    if (s.dmu_cs)
      for (int j = 0; j < p.A; ++j) s.dmu_cs[(int64_t)blockIdx.x * p.A + j] = v[3 + NA + j];
    if (s.dvalue_cs) s.dvalue_cs[blockIdx.x] = v[3 + 2 * NA];
  }
  if (last_block(p.counter)) {
    float t[3 + NA];
    final_sum<3 + NA>(p.ws, 3 + HMAXA, gridDim.x, t, red);
    if (threadIdx.x == 0) {
      p.out[0] = t[0] / p.B;
      p.out[1] = t[1] / p.B;
      p.out[3] = t[2] / p.B;
      if (p.kl_dst) *p.kl_dst = t[2] / p.B;
      float ent = 0.f;
      for (int j = 0; j < p.A; ++j) ent += 0.5f + 0.9189385332046727f + lstd[j];
      p.out[2] = ent;
      for (int j = 0; j < p.A; ++j) {
        const float d = t[3 + j] + ge / stdv[j];
        p.dstd[j] = p.accumulate_dstd ? p.dstd[j] + d : d;
      }
      *p.counter = 0u;
    }
  }
}

template <int NA>
__device__ __forceinline__ void ppo_head_fused_body(const lgx_ppo_head_args& p, const lgx_heads_s8_args& s) {
  constexpr int NV = 3 + 2 * NA + 1;  // forward sums | dstd partial | dmu column sums | dvalue sum
  __shared__ float red[4 * NV];
  __shared__ float stdv[HMAXA], lstd[HMAXA];
  if (threadIdx.x < HMAXA) {
    const float sd = p.std[min((int)threadIdx.x, p.A - 1)];
    stdv[threadIdx.x] = sd;
    lstd[threadIdx.x] = logf(sd);
  }
  __syncthreads();
  const float gs = p.g[0] / p.B, gv = p.g[1] / p.B, ge = p.g[2];
  float v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = 0.f;
  for (int i = blockIdx.x * HT + threadIdx.x; i < p.B; i += gridDim.x * HT) {
    float mu[NA], dmu[NA], dv;
    load_cols(p.mu, i, p.A, mu);
    HeadIn<NA> x;
    x.load(p, i);
    head_fused_row<NA>(p, s, i, stdv, lstd, mu, p.value[i], x, gs, gv, v, dmu, dv);
  }
  head_block_finish<NA>(p, s, v, red, stdv, lstd, ge);
}

// nblk: the blocks that take part (blockIdx.x < nblk; 0: the grid's)
// st: the row staging ([HT][AUX_CW + 1] floats of LDS)
__device__ __forceinline__ void aux_loss_fused_core(const lgx_aux_loss_args& p, const lgx_heads_s8_args& s,
                                                    unsigned nblk, float* st) {
  const unsigned nb = nblk ? nblk : gridDim.x;
  if (blockIdx.x >= nb) return;
  constexpr int NV = 2 + 8;  // forward sums | de column sums (E <= 8 on the S8 path)
  __shared__ float red[4 * NV];
  const int i0 = blockIdx.x * HT, i = i0 + threadIdx.x;
  const int64_t ic = min(i, p.B - 1);
  const float gr = p.g[0] / p.B, ge = p.g[1] / p.B;
  const int64_t ldp = p.ld_p > 0 ? p.ld_p : p.L;
  float v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = 0.f;
  const float n = sqrtf(aux_row_sq(p, ldp, i0, st));
  const float q = aux_est_sq(p, ic);
  if (i < p.B) {
    v[0] = n;
    const float nq = sqrtf(q);  // torch: norm(dim=1).pow(2)
    v[1] = nq * nq;
  }
  const float k = n > 0.f ? gr / n : 0.f;
  for (int j0 = 0; j0 < p.L; j0 += AUX_CW) {
    const int w = min(AUX_CW, p.L - j0);
    float a[AUX_CW];
#pragma unroll
    for (int j = 0; j < AUX_CW; ++j) a[j] = p.a[ic * p.L + j0 + min(j, w - 1)];
    aux_stage_p(p, ldp, i0, j0, w, st);
#pragma unroll
    for (int j = 0; j < AUX_CW; ++j)
      if (i < p.B && j < w) p.dp[ic * p.L + j0 + j] = k * (st[threadIdx.x * (AUX_CW + 1) + j] - a[j]);
  }
  float de[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int64_t c = ic * p.E + min(u, p.E - 1);
    de[u] = u < p.E && i < p.B ? ge * 2.f * (p.e[c] - p.t[c]) : 0.f;
    v[2 + u] = de[u];
  }
  if (i < p.B) {
    if (p.de)
      for (int u = 0; u < p.E; ++u) p.de[ic * p.E + u] = de[u];
    if (s.de_s8) store_s8_group(static_cast<char*>(s.de_s8) + ic * s.ld_de * 4, de);
  }
  block_sum<NV>(v, red);
  if (threadIdx.x == 0) {
    p.ws[blockIdx.x * 2] = v[0];
    p.ws[blockIdx.x * 2 + 1] = v[1];
    if (s.de_cs)
      for (int u = 0; u < p.E; ++u) s.de_cs[(int64_t)blockIdx.x * p.E + u] = v[2 + u];
  }
  if (last_block(p.counter, nb)) {
    float t[2];
    final_sum<2>(p.ws, 2, nb, t, red);
    if (threadIdx.x == 0) {
      p.out[0] = t[0] / p.B;
      p.out[1] = t[1] / p.B;
      *p.counter = 0u;
    }
  }
}

__device__ __forceinline__ void aux_loss_fused_body(const lgx_aux_loss_args& p, const lgx_heads_s8_args& s) {
  __shared__ float st[HT * (AUX_CW + 1)];
  aux_loss_fused_core(p, s, 0, st);
}

template <int NA>
__global__ __launch_bounds__(HT) void loss_heads_fused(lgx_ppo_head_args h, lgx_aux_loss_args a, lgx_heads_s8_args s) {
  if (blockIdx.y == 0) ppo_head_fused_body<NA>(h, s);
  else aux_loss_fused_body(a, s);
}

// ---- the PPO head with the actor's / critic's last layers around it (lgx_loss_heads_tail):
// block = TR rows, 256 threads. LDS (dynamic, floats): the rows' hidden activations y, y_c
// [TR][H + 4] (then, in place, the input gradients dy, dy_c), W [NA][H + 4], W_c [H_c + 4],
// mu [TR][NA], value [TR], dmu [TR][NA], dvalue [TR].
constexpr int TR = LGX_HEADS_TAIL_ROWS;
// per-block phase clocks (dev builds only: -DLGX_TAIL_CLOCK, tools/tail_clock.py): thread 0 of
// every PPO block writes clock64 deltas of its phases to g_tailclk[block][8]
#ifdef LGX_TAIL_CLOCK
__device__ uint32_t* g_tailclk = nullptr;
#define TCK(q) do { if (tid == 0) { const uint64_t t_ = clock64(); ck[q] = (uint32_t)(t_ - ckl); ckl = t_; } } while (0)
#else
#define TCK(q) do { } while (0)
#endif
__host__ __device__ constexpr int tail_pitch(int h) { return h + 4; }
__host__ __device__ inline size_t tail_lds_floats(int NA, int H, int Hc) {
  return (size_t)TR * tail_pitch(H) + (size_t)TR * tail_pitch(Hc) + (size_t)NA * tail_pitch(H) + tail_pitch(Hc) +
         2 * (size_t)TR * NA + 2 * TR;
}

// dot over k < n of two LDS rows (16-B aligned), k in order
__device__ __forceinline__ float lds_dot(const float* x, const float* w, int n) {
  float acc = 0.f;
#pragma unroll 8
  for (int k = 0; k < n; k += 4) {
    const float4 a = *reinterpret_cast<const float4*>(x + k);
    const float4 b = *reinterpret_cast<const float4*>(w + k);
    acc = fmaf(a.x, b.x, acc);
    acc = fmaf(a.y, b.y, acc);
    acc = fmaf(a.z, b.z, acc);
    acc = fmaf(a.w, b.w, acc);
  }
  return acc;
}

template <int NA>
__device__ __forceinline__ void ppo_tail_body(const lgx_ppo_head_args& p, const lgx_heads_s8_args& s,
                                              const lgx_heads_tail_args& t, int bx) {
  constexpr int NV = 3 + 2 * NA + 1;
  extern __shared__ __align__(16) float tl[];
  __shared__ float stdv[HMAXA], lstd[HMAXA];
  // the head rows' inputs (act | old_sigma | old_mu | old_logp adv tv R), later their sums
  __shared__ float hin_[TR * (3 * NA + 4)];
  float(*hin)[3 * NA + 4] = reinterpret_cast<float(*)[3 * NA + 4]>(hin_);
  const int H = t.H, Hc = t.Hc, PH = tail_pitch(H), PC = tail_pitch(Hc), A = p.A;
  float* ys = tl;                   // [TR][PH]
  float* yc = ys + TR * PH;         // [TR][PC]
  float* Ws = yc + TR * PC;         // [NA][PH] (rows past A zero)
  float* Wc = Ws + NA * PH;         // [PC]
  float* mus = Wc + PC;             // [TR][NA]
  float* vals = mus + TR * NA;      // [TR]
  float* dmus = vals + TR;          // [TR][NA] (columns past A zero)
  float* dvs = dmus + TR * NA;      // [TR]
  const int r0 = bx * TR, tid = threadIdx.x;
#ifdef LGX_TAIL_CLOCK
  uint64_t ckl = clock64(), ck0 = ckl;
  uint32_t ck[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  if (tid < HMAXA) {
    const float sd = p.std[min(tid, A - 1)];
    stdv[tid] = sd;
    lstd[tid] = logf(sd);
  }
  // every global input of the block, by all threads: all requests first (registers), then the
  // LDS writes — one memory round trip instead of one per loop
  typedef unsigned u4 __attribute__((ext_vector_type(4)));
  constexpr int YS = TR * 32 / 256;     // S8 groups per thread and network (H <= 256)
  constexpr int WS = HMAXA * 256 / 256;  // weight elements per thread (A <= 16, H <= 256)
  constexpr int IS = TR * (3 * NA + 4) / 256 + 1;
  u4 yh[2][YS], yl[2][YS];
  float wv[WS], wcv, iv[IS];
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const int G = (n ? Hc : H) / 8;
    const char* src = static_cast<const char*>(n ? t.yc : t.y);
    const int64_t ld = n ? t.ld_yc : t.ld_y;
#pragma unroll
    for (int q = 0; q < YS; ++q) {
      const int it = tid + 256 * q, r = it / G, g = it % G;
      const bool ok = it < TR * G && r0 + r < p.B;
      const u4* gp = reinterpret_cast<const u4*>(src + ((int64_t)min(r0 + r, p.B - 1) * ld + 8 * g) * 4);
      yh[n][q] = ok ? gp[0] : u4{0u, 0u, 0u, 0u};
      yl[n][q] = ok ? gp[1] : u4{0u, 0u, 0u, 0u};
    }
  }
#pragma unroll
  for (int q = 0; q < WS; ++q) {
    const int it = tid + 256 * q, a = it / H;
    wv[q] = a < A ? t.W[min(it, A * H - 1)] : 0.f;
  }
  wcv = t.Wc[min(tid, Hc - 1)];
#pragma unroll
  for (int q = 0; q < IS; ++q) {
    const int it = tid + 256 * q, r = it / (3 * NA + 4), c = it % (3 * NA + 4);
    const int i = min(r0 + min(r, TR - 1), p.B - 1);
    float x;
    if (c < 3 * NA) {
      const int qq = c / NA, j = c % NA;
      const float* src = qq == 0 ? p.actions : (qq == 1 ? p.old_sigma : p.old_mu);
      x = src[(int64_t)i * A + min(j, A - 1)];
    } else if (c == 3 * NA) {
      x = p.old_logp[i];
    } else if (c == 3 * NA + 1) {
      x = p.adv[i];
    } else if (c == 3 * NA + 2) {
      x = p.clipped_value ? p.target_values[i] : 0.f;
    } else {
      x = p.returns[i];
    }
    iv[q] = x;
  }
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const int G = (n ? Hc : H) / 8, P = n ? PC : PH;
    float* dst = n ? yc : ys;
#pragma unroll
    for (int q = 0; q < YS; ++q) {
      const int it = tid + 256 * q, r = it / G, g = it % G;
      if (it >= TR * G) continue;
      const u4 Hh = yh[n][q], Ll = yl[n][q];
      *reinterpret_cast<float4*>(dst + r * P + 8 * g) =
          float4{__uint_as_float(Hh[0] << 16) + __uint_as_float(Ll[0] << 16),
                 __uint_as_float(Hh[0] & 0xffff0000u) + __uint_as_float(Ll[0] & 0xffff0000u),
                 __uint_as_float(Hh[1] << 16) + __uint_as_float(Ll[1] << 16),
                 __uint_as_float(Hh[1] & 0xffff0000u) + __uint_as_float(Ll[1] & 0xffff0000u)};
      *reinterpret_cast<float4*>(dst + r * P + 8 * g + 4) =
          float4{__uint_as_float(Hh[2] << 16) + __uint_as_float(Ll[2] << 16),
                 __uint_as_float(Hh[2] & 0xffff0000u) + __uint_as_float(Ll[2] & 0xffff0000u),
                 __uint_as_float(Hh[3] << 16) + __uint_as_float(Ll[3] << 16),
                 __uint_as_float(Hh[3] & 0xffff0000u) + __uint_as_float(Ll[3] & 0xffff0000u)};
    }
  }
#pragma unroll
  for (int q = 0; q < WS; ++q) {
    const int it = tid + 256 * q, a = it / H, k = it % H;
    if (a < NA) Ws[a * PH + k] = wv[q];
  }
  if (tid < Hc) Wc[tid] = wcv;
#pragma unroll
  for (int q = 0; q < IS; ++q) {
    const int it = tid + 256 * q, r = it / (3 * NA + 4), c = it % (3 * NA + 4);
    if (r < TR) hin[r][c] = iv[q];
  }
  __syncthreads();
  TCK(0);
  // the last layers' forward: TR x A actor outputs, then TR values (k in order)
  for (int o = tid; o < TR * A + TR; o += blockDim.x) {
    if (o < TR * A) {
      const int r = o / A, a = o % A;
      const float m = lds_dot(ys + r * PH, Ws + a * PH, H) + t.b[a];
      mus[r * NA + a] = m;
      if (t.mu_out && r0 + r < p.B) t.mu_out[(int64_t)(r0 + r) * A + a] = m;
    } else {
      const int r = o - TR * A;
      const float v = lds_dot(yc + r * PC, Wc, Hc) + t.bc[0];
      vals[r] = v;
      if (t.value_out && r0 + r < p.B) t.value_out[r0 + r] = v;
    }
  }
  __syncthreads();
  TCK(1);
  const float gs = p.g[0] / p.B, gv = p.g[1] / p.B, ge = p.g[2];
  // The PPO head rows (head_fused_row's arithmetic, bit for bit) with the per-action work spread
  // over (row, action) threads: (1) each action's log-prob and KL terms; (2) per row, their sums in
  // action order, the ratio, the clip / max decisions, the value loss and dlogp; (3) each action's
  // dmu and std-gradient term. The row sums are the serial sums of head_fused_row (same order).
  __shared__ float tlp[TR][NA], tkl[TR][NA];  // log-prob / KL terms (then tvs: std-gradient terms)
  __shared__ float rowv[TR][4];                // surrogate, value loss, KL, dlogp
  float(*tvs)[NA] = tlp;                       // the log-prob terms are dead after the row sums
  for (int o = tid; o < TR * NA; o += blockDim.x) {
    const int r = o / NA, j = o % NA;
    const float sd = stdv[j], mu = mus[r * NA + min(j, A - 1)];
    const float d = hin[r][j] - mu;
    tlp[r][j] = -(d * d) / (2.f * sd * sd) - lstd[j] - 0.9189385332046727f;
    const float os = hin[r][NA + j], dm = hin[r][2 * NA + j] - mu;
    tkl[r][j] = logf(sd / os + 1.0e-5f) + (os * os + dm * dm) / (2.f * (sd * sd)) - 0.5f;
  }
  __syncthreads();
  if (tid < TR) {
    const int i = r0 + tid;
    float r4[4] = {0.f, 0.f, 0.f, 0.f}, dv = 0.f;
    if (i < p.B) {
      float lp = 0.f;
#pragma unroll
      for (int j = 0; j < NA; ++j) lp = j < A ? lp + tlp[tid][j] : lp;
      const float ratio = expf(lp - hin[tid][3 * NA]);
      const float a = hin[tid][3 * NA + 1];
      const float lo = 1.f - p.clip, hi = 1.f + p.clip;
      const float s1 = -a * ratio, s2 = -a * fminf(fmaxf(ratio, lo), hi);
      const float R = hin[tid][3 * NA + 3], val = vals[tid];
      const float tv = p.clipped_value ? hin[tid][3 * NA + 2] : val;
      const float vc = p.clipped_value ? tv + fminf(fmaxf(val - tv, -p.clip), p.clip) : 0.f;
      const float l1 = (val - R) * (val - R), l2 = (vc - R) * (vc - R);
      float w1 = s1 > s2 ? 1.f : (s1 == s2 ? 0.5f : 0.f);
      float in = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
      float u1 = l1 > l2 ? 1.f : (l1 == l2 ? 0.5f : 0.f);
      float inv = (val - tv >= -p.clip && val - tv <= p.clip) ? 1.f : 0.f;
      if (s.decisions_out)
        s.decisions_out[i] = (uint8_t)((unsigned)(2.f * w1) | ((unsigned)in << 2) | ((unsigned)(2.f * u1) << 3) |
                                       ((unsigned)inv << 5));
      const bool forced = s.decisions_in != nullptr && !(s.decisions_in[i] & 0x40u);
      if (forced) {
        const unsigned dd = s.decisions_in[i];
        w1 = 0.5f * (float)(dd & 3u);
        in = (float)((dd >> 2) & 1u);
        u1 = 0.5f * (float)((dd >> 3) & 3u);
        inv = (float)((dd >> 5) & 1u);
      }
      if (!forced) {
        r4[0] = 0.f + fmaxf(s1, s2);
        r4[1] = 0.f + (p.clipped_value ? fmaxf(l1, l2) : (R - val) * (R - val));
      } else {
        r4[0] = 0.f + (w1 > 0.75f ? s1 : (w1 < 0.25f ? s2 : fmaxf(s1, s2)));
        r4[1] = 0.f + (p.clipped_value ? (u1 > 0.75f ? l1 : (u1 < 0.25f ? l2 : fmaxf(l1, l2))) : (R - val) * (R - val));
      }
      float kl = 0.f;
#pragma unroll
      for (int j = 0; j < NA; ++j) kl = j < A ? kl + tkl[tid][j] : kl;
      r4[2] = 0.f + kl;
      const float w2 = 1.f - w1;
      const float dratio = gs * (w1 * -a + w2 * -a * in);
      r4[3] = dratio * ratio;  // dlogp
      if (p.clipped_value) dv = gv * (u1 * 2.f * (val - R) + (1.f - u1) * 2.f * (vc - R) * inv);
      else dv = gv * 2.f * (val - R);
      if (p.dvalue) p.dvalue[i] = dv;
      if (s.dvalue_s8) {
        const float q[8] = {dv, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        store_s8_group(static_cast<char*>(s.dvalue_s8) + (int64_t)i * s.ld_dvalue * 4, q);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) rowv[tid][k] = r4[k];
    dvs[tid] = dv;
  }
  __syncthreads();
  for (int o = tid; o < TR * NA; o += blockDim.x) {
    const int r = o / NA, j = o % NA, i = r0 + r;
    float dmu = 0.f, vs = 0.f;
    if (i < p.B && j < A) {
      const float sd = stdv[j], dlogp = rowv[r][3];
      const float d = hin[r][j] - mus[r * NA + j];
      const float var = sd * sd;
      dmu = dlogp * d / var;
      if (p.dmu) p.dmu[(int64_t)i * p.A + j] = dmu;
      vs = 0.f + dlogp * (d * d / (var * sd) - 1.f / sd);
    }
    dmus[r * NA + j] = dmu;
    tvs[r][j] = vs;
  }
  __syncthreads();
  if (s.dmu_s8) {  // the rows' dmu as S8 groups (columns past A zero)
    constexpr int GN = (NA + 7) / 8;
    for (int o = tid; o < TR * GN; o += blockDim.x) {
      const int r = o / GN, g0 = 8 * (o % GN), i = r0 + r;
      if (i >= p.B || g0 >= A) continue;
      float q[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) q[e] = g0 + e < NA ? dmus[r * NA + g0 + e] : 0.f;
      store_s8_group(static_cast<char*>(s.dmu_s8) + ((int64_t)i * s.ld_dmu + g0) * 4, q);
    }
  }
  TCK(2);
  // the last layers' input gradients, in place of y / y_c: (dmu W) * ELU'(y), (dvalue W_c) * ELU'(y_c)
  {
    const int G = H / 8, Gc = Hc / 8;
    for (int it = tid; it < TR * (G + Gc); it += blockDim.x) {
      const bool critic = it >= TR * G;
      const int jt = critic ? it - TR * G : it;
      const int gg = critic ? Gc : G;
      const int r = jt / gg, q = jt % gg;
      float* y = critic ? yc + r * PC + 8 * q : ys + r * PH + 8 * q;
      float x[8];
      if (critic) {
        const float d = dvs[r];
        const float4 w0 = *reinterpret_cast<const float4*>(Wc + 8 * q);
        const float4 w1 = *reinterpret_cast<const float4*>(Wc + 8 * q + 4);
        x[0] = d * w0.x; x[1] = d * w0.y; x[2] = d * w0.z; x[3] = d * w0.w;
        x[4] = d * w1.x; x[5] = d * w1.y; x[6] = d * w1.z; x[7] = d * w1.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = 0.f;
#pragma unroll
        for (int a = 0; a < NA; ++a) {  // a in order; rows past A are zero
          const float d = dmus[r * NA + a];
          const float4 w0 = *reinterpret_cast<const float4*>(Ws + a * PH + 8 * q);
          const float4 w1 = *reinterpret_cast<const float4*>(Ws + a * PH + 8 * q + 4);
          x[0] = fmaf(d, w0.x, x[0]); x[1] = fmaf(d, w0.y, x[1]); x[2] = fmaf(d, w0.z, x[2]);
          x[3] = fmaf(d, w0.w, x[3]); x[4] = fmaf(d, w1.x, x[4]); x[5] = fmaf(d, w1.y, x[5]);
          x[6] = fmaf(d, w1.z, x[6]); x[7] = fmaf(d, w1.w, x[7]);
        }
      }
      const float4 y0 = *reinterpret_cast<const float4*>(y);
      const float4 y1 = *reinterpret_cast<const float4*>(y + 4);
      const float yy[8] = {y0.x, y0.y, y0.z, y0.w, y1.x, y1.y, y1.z, y1.w};
      float d[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = x[e] * (yy[e] > 0.f ? 1.f : yy[e] + 1.f);
      *reinterpret_cast<float4*>(y) = {d[0], d[1], d[2], d[3]};
      *reinterpret_cast<float4*>(y + 4) = {d[4], d[5], d[6], d[7]};
      if (r0 + r < p.B) {
        if (critic) store_s8_group(static_cast<char*>(t.dyc) + ((int64_t)(r0 + r) * t.ld_dyc + 8 * q) * 4, d);
        else store_s8_group(static_cast<char*>(t.dy) + ((int64_t)(r0 + r) * t.ld_dy + 8 * q) * 4, d);
      }
    }
  }
  __syncthreads();
  TCK(3);
  // their column sums over the block's rows (rows past B hold zeros), rows in order
  for (int o = tid; o < H + Hc; o += blockDim.x) {
    const bool critic = o >= H;
    const int k = critic ? o - H : o;
    float* cs = critic ? t.dyc_cs : t.dy_cs;
    if (!cs) continue;
    const float* y = critic ? yc : ys;
    const int P = critic ? PC : PH;
    float sum = 0.f;
#pragma unroll 8
    for (int r = 0; r < TR; ++r) sum += y[r * P + k];
    cs[(int64_t)bx * (critic ? Hc : H) + k] = sum;
  }
  // the block's partials only — no last-block pass (an agent-scope fence per block costs the L2's
  // write-back: ~1 us each): ws[b] = {surr / B, vloss / B, kl / B, dstd partial [A]}, block 0's
  // dstd partial with the entropy term ge / std; the launch's totals are flat sums of these
  // (lgx_s8_reduce jobs of the caller). Block 0 writes the entropy (a constant) into out[2].
  TCK(4);
  // the block's sums of the rows' values, summed in row order
  if (tid < NV) {
    float sum = 0.f;
    for (int q = 0; q < TR; ++q) {
      const float x = tid < 3 ? rowv[q][tid]
                              : (tid < 3 + NA ? tvs[q][tid - 3]
                                              : (tid < 3 + 2 * NA ? dmus[q * NA + tid - 3 - NA] : dvs[q]));
      sum += x;
    }
    const float inv = 1.f / p.B;
    float* w = p.ws + (int64_t)bx * (3 + HMAXA);
    if (tid < 3) w[tid] = sum * inv;
    else if (tid < 3 + NA) {
      const int j = tid - 3;
      if (j < A) w[3 + j] = sum + (bx == 0 ? ge / stdv[j] : 0.f);
    } else if (tid < 3 + 2 * NA) {
      const int j = tid - 3 - NA;
      if (s.dmu_cs && j < A) s.dmu_cs[(int64_t)bx * A + j] = sum;
    } else if (s.dvalue_cs) {
      s.dvalue_cs[bx] = sum;
    }
  }
  TCK(5);
  if (tid == 0) {
    if (bx == 0) {
      float ent = 0.f;
      for (int j = 0; j < A; ++j) ent += 0.5f + 0.9189385332046727f + lstd[j];
      p.out[2] = ent;
    }
  }
#ifdef LGX_TAIL_CLOCK
  if (tid == 0 && g_tailclk) {
    ck[6] = (uint32_t)(clock64() - ck0);
    for (int q = 0; q < 7; ++q) g_tailclk[(size_t)bx * 8 + q] = ck[q];
  }
#endif
}

// one grid: blocks [0, naux) the aux head's 256-row blocks (first, so that they run beside the
// PPO head's blocks rather than after them), then the PPO head's TR-row blocks
template <int NA>
__global__ __launch_bounds__(256) void loss_heads_tail(lgx_ppo_head_args h, lgx_aux_loss_args a, lgx_heads_s8_args s,
                                                       lgx_heads_tail_args t) {
  const int naux = (int)head_grid(a.B);
  extern __shared__ __align__(16) float tl[];
  if ((int)blockIdx.x < naux) aux_loss_fused_core(a, s, naux, tl);  // staging in the dynamic LDS
  else ppo_tail_body<NA>(h, s, t, (int)blockIdx.x - naux);
}

// ---------------------------------------------------------------- PPO minibatch optimizer tail
#ifndef LGX_TAIL_BLOCKS
#define LGX_TAIL_BLOCKS 128
#endif
constexpr int TAIL_BLOCKS = LGX_TAIL_BLOCKS;  // each block ends with a release + counter atomic

// A flat segment [lo, hi) of the 16-B aligned grads/params/moments buffers as a scalar head
// (up to the first multiple of 4), a float4 body [a, b) and a scalar tail: every segment
// offset is arbitrary, the buffers' bases are aligned (torch allocations), so the body of
// every array is float4-aligned at the same indices.
__device__ __forceinline__ void body4(int64_t lo, int64_t hi, int64_t& a, int64_t& b) {
  a = min(hi, (lo + 3) & ~(int64_t)3);
  b = max(a, hi & ~(int64_t)3);
}

// squared norm partial of one thread: float4 body, four loads in flight per pass, four
// accumulators (one per lane of the float4) combined in a fixed order (the float4s in index order)
__device__ __forceinline__ float sumsq_range(const float* __restrict__ g, int64_t lo, int64_t hi, int64_t i0,
                                             int64_t stride) {
  int64_t a, b;
  body4(lo, hi, a, b);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  const float4* g4 = reinterpret_cast<const float4*>(g + a);
  const int64_t n4 = (b - a) >> 2;
  int64_t j = i0;
  for (; j + 3 * stride < n4; j += 4 * stride) {
    float4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) x[u] = g4[j + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s0 += x[u].x * x[u].x; s1 += x[u].y * x[u].y; s2 += x[u].z * x[u].z; s3 += x[u].w * x[u].w;
    }
  }
  for (; j < n4; j += stride) {
    const float4 x = g4[j];
    s0 += x.x * x.x; s1 += x.y * x.y; s2 += x.z * x.z; s3 += x.w * x.w;
  }
  if (i0 < a - lo) s0 += g[lo + i0] * g[lo + i0];
  if (i0 < hi - b) s1 += g[b + i0] * g[b + i0];
  return (s0 + s1) + (s2 + s3);
}

// grid TAIL_BLOCKS: squared norms (estimator; main + adaptation) as block partials; block 0 also
// runs the KL schedule, bumps the Adam steps and the loss sums (none of which needs the norms).
// No last-block pass (an agent-scope fence per block costs an L2 write-back, ~1 us each): every
// tail_adam block sums the partials itself, in one fixed order, after the launch boundary.
__global__ __launch_bounds__(256) void tail_norms(lgx_ppo_tail_args p) {
  __shared__ float red[4 * 2];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float v[2];
  v[0] = sumsq_range(p.grads, p.est_lo, p.est_hi, i0, stride);
  v[1] = sumsq_range(p.grads, p.main_lo, p.main_hi, i0, stride) + sumsq_range(p.grads, p.adapt_lo, p.adapt_hi, i0, stride);
  block_sum<2>(v, red);
  if (threadIdx.x == 0) { p.ws[blockIdx.x * 2] = v[0]; p.ws[blockIdx.x * 2 + 1] = v[1]; }
  if (blockIdx.x == 0) {
    // the scalar bookkeeping on separate threads (each one dependent memory round trip,
    // not one thread's serial chain of loads behind possibly-aliasing stores)
    const int tid = threadIdx.x;
    if (tid == 0) {
      if (p.kl_index >= 0) {
        const double kl = (double)p.grads[p.kl_index];
        double lr = *p.lr64;
        if (kl > p.desired_kl * 2.0) lr = fmax(lr / 1.5, 1e-5);
        else if (kl < p.desired_kl / 2.0 && kl > 0.0) lr = fmin(lr * 1.5, 1e-2);
        *p.lr64 = lr;
        *p.lr32 = (float)lr;
      }
    } else if (tid == 1) {
      *p.step_main += 1.f;
    } else if (tid == 2) {
      *p.step_est += 1.f;
    } else if (tid - 3 < p.nloss) {
      p.sums[tid - 3] += *p.loss_ptrs[tid - 3];
    }
  }
}

// Adam over one segment: float4 body (params, grads, moments at the same aligned indices),
// scalar head and tail
__device__ __forceinline__ void adam_range(const lgx_ppo_tail_args& p, int64_t lo, int64_t hi, int64_t i0,
                                           int64_t stride, float c, float b1, float b2, float eps, float ss,
                                           float sq) {
  int64_t a, b;
  body4(lo, hi, a, b);
  float4* P = reinterpret_cast<float4*>(p.params + a);
  const float4* G = reinterpret_cast<const float4*>(p.grads + a);
  float4* M = reinterpret_cast<float4*>(p.exp_avg + a);
  float4* V = reinterpret_cast<float4*>(p.exp_avg_sq + a);
  // one float4 item per pass (4 items per pass with every load before the first store measured
  // slower: 13.1 -> 15.5 us per launch)
  const int64_t n4 = (b - a) >> 2;
  int64_t j = i0;
  for (; j < n4; j += stride) {
    float4 x = P[j], m = M[j], v = V[j];
    const float4 g = G[j];
    adam1(x.x, g.x * c, m.x, v.x, b1, b2, eps, ss, sq);
    adam1(x.y, g.y * c, m.y, v.y, b1, b2, eps, ss, sq);
    adam1(x.z, g.z * c, m.z, v.z, b1, b2, eps, ss, sq);
    adam1(x.w, g.w * c, m.w, v.w, b1, b2, eps, ss, sq);
    P[j] = x; M[j] = m; V[j] = v;
  }
  if (i0 < a - lo) {
    const int64_t i = lo + i0;
    adam1(p.params[i], p.grads[i] * c, p.exp_avg[i], p.exp_avg_sq[i], b1, b2, eps, ss, sq);
  }
  if (i0 < hi - b) {
    const int64_t i = b + i0;
    adam1(p.params[i], p.grads[i] * c, p.exp_avg[i], p.exp_avg_sq[i], b1, b2, eps, ss, sq);
  }
}

__global__ __launch_bounds__(256) void tail_adam(lgx_ppo_tail_args p) {
  __shared__ float red[4 * 2];
  __shared__ float sc[2];
  {  // the clip coefficients from tail_norms' partials (the same fixed order in every block)
    float t[2];
    final_sum<2>(p.ws, 2, TAIL_BLOCKS, t, red);
    if (threadIdx.x == 0) {
      sc[0] = fminf(p.max_norm / (sqrtf(t[0]) + 1e-6f), 1.f);
      sc[1] = fminf(p.max_norm / (sqrtf(t[1]) + 1e-6f), 1.f);
    }
    __syncthreads();
  }
  const float ce = sc[0], cm = sc[1];
  const float tm = *p.step_main, te = *p.step_est;
  const float lrm = *p.lr32;
  const float bcm1 = 1.f - powf(p.b1_main, tm), bcm2 = 1.f - powf(p.b2_main, tm);
  const float bce1 = 1.f - powf(p.b1_est, te), bce2 = 1.f - powf(p.b2_est, te);
  const float ssm = lrm / bcm1, sqm = sqrtf(bcm2), sse = p.est_lr / bce1, sqe = sqrtf(bce2);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  adam_range(p, p.main_lo, p.main_hi, i0, stride, cm, p.b1_main, p.b2_main, p.eps_main, ssm, sqm);
  adam_range(p, p.est_lo, p.est_hi, i0, stride, ce, p.b1_est, p.b2_est, p.eps_est, sse, sqe);
  int64_t a, b;
  body4(p.adapt_lo, p.adapt_hi, a, b);
  float4* g4 = reinterpret_cast<float4*>(p.grads + a);
  for (int64_t j = i0; j < (b - a) >> 2; j += stride) {
    float4 x = g4[j];
    x.x *= cm; x.y *= cm; x.z *= cm; x.w *= cm;
    g4[j] = x;
  }
  if (i0 < a - p.adapt_lo) p.grads[p.adapt_lo + i0] *= cm;
  if (i0 < p.adapt_hi - b) p.grads[b + i0] *= cm;
}

// The tail's Adam launch with the S8 copies (lgx_ppo_tail_args.n_s8 > 0): the host cuts the
// three segments at the weights' boundaries into ranges, each with its own blocks (a block's
// range is uniform: no per-element table lookup), and a weight's range writes every updated
// value's S8 copies (lgx_s8_split's conversion and layouts) right after its Adam update.
constexpr int TAIL_RMAX = 48;
struct TailRange {
  int64_t lo, hi;   // flat elements
  int32_t opt;      // 0: main Adam, 1: estimator Adam, 2: the adaptation gradients' clip scaling
  int32_t seg0, nseg;  // this weight's S8 entries (nseg 0: not a weight)
  int32_t blk0;     // first block
};
struct TailK {
  lgx_ppo_tail_args p;
  int32_t nr;
  TailRange r[TAIL_RMAX + 1];  // r[nr].blk0 = the grid
  lgx_tail_s8_seg s[LGX_TAIL_S8_MAX];
};
static_assert(sizeof(TailK) <= 4096, "kernel argument segment");

__device__ __forceinline__ void s8_put(const lgx_tail_s8_seg& S, int r, int c, float x) {
  const __bf16 h = (__bf16)x;
  const __bf16 l = (__bf16)(x - (float)h);
  char* q;
  int lo;
  if (S.packed) {
    q = S.dst + ((int64_t)(r >> 4) * S.ld + (c >> 5)) * 2048 + ((((c >> 3) & 3) << 4) | (r & 15)) * 16 + (c & 7) * 2;
    lo = 1024;
  } else {
    q = S.dst + (int64_t)r * S.ld * 4 + (c >> 3) * 32 + (c & 7) * 2;
    lo = 16;
  }
  *reinterpret_cast<__bf16*>(q) = h;
  *reinterpret_cast<__bf16*>(q + lo) = l;
}

// 4 consecutive columns c..c+3 (c % 4 == 0) of row r: 8 B of hi, 8 B of lo (same group half)
__device__ __forceinline__ void s8_put4(const lgx_tail_s8_seg& S, int r, int c, const float (&x)[4]) {
  uint32_t h[2], l[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const __bf16 h0 = (__bf16)x[2 * e], h1 = (__bf16)x[2 * e + 1];
    const __bf16 l0 = (__bf16)(x[2 * e] - (float)h0), l1 = (__bf16)(x[2 * e + 1] - (float)h1);
    h[e] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
    l[e] = (uint32_t)__builtin_bit_cast(uint16_t, l0) | ((uint32_t)__builtin_bit_cast(uint16_t, l1) << 16);
  }
  char* q;
  int lo;
  if (S.packed) {
    q = S.dst + ((int64_t)(r >> 4) * S.ld + (c >> 5)) * 2048 + ((((c >> 3) & 3) << 4) | (r & 15)) * 16 + (c & 7) * 2;
    lo = 1024;
  } else {
    q = S.dst + (int64_t)r * S.ld * 4 + (c >> 3) * 32 + (c & 7) * 2;
    lo = 16;
  }
  *reinterpret_cast<uint2*>(q) = make_uint2(h[0], h[1]);
  *reinterpret_cast<uint2*>(q + lo) = make_uint2(l[0], l[1]);
}

__global__ __launch_bounds__(256) void tail_adam_ranges(TailK k) {
  __shared__ float red[4 * 2];
  __shared__ float sc[2];
  const lgx_ppo_tail_args& p = k.p;
  {  // the clip coefficients from tail_norms' partials (as tail_adam)
    float t[2];
    final_sum<2>(p.ws, 2, TAIL_BLOCKS, t, red);
    if (threadIdx.x == 0) {
      sc[0] = fminf(p.max_norm / (sqrtf(t[0]) + 1e-6f), 1.f);
      sc[1] = fminf(p.max_norm / (sqrtf(t[1]) + 1e-6f), 1.f);
    }
    __syncthreads();
  }
  int ri = 0, hi_ = k.nr - 1;  // this block's range (binary search on the first blocks)
  while (ri < hi_) {
    const int mid = (ri + hi_ + 1) >> 1;
    if ((int)blockIdx.x >= k.r[mid].blk0) ri = mid;
    else hi_ = mid - 1;
  }
  TailRange R = k.r[ri];
  const float c = R.opt == 1 ? sc[0] : sc[1];
  const int64_t nb = k.r[ri + 1].blk0 - R.blk0;
  const int64_t stride = nb * blockDim.x;
  const int64_t i0 = (int64_t)(blockIdx.x - R.blk0) * blockDim.x + threadIdx.x;
  int64_t a, b;
  body4(R.lo, R.hi, a, b);
  if (R.opt == 2) {  // g[adapt] *= coef_m
    float4* g4 = reinterpret_cast<float4*>(p.grads + a);
    for (int64_t j = i0; j < (b - a) >> 2; j += stride) {
      float4 x = g4[j];
      x.x *= c; x.y *= c; x.z *= c; x.w *= c;
      g4[j] = x;
    }
    if (i0 < a - R.lo) p.grads[R.lo + i0] *= c;
    if (i0 < R.hi - b) p.grads[b + i0] *= c;
    return;
  }
  const bool est = R.opt == 1;
  const float t = est ? *p.step_est : *p.step_main;
  const float b1 = est ? p.b1_est : p.b1_main, b2 = est ? p.b2_est : p.b2_main, eps = est ? p.eps_est : p.eps_main;
  const float lr = est ? p.est_lr : *p.lr32;
  const float ss = lr / (1.f - powf(b1, t)), sq = sqrtf(1.f - powf(b2, t));
  // the weight's S8 entries (all share p0, N, K)
#ifdef LGX_TAIL_NOEMIT  // dev builds: the ranges kernel without its S8 stores (timing only)
  R.nseg = 0;
#endif
  const int64_t p0 = R.nseg > 0 ? k.s[R.seg0].p0 : 0;
  const int K = R.nseg > 0 ? k.s[R.seg0].K : 1;
  // the weight's entries (<= 4 used here: the segmented first layer's spans, or a row-major and
  // a packed copy), hoisted out of the element loop
  constexpr int NSEG = 4;
  lgx_tail_s8_seg sg[NSEG];
  const int ns = min(R.nseg, NSEG);
#pragma unroll
  for (int e = 0; e < NSEG; ++e) sg[e] = k.s[R.seg0 + min(e, max(ns - 1, 0))];
  auto emit_rc = [&](int r, int col, float x) {
#pragma unroll
    for (int e = 0; e < NSEG; ++e) {
      const int cc = col - sg[e].c0;
      if (e < ns && cc >= 0 && cc < sg[e].w) s8_put(sg[e], r, cc, x);
    }
  };
  auto emit = [&](int64_t i, float x) {
    const int d = (int)(i - p0);
    const int r = d / K;
    emit_rc(r, d - r * K, x);
  };
  float4* P = reinterpret_cast<float4*>(p.params + a);
  const float4* G = reinterpret_cast<const float4*>(p.grads + a);
  float4* M = reinterpret_cast<float4*>(p.exp_avg + a);
  float4* V = reinterpret_cast<float4*>(p.exp_avg_sq + a);
  for (int64_t j = i0; j < (b - a) >> 2; j += stride) {
    float4 x = P[j], m = M[j], v = V[j];
    const float4 g = G[j];
    adam1(x.x, g.x * c, m.x, v.x, b1, b2, eps, ss, sq);
    adam1(x.y, g.y * c, m.y, v.y, b1, b2, eps, ss, sq);
    adam1(x.z, g.z * c, m.z, v.z, b1, b2, eps, ss, sq);
    adam1(x.w, g.w * c, m.w, v.w, b1, b2, eps, ss, sq);
    P[j] = x; M[j] = m; V[j] = v;
    if (R.nseg > 0) {  // one division per float4: the next three elements by carry
      const int d = (int)(a + 4 * j - p0);
      int r = d / K, col = d - r * K;
      const float xs[4] = {x.x, x.y, x.z, x.w};
      if ((col & 3) == 0 && col + 4 <= K) {  // one row: whole 4-column pieces where they fit
#pragma unroll
        for (int e = 0; e < NSEG; ++e) {
          const int cc = col - sg[e].c0;
          if (e >= ns || cc + 4 <= 0 || cc >= sg[e].w) continue;
          if ((cc & 3) == 0 && cc >= 0 && cc + 4 <= sg[e].w) {
            s8_put4(sg[e], r, cc, xs);
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q)
              if (cc + q >= 0 && cc + q < sg[e].w) s8_put(sg[e], r, cc + q, xs[q]);
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          emit_rc(r, col, xs[e]);
          if (++col == K) { col = 0; ++r; }
        }
      }
    }
  }
  if (i0 < a - R.lo) {
    const int64_t i = R.lo + i0;
    adam1(p.params[i], p.grads[i] * c, p.exp_avg[i], p.exp_avg_sq[i], b1, b2, eps, ss, sq);
    if (R.nseg > 0) emit(i, p.params[i]);
  }
  if (i0 < R.hi - b) {
    const int64_t i = b + i0;
    adam1(p.params[i], p.grads[i] * c, p.exp_avg[i], p.exp_avg_sq[i], b1, b2, eps, ss, sq);
    if (R.nseg > 0) emit(i, p.params[i]);
  }
}

// dynamic LDS: two K-step stages of hi/lo A and B images, or the fp32 C image (reused)
constexpr size_t lds_bytes(int bn, int bm = BM) {
  const size_t stages = 2 * (2 * bm * PITCH + 2 * bn * PITCH) * sizeof(__bf16);
  const size_t cimg = (size_t)bm * (bn + 4) * sizeof(float);
  return stages > cimg ? stages : cimg;
}

template <int AM, int BMODE, bool CS>
void launch(Params p, int bn, hipStream_t s) {
  p.tiles_m = (p.M + BM - 1) / BM;
  p.tiles_n = (p.N + bn - 1) / bn;
  p.tiles = p.tiles_m * p.tiles_n * p.split;
  const int grid = (p.tiles + 7) / 8 * 8;
  if (bn == 128) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_kernel<AM, BMODE, CS, 128>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes(128));
      attr = true;
    }
    hipLaunchKernelGGL((gemm_kernel<AM, BMODE, CS, 128>), dim3(grid), dim3(NT), lds_bytes(128), s, p);
  } else {
    hipLaunchKernelGGL((gemm_kernel<AM, BMODE, CS, 64>), dim3(grid), dim3(NT), lds_bytes(64), s, p);
  }
}

}  // namespace lgxm

static thread_local char g_err[256] = "";

static int fail(const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return -1;
}


static int tile_n(int N) {
  static int forced = -1;
  if (forced < 0) {
    const char* e = LGX_DEV_KNOB("LGX_MLP_BN");  // dev knob: force 64 or 128
    forced = e ? atoi(e) : 0;
  }
  if (forced == 64 || forced == 128) return forced;
  return N > 128 ? 128 : 64;
}

// Forward / input-gradient launches over few rows (the rollout's 4096-env batches): 64-wide
// tiles double the block count of a launch that would otherwise leave most CUs idle
// (4096 x 736 -> 512 forward: 33 -> 23 us, tools/gemm_variants.py); weight gradients and
// the update's 24,576-row launches keep tile_n.
static int tile_n_for(int M, int N, bool rows_are_batch) {
  static int forced = -1;
  if (forced < 0) {
    const char* e = LGX_DEV_KNOB("LGX_MLP_BN");
    forced = e ? atoi(e) : 0;
  }
  if (forced == 64 || forced == 128) return forced;
  if (rows_are_batch && M <= 8192) return 64;
  return tile_n(N);
}

// Tile width of a grouped weight-gradient launch (LGX_DW_BN: dev knob, 64 or 128)
static int dw_tile_n(int N) {
  static int forced = -1;
  if (forced < 0) {
    const char* e = LGX_DEV_KNOB("LGX_DW_BN");
    forced = e ? atoi(e) : 0;
  }
  if (forced == 64 || forced == 128) return forced;
  return tile_n_for(0, N, false);
}

// Rows per tile of a grouped launch: 64 for forward-kind launches (forward, and input
// gradients on transposed weights) with 64-wide tiles and fewer than 2 blocks per CU at 128
// rows — the rollout's 4096-env batches and the update's narrow layers: twice the blocks per
// launch, so twice the waves per CU to hide each K step's latency — else BM. LGX_MLP_BM=128 forces the 128-row tile (dev knob).
static int group_tile_m(int kind, int bn, int64_t tiles128) {
  static int forced = -1;
  if (forced < 0) {
    const char* e = LGX_DEV_KNOB("LGX_MLP_BM");
    forced = e ? atoi(e) : 0;
  }
  if (forced == 128) return lgxm::BM;
  if (forced == 64) return kind != lgxm::G_DW && bn == 64 ? 64 : lgxm::BM;  // dev: every 64-wide fwd / dx launch
  // (a launch that already has 2 blocks per CU at 128 rows — the 4096-row actor/critic
  // layer 0, 512 tiles — measured faster with them: 32 vs 35 us)
  return kind == lgxm::G_FWD && bn == 64 && tiles128 < 512 ? 64 : lgxm::BM;
}

// Waves per block of the 128 x 128 grouped launches: 8 for the forward and input-gradient kinds
// (4 waves per SIMD at 108-122 VGPRs instead of 2 at 194-210: +1.5-2 % per iteration, r03,
// profiles/r03_gemm_waves.txt), 4 for the weight gradient (8 measured equal, and its bias-gradient
// sums would change order vs the single-launch path). Dev knobs: LGX_MLP_NW, LGX_MLP_NW_DW (4 or 8).
static int group_waves(int kind) {
  static int fwd = -1, dw = -1;
  if (fwd < 0) {
    const char* e = LGX_DEV_KNOB("LGX_MLP_NW");
    fwd = e ? (atoi(e) == 4 ? 4 : 8) : 8;
    const char* d = LGX_DEV_KNOB("LGX_MLP_NW_DW");
    dw = d && atoi(d) == 8 ? 8 : 4;
  }
  return kind == lgxm::G_DW ? dw : fwd;
}

// ================================================================ rollout bookkeeping
namespace lgxm {

struct CopyBatch {
  lgx_copy_desc d[LGX_COPY_MAX];
  int32_t n;
};

// blockIdx.y = entry; blocks stride over the entry's 16-byte chunks
__global__ __launch_bounds__(256) void copy_batch_kernel(CopyBatch cb) {
  const lgx_copy_desc& d = cb.d[blockIdx.y];
  const bool vec = ((reinterpret_cast<uintptr_t>(d.src) | reinterpret_cast<uintptr_t>(d.dst) | (uintptr_t)d.nbytes) &
                    15) == 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if (vec) {
    const int64_t n16 = d.nbytes >> 4;
    const float4* __restrict__ s = reinterpret_cast<const float4*>(d.src);
    float4* __restrict__ t = reinterpret_cast<float4*>(d.dst);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) t[i] = s[i];
  } else {
    const uint8_t* __restrict__ s = reinterpret_cast<const uint8_t*>(d.src);
    uint8_t* __restrict__ t = reinterpret_cast<uint8_t*>(d.dst);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < d.nbytes; i += stride) t[i] = s[i];
  }
}

// blockIdx.y = entry (nbytes = bytes per row); threads stride over (row, chunk) pairs
// item i = (row r, chunk c) with 32-bit index math (host: rows * per < 2^31); the
// destination row stride may exceed the row (rows placed inside a wider buffer)
__global__ __launch_bounds__(256) void gather_rows_kernel(CopyBatch cb, const int64_t* __restrict__ idx, int64_t rows) {
  const lgx_copy_desc& d = cb.d[blockIdx.y];
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t i0 = blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t dstr = d.dst_stride > 0 ? d.dst_stride : d.nbytes;
  const bool vec = ((reinterpret_cast<uintptr_t>(d.src) | reinterpret_cast<uintptr_t>(d.dst) | (uintptr_t)d.nbytes |
                     (uintptr_t)dstr) & 15) == 0;
  if (vec) {
    const uint32_t per = (uint32_t)(d.nbytes >> 4), tpr = (uint32_t)(dstr >> 4);
    const uint32_t n = (uint32_t)rows * per;
    const float4* __restrict__ s = reinterpret_cast<const float4*>(d.src);
    float4* __restrict__ t = reinterpret_cast<float4*>(d.dst);
    for (uint32_t i = i0; i < n; i += stride) {
      const uint32_t r = i / per, c = i - r * per;
      t[(int64_t)r * tpr + c] = s[idx[r] * per + c];
    }
  } else {
    const uint32_t per = (uint32_t)(d.nbytes >> 2), tpr = (uint32_t)(dstr >> 2);  // 4-B elements (host checks)
    const uint32_t n = (uint32_t)rows * per;
    const float* __restrict__ s = reinterpret_cast<const float*>(d.src);
    float* __restrict__ t = reinterpret_cast<float*>(d.dst);
    for (uint32_t i = i0; i < n; i += stride) {
      const uint32_t r = i / per, c = i - r * per;
      t[(int64_t)r * tpr + c] = s[idx[r] * per + c];
    }
  }
}

// eps == NULL: the standard normal of action j of global env `gid` at env step `step` is
// Philox4x32-10 with the env's counter layout on stream LGX_ACT_NOISE_STREAM, block j / 4; its
// 4 uniforms make 2 Box-Muller pairs (u1 = 1 - u[2q], u2 = u[2q + 1], r = sqrt(-2 log u1),
// theta = 2 pi u2), action j takes r cos theta (even j) or r sin theta (odd j) of pair
// (j / 2) % 2. oracle/philox.py act_noise states the same.
__global__ __launch_bounds__(256) void act_head_kernel(lgx_act_head_args p) {
  // four lanes per row: lane q of a row's group handles actions 4q..4q+3 (one Philox call: the
  // 2 Box-Muller pairs of act_noise's block q); lane 0 then sums the row's log-prob terms in
  // action order (the same sum as one lane looping over the actions). std and log std once per block.
  __shared__ float s_sd[HMAXA], s_lsd[HMAXA];
  if ((int)threadIdx.x < p.A) {
    s_sd[threadIdx.x] = p.std[threadIdx.x];
    s_lsd[threadIdx.x] = logf(p.std[threadIdx.x]);
  }
  __syncthreads();
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = t >> 2, q = t & 3;  // row, block of 4 actions (B * 4 threads: whole groups)
  const bool row = i < p.B, on = row && 4 * q < p.A;
  const float c = 0.91893853320467274178f;  // log(sqrt(2 pi))
  float term[4] = {0.f, 0.f, 0.f, 0.f};
  if (on) {
    float e4[4];
    if (p.eps == nullptr) {
      const uint64_t step = (uint64_t)*p.step_dev;
      const uint32_t gid = (uint32_t)(p.env_offset + i);
      uint32_t o[4];
      philox4x32_10(gid, (uint32_t)step, (uint32_t)q | ((uint32_t)LGX_ACT_NOISE_STREAM << 16), (uint32_t)(step >> 32),
                    (uint32_t)p.seed, (uint32_t)(p.seed >> 32), o);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float u1 = 1.0f - u01(o[2 * h]);
        const float u2 = u01(o[2 * h + 1]);
        const float r = sqrtf(-2.0f * logf(u1));
        const float th = 6.28318530717958647692f * u2;
        e4[2 * h] = r * cosf(th);
        e4[2 * h + 1] = r * sinf(th);
      }
    } else {
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) e4[jj] = 4 * q + jj < p.A ? p.eps[(size_t)i * p.A + 4 * q + jj] : 0.f;
    }
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = 4 * q + jj;
      if (j >= p.A) break;
      const size_t k = (size_t)i * p.A + j;
      const float m = p.mean[k], sd = s_sd[j];
      const float a = m + sd * e4[jj];
      const float d = a - m;
      term[jj] = -(d * d) / (2.0f * (sd * sd)) - s_lsd[j] - c;
      p.actions[k] = a;
      if (p.actions_copy) p.actions_copy[k] = a;
      p.mu[k] = m;
      p.sigma[k] = sd;
    }
  }
  // the row's terms to its lane 0, summed in action order
  float all[HMAXA];
#pragma unroll
  for (int qq = 0; qq < 4; ++qq)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) all[4 * qq + jj] = __shfl(term[jj], (threadIdx.x & ~3) + qq, 64);
  if (row && q == 0) {
    float lp = 0.0f;
    for (int j = 0; j < p.A; ++j) lp += all[j];
    p.logp[i] = lp;
  }
}

__global__ __launch_bounds__(256) void transition_kernel(lgx_transition_args p) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.B) return;
  const float v = p.values[i];
  float r = p.rewards[i];
  const bool d = p.dones[i] != 0;  // every load before the first store (no aliasing stall)
  if (p.time_outs) r = r + p.gamma * (v * (float)p.time_outs[i]);
  p.rewards_out[i] = r;
  p.dones_out[i] = d ? 1 : 0;
  p.values_out[i] = v;
}

// GAE (lgx_gae): one thread per env, the T steps backwards in torch's operation order;
// fp64 block partials of the advantages' sum and sum of squares, summed by the last block.
__global__ __launch_bounds__(256) void gae_kernel(lgx_gae_args p) {
  __shared__ double red[2 * 4];
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  double s1 = 0.0, s2 = 0.0;
  if (n < p.N) {
    const int64_t N = p.N;
    const float g = p.gamma, lam = p.lam;
    float adv = 0.f;
    // the env's rows of up to GT steps requested before the recursion (the stores of returns /
    // advantages would otherwise hold each step's loads behind the previous step's stores: one
    // memory round trip per step); clamped steps, no load under a condition
    constexpr int GT = 32;
    const int T = p.T;
    if (T <= GT) {
      float vv[GT], rr[GT], dd[GT];
#pragma unroll
      for (int t = 0; t < GT; ++t) {
        const int64_t i = (int64_t)min(t, T - 1) * N + n;
        vv[t] = p.values[i];
        rr[t] = p.rewards[i];
        dd[t] = (float)p.dones[i];
      }
      const float last = p.last_values[n];
#pragma unroll
      for (int t = GT - 1; t >= 0; --t) {
        if (t >= T) continue;
        const int64_t i = (int64_t)t * N + n;
        const float v = vv[t];
        const float next = t == T - 1 ? last : vv[t + 1 < GT ? t + 1 : t];
        const float nt = 1.0f - dd[t];
        const float delta = (rr[t] + (nt * g) * next) - v;
        adv = delta + ((nt * g) * lam) * adv;
        const float ret = adv + v;
        const float a = ret - v;
        p.returns[i] = ret;
        p.advantages[i] = a;
        s1 += (double)a;
        s2 += (double)a * (double)a;
      }
    } else {
      for (int t = T - 1; t >= 0; --t) {
        const int64_t i = (int64_t)t * N + n;
        const float v = p.values[i];
        const float next = t == T - 1 ? p.last_values[n] : p.values[i + N];
        const float nt = 1.0f - (float)p.dones[i];
        const float delta = (p.rewards[i] + (nt * g) * next) - v;
        adv = delta + ((nt * g) * lam) * adv;
        const float ret = adv + v;
        const float a = ret - v;
        p.returns[i] = ret;
        p.advantages[i] = a;
        s1 += (double)a;
        s2 += (double)a * (double)a;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_down(s1, o, 64);
    s2 += __shfl_down(s2, o, 64);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) { red[wv] = s1; red[4 + wv] = s2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    p.ws[2 * blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
    p.ws[2 * blockIdx.x + 1] = ((red[4] + red[5]) + red[6]) + red[7];
    __threadfence();
    if (atomicAdd(p.counter, 1u) == gridDim.x - 1) {  // last block: partials in block order
      __threadfence();
      double t1 = 0.0, t2 = 0.0;
      for (int b = 0; b < (int)gridDim.x; ++b) { t1 += p.ws[2 * b]; t2 += p.ws[2 * b + 1]; }
      p.moments[0] = t1;
      p.moments[1] = t2;
      *p.counter = 0u;
    }
  }
}

__global__ __launch_bounds__(256) void adv_norm_kernel(float* __restrict__ a, int64_t n, const double* __restrict__ m,
                                                       double count) {
  const double mean = m[0] / count;
  const double var = (m[1] - count * mean * mean) / (count - 1.0);
  const float mf = (float)mean, den = (float)sqrt(var > 0.0 ? var : 0.0) + 1e-8f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) a[i] = (a[i] - mf) / den;
}

}  // namespace lgxm

extern "C" {

int32_t lgx_mlp_abi_version(void) { return LGX_MLP_ABI_VERSION; }

int32_t lgx_mlp_sizeof_gemm_args(void) { return (int32_t)sizeof(lgx_gemm_args); }

const char* lgx_mlp_last_error(void) { return g_err; }

int32_t lgx_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                      const float* lr_dev, float lr, float beta1, float beta2, float eps, const float* step,
                      const float* grad_scale, void* stream) {
  if (n < 0) return fail("lgx_adam_step: negative size");
  if (n == 0) return 0;
  if (!param || !grad || !exp_avg || !exp_avg_sq || !step) return fail("lgx_adam_step: null pointer");
  const int64_t work = (n + 3) / 4;
  int blocks = (int)((work + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(lgxm::adam_kernel, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), param, grad,
                     exp_avg, exp_avg_sq, n, lr_dev, lr, beta1, beta2, eps, step, grad_scale);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_clip_adam(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, const float* lr_dev,
                      float lr, float beta1, float beta2, float eps, float* step, float max_norm, float* coef_out,
                      void* stream) {
  if (n < 1 || n > LGX_CLIP_ADAM_MAX) return fail("lgx_clip_adam: 1 <= n <= LGX_CLIP_ADAM_MAX");
  if (!param || !grad || !exp_avg || !exp_avg_sq || !step) return fail("lgx_clip_adam: null pointer");
  hipLaunchKernelGGL(lgxm::clip_adam_kernel, dim3(1), dim3(lgxm::CLIP_ADAM_NT), 0, static_cast<hipStream_t>(stream),
                     param, grad, exp_avg, exp_avg_sq, (int)n, lr_dev, lr, beta1, beta2, eps, step, max_norm, coef_out);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

static int head_check(const lgx_ppo_head_args* a) {
  if (!a) return fail("lgx_ppo_head: null args");
  if (a->A < 1 || a->A > lgxm::HMAXA) return fail("lgx_ppo_head: 1 <= A <= 16");
  if (a->B < 1) return fail("lgx_ppo_head: B >= 1");
  if (!a->mu || !a->value || !a->std || !a->actions || !a->old_logp || !a->adv || !a->returns || !a->ws || !a->counter)
    return fail("lgx_ppo_head: null pointer");
  if (a->clipped_value && !a->target_values) return fail("lgx_ppo_head: clipped_value needs target_values");
  return 0;
}

int32_t lgx_ppo_head_forward(const lgx_ppo_head_args* a, void* stream) {
  if (head_check(a)) return -1;
  if (!a->out || !a->old_mu || !a->old_sigma) return fail("lgx_ppo_head_forward: null out/old_mu/old_sigma");
  hipLaunchKernelGGL(a->A <= 12 ? lgxm::ppo_head_fwd<12> : lgxm::ppo_head_fwd<lgxm::HMAXA>, dim3(lgxm::head_grid(a->B)),
                     dim3(lgxm::HT), 0, static_cast<hipStream_t>(stream), *a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_ppo_head_backward(const lgx_ppo_head_args* a, void* stream) {
  if (head_check(a)) return -1;
  if (!a->g || !a->dmu || !a->dvalue || !a->dstd) return fail("lgx_ppo_head_backward: null g/dmu/dvalue/dstd");
  hipLaunchKernelGGL(a->A <= 12 ? lgxm::ppo_head_bwd<12> : lgxm::ppo_head_bwd<lgxm::HMAXA>, dim3(lgxm::head_grid(a->B)),
                     dim3(lgxm::HT), 0, static_cast<hipStream_t>(stream), *a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_aux_loss_forward(const lgx_aux_loss_args* a, void* stream) {
  if (!a || a->B < 1 || a->L < 1 || a->E < 1 || !a->p || !a->a || !a->e || !a->t || !a->out || !a->ws || !a->counter)
    return fail("lgx_aux_loss_forward: bad arguments");
  hipLaunchKernelGGL(lgxm::aux_loss_fwd, dim3(lgxm::head_grid(a->B)), dim3(lgxm::HT), 0,
                     static_cast<hipStream_t>(stream), *a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_aux_loss_backward(const lgx_aux_loss_args* a, void* stream) {
  if (!a || a->B < 1 || a->L < 1 || a->E < 1 || !a->p || !a->a || !a->e || !a->t || !a->g || !a->dp || !a->de)
    return fail("lgx_aux_loss_backward: bad arguments");
  hipLaunchKernelGGL(lgxm::aux_loss_bwd, dim3((a->B + lgxm::HT - 1) / lgxm::HT), dim3(lgxm::HT), 0,
                     static_cast<hipStream_t>(stream), *a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_loss_heads_forward(const lgx_ppo_head_args* h, const lgx_aux_loss_args* a, void* stream) {
  if (head_check(h)) return -1;
  if (!h->out || !h->old_mu || !h->old_sigma) return fail("lgx_loss_heads_forward: null out/old_mu/old_sigma");
  if (!a || a->B != h->B || a->L < 1 || a->E < 1 || !a->p || !a->a || !a->e || !a->t || !a->out || !a->ws ||
      !a->counter)
    return fail("lgx_loss_heads_forward: bad aux arguments");
  hipLaunchKernelGGL(h->A <= 12 ? lgxm::loss_heads_fwd<12> : lgxm::loss_heads_fwd<lgxm::HMAXA>, dim3(lgxm::head_grid(h->B), 2),
                     dim3(lgxm::HT), 0, static_cast<hipStream_t>(stream), *h, *a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_loss_heads_backward(const lgx_ppo_head_args* h, const lgx_aux_loss_args* a, void* stream) {
  if (head_check(h)) return -1;
  if (!h->g || !h->dmu || !h->dvalue || !h->dstd) return fail("lgx_loss_heads_backward: null g/dmu/dvalue/dstd");
  if (!a || a->B != h->B || a->L < 1 || a->E < 1 || !a->p || !a->a || !a->e || !a->t || !a->g || !a->dp || !a->de)
    return fail("lgx_loss_heads_backward: bad aux arguments");
  hipLaunchKernelGGL(h->A <= 12 ? lgxm::loss_heads_bwd<12> : lgxm::loss_heads_bwd<lgxm::HMAXA>, dim3(lgxm::head_grid(h->B), 2),
                     dim3(lgxm::HT), 0, static_cast<hipStream_t>(stream), *h, *a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_loss_heads_fused(const lgx_ppo_head_args* h, const lgx_aux_loss_args* a, const lgx_heads_s8_args* s,
                             void* stream) {
  if (head_check(h)) return -1;
  if (!h->out || !h->old_mu || !h->old_sigma || !h->g || !h->dstd)
    return fail("lgx_loss_heads_fused: null out/old_mu/old_sigma/g/dstd");
  if (!a || a->B != h->B || a->L < 1 || a->E < 1 || !a->p || !a->a || !a->e || !a->t || !a->out || !a->ws ||
      !a->counter || !a->g || !a->dp)
    return fail("lgx_loss_heads_fused: bad aux arguments");
  if (!s) return fail("lgx_loss_heads_fused: null S8 arguments");
  if ((!h->dmu && !s->dmu_s8) || (!h->dvalue && !s->dvalue_s8) || (!a->de && !s->de_s8))
    return fail("lgx_loss_heads_fused: dmu / dvalue / de need an fp32 or an S8 destination");
  if (a->E > 8) return fail("lgx_loss_heads_fused: E <= 8");
  if ((s->dmu_cs || s->dvalue_cs || s->de_cs) && lgxm::HT != 256)
    return fail("lgx_loss_heads_fused: column-sum partials need 256-row blocks (LGX_HT 256)");
  if ((s->dmu_s8 && (s->ld_dmu % 8 || s->ld_dmu < (h->A + 7) / 8 * 8)) || (s->dvalue_s8 && s->ld_dvalue % 8) ||
      (s->de_s8 && s->ld_de % 8))
    return fail("lgx_loss_heads_fused: S8 pitches are multiples of 8 covering the columns");
  if ((((uintptr_t)s->dmu_s8) | ((uintptr_t)s->dvalue_s8) | ((uintptr_t)s->de_s8)) & 15)
    return fail("lgx_loss_heads_fused: S8 destinations must be 16-B aligned");
  hipLaunchKernelGGL(h->A <= 12 ? lgxm::loss_heads_fused<12> : lgxm::loss_heads_fused<lgxm::HMAXA>,
                     dim3(lgxm::head_grid(h->B), 2), dim3(lgxm::HT), 0, static_cast<hipStream_t>(stream), *h, *a, *s);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

#ifdef LGX_TAIL_CLOCK
int32_t lgx_tail_set_clock(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(lgxm::g_tailclk), &buf, sizeof(void*)) == hipSuccess ? 0 : -1;
}
#endif
int32_t lgx_loss_heads_tail(const lgx_ppo_head_args* h, const lgx_aux_loss_args* a, const lgx_heads_s8_args* s,
                            const lgx_heads_tail_args* t, void* stream) {
  if (!h || !t || !s) return fail("lgx_loss_heads_tail: null arguments");
  if (h->B < 1 || h->A < 1 || h->A > lgxm::HMAXA || !h->std || !h->actions || !h->old_logp || !h->adv ||
      !h->returns || (h->clipped_value && !h->target_values) || !h->ws || !h->counter)
    return fail("lgx_loss_heads_tail: bad head arguments");
  if (!h->out || !h->old_mu || !h->old_sigma || !h->g || !h->dstd)
    return fail("lgx_loss_heads_tail: null out/old_mu/old_sigma/g/dstd");
  if (!a || a->B != h->B || a->L < 1 || a->E < 1 || !a->p || !a->a || !a->e || !a->t || !a->out || !a->ws ||
      !a->counter || !a->g || !a->dp)
    return fail("lgx_loss_heads_tail: bad aux arguments");
  if ((!h->dmu && !s->dmu_s8) || (!h->dvalue && !s->dvalue_s8) || (!a->de && !s->de_s8))
    return fail("lgx_loss_heads_tail: dmu / dvalue / de need an fp32 or an S8 destination");
  if (a->E > 8) return fail("lgx_loss_heads_tail: E <= 8");
  if (s->de_cs && lgxm::HT != 256) return fail("lgx_loss_heads_tail: de column sums need LGX_HT 256");
  if ((s->dmu_s8 && (s->ld_dmu % 8 || s->ld_dmu < (h->A + 7) / 8 * 8)) || (s->dvalue_s8 && s->ld_dvalue % 8) ||
      (s->de_s8 && s->ld_de % 8))
    return fail("lgx_loss_heads_tail: S8 pitches are multiples of 8 covering the columns");
  if (t->H < 8 || t->H > 256 || t->H % 8 || t->Hc < 8 || t->Hc > 256 || t->Hc % 8 || !t->y || !t->W || !t->b ||
      !t->dy || !t->yc || !t->Wc || !t->bc || !t->dyc || t->ld_y % 8 || t->ld_y < t->H || t->ld_yc % 8 ||
      t->ld_yc < t->Hc || t->ld_dy % 8 || t->ld_dy < t->H || t->ld_dyc % 8 || t->ld_dyc < t->Hc)
    return fail("lgx_loss_heads_tail: bad tail arguments (H, H_c multiples of 8 in [8, 256]; S8 pitches)");
  if ((((uintptr_t)s->dmu_s8) | ((uintptr_t)s->dvalue_s8) | ((uintptr_t)s->de_s8) | ((uintptr_t)t->y) |
       ((uintptr_t)t->yc) | ((uintptr_t)t->dy) | ((uintptr_t)t->dyc)) & 15)
    return fail("lgx_loss_heads_tail: S8 operands must be 16-B aligned");
  const int na = h->A <= 12 ? 12 : lgxm::HMAXA;
  const size_t lds = std::max(lgxm::tail_lds_floats(na, t->H, t->Hc), (size_t)lgxm::HT * (lgxm::AUX_CW + 1)) *
                     sizeof(float);
  const unsigned nb = (unsigned)((h->B + lgxm::TR - 1) / lgxm::TR);
  auto* k = h->A <= 12 ? lgxm::loss_heads_tail<12> : lgxm::loss_heads_tail<lgxm::HMAXA>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)lgxm::loss_heads_tail<12>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lgxm::tail_lds_floats(12, 256, 256) * 4);
    (void)hipFuncSetAttribute((const void*)lgxm::loss_heads_tail<lgxm::HMAXA>,
                              hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lgxm::tail_lds_floats(lgxm::HMAXA, 256, 256) * 4);
    attr = true;
  }
  hipLaunchKernelGGL(k, dim3(nb + lgxm::head_grid(h->B)), dim3(256), lds, static_cast<hipStream_t>(stream), *h, *a, *s,
                     *t);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_ppo_tail(const lgx_ppo_tail_args* a, void* stream) {
  if (!a || !a->grads || !a->params || !a->exp_avg || !a->exp_avg_sq || !a->lr32 || !a->lr64 || !a->step_main ||
      !a->step_est || !a->ws || !a->counter)
    return fail("lgx_ppo_tail: null pointer");
  if (a->main_lo > a->main_hi || a->est_lo > a->est_hi || a->adapt_lo > a->adapt_hi || a->nloss < 0 ||
      a->nloss > LGX_TAIL_MAX_LOSSES || (a->nloss > 0 && !a->sums))
    return fail("lgx_ppo_tail: bad ranges");
  for (int k = 0; k < a->nloss; ++k)
    if (!a->loss_ptrs[k]) return fail("lgx_ppo_tail: null loss pointer");
  if (a->n_s8 < 0 || a->n_s8 > LGX_TAIL_S8_MAX || (a->n_s8 > 0 && !a->s8))
    return fail("lgx_ppo_tail: bad S8 segment table");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (a->n_s8 > 0) {
    // ranges: the main / estimator segments cut at every S8 weight's [p0, p0 + N K), then the
    // adaptation scaling; a weight's entries are consecutive in the table (same p0)
#ifndef LGX_TAIL_ELEMS
#define LGX_TAIL_ELEMS 1024
#endif
    constexpr int64_t TAIL_ELEMS = LGX_TAIL_ELEMS;  // elements per block (one float4 per thread)
    lgxm::TailK k{};  // ~3.4 KB, copied into the launch's argument segment by the launch
    k.p = *a;
    for (int i = 0; i < a->n_s8; ++i) {
      const lgx_tail_s8_seg& q = a->s8[i];
      if (q.N <= 0 || q.K <= 0 || q.w <= 0 || q.c0 < 0 || q.c0 + q.w > q.K || !q.dst || q.ld <= 0 ||
          (int64_t)q.N * q.K >= (1ll << 31))
        return fail("lgx_ppo_tail: bad S8 entry");
      if (i > 0 && q.p0 < a->s8[i - 1].p0) return fail("lgx_ppo_tail: S8 entries must be sorted by p0");
      if (i > 0 && q.p0 == a->s8[i - 1].p0 && (q.N != a->s8[i - 1].N || q.K != a->s8[i - 1].K))
        return fail("lgx_ppo_tail: S8 entries of one weight disagree on its shape");
      k.s[i] = q;
    }
    int nr = 0, blk = 0;
    auto add = [&](int64_t lo, int64_t hi, int opt, int seg0, int nseg) -> bool {
      if (hi <= lo) return true;
      if (nr >= lgxm::TAIL_RMAX) return false;
      lgxm::TailRange& r = k.r[nr++];
      r.lo = lo; r.hi = hi; r.opt = opt; r.seg0 = seg0; r.nseg = nseg; r.blk0 = blk;
      blk += (int)std::max<int64_t>(1, (hi - lo + TAIL_ELEMS - 1) / TAIL_ELEMS);
      return true;
    };
    const int64_t segs[2][2] = {{a->main_lo, a->main_hi}, {a->est_lo, a->est_hi}};
    bool ok = true;
    for (int o = 0; o < 2 && ok; ++o) {
      int64_t cur = segs[o][0];
      for (int i = 0; i < a->n_s8 && ok;) {
        int j = i;
        while (j < a->n_s8 && a->s8[j].p0 == a->s8[i].p0) ++j;
        if (j - i > 4) return fail("lgx_ppo_tail: more than 4 S8 entries for one weight");
        const int64_t w0 = a->s8[i].p0, w1 = w0 + (int64_t)a->s8[i].N * a->s8[i].K;
        if (w0 >= segs[o][0] && w1 <= segs[o][1]) {
          if (w0 < cur) return fail("lgx_ppo_tail: overlapping S8 weights");
          ok = add(cur, w0, o, 0, 0) && add(w0, w1, o, i, j - i);
          cur = w1;
        } else if (w0 < segs[o][1] && w1 > segs[o][0]) {
          return fail("lgx_ppo_tail: an S8 weight straddles a segment boundary");
        }
        i = j;
      }
      ok = ok && add(cur, segs[o][1], o, 0, 0);
    }
    ok = ok && add(a->adapt_lo, a->adapt_hi, 2, 0, 0);
    if (!ok) return fail("lgx_ppo_tail: too many ranges");
    k.nr = nr;
    k.r[nr].blk0 = blk;
    hipLaunchKernelGGL(lgxm::tail_norms, dim3(lgxm::TAIL_BLOCKS), dim3(256), 0, s, *a);
    if (blk > 0) hipLaunchKernelGGL(lgxm::tail_adam_ranges, dim3(blk), dim3(256), 0, s, k);
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
  }
  hipLaunchKernelGGL(lgxm::tail_norms, dim3(lgxm::TAIL_BLOCKS), dim3(256), 0, s, *a);
  hipLaunchKernelGGL(lgxm::tail_adam, dim3(1024), dim3(256), 0, s, *a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_gae(const lgx_gae_args* a, void* stream) {
  if (!a || a->T < 1 || a->N < 1 || !a->rewards || !a->dones || !a->values || !a->last_values || !a->returns ||
      !a->advantages || !a->moments || !a->ws || !a->counter)
    return fail("lgx_gae: bad arguments");
  hipLaunchKernelGGL(lgxm::gae_kernel, dim3((a->N + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream), *a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_normalize_advantages(float* adv, int64_t n, const double* moments, double count, void* stream) {
  if (n < 0 || (n > 0 && (!adv || !moments)) || !(count >= 2.0)) return fail("lgx_normalize_advantages: bad arguments");
  if (n == 0) return 0;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(lgxm::adv_norm_kernel, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream), adv, n,
                     moments, count);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_mlp_pick_split(int32_t M, int32_t N, int32_t K) {
  const int bn = tile_n(N);
  const int tiles = ((M + lgxm::BM - 1) / lgxm::BM) * ((N + bn - 1) / bn);
  int s = (768 + tiles - 1) / tiles;            // ~3 blocks per CU over 256 CUs
  const int kmax = (K + 255) / 256;             // keep >= 256 rows of K per split
  if (s > kmax) s = kmax;
  if (s > 48) s = 48;
  // cap the partial-sum workspace at ~8 M floats (32 MB)
  const int64_t mn = (int64_t)M * N;
  while (s > 2 && (int64_t)s * mn > (8 << 20)) --s;
  if (s < 1) s = 1;
  return s;
}

// Validates one lgx_gemm_args and fills the kernel's Params; nullptr on success, else the
// reason. *empty: M or N is 0 (nothing to launch).
static const char* to_params(const lgx_gemm_args* a, lgxm::Params& p, bool* empty) {
  using namespace lgxm;
  *empty = false;
  if (!a) return "null args";
  if (a->M < 0 || a->N < 0 || a->K < 0) return "negative size";
  if (a->M == 0 || a->N == 0) { *empty = true; return nullptr; }
  if (!a->A || !a->B || !a->C) return "null operand";
  if ((a->epilogue & LGX_EPI_BIAS) && !a->bias) return "EPI_BIAS without bias";
  if ((a->epilogue & LGX_EPI_DELU) && !a->act) return "EPI_DELU without act";
  const int split = a->split_k < 1 ? 1 : a->split_k;
  if (split > 1 && !a->workspace) return "split_k > 1 needs a workspace";
  const bool cs = a->colsum != nullptr;
  if (cs && (a->a_kcontig || !a->colsum_ws)) return "colsum needs a_kcontig = 0 and colsum_ws";
  if (cs && split == 1) return "colsum requires split_k > 1";
  if (!a->a_kcontig && a->b_kcontig) return "a_kcontig = 0 with b_kcontig = 1 is not built";
  p.A = a->A; p.lda = a->lda; p.B = a->B; p.ldb = a->ldb; p.C = a->C; p.ldc = a->ldc;
  p.M = a->M; p.N = a->N; p.K = a->K; p.epi = a->epilogue; p.bias = a->bias; p.act = a->act;
  p.ld_act = a->ld_act; p.split = split;
  p.kchunk = ((a->K + split - 1) / split + BKS - 1) / BKS * BKS;
  if (p.kchunk == 0) p.kchunk = BKS;
  p.ws = a->workspace;
  p.colsum_ws = a->colsum_ws;
  p.ws_vec = a->N % 4 == 0;  // a float4 of the flat workspace stays inside one row
  return nullptr;
}

int32_t lgx_gemm(const lgx_gemm_args* a, void* stream) {
  using namespace lgxm;
  Params p;
  bool empty;
  if (const char* why = to_params(a, p, &empty)) {
    snprintf(g_err, sizeof(g_err), "lgx_gemm: %s", why);
    return -1;
  }
  if (empty) return 0;
  const int split = p.split;
  const bool cs = a->colsum != nullptr;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int bn = tile_n_for(a->M, a->N, a->a_kcontig != 0);
  const bool ma = a->M % 4 == 0, nb = a->N % 4 == 0;  // m/n-contiguous stagers: whole 4-row groups
  if (a->a_kcontig && !a->b_kcontig) {  // input gradient, W read in place
    if (nb) launch<KV, MV, false>(p, bn, s);
    else launch<KV, MVE, false>(p, bn, s);
  } else if (a->a_kcontig) {
    launch<KV, KV, false>(p, bn, s);
  } else if (cs) {
    if (ma && nb) launch<MV, MV, true>(p, bn, s);
    else if (ma) launch<MV, MVE, true>(p, bn, s);
    else if (nb) launch<MVE, MV, true>(p, bn, s);
    else launch<MVE, MVE, true>(p, bn, s);
  } else {
    if (ma && nb) launch<MV, MV, false>(p, bn, s);
    else launch<MVE, MVE, false>(p, bn, s);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(hipGetErrorString(e));
  if (split > 1 && !a->defer_reduce) {
    const int64_t n = ((int64_t)a->M * a->N + 3) / 4 + (cs ? a->M : 0);  // float4 outputs + bias rows
    hipLaunchKernelGGL(splitk_reduce, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, a->colsum);
    e = hipGetLastError();
    if (e != hipSuccess) return fail(hipGetErrorString(e));
  }
  return 0;
}

// Slots of one residency wave of the GEMM kernel: 256 CUs x blocks per CU (LDS-bound:
// 2 at BN = 128, 3 at BN = 64).
static int group_slots(int bn) { return 256 * (bn == 128 ? 2 : 3); }

int32_t lgx_gemm_group(const lgx_gemm_args* args, int32_t n, void* stream) {
  using namespace lgxm;
  if (n < 0 || n > LGX_GEMM_GROUP_MAX || (n > 0 && !args)) return fail("lgx_gemm_group: 0 <= n <= LGX_GEMM_GROUP_MAX");
  GroupParams g;
  g.n = 0;
  int kind = -1, maxn = 0, maxm = 0;
  for (int i = 0; i < n; ++i) {
    const lgx_gemm_args* a = args + i;
    Params p;
    bool empty;
    if (const char* why = to_params(a, p, &empty)) {
      snprintf(g_err, sizeof(g_err), "lgx_gemm_group: entry %d: %s", i, why);
      return -1;
    }
    if (empty) continue;
    const int k = a->a_kcontig ? (a->b_kcontig ? G_FWD : G_DX) : G_DW;
    if (k == G_DW && !a->colsum) return fail("lgx_gemm_group: weight-gradient entries need colsum");
    if (kind >= 0 && k != kind) return fail("lgx_gemm_group: entries of different kinds");
    if (p.split > 1 && !a->defer_reduce) return fail("lgx_gemm_group: split-K entries need defer_reduce");
    kind = k;
    int mode = 0;
    if (k == G_DX) mode = a->N % 4 != 0;
    if (k == G_DW) mode = (a->M % 4 != 0) | ((a->N % 4 != 0) << 1);
    g.mode[g.n] = mode;
    g.p[g.n] = p;
    maxn = std::max(maxn, a->N);
    maxm = std::max(maxm, a->M);
    ++g.n;
  }
  if (g.n == 0) return 0;
  // longest K chunk first: every XCD starts its costliest tiles first
  for (int i = 1; i < g.n; ++i)
    for (int k = i; k > 0 && g.p[k].kchunk > g.p[k - 1].kchunk; --k) {
      std::swap(g.p[k], g.p[k - 1]);
      std::swap(g.mode[k], g.mode[k - 1]);
    }
  const int bn = kind == G_DW ? dw_tile_n(maxn) : tile_n_for(maxm, maxn, true);
  int64_t tiles128 = 0;
  for (int i = 0; i < g.n; ++i)
    tiles128 += (int64_t)((g.p[i].M + BM - 1) / BM) * ((g.p[i].N + bn - 1) / bn) * g.p[i].split;
  const int bm = group_tile_m(kind, bn, tiles128);
  int total = 0;
  for (int i = 0; i < g.n; ++i) {
    Params& p = g.p[i];
    p.tiles_m = (p.M + bm - 1) / bm;
    p.tiles_n = (p.N + bn - 1) / bn;
    p.tiles = p.tiles_m * p.tiles_n * p.split;
    g.start[i] = total;
    total += (p.tiles + 7) / 8;
  }
  g.start[g.n] = total;
  g.per_xcd = total;
  const int grid = 8 * total;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int nw = group_waves(kind);
#define LGX_GROUP_LAUNCH(K)                                                                                     \
  if (bn == 128 && nw == 8) {                                                                                   \
    static bool attr8 = false;                                                                                  \
    if (!attr8) {                                                                                               \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_group_kernel<K, 128, BM, 8>),              \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes(128));               \
      attr8 = true;                                                                                             \
    }                                                                                                           \
    hipLaunchKernelGGL((gemm_group_kernel<K, 128, BM, 8>), dim3(grid), dim3(512), lds_bytes(128), s, g);       \
  } else if (bn == 128) {                                                                                       \
    static bool attr = false;                                                                                   \
    if (!attr) {                                                                                                \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_group_kernel<K, 128>),                     \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes(128));               \
      attr = true;                                                                                              \
    }                                                                                                           \
    hipLaunchKernelGGL((gemm_group_kernel<K, 128>), dim3(grid), dim3(NT), lds_bytes(128), s, g);               \
  } else {                                                                                                      \
    hipLaunchKernelGGL((gemm_group_kernel<K, 64>), dim3(grid), dim3(NT), lds_bytes(64), s, g);                 \
  }
  if (kind == G_FWD && bm == 64) {
    hipLaunchKernelGGL((gemm_group_kernel<G_FWD, 64, 64>), dim3(grid), dim3(NT), lds_bytes(64, 64), s, g);
  } else if (kind == G_DX && bm == 64) {
    hipLaunchKernelGGL((gemm_group_kernel<G_DX, 64, 64>), dim3(grid), dim3(NT), lds_bytes(64, 64), s, g);
  } else if (kind == G_FWD) {
    LGX_GROUP_LAUNCH(G_FWD)
  } else if (kind == G_DX) {
    LGX_GROUP_LAUNCH(G_DX)
  } else {
    LGX_GROUP_LAUNCH(G_DW)
  }
#undef LGX_GROUP_LAUNCH
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_adaptation_forward(const lgx_adapt_args* a, void* stream) {
  using namespace lgxm;
  if (!a) return fail("lgx_adaptation_forward: null args");
  if (a->B < 0) return fail("lgx_adaptation_forward: B >= 0");
  if (a->B == 0) return 0;
  if (a->H < 1 || a->P < 1 || a->C1 < 1 || a->C2 < 1 || a->C3 < 1 || a->NO < 1 || a->k1 < 1 || a->s1 < 1 ||
      a->k2 < 1 || a->s2 < 1)
    return fail("lgx_adaptation_forward: dimensions must be positive");
  AdaptParams P;
  P.a = *a;
  P.L1 = (a->H - a->k1) / a->s1 + 1;
  P.L2 = (P.L1 - a->k2) / a->s2 + 1;
  if (a->H < a->k1 || P.L1 < a->k2) return fail("lgx_adaptation_forward: history shorter than a kernel");
  if (!a->x || a->ldx < (int64_t)a->H * a->P || !a->w0 || !a->b0 || !a->w1 || !a->b1 || !a->w2 || !a->b2 || !a->wf ||
      !a->bf || !a->out || a->ldo < a->NO)
    return fail("lgx_adaptation_forward: bad operands");
  const int64_t floats = (int64_t)AR * ((int64_t)a->H * a->C1 + (int64_t)P.L1 * a->C2 + (int64_t)P.L2 * a->C3);
  if (floats * 4 > 64 * 1024 || (int64_t)a->B * a->ldx > INT32_MAX)
    return fail("lgx_adaptation_forward: sizes beyond the fused kernel's LDS / 32-bit offsets");
  hipLaunchKernelGGL(adapt_fwd_kernel, dim3((unsigned)((a->B + AR - 1) / AR)), dim3(NT), (size_t)floats * 4,
                     static_cast<hipStream_t>(stream), P);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

#ifdef LGX_ADAPT_CLOCK
int32_t lgx_adapt_set_clock(void* buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(lgxm::g_adclk), &buf, sizeof(void*)) == hipSuccess ? 0 : -1;
}
#endif
int32_t lgx_adaptation_train(const lgx_adapt_train_args* t, void* stream) {
  using namespace lgxm;
  if (!t) return fail("lgx_adaptation_train: null args");
  const lgx_adapt_args* a = &t->f;
  if (a->B < 1 || a->H < 1 || a->P < 1 || a->C1 < 1 || a->C2 < 1 || a->C3 < 1 || a->NO < 1 || a->k1 < 1 ||
      a->s1 < 1 || a->k2 < 1 || a->s2 < 1 || t->blocks < 1)
    return fail("lgx_adaptation_train: dimensions must be positive");
  AdaptTrainParams Q;
  Q.t = *t;
  Q.L1 = (a->H - a->k1) / a->s1 + 1;
  Q.L2 = (Q.L1 - a->k2) / a->s2 + 1;
  if (a->H < a->k1 || Q.L1 < a->k2) return fail("lgx_adaptation_train: history shorter than a kernel");
  if (!a->x || a->ldx < (int64_t)a->H * a->P || !a->w0 || !a->b0 || !a->w1 || !a->b1 || !a->w2 || !a->b2 || !a->wf ||
      !a->bf || (a->out && a->ldo < a->NO) || !t->target || t->ldt < a->NO || !t->gws || !t->loss_ws)
    return fail("lgx_adaptation_train: bad operands");
  auto r4 = [](int v) { return (v + 3) / 4 * 4; };
  auto tiles = [](int m, int n) { return ((m + 15) / 16) * ((n + 15) / 16); };
  Q.Y0P = a->C1 | 1;  // odd pitch: the conv1 windows of a 16-row tile spread over the banks
  Q.W1P = r4(a->k1 * Q.Y0P);
  Q.W2P = r4(a->k2 * a->C2);
  Q.Y2P = r4(Q.L2 * a->C3);
  Q.C2P = r4(a->C2);
  Q.C3P = r4(a->C3);
  Q.NOP = r4(a->NO);
  const int ntn0 = (a->C1 + 15) / 16;
  if (Q.L1 > 4 || Q.L2 > 4 || 4 % ntn0 || (a->P + 3) / 4 > AT_K0 || ATR * a->H * a->P > AT_XPT * NT ||
      ATR * a->NO > AT_TPT * NT || tiles(a->C1, a->P + 1) > 4 * AT_W0 || tiles(a->C2, a->k1 * Q.Y0P + 1) > 4 * AT_W1 ||
      tiles(a->C3, a->k2 * a->C2 + 1) > 4 * AT_W2 || tiles(a->NO, Q.L2 * a->C3 + 1) > 4 * AT_WF)
    return fail("lgx_adaptation_train: encoder shape outside the fused kernel's tiling");
  const int sizes[8] = {a->C1 * a->P, a->C1, a->C2 * a->C1 * a->k1, a->C2, a->C3 * a->C2 * a->k2, a->C3,
                        a->NO * a->C3 * Q.L2, a->NO};
  Q.off[0] = 0;
  for (int i = 0; i < 8; ++i) Q.off[i + 1] = Q.off[i] + sizes[i];
  Q.NP = Q.off[8];
  const int region[AL_END] = {ATR * a->H * a->P, ATR * a->H * Q.Y0P, ATR * Q.L1 * a->C2, ATR * Q.Y2P, ATR * a->NO,
                              ATR * a->NO, Q.C2P * Q.W1P, Q.C3P * Q.W2P, Q.NOP * Q.Y2P,
                              a->C1 + a->C2 + a->C3 + a->NO, 8};
  Q.lds[0] = 0;
  for (int i = 0; i < AL_END; ++i) Q.lds[i + 1] = Q.lds[i] + r4(region[i]);
  const int64_t bytes = (int64_t)Q.lds[AL_END] * 4;
  if (bytes > 80 * 1024 || (int64_t)a->B * a->ldx > INT32_MAX)
    return fail("lgx_adaptation_train: sizes beyond the fused kernel's LDS / 32-bit offsets");
  const int nchunk = (a->B + ATR - 1) / ATR;
  Q.chunks = (nchunk + t->blocks - 1) / t->blocks;
  const unsigned grid = (unsigned)((nchunk + Q.chunks - 1) / Q.chunks);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)adapt_train_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(adapt_train_kernel, dim3(grid), dim3(NT), (size_t)bytes, static_cast<hipStream_t>(stream), Q);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_chain(const lgx_chain_desc* chains, int32_t n, void* stream) {
  using namespace lgxm;
  if (n < 0 || n > LGX_CHAIN_MAX || (n > 0 && !chains)) return fail("lgx_chain: 0 <= n <= LGX_CHAIN_MAX");
  ChainParams P;
  P.n = 0;
  int maxw = 0, maxn = 0, maxrows = 0;
  for (int i = 0; i < n; ++i) {
    const lgx_chain_desc& d = chains[i];
    if (d.rows < 0 || d.nlayers < 1 || d.nlayers > LGX_CHAIN_MAXL) return fail("lgx_chain: rows >= 0, 1 <= nlayers <= LGX_CHAIN_MAXL");
    if (d.rows == 0) continue;
    if (!d.A || d.lda < d.layers[0].K) return fail("lgx_chain: bad input");
    for (int l = 0; l < d.nlayers; ++l) {
      const lgx_chain_layer& L = d.layers[l];
      if (L.K < 1 || L.N < 1 || L.K > LGX_CHAIN_MAXW || L.N > LGX_CHAIN_MAXW)
        return fail("lgx_chain: layer widths must lie in [1, LGX_CHAIN_MAXW]");
      if (l > 0 && L.K != d.layers[l - 1].N) return fail("lgx_chain: K of a layer must be N of the previous one");
      if (!L.B || L.ldb < L.K || !L.C || L.ldc < L.N) return fail("lgx_chain: bad layer operands");
      if (L.epilogue & ~(LGX_EPI_BIAS | LGX_EPI_ELU | LGX_EPI_DELU)) return fail("lgx_chain: epilogue bits BIAS/ELU/DELU only");
      if (((L.epilogue & LGX_EPI_BIAS) && !L.bias) || ((L.epilogue & LGX_EPI_DELU) && (!L.act || L.ld_act < L.N)))
        return fail("lgx_chain: epilogue operand missing");
      maxw = std::max(maxw, std::max((int)L.K, (int)L.N));
      maxn = std::max(maxn, (int)L.N);
    }
    P.c[P.n++] = d;
    maxrows = std::max(maxrows, (int)d.rows);
  }
  if (P.n == 0) return 0;
  // 64-row blocks for narrow chains over many rows, else 32 (LDS: 2 images x 2 planes)
  const int br = (maxw <= 128 && maxrows > 8192) ? 64 : 32;
  P.ip = ((maxw + 31) / 32) * 32 + 8;
  int total = 0;
  for (int i = 0; i < P.n; ++i) {
    P.start[i] = total;
    total += (P.c[i].rows + br - 1) / br;
  }
  P.start[P.n] = total;
  const int njw = ((maxn + 15) / 16 + 3) / 4;  // 16-wide column tiles per wave
  const size_t lds = (size_t)2 * br * P.ip * sizeof(__bf16);  // one image, hi | lo
  hipStream_t s = static_cast<hipStream_t>(stream);
#define LGX_CHAIN_LAUNCH(BR_, NJ_)                                                                     \
  {                                                                                                    \
    static bool attr = false;                                                                          \
    if (!attr) {                                                                                       \
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&chain_kernel<BR_, NJ_>),                \
                                hipFuncAttributeMaxDynamicSharedMemorySize, 2 * BR_ * (256 + 8) * 2);  \
      attr = true;                                                                                     \
    }                                                                                                  \
    hipLaunchKernelGGL((chain_kernel<BR_, NJ_>), dim3(total), dim3(NT), lds, s, P);                   \
  }
  if (br == 64) {
    if (njw == 1) LGX_CHAIN_LAUNCH(64, 1) else LGX_CHAIN_LAUNCH(64, 2)
  } else {
    if (njw == 1) LGX_CHAIN_LAUNCH(32, 1) else if (njw == 2) LGX_CHAIN_LAUNCH(32, 2) else LGX_CHAIN_LAUNCH(32, 4)
  }
#undef LGX_CHAIN_LAUNCH
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_mlp_pick_split_group(const int32_t* M, const int32_t* N, const int32_t* K, int32_t n, int32_t* split) {
  if (n < 1 || n > LGX_GEMM_GROUP_MAX || !M || !N || !K || !split) return fail("lgx_mlp_pick_split_group: bad arguments");
  int maxn = 0;
  for (int i = 0; i < n; ++i) {
    if (M[i] < 0 || N[i] < 0 || K[i] < 0) return fail("lgx_mlp_pick_split_group: negative size");
    maxn = std::max(maxn, (int)N[i]);
  }
  const int bn = dw_tile_n(maxn);
  // LGX_DW_SLOTS: dev knob (block budget of the grouped weight-gradient launch)
  const char* knob = LGX_DEV_KNOB("LGX_DW_SLOTS");
  const int slots = knob ? std::max(64, atoi(knob)) : group_slots(bn);
  // equal K chunks for every problem: the smallest chunk (a multiple of the K step, at least
  // 256 rows) whose block count fits one residency wave; every split >= 2 (bias gradient)
  int chunk = 256;
  for (;; chunk += lgxm::BKS) {
    int64_t blocks = 0, kmax = 0;
    for (int i = 0; i < n; ++i) {
      const int64_t tiles = (int64_t)((M[i] + lgxm::BM - 1) / lgxm::BM) * ((N[i] + bn - 1) / bn);
      blocks += tiles * std::max(2, (K[i] + chunk - 1) / chunk);
      kmax = std::max<int64_t>(kmax, K[i]);
    }
    if (blocks <= slots || chunk >= kmax) break;
  }
  for (int i = 0; i < n; ++i) split[i] = std::max(2, (K[i] + chunk - 1) / chunk);
  return 0;
}

int32_t lgx_splitk_reduce_batch(const lgx_splitk_desc* descs, int32_t n, void* stream) {
  if (n < 0 || n > LGX_SPLITK_MAX || (n > 0 && !descs)) return fail("lgx_splitk_reduce_batch: 0 <= n <= LGX_SPLITK_MAX");
  if (n == 0) return 0;
  lgxm::SplitkBatch b;
  int64_t most = 0;
  for (int i = 0; i < n; ++i) {
    const lgx_splitk_desc& d = descs[i];
    if (d.M < 0 || d.N < 0 || d.split < 1 || !d.ws || !d.C || (d.colsum && !d.colsum_ws))
      return fail("lgx_splitk_reduce_batch: bad entry");
    if (d.N % 4 == 0 && (reinterpret_cast<uintptr_t>(d.ws) & 15) != 0)
      return fail("lgx_splitk_reduce_batch: workspace must be 16-B aligned");
    b.d[i] = d;
    const int64_t items = ((int64_t)d.M * d.N + 3) / 4 + (d.colsum ? d.M : 0);
    most = items > most ? items : most;
  }
  if (most == 0) return 0;
  const unsigned bx = (unsigned)std::min<int64_t>((most + 255) / 256, 2048);
  hipLaunchKernelGGL(lgxm::splitk_reduce_batch, dim3(bx, (unsigned)n), dim3(256), 0, static_cast<hipStream_t>(stream),
                     b);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_transpose_batch(const lgx_transpose_desc* descs, int32_t n, void* stream) {
  if (n < 0 || n > LGX_TRANSPOSE_MAX || (n > 0 && !descs)) return fail("lgx_transpose_batch: 0 <= n <= LGX_TRANSPOSE_MAX");
  if (n == 0) return 0;
  lgxm::TransposeBatch b;
  int most = 0;
  for (int i = 0; i < n; ++i) {
    const lgx_transpose_desc& d = descs[i];
    if (d.rows < 0 || d.cols < 0 || d.ld < d.cols || ((int64_t)d.rows * d.cols > 0 && (!d.src || !d.dst)))
      return fail("lgx_transpose_batch: bad entry");
    b.d[i] = d;
    most = std::max(most, ((d.rows + 31) / 32) * ((d.cols + 31) / 32));
  }
  if (most == 0) return 0;
  hipLaunchKernelGGL(lgxm::transpose_batch_kernel, dim3((unsigned)std::min(most, 256), 1, (unsigned)n), dim3(256), 0,
                     static_cast<hipStream_t>(stream), b);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_copy_batch(const lgx_copy_desc* descs, int32_t n, void* stream) {
  if (n < 0 || n > LGX_COPY_MAX || (n > 0 && !descs)) return fail("lgx_copy_batch: 0 <= n <= LGX_COPY_MAX");
  if (n == 0) return 0;
  lgxm::CopyBatch cb;
  int64_t most = 0;
  for (int i = 0; i < n; ++i) {
    if (descs[i].nbytes < 0 || (descs[i].nbytes > 0 && (!descs[i].src || !descs[i].dst)))
      return fail("lgx_copy_batch: bad entry");
    cb.d[i] = descs[i];
    most = descs[i].nbytes > most ? descs[i].nbytes : most;
  }
  cb.n = n;
  if (most == 0) return 0;
  // enough blocks per entry to stream the largest at full rate (16 B per thread per pass)
  const int64_t chunks = (most + 15) / 16;
  const unsigned bx = (unsigned)std::min<int64_t>((chunks + 255) / 256, 1024);
  hipLaunchKernelGGL(lgxm::copy_batch_kernel, dim3(bx, (unsigned)n), dim3(256), 0, static_cast<hipStream_t>(stream),
                     cb);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_gather_rows(const lgx_copy_desc* descs, int32_t n, const int64_t* idx, int64_t rows, void* stream) {
  if (n < 0 || n > LGX_COPY_MAX || (n > 0 && !descs) || rows < 0 || (rows > 0 && !idx))
    return fail("lgx_gather_rows: bad arguments");
  if (n == 0 || rows == 0) return 0;
  lgxm::CopyBatch cb;
  int64_t most = 0;
  for (int i = 0; i < n; ++i) {
    if (descs[i].nbytes < 0 || descs[i].nbytes % 4 != 0 || (descs[i].nbytes > 0 && (!descs[i].src || !descs[i].dst)))
      return fail("lgx_gather_rows: bad entry (row bytes must be a multiple of 4)");
    if (descs[i].dst_stride != 0 && (descs[i].dst_stride < descs[i].nbytes || descs[i].dst_stride % 4 != 0))
      return fail("lgx_gather_rows: dst_stride must be 0 or a multiple of 4 >= the row bytes");
    if (rows * (descs[i].nbytes / 4) >= (int64_t)1 << 31) return fail("lgx_gather_rows: rows * row elements >= 2^31");
    cb.d[i] = descs[i];
    most = descs[i].nbytes > most ? descs[i].nbytes : most;
  }
  cb.n = n;
  const int64_t work = rows * ((most + 15) / 16);
  const unsigned bx = (unsigned)std::min<int64_t>((work + 255) / 256, 2048);
  hipLaunchKernelGGL(lgxm::gather_rows_kernel, dim3(bx, (unsigned)n), dim3(256), 0, static_cast<hipStream_t>(stream),
                     cb, idx, rows);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_act_head(const lgx_act_head_args* a, void* stream) {
  if (!a || !a->mean || !a->std || !a->actions || !a->mu || !a->sigma || !a->logp || a->B < 0 || a->A <= 0 ||
      a->A > lgxm::HMAXA)
    return fail("lgx_act_head: bad arguments");
  if (!a->eps && (!a->step_dev || a->env_offset < 0 || a->env_offset + a->B > (int64_t)UINT32_MAX))
    return fail("lgx_act_head: eps == NULL needs step_dev and a 32-bit global env range");
  if (a->B == 0) return 0;
  hipLaunchKernelGGL(lgxm::act_head_kernel, dim3((unsigned)((4 * (int64_t)a->B + 255) / 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), *a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

}  // extern "C"

namespace lgxm {
// on_policy_runner.py:160-170 bookkeeping: one workgroup of 1024 threads, each owning a
// contiguous chunk of envs; the done count per chunk is scanned across the block so every
// done env knows its rank among all done envs (env order, as torch.cumsum gives).
__device__ __forceinline__ void track_block(const lgx_track_args& a);
__global__ __launch_bounds__(1024) void track_kernel(lgx_track_args a) { track_block(a); }

// The rollout step's transition row and episode bookkeeping in ONE launch (lgx_post_step):
// blocks 0 .. nt-1 (1024 threads) store the transition, block nt runs track_block. The two read
// the same env outputs and write disjoint buffers, so their blocks need no ordering.
__global__ __launch_bounds__(1024) void post_step_kernel(lgx_transition_args p, lgx_track_args a, int nt) {
  if ((int)blockIdx.x < nt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.B) return;
    const float v = p.values[i];
    float r = p.rewards[i];
    const bool d = p.dones[i] != 0;
    if (p.time_outs) r = r + p.gamma * (v * (float)p.time_outs[i]);
    p.rewards_out[i] = r;
    p.dones_out[i] = d ? 1 : 0;
    p.values_out[i] = v;
    return;
  }
  track_block(a);
}

__device__ __forceinline__ void track_block(const lgx_track_args& a) {
  __shared__ int wsum[16];
  __shared__ int k_all;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int chunk = (a.N + 1023) / 1024;
  const int i0 = min(tid * chunk, a.N), i1 = min(i0 + chunk, a.N);
  const int64_t ptr = *a.ptr;  // every thread reads it before thread 0 moves it (barriers below)
  // 4 or 8 envs per thread with aligned rows (N = 4096 / 8192): the thread's rows as float4 /
  // 4-byte loads, all issued before any use — one memory round trip instead of one per env
  const bool vec = (chunk == 4 || chunk == 8) && a.N % chunk == 0 &&
                   ((reinterpret_cast<uintptr_t>(a.cur_rew) | reinterpret_cast<uintptr_t>(a.cur_len) |
                     reinterpret_cast<uintptr_t>(a.rewards)) & 15) == 0 && (reinterpret_cast<uintptr_t>(a.dones) & 3) == 0;
  float4 cr[2], rw[2], cl[2];
  uint32_t dn[2] = {0u, 0u};
  int cnt = 0;
  if (vec) {
    const int nv = chunk / 4, q0 = tid * nv;
    for (int v = 0; v < 2; ++v) {
      if (v >= nv || i0 >= i1) continue;
      cr[v] = reinterpret_cast<const float4*>(a.cur_rew)[q0 + v];
      cl[v] = reinterpret_cast<const float4*>(a.cur_len)[q0 + v];
      rw[v] = reinterpret_cast<const float4*>(a.rewards)[q0 + v];
      dn[v] = reinterpret_cast<const uint32_t*>(a.dones)[q0 + v];
    }
    for (int v = 0; v < 2; ++v)
      for (int e = 0; e < 4; ++e) cnt += ((dn[v] >> (8 * e)) & 0xffu) != 0u;
  } else {
    for (int i = i0; i < i1; ++i) cnt += a.dones[i] != 0;
  }
  // inclusive scan over the block: within the wave by shuffles, then over the 16 waves
  int x = cnt;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wv] = x;
  __syncthreads();
  if (tid == 0) {
    int t = 0;
    for (int w = 0; w < 16; ++w) {
      const int v = wsum[w];
      wsum[w] = t;
      t += v;
    }
    k_all = t;
  }
  __syncthreads();
  const int k = k_all;
  int rank = wsum[wv] + x - cnt;  // exclusive prefix of this thread's chunk
  // env i's update; returns its new (cur_rew, cur_len)
  auto one = [&](float cur_r, float rew, float cur_l, bool done, float& nr, float& nl) {
    const float r = cur_r + rew;
    const float l = cur_l + 1.0f;
    if (done) {
      if (rank >= k - 100) {
        const int slot = (int)((ptr + rank) % 100);
        a.rew_ring[slot] = r;
        a.len_ring[slot] = l;
      }
      ++rank;
      nr = 0.f;
      nl = 0.f;
    } else {
      nr = r;
      nl = l;
    }
  };
  if (vec) {
    const int nv = chunk / 4, q0 = tid * nv;
    for (int v = 0; v < 2; ++v) {
      if (v >= nv || i0 >= i1) continue;
      float4 R, L;
      one(cr[v].x, rw[v].x, cl[v].x, (dn[v] & 0xffu) != 0u, R.x, L.x);
      one(cr[v].y, rw[v].y, cl[v].y, ((dn[v] >> 8) & 0xffu) != 0u, R.y, L.y);
      one(cr[v].z, rw[v].z, cl[v].z, ((dn[v] >> 16) & 0xffu) != 0u, R.z, L.z);
      one(cr[v].w, rw[v].w, cl[v].w, ((dn[v] >> 24) & 0xffu) != 0u, R.w, L.w);
      reinterpret_cast<float4*>(a.cur_rew)[q0 + v] = R;
      reinterpret_cast<float4*>(a.cur_len)[q0 + v] = L;
    }
  } else {
    for (int i = i0; i < i1; ++i) {
      float nr, nl;
      one(a.cur_rew[i], a.rewards[i], a.cur_len[i], a.dones[i] != 0, nr, nl);
      a.cur_rew[i] = nr;
      a.cur_len[i] = nl;
    }
  }
  __syncthreads();  // every thread read *ptr before it moves
  if (tid == 0) {
    *a.ptr = (ptr + k) % 100;
    const int64_t n = *a.n + k;
    *a.n = n < 100 ? n : 100;
    if (a.ep_cnt) *a.ep_cnt += 1.0f;
  }
  if (a.ep_sum) {
    if (tid < a.na) a.ep_sum[tid] += a.ep_a[tid];
    else if (tid < a.na + a.nb) a.ep_sum[tid] += a.ep_b[tid - a.na];
  }
}
}  // namespace lgxm

extern "C" {

int32_t lgx_track_episodes(const lgx_track_args* a, void* stream) {
  if (!a || !a->rewards || !a->dones || !a->cur_rew || !a->cur_len || !a->rew_ring || !a->len_ring || !a->ptr ||
      !a->n || a->N < 0 || a->na < 0 || a->nb < 0 || a->na + a->nb > 1024 ||
      (a->ep_sum && (!a->ep_cnt || (a->na && !a->ep_a) || (a->nb && !a->ep_b))))
    return fail("lgx_track_episodes: bad arguments");
  hipLaunchKernelGGL(lgxm::track_kernel, dim3(1), dim3(1024), 0, static_cast<hipStream_t>(stream), *a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

int32_t lgx_post_step(const lgx_transition_args* t, const lgx_track_args* a, void* stream) {
  if (!a) return lgx_store_transition(t, stream);
  if (!t || !t->rewards || !t->dones || !t->values || !t->rewards_out || !t->dones_out || !t->values_out || t->B < 0)
    return fail("lgx_post_step: bad transition arguments");
  if (!a->rewards || !a->dones || !a->cur_rew || !a->cur_len || !a->rew_ring || !a->len_ring || !a->ptr ||
      !a->n || a->N < 0 || a->na < 0 || a->nb < 0 || a->na + a->nb > 1024 ||
      (a->ep_sum && (!a->ep_cnt || (a->na && !a->ep_a) || (a->nb && !a->ep_b))))
    return fail("lgx_post_step: bad tracking arguments");
  const int nt = (t->B + 1023) / 1024;
  hipLaunchKernelGGL(lgxm::post_step_kernel, dim3(nt + 1), dim3(1024), 0, static_cast<hipStream_t>(stream), *t, *a, nt);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}
int32_t lgx_store_transition(const lgx_transition_args* a, void* stream) {
  if (!a || !a->rewards || !a->dones || !a->values || !a->rewards_out || !a->dones_out || !a->values_out || a->B < 0)
    return fail("lgx_store_transition: bad arguments");
  if (a->B == 0) return 0;
  hipLaunchKernelGGL(lgxm::transition_kernel, dim3((a->B + 255) / 256), dim3(256), 0,
                     static_cast<hipStream_t>(stream), *a);
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : fail(hipGetErrorString(e));
}

}  // extern "C"
