// lgx_s8.hip — the learner's GEMM core on pre-split (S8) operands, gfx950 (include/lgx_s8.h).
//
// Every operand arrives as bf16 hi/lo planes interleaved per 8 columns (S8), written by the
// kernel that produced it (forward / input-gradient epilogues here, lgx_s8_split for weights,
// inputs and the loss heads' gradients). So the K loop moves bytes and multiplies: no fp32 ->
// bf16 split, no VGPR round trip.
//
// Block: 256 threads = 4 waves as 2 x 2, output tile 128 x 128, each wave 64 x 64 = 4 x 4
// tiles of v_mfma_f32_16x16x32_bf16; per product lo*hi + hi*lo + hi*hi (3 x bf16, fp32
// accumulation; lgx_mlp.hip's order). K step 32, 2 LDS stages, 2 blocks per CU (lgxs::Cfg).
// Staging: global_load_lds_dwordx4 (LDS-DMA; destination = wave base + 16 B x lane), 8 per wave
// per K step, NS - 1 steps in flight across raw s_barriers with a counted vmcnt — no barrier
// drains the DMA (cdna_hip_programming.md §5 "Pipelining across barriers"). Images:
//   ROW operand (k along the source row): [128 rows][32 k] = 128-B rows, 8 slots of 16 B
//       (hi g0, lo g0, hi g1, ...); fragments by ds_read_b128 (8 consecutive k of one row).
//   TR operand (k = source row): [32 k][128 cols] = 512-B rows (the source row's 128-column
//       span verbatim); fragments by ds_read_b64_tr_b16 (4 k x 16 columns, delivered per column).
// The 16-B slots are XOR-swizzled by a function of the image row — applied to the DMA's per-lane
// SOURCE address (the destination is lane-linear) and to the read address — so every fragment
// read is bank-conflict free (tools/exp/s8_banks.py, MI355X_MICROARCH.md §LDS bank model).
// Epilogue through an fp32 LDS image of the tile: FWD bias + ELU, DX * ELU'(y_prev) (+ addend),
// both written as S8 (32 B per lane: 8 columns' hi + lo) and/or fp32, with the column sums of each
// 128-row tile (the next weight gradient's bias gradient); DW fp32 split-K partials.
#include <hip/hip_runtime.h>
#include "lgx_knobs.h"
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

#include "../../include/lgx_s8.h"

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4u __attribute__((ext_vector_type(4), aligned(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// MFMA issue order of a K step: each accumulator's three products back to back (lo*hi, hi*lo,
// hi*hi), then the next accumulator. Left to itself the scheduler groups the MFMAs by a shared
// operand register (one fragment held over 4 consecutive MFMAs, the accumulators rotating); the
// per-accumulator chain draws less power at the same per-clock MFMA issue rate, so the chip holds
// a higher clock under the K loop (measured: tools/exp/mfma_power.hip). A
// scheduling barrier after each MFMA pins the source order; the products and their accumulation
// order are the same either way (bit-identical results).
#ifndef LGX_S8_MFMA_CHAIN
#define LGX_S8_MFMA_CHAIN 1
#endif
#if LGX_S8_MFMA_CHAIN
#define S8_MFMA_ORDER() __builtin_amdgcn_sched_barrier(0)
#else
#define S8_MFMA_ORDER() do { } while (0)
#endif
#define LDS_AS __attribute__((address_space(3)))

#ifndef LGX_S8_BK
#define LGX_S8_BK 32
#endif

namespace lgxs {

constexpr int BK = LGX_S8_BK, BN = 128, NJ = 4, GMAX = LGX_S8_GROUP_MAX;
static_assert(BK == 32, "K step 32 (a 64-deep build fails the whole-update test: profiles/r06_bk64_note.txt)");
constexpr int CP = BN + 4;  // fp32 epilogue image pitch (floats)
// Output tile 128 x 128, 4 waves as 2 x 2 (each 64 x 64 = 4 x 4 MFMA tiles), 2 LDS stages of
// 32 KB, 2 blocks per CU. Measured and not kept: 256 x 128 and 128 x 128 tiles
// at 3-4 stages and 1 block per CU, and a 256 x 256 tile whose two wave rows run a barrier apart
// (reads of one row beside the MFMAs of the other) — all slower on these shapes.
struct Cfg {
  static constexpr int BM = 128, NS = 2, NW = 4, NT = 256, WR = 2;
  static constexpr int LDS_STAGES = NS * (BM + BN) * BK * 4, LDS_EPI = BM * CP * 4;
  static constexpr int LDS = LDS_STAGES > LDS_EPI ? LDS_STAGES : LDS_EPI;
};

// ---- per-block cycle accounts (dev builds only: -DLGX_S8_CLOCK, tools/s8_clock.py): waves 0 and
// NW - 1 of every block sum clock64 deltas of the K loop's DMA wait, barrier and issue + compute
// sections and of the epilogue, into g_s8clk[block][wave slot][12]. Compiled out of the product.
#ifdef LGX_S8_CLOCK
__device__ uint32_t* g_s8clk = nullptr;
#endif

// slot swizzles (16-B slot index XOR), image row -> mask
__device__ __forceinline__ int fsw_row(int r) {
  if constexpr (BK == 32) return ((r >> 1) & 1) | (((r >> 3) & 1) << 2);  // 8 slots per 128-B row
  return (r & 15) ^ ((((r >> 2) ^ (r >> 3)) & 1) << 1);                     // 16 slots per 256-B row
}
__device__ __forceinline__ int fsw_tr(int k) { return (k & 1) | ((k & 2) << 1) | (k & 8); }

struct Prob {
  const char* A; const char* B;
  int64_t lda, ldb;            // bytes
  int M, N, K;
  int tiles_m, tiles_n, tiles;  // tiles includes the split
  int kchunk, epi;
  char* C; int64_t ldc;         // bytes (S8)
  float* C32; int64_t ldc32;    // floats
  const float* bias;
  const char* act; int64_t ld_act;  // bytes (S8)
  const float* addend; int64_t ld_add;
  int add_cols, pad;
  float* colsum_ws;
};

// XCD units (weight gradients): whole K-chunk slices of a problem (all its output tiles of one
// K chunk) dealt to one XCD each, so that every operand byte of a chunk is fetched into one L2
// only (the tiles of a slice share its dY and X rows). units[ustart[x] .. ustart[x + 1]) are XCD
// slot x's slices in order, each pi | z << 5, covering tiles_m * tiles_n consecutive jb.
constexpr int UMAX = 256;
struct Group {
  int n, per_xcd;
  int start[GMAX + 1];
  Prob p[GMAX];
  int nunits;
  uint16_t ustart[9];
  uint16_t units[UMAX];
};
static_assert(sizeof(Group) <= 4096, "kernel argument segment");

// An operand's staging geometry (one K step).
// T = the tile's extent along this operand (BM for A, BN for B); NW = waves of the block.
template <bool TR, int T, int NW>
struct Op {
  static constexpr int PITCH = TR ? T * 4 : BK * 4;  // image row bytes
  static constexpr int SLOTS = PITCH / 16;
  static constexpr int RPI = 1024 / PITCH;           // image rows per DMA wave-instruction
  static constexpr int NI = T * BK * 4 / 1024;       // DMA wave-instructions per step
  static constexpr int PW = NI / NW;                 // per wave
  static constexpr int IMG = T * BK * 4;             // bytes
  static_assert(PW * NW == NI && RPI >= 1, "DMA split");

  // per-lane 32-bit source offsets of this wave's instructions (step 0); t0 = the tile's first
  // m / n, R = M / N (the operand's extent along the tile), ld = row pitch (bytes)
  __device__ __forceinline__ static void offsets(uint32_t (&off)[PW], int wave, int lane, int t0, int R,
                                                 int64_t ld, int kbeg) {
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      const int i = wave + NW * j;
      const int r = i * RPI + lane / SLOTS, ps = lane % SLOTS;
      if (TR) {  // r = k (source row kbeg + r), columns t0 .. t0 + 127
        // columns clamped to the operand's own groups [0, round_up(R, 8)) — the span the
        // producer wrote — never the row pitch: an operand may start past column 0 of a wider
        // row (a column span), and reading to the pitch would run past the buffer's last row
        const int ls = ps ^ fsw_tr(r);
        const int64_t cb = std::min<int64_t>((int64_t)t0 * 4 + ls * 16, (int64_t)((R + 7) / 8) * 32 - 16);
        off[j] = (uint32_t)((int64_t)(kbeg + r) * ld + cb);
      } else {   // r = tile row (source row t0 + r, clamped), k from kbeg
        const int ls = ps ^ fsw_row(r);
        const int row = std::min(t0 + r, R - 1);
        off[j] = (uint32_t)((int64_t)row * ld + (int64_t)kbeg * 4 + ls * 16);
      }
    }
  }
  // step s's source advance (uniform)
  __device__ __forceinline__ static int64_t step_bytes(int64_t ld) { return TR ? (int64_t)BK * ld : BK * 4; }

  // The DMA is issued by inline asm so that hipcc does not see an LDS write in flight: with the
  // builtin it waits vmcnt(0) before every ds_read of the tile (alias analysis cannot separate
  // the stages of one LDS array), which would serialise the load of step k + 1 with the compute
  // of step k. The ring's own counted vmcnt + s_barrier order it (the main loop). `lds_addr` is
  // the wave-uniform LDS byte address of this operand's image in the stage.
  __device__ __forceinline__ static void issue(const char* base, const uint32_t (&off)[PW], uint32_t lds_addr,
                                               int wave) {
#pragma unroll
    for (int j = 0; j < PW; ++j) {
      const uint32_t m0 = lds_addr + (uint32_t)(wave + NW * j) * 1024u;
      asm volatile(
          "s_mov_b32 m0, %2\n\t"
          "s_nop 0\n\t"
          "global_load_lds_dwordx4 %0, %1"
          :
          : "v"(off[j]), "s"(base), "s"(m0)
          : "memory", "m0");
    }
  }

  // fragment (hi, lo) of 16 tile rows/cols starting at t (multiple of 16), k 32 kk .. 32 kk + 31
  __device__ __forceinline__ static void frag(const char* img, int t, int kk, int lane, bf16x8& hi, bf16x8& lo) {
    if (TR) {
      const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
      const int ls = 2 * ((t >> 3) + (p >> 1));
      s16x4 h[2], l[2];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int k = 32 * kk + 8 * G + 4 * hh + q;
        const char* row = img + k * PITCH + (p & 1) * 8;
        const int f = fsw_tr(k);
        h[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(row + ((ls ^ f) << 4)));
        l[hh] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(row + (((ls + 1) ^ f) << 4)));
      }
      const s16x8 H = {h[0][0], h[0][1], h[0][2], h[0][3], h[1][0], h[1][1], h[1][2], h[1][3]};
      const s16x8 L = {l[0][0], l[0][1], l[0][2], l[0][3], l[1][0], l[1][1], l[1][2], l[1][3]};
      hi = __builtin_bit_cast(bf16x8, H);
      lo = __builtin_bit_cast(bf16x8, L);
    } else {
      const int r = t + (lane & 15), g = lane >> 4;
      const int f = fsw_row(r);
      const char* row = img + r * PITCH;
      hi = *reinterpret_cast<const bf16x8*>(row + (((8 * kk + 2 * g) ^ f) << 4));
      lo = *reinterpret_cast<const bf16x8*>(row + (((8 * kk + 2 * g + 1) ^ f) << 4));
    }
  }
};

__device__ __forceinline__ float elu(float v) {  // lgx_mlp.hip's ELU (same polynomial / exp switch)
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

__device__ __forceinline__ unsigned pack2(__bf16 a, __bf16 b) {
  return (unsigned)__builtin_bit_cast(unsigned short, a) | ((unsigned)__builtin_bit_cast(unsigned short, b) << 16);
}
// 8 fp32 -> hi x 8 at h, lo x 8 at l
__device__ __forceinline__ void store_s8x(char* hp, char* lp, const float (&v)[8]) {
  __bf16 h[8], l[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    h[e] = (__bf16)v[e];
    l[e] = (__bf16)(v[e] - (float)h[e]);
  }
  const u32x4 H = {pack2(h[0], h[1]), pack2(h[2], h[3]), pack2(h[4], h[5]), pack2(h[6], h[7])};
  const u32x4 L = {pack2(l[0], l[1]), pack2(l[2], l[3]), pack2(l[4], l[5]), pack2(l[6], l[7])};
  *reinterpret_cast<u32x4*>(hp) = H;
  *reinterpret_cast<u32x4*>(lp) = L;
}
// 8 fp32 -> S8 group (32 B: hi x 8, lo x 8)
__device__ __forceinline__ void store_s8(char* dst, const float (&v)[8]) { store_s8x(dst, dst + 16, v); }
__device__ __forceinline__ void load_s8(const char* src, float (&v)[8]) {
  const u32x4 H = reinterpret_cast<const u32x4*>(src)[0];
  const u32x4 L = reinterpret_cast<const u32x4*>(src)[1];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = __uint_as_float(H[e] << 16) + __uint_as_float(L[e] << 16);
    v[2 * e + 1] = __uint_as_float(H[e] & 0xffff0000u) + __uint_as_float(L[e] & 0xffff0000u);
  }
}

// ---- epilogues over an fp32 LDS image [ROWS][CPI] of output rows m_base.., columns n_base..
// DW: fp32 rows (float4): split partial slab z, or the output itself (split 1, optional accumulate)
template <int NT, int ROWS, int COLS, int CPI>
__device__ __forceinline__ void epi_dw(const Prob& P, const float* img, int m_base, int n_base, int z, int tid) {
  const bool part = P.tiles > P.tiles_m * P.tiles_n;
  float* dst = part ? P.C32 + (int64_t)z * P.M * P.N : P.C32;
  const int64_t ldd = part ? P.N : P.ldc32;
  const bool accum = !part && (P.epi & LGX_S8_EPI_ACCUM);
  constexpr int Q = COLS / 4;  // float4 per row
#pragma unroll
  for (int it = 0; it < ROWS * Q / NT; ++it) {
    const int idx = tid + it * NT;
    const int row = idx / Q, c = (idx % Q) * 4;
    const int m = m_base + row, n = n_base + c;
    if (m >= P.M || n >= P.N) continue;
    const f32x4 t = *reinterpret_cast<const f32x4*>(img + row * CPI + c);
    float* d = dst + (int64_t)m * ldd + n;
    if (n + 4 <= P.N) {
      f32x4u o = {t[0], t[1], t[2], t[3]};
      if (accum) o += *reinterpret_cast<const f32x4u*>(d);
      *reinterpret_cast<f32x4u*>(d) = o;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (n + e < P.N) d[e] = accum ? d[e] + t[e] : t[e];
    }
  }
}

// FWD / DX: thread = one 8-column group (gq) of rows r0 + RS it; FWD bias + ELU, DX ELU'(y_prev)
// (+ addend); S8 and/or fp32 out; the column sums of each 128-row span (partial part0 + h), in a
// fixed order (the same order for every tile configuration: RS = 16 row slots)
template <int KIND, int NT, int ROWS, int COLS, int CPI>
__device__ __forceinline__ void epi_act(const Prob& P, float* img, int m_base, int n_base, int part0, int tid) {
  constexpr int G = COLS / 8, RS = NT / G, NH = ROWS / LGX_S8_TILE_M;
  static_assert(RS == 16 && ROWS % LGX_S8_TILE_M == 0, "epilogue row slots");
  const int gq = tid % G, r0 = tid / G;
  const int n = n_base + 8 * gq;
  float cs[NH][8];
#pragma unroll
  for (int h = 0; h < NH; ++h)
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[h][e] = 0.f;
  float bias[8];
  if constexpr (KIND == LGX_S8_FWD) {
#pragma unroll
    for (int e = 0; e < 8; ++e) bias[e] = (P.epi & LGX_S8_EPI_BIAS) && n + e < P.N ? P.bias[n + e] : 0.f;
  }
  // DX: the ELU' operand y (the layer below's S8 output) of every row slot requested before the
  // first use — one memory round trip for the tile instead of one per row slot (a load after a
  // store of the previous slot cannot be hoisted: the compiler cannot rule out aliasing).
  // Clamped rows / groups: no load under a condition.
  constexpr int NIT = KIND == LGX_S8_FWD ? 1 : ROWS / RS;
  u32x4 yh[NIT], yl[NIT];
  float adv[NIT][8];  // the addend (the regulariser's latent gradient), requested the same way
  const bool delu = KIND != LGX_S8_FWD && (P.epi & LGX_S8_EPI_DELU);
  if constexpr (KIND != LGX_S8_FWD) {
    if (delu) {
      const int64_t gofs = (int64_t)(std::min(n, P.N - 1) >> 3) * 32;
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int m = std::min(m_base + r0 + RS * it, P.M - 1);
        const char* src = P.act + (int64_t)m * P.ld_act + gofs;
        yh[it] = reinterpret_cast<const u32x4*>(src)[0];
        yl[it] = reinterpret_cast<const u32x4*>(src)[1];
      }
    }
    if (P.addend != nullptr && P.add_cols > 0) {
#pragma unroll
      for (int it = 0; it < NIT; ++it) {
        const int m = std::min(m_base + r0 + RS * it, P.M - 1);
#pragma unroll
        for (int e = 0; e < 8; ++e) adv[it][e] = P.addend[(int64_t)m * P.ld_add + std::min(n + e, P.add_cols - 1)];
      }
    }
  }
#pragma unroll
  for (int it = 0; it < ROWS / RS; ++it) {
    const int h = RS * it / LGX_S8_TILE_M;  // compile-time: r0 < RS and RS divides 128
    const int row = r0 + RS * it, m = m_base + row;
    if (m >= P.M || n >= P.N) continue;
    const f32x4 t0 = *reinterpret_cast<const f32x4*>(img + row * CPI + 8 * gq);
    const f32x4 t1 = *reinterpret_cast<const f32x4*>(img + row * CPI + 8 * gq + 4);
    float v[8] = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
    if constexpr (KIND == LGX_S8_FWD) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += bias[e];
      if (P.epi & LGX_S8_EPI_ELU) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = elu(v[e]);
      }
    } else {
      if (delu) {  // y = hi + lo, as load_s8
        const int q = KIND == LGX_S8_FWD ? 0 : it;
        float y[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          y[2 * e] = __uint_as_float(yh[q][e] << 16) + __uint_as_float(yl[q][e] << 16);
          y[2 * e + 1] = __uint_as_float(yh[q][e] & 0xffff0000u) + __uint_as_float(yl[q][e] & 0xffff0000u);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= y[e] > 0.f ? 1.f : y[e] + 1.f;
      }
      if (P.addend != nullptr && P.add_cols > 0) {
        const int q = KIND == LGX_S8_FWD ? 0 : it;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (n + e < P.add_cols) v[e] += adv[q][e];
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = n + e < P.N ? v[e] : 0.f;  // zero pad columns
    if (P.C != nullptr) store_s8(P.C + (int64_t)m * P.ldc + (n >> 3) * 32, v);
    if (P.C32 != nullptr) {
      float* d = P.C32 + (int64_t)m * P.ldc32 + n;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (n + e < P.N) d[e] = v[e];
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[h][e] += v[e];
  }
  if (P.colsum_ws != nullptr) {
    __syncthreads();
    float* red = img;  // [NH][RS row slots][COLS]
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int e = 0; e < 8; ++e) red[(h * RS + r0) * COLS + 8 * gq + e] = cs[h][e];
    __syncthreads();
    for (int t = tid; t < NH * COLS; t += NT) {
      const int h = t / COLS, c = t % COLS;
      if (n_base + c < P.N && m_base + h * LGX_S8_TILE_M < P.M) {
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < RS; ++q) s += red[(h * RS + q) * COLS + c];
        P.colsum_ws[(int64_t)(part0 + h) * P.N + n_base + c] = s;
      }
    }
  }
}

template <int KIND>
__global__ __launch_bounds__(Cfg::NT, 2) __attribute__((amdgpu_waves_per_eu(1, 2))) void s8_gemm_kernel(Group g) {
  constexpr bool ATR = KIND == LGX_S8_DW, BTR = KIND != LGX_S8_FWD;
  constexpr int BM = Cfg::BM, NW = Cfg::NW, NT = Cfg::NT, NS = Cfg::NS;
  using OA = Op<ATR, BM, NW>;
  using OB = Op<BTR, BN, NW>;
  constexpr int STAGE = OA::IMG + OB::IMG;
  extern __shared__ __align__(16) char lds[];

  const int x = blockIdx.x & 7, jb = blockIdx.x >> 3;
  if (jb >= g.per_xcd) return;
  int pi = 0, l = -1;
  if (g.nunits > 0) {
    int j = jb;
    for (int u = g.ustart[x]; u < g.ustart[x + 1]; ++u) {
      const int e = g.units[u], q = e & 31, sz = g.p[q].tiles_m * g.p[q].tiles_n;
      if (j < sz) {
        pi = q;
        l = (e >> 5) * sz + j;
        break;
      }
      j -= sz;
    }
    if (l < 0) return;
  } else {
    while (pi + 1 < g.n && jb >= g.start[pi + 1]) ++pi;
    l = x * (g.start[pi + 1] - g.start[pi]) + (jb - g.start[pi]);
  }
  const Prob P = g.p[pi];
  if (l >= P.tiles) return;
  const int tn = l % P.tiles_n, tm = (l / P.tiles_n) % P.tiles_m, z = l / (P.tiles_n * P.tiles_m);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = z * P.kchunk;
  const int kend = std::min(P.K, kbeg + P.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave % Cfg::WR) * 64, wn = (wave / Cfg::WR) * 64;

  uint32_t offA[OA::PW], offB[OB::PW];
  // ROW operands: source rows = tile rows (M or N); TR operands: source rows = k
  OA::offsets(offA, wave, lane, m0, P.M, P.lda, kbeg);
  OB::offsets(offB, wave, lane, n0, P.N, P.ldb, kbeg);
  const int64_t sa = OA::step_bytes(P.lda), sb = OB::step_bytes(P.ldb);

  const uint32_t lds0 = (uint32_t)(uintptr_t)((LDS_AS char*)lds);
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  auto issue = [&](int stage, int s) {
    const uint32_t st = lds0 + (uint32_t)(stage * STAGE);
    OA::issue(P.A + s * sa, offA, st, wv);
    OB::issue(P.B + s * sb, offB, st + OA::IMG, wv);
  };

  f32x4 acc[4][NJ];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int stage) {
    const char* st = lds + stage * STAGE;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 ah[4], al[4], bh[NJ], bl[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) OB::frag(st + OA::IMG, wn + 16 * j, kk, lane, bh[j], bl[j]);
#pragma unroll
      for (int i = 0; i < 4; ++i) OA::frag(st, wm + 16 * i, kk, lane, ah[i], al[i]);
      // every fragment read is issued before the first MFMA (the scheduler would otherwise
      // re-load A fragments one at a time behind lgkmcnt(0), exposing the LDS latency 8 times
      // per step); the MFMAs then wait on counted lgkmcnt in issue order
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[i], bh[j], acc[i][j], 0, 0, 0);
          S8_MFMA_ORDER();
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bl[j], acc[i][j], 0, 0, 0);
          S8_MFMA_ORDER();
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[i], bh[j], acc[i][j], 0, 0, 0);
          S8_MFMA_ORDER();
        }
    }
  };

  // pipeline: step s lives in stage s % NS; NS - 1 steps in flight. Each wave waits for its own
  // DMA of step k (counted vmcnt: the younger steps stay in flight), then the barrier makes
  // every wave's DMA of step k visible and retires every wave's reads of step k - 1, whose
  // stage the next DMA overwrites.
  constexpr int PW = OA::PW + OB::PW;  // DMA instructions per wave per step
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nk) issue(s, s);
#ifdef LGX_S8_CLOCK
  uint64_t ck0 = clock64(), ckl = ck0;
  uint32_t ckw = 0, ckb = 0, ckc = 0;
#define S8CK(acc_) do { const uint64_t t_ = clock64(); acc_ += (uint32_t)(t_ - ckl); ckl = t_; } while (0)
#else
#define S8CK(acc_) do { } while (0)
#endif
  for (int k = 0; k < nk; ++k) {
    S8CK(ckc);
    if (k + NS - 2 < nk) {
      if constexpr (NS == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else if constexpr (NS == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PW) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PW) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    S8CK(ckw);
    asm volatile("s_barrier" ::: "memory");
    S8CK(ckb);
    if (k + NS - 1 < nk) issue((k + NS - 1) % NS, k + NS - 1);
    compute(k % NS);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  S8CK(ckc);

  // ---- epilogue: the fp32 tile into LDS (MFMA C/D map: col = lane & 15, row = (lane >> 4) * 4 + r)
  float* img = reinterpret_cast<float*>(lds);
  {
    const int ec = lane & 15, er = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) img[(wm + 16 * i + er + r) * CP + wn + 16 * j + ec] = acc[i][j][r];
  }
  __syncthreads();
  if constexpr (KIND == LGX_S8_DW)
    epi_dw<NT, BM, BN, CP>(P, img, m0, n0, z, tid);
  else
    epi_act<KIND, NT, BM, BN, CP>(P, img, m0, n0, tm * (BM / LGX_S8_TILE_M), tid);
#ifdef LGX_S8_CLOCK
  if (lane == 0 && (wave == 0 || wave == NW - 1) && g_s8clk != nullptr) {
    const uint64_t t = clock64();
    uint32_t* o = g_s8clk + ((size_t)blockIdx.x * 2 + (wave != 0)) * 12;
    o[0] = ckw; o[1] = ckb; o[2] = ckc; o[3] = (uint32_t)(t - ckl); o[4] = (uint32_t)(t - ck0);
    o[5] = (uint32_t)nk; o[6] = __builtin_amdgcn_s_getreg(20 | (31 << 11)) & 15;  // XCC_ID
  }
#endif
}

// ---------------------------------------------------------------- FWD with a register epilogue (round 6)
// The forward kind's tile with its epilogue run from the accumulator registers (no fp32 LDS image,
// no barrier): one tile per block, the blocks dispatched by the hardware as slots free up (a
// static persistent tile list measured slower: it loses that dynamic balance).
// The MFMA operands are swapped (weights as the MFMA's A operand, activations as its B operand):
// the same three products per K step in the same accumulation order (lo*hi, hi*lo, hi*hi; bit-
// identical outputs, tests/test_gpu_s8.py), but each lane then holds 4 CONSECUTIVE output columns
// of one row (C/D map: column = 4 (lane >> 4) + r, row = lane & 15). Lanes l and l + 16 hold the
// two halves of one 8-column S8 group: after the bf16 hi / lo split one v_permlane16_swap per
// dword gives lane l the group's 8 hi values and lane l + 16 its 8 lo values — one 16-B store
// each, the 32-B group written whole. Column sums (optional for FWD) per 64-row half tile: the
// wave's 4 row tiles summed in registers, then the 16 lanes of a row by DPP (fixed order).
// The input-gradient kind keeps lgxs::s8_gemm_kernel: its ELU' operand loads coalesce better
// through the LDS image's row-slot map (measured, §4.2b).
struct FGroup {
  int n, per_xcd;
  int start[GMAX + 1];   // first tile of each problem in the launch's tile list
  int xstart[9];         // XCD slot x: tiles [xstart[x], xstart[x + 1]); its block s runs tile xstart[x] + s
  Prob p[GMAX];
};
static_assert(sizeof(FGroup) <= 4096, "kernel argument segment");

__device__ __forceinline__ float dpp_row_sum(float v) {
  // sum over the 16 lanes of each DPP row (every lane of the row gets it): quad swaps, then
  // rotations by 4 and 8 within the row — a fixed order, so the result is deterministic
  int x = __float_as_int(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0xB1, 0xf, 0xf, false));  // quad_perm [1,0,3,2]
  x = __float_as_int(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x4E, 0xf, 0xf, false));  // quad_perm [2,3,0,1]
  x = __float_as_int(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x124, 0xf, 0xf, false));  // row_ror:4
  x = __float_as_int(v);
  v += __int_as_float(__builtin_amdgcn_update_dpp(x, x, 0x128, 0xf, 0xf, false));  // row_ror:8
  return v;
}

__global__ __launch_bounds__(Cfg::NT, 2) __attribute__((amdgpu_waves_per_eu(1, 2))) void s8f_kernel(FGroup g) {
  constexpr int BM = Cfg::BM, NW = Cfg::NW;
  using OA = Op<false, BM, NW>;
  using OB = Op<false, BN, NW>;
  constexpr int STAGE = OA::IMG + OB::IMG;
  static_assert(2 * STAGE <= Cfg::LDS_STAGES, "two stages");
  extern __shared__ __align__(16) char lds[];

  const int x = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int t = g.xstart[x] + slot;
  if (t >= g.xstart[x + 1]) return;
  int pi = 0;
  while (pi + 1 < g.n && t >= g.start[pi + 1]) ++pi;
  const Prob& P = g.p[pi];
  const int M = P.M, N = P.N, epi = P.epi;
  const int l = t - g.start[pi];
  const int n0 = (l % P.tiles_n) * BN, m0 = (l / P.tiles_n) * BM;
  const int nk = (P.K + BK - 1) / BK;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave % Cfg::WR) * 64, wn = (wave / Cfg::WR) * 64;
  const uint32_t lds0 = (uint32_t)(uintptr_t)((LDS_AS char*)lds);
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  uint32_t offA[OA::PW], offB[OB::PW];
  OA::offsets(offA, wave, lane, m0, M, P.lda, 0);
  OB::offsets(offB, wave, lane, n0, N, P.ldb, 0);
  auto issue = [&](int stage, int step) {
    const uint32_t st = lds0 + (uint32_t)(stage * STAGE);
    OA::issue(P.A + step * OA::step_bytes(P.lda), offA, st, wv);
    OB::issue(P.B + step * OB::step_bytes(P.ldb), offB, st + OA::IMG, wv);
  };
  f32x4 acc[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int stage) {
    const char* st = lds + stage * STAGE;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 ah[4], al[4], bh[NJ], bl[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) OB::frag(st + OA::IMG, wn + 16 * j, kk, lane, bh[j], bl[j]);
#pragma unroll
      for (int i = 0; i < 4; ++i) OA::frag(st, wm + 16 * i, kk, lane, ah[i], al[i]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[j], al[i], acc[j][i], 0, 0, 0);
          S8_MFMA_ORDER();
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bl[j], ah[i], acc[j][i], 0, 0, 0);
          S8_MFMA_ORDER();
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bh[j], ah[i], acc[j][i], 0, 0, 0);
          S8_MFMA_ORDER();
        }
    }
  };
  // pipeline as lgxs::s8_gemm_kernel (2 stages, counted waits, raw barriers); the bias is
  // requested before the last step's MFMAs, so its latency runs beside them
  if (nk > 0) issue(0, 0);
  const int q4 = lane >> 4, lr = lane & 15, odd = q4 & 1;
  float bv[NJ][4];
  for (int k = 0; k < nk; ++k) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_barrier" ::: "memory");
    if (k + 1 < nk) issue((k + 1) & 1, k + 1);
    compute(k & 1);
  }
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int nq = n0 + wn + 16 * j + 4 * q4;
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[j][r] = (epi & LGX_S8_EPI_BIAS) ? P.bias[min(nq + r, N - 1)] : 0.f;
  }

  // ---- epilogue from the accumulators: lane (lr, q4) holds rows m0 + wm + 16 i + lr, columns
  // n0 + wn + 16 j + 4 q4 + r of acc[j][i][r]
  char* const Cp = P.C;
  float* const C32p = P.C32;
  const int64_t ldc = P.ldc, ldc32 = P.ldc32;
  const bool full = m0 + BM <= M && n0 + BN <= N;  // no row / column checks
  float cs[NJ][4];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) cs[j][r] = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int nq = n0 + wn + 16 * j + 4 * q4;  // this lane's first column
    const int grp = (n0 + wn + 16 * j) / 8 + (q4 >> 1);
    bool colok[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) colok[r] = full || nq + r < N;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm + 16 * i + lr;
      const bool rowok = full || m < M;
      float v[4] = {acc[j][i][0], acc[j][i][1], acc[j][i][2], acc[j][i][3]};
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += bv[j][r];
      if (epi & LGX_S8_EPI_ELU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = elu(v[r]);
      }
      if (!full) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = colok[r] ? v[r] : 0.f;  // zero pad columns
      }
      if (Cp != nullptr) {
        __bf16 h[4], lo[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          h[r] = (__bf16)v[r];
          lo[r] = (__bf16)(v[r] - (float)h[r]);
        }
        const auto s0 = __builtin_amdgcn_permlane16_swap(pack2(h[0], h[1]), pack2(lo[0], lo[1]), false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(pack2(h[2], h[3]), pack2(lo[2], lo[3]), false, false);
        // even-row lanes: {own hi, partner hi} = the group's 8 hi; odd-row: its 8 lo
        const u32x4 out = {s0[0], s1[0], s0[1], s1[1]};
        if (rowok && (full || grp * 8 < N))
          *reinterpret_cast<u32x4*>(Cp + (int64_t)m * ldc + grp * 32 + odd * 16) = out;
      }
      if (C32p != nullptr && rowok) {
        float* d = C32p + (int64_t)m * ldc32 + nq;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (colok[r]) d[r] = v[r];
      }
      if (rowok) {
#pragma unroll
        for (int r = 0; r < 4; ++r) cs[j][r] += v[r];
      }
    }
  }
  if (P.colsum_ws != nullptr) {
    // per 64-row half tile: partial index (m0 + wm) / 64, columns n of this wave
    const int part = (m0 + wm) / LGX_S8_TILE_M;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int nq = n0 + wn + 16 * j + 4 * q4;
      float sv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) sv[r] = dpp_row_sum(cs[j][r]);
      if (lr == 0 && m0 + wm < M) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (nq + r < N) P.colsum_ws[(int64_t)part * N + nq + r] = sv[r];
      }
    }
  }
}

// ---------------------------------------------------------------- fp32 -> S8 (+ column sums)
#define LGX_S8_SPLIT_WIDE 512  // (row, 8-column group) items per block of a wide split job

struct SplitJob {
  const float* src; int64_t ld_src;
  char* dst; int64_t ld_dst;  // bytes
  int rows, cols;
  float* colsum_ws;
  const int64_t* idx;
  int blk0;     // first block of this job
  int psteps;   // > 0: fragment-packed destination (lgx_s8_chain_layer.packed)
  int tr;       // packed only: src is [cols][rows] (the destination is its transpose)
};
struct SplitBatch {
  int n;
  SplitJob j[LGX_S8_BATCH_MAX];
};
static_assert(sizeof(SplitBatch) <= 4096, "kernel argument segment");

// Narrow jobs (<= 8 groups, the only ones with column sums): block = 256 rows, thread t owns
// group t & 7 of rows (t >> 3) + 32 it (fixed order). Wide jobs: block = SPLIT_WIDE (row, group)
// items, so a few-row job (a weight matrix) still spreads over many blocks.
__global__ __launch_bounds__(256) void s8_split_kernel(SplitBatch b) {
  int ji = 0, hi = b.n - 1;  // the block's job: binary search on the jobs' first blocks
  while (ji < hi) {
    const int mid = (ji + hi + 1) >> 1;
    if ((int)blockIdx.x >= b.j[mid].blk0) ji = mid;
    else hi = mid - 1;
  }
  const SplitJob J = b.j[ji];
  const int blk = blockIdx.x - J.blk0;
  const int rbase = blk * LGX_S8_SPLIT_ROWS;
  const int G = (J.cols + 7) / 8;
  const int tid = threadIdx.x;
  auto load8 = [&](int r, int gg, float (&v)[8]) {
    if (J.tr) {  // element (r, c) = src[c][r]
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 8 * gg + e < J.cols ? J.src[(int64_t)(8 * gg + e) * J.ld_src + r] : 0.f;
      return;
    }
    const int64_t sr = J.idx ? J.idx[r] : r;
    const float* s = J.src + sr * J.ld_src + 8 * gg;
    if (8 * gg + 8 <= J.cols) {
      const f32x4u a = *reinterpret_cast<const f32x4u*>(s), b = *reinterpret_cast<const f32x4u*>(s + 4);
      v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = 8 * gg + e < J.cols ? s[e] : 0.f;
    }
  };
  // row r, group gg -> its 16 B of hi (lo: + 16 in rows; + 1024 packed: tile r / 16, step gg / 4,
  // lane 16 (gg % 4) + r % 16 — the MFMA B fragment of that lane)
  auto put = [&](int r, int gg, const float (&v)[8]) {
    if (J.psteps) {
      char* q = J.dst + ((int64_t)(r >> 4) * J.psteps + (gg >> 2)) * 2048 + (((gg & 3) << 4) | (r & 15)) * 16;
      store_s8x(q, q + 1024, v);
    } else {
      store_s8(J.dst + (int64_t)r * J.ld_dst + gg * 32, v);
    }
  };
  if (G <= 8) {
    // every row's loads first (clamped rows, no load under a condition), then the stores: one
    // memory round trip per thread instead of one per row (src and dst never alias)
    constexpr int NI = LGX_S8_SPLIT_ROWS / 32;
    const int gg = tid & 7, ggc = min(gg, G - 1);
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float v[NI][8];
#pragma unroll
    for (int it = 0; it < NI; ++it) load8(min(rbase + (tid >> 3) + 32 * it, J.rows - 1), ggc, v[it]);
#pragma unroll
    for (int it = 0; it < NI; ++it) {
      const int r = rbase + (tid >> 3) + 32 * it;
      if (gg >= G || r >= J.rows) continue;
      put(r, gg, v[it]);
#pragma unroll
      for (int e = 0; e < 8; ++e) cs[e] += v[it][e];
    }
    if (J.colsum_ws != nullptr) {
      __shared__ float red[32][64];
#pragma unroll
      for (int e = 0; e < 8; ++e) red[tid >> 3][8 * gg + e] = cs[e];
      __syncthreads();
      if (tid < J.cols) {
        float s = 0.f;
        for (int q = 0; q < 32; ++q) s += red[q][tid];
        J.colsum_ws[(int64_t)blk * J.cols + tid] = s;
      }
    }
    return;
  }
  // wide jobs: block = SPLIT_WIDE consecutive (row, group) items, row-major; a thread's items
  // are all loaded before any is stored (src and dst may not alias; the loads overlap)
  constexpr int IT = LGX_S8_SPLIT_WIDE / 256;
  const int64_t i0 = (int64_t)blk * LGX_S8_SPLIT_WIDE;
  float v[IT][8];
  int rr[IT], gs[IT];
#pragma unroll
  for (int k = 0; k < IT; ++k) {
    const int64_t i = i0 + tid + 256 * k;
    rr[k] = (int)(i / G);
    gs[k] = (int)(i - (int64_t)rr[k] * G);
    if (rr[k] < J.rows) load8(rr[k], gs[k], v[k]);
  }
#pragma unroll
  for (int k = 0; k < IT; ++k)
    if (rr[k] < J.rows) put(rr[k], gs[k], v[k]);
}

struct ReduceBatch {
  int n;
  int64_t start[LGX_S8_BATCH_MAX + 1];  // first thread of each job (256-aligned: one job per block)
  lgx_s8_reduce_args j[LGX_S8_BATCH_MAX];
  unsigned char wave[LGX_S8_BATCH_MAX];  // one wave per output (long sums: the bias partials)
  unsigned char vec[LGX_S8_BATCH_MAX];   // 4 consecutive outputs per thread (flat, 16-B aligned jobs)
};
static_assert(sizeof(ReduceBatch) <= 4096, "kernel argument segment");

__global__ __launch_bounds__(256) void s8_reduce_kernel(ReduceBatch b) {
  // jobs start at multiples of 256 threads: a block belongs to one job, found by a binary search
  // on the block's first thread (wave-uniform: scalar loads of the job, no per-lane job fetch)
  const int64_t b0 = (int64_t)blockIdx.x * 256;
  int lo = 0, hi = b.n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (b.start[mid] <= b0) lo = mid;
    else hi = mid - 1;
  }
  const int ji = __builtin_amdgcn_readfirstlane(lo);
  const int64_t i = b0 + threadIdx.x;
  if (i >= b.start[b.n]) return;
  const lgx_s8_reduce_args& J = b.j[ji];
  if (b.wave[ji]) {
    // a long sum (one partial per 128-row tile): lane l takes partials l, l + 64, ... in order,
    // then a fixed butterfly over the wave — a few loads per lane instead of one thread's
    // nsplit / 16 dependent rounds (deterministic; the job's threads are whole waves)
    const int64_t e = (i - b.start[ji]) >> 6;
    const int lane = (int)(i & 63);
    if (e >= (int64_t)J.rows * J.cols) return;  // (never splits a wave: 64-aligned, whole waves)
    const int64_t r = e / J.cols, c = e - r * J.cols;
    const float* w = J.ws + r * J.ld_ws + c;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    int q = lane;
    for (; q + 192 < J.nsplit; q += 256) {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] += w[(int64_t)(q + 64 * u) * J.stride];
    }
    for (; q < J.nsplit; q += 64) v[0] += w[(int64_t)q * J.stride];
    float s = (v[0] + v[1]) + (v[2] + v[3]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) {
      float* o = J.out + r * J.ld_out + c;
      *o = J.accumulate ? *o + s : s;
    }
    return;
  }
  if (b.vec[ji]) {
    // a flat job (the split-K weight partials): float4 per thread, the partials requested 8 at a
    // time (clamped indices, no load under a condition), summed in split order per component
    const int64_t e = (i - b.start[ji]) * 4;
    if (e >= J.cols) return;
    const float* w = J.ws + e;
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int q = 0; q < J.nsplit; q += 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const f32x4*>(w + (int64_t)min(q + u, J.nsplit - 1) * J.stride);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (q + u < J.nsplit) s += v[u];
    }
    f32x4* o = reinterpret_cast<f32x4*>(J.out + e);
    *o = J.accumulate ? *o + s : s;
    return;
  }
  const int64_t e = i - b.start[ji];
  if (e >= (int64_t)J.rows * J.cols) return;  // the alignment gap before a wave job
  const int64_t r = e / J.cols, c = e - r * J.cols;
  const float* w = J.ws + r * J.ld_ws + c;
  // partials summed in split order; loaded 16 at a time so the bias jobs' long (one partial per
  // 128-row tile) sums are not a chain of dependent memory latencies
  float s = 0.f;
  int q = 0;
  for (; q + 16 <= J.nsplit; q += 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = w[(int64_t)(q + u) * J.stride];
#pragma unroll
    for (int u = 0; u < 16; ++u) s += v[u];
  }
  for (; q < J.nsplit; ++q) s += w[(int64_t)q * J.stride];
  float* o = J.out + r * J.ld_out + c;
  *o = J.accumulate ? *o + s : s;
}

}  // namespace lgxs

// ---------------------------------------------------------------- host
static thread_local char g_err[256] = "";
static int fail(const char* msg) {
  snprintf(g_err, sizeof g_err, "%s", msg);
  return -1;
}
static int launched(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
    return -2;
  }
  return 0;
}
static int cdiv(int a, int b) { return (a + b - 1) / b; }
int lgxs_fail(const char* msg) { return fail(msg); }  // for the library's other sources
int lgxs_launched(const char* what) { return launched(what); }

static bool dw_xcd_units() {
  static int on = -1;
  if (on < 0) {
    const char* e = LGX_DEV_KNOB("LGX_S8_DW_XCD");  // dev knob: 0 = tiles dealt per problem
    on = e ? atoi(e) != 0 : 1;
  }
  return on != 0;
}

// Deal the weight-gradient slices (problem, K chunk) to the 8 XCD slots, largest first onto the
// least-loaded slot (LPT); kept only if it needs no more block slots per XCD than one residency
// round (2 blocks x 32 CUs) or than the per-problem deal. Measured (tools/dw_probe.py, the go2
// minibatch's group alone): fabric reads 958 -> 687 MB per launch (FETCH_SIZE x 2; the operands
// are 661 MB), 196.6 -> 193.7 us — the group is not bound by its HBM traffic.
static void deal_units(lgxs::Group& g) {
  struct U { int pi, z, sz; };
  U u[lgxs::UMAX];
  int nu = 0;
  for (int pi = 0; pi < g.n; ++pi) {
    const lgxs::Prob& p = g.p[pi];
    const int sz = p.tiles_m * p.tiles_n, split = p.tiles / sz;
    if (split > 2047 || nu + split > lgxs::UMAX) return;
    for (int z = 0; z < split; ++z) u[nu++] = U{pi, z, sz};
  }
  std::stable_sort(u, u + nu, [](const U& a, const U& b) { return a.sz > b.sz; });
  int load[8] = {0}, cnt[8] = {0}, slot[lgxs::UMAX];
  for (int i = 0; i < nu; ++i) {
    int x = 0;
    for (int y = 1; y < 8; ++y)
      if (load[y] < load[x]) x = y;
    slot[i] = x;
    load[x] += u[i].sz;
    ++cnt[x];
  }
  const int mx = *std::max_element(load, load + 8);
  if (mx > std::max(g.per_xcd, 64)) return;
  g.ustart[0] = 0;
  for (int x = 0; x < 8; ++x) g.ustart[x + 1] = (uint16_t)(g.ustart[x] + cnt[x]);
  int fill[8];
  for (int x = 0; x < 8; ++x) fill[x] = g.ustart[x];
  for (int i = 0; i < nu; ++i) g.units[fill[slot[i]]++] = (uint16_t)(u[i].pi | (u[i].z << 5));
  g.nunits = nu;
  g.per_xcd = mx;
}

// The FWD launch: problems ordered by K (longest first: the dispatcher then starts the longest
// tiles first); the tile list cut into 8 contiguous XCD ranges of equal cost (an XCD's blocks
// share its L2: a row tile's column tiles stay together); block s of XCD slot x runs tile
// xstart[x] + s, one tile per block.
static bool fwd_register_epilogue() {
  static int on = -1;
  if (on < 0) {
    const char* e = LGX_DEV_KNOB("LGX_S8_FWD_REG");  // dev knob: 0 = the LDS-image epilogue kernel for FWD
#ifndef LGX_S8_FWD_REG_DEFAULT
#define LGX_S8_FWD_REG_DEFAULT 1  // (dev builds: -DLGX_S8_FWD_REG_DEFAULT=0 for the A/B variant)
#endif
    on = e ? atoi(e) != 0 : LGX_S8_FWD_REG_DEFAULT;
  }
  return on != 0;
}

static void launch_fwd(const lgxs::Group& g0, hipStream_t s) {
  lgxs::FGroup g;
  memset(&g, 0, sizeof g);
  int order[lgxs::GMAX];
  for (int i = 0; i < g0.n; ++i) order[i] = i;
  constexpr int EPI = 4;  // epilogue allowance in K steps
  auto nk = [&](int i) { return (g0.p[i].K + lgxs::BK - 1) / lgxs::BK; };
  std::stable_sort(order, order + g0.n, [&](int a, int b) { return nk(a) > nk(b); });
  int64_t total = 0;
  int ntiles = 0;
  for (int k = 0; k < g0.n; ++k) {
    g.p[k] = g0.p[order[k]];
    g.start[k] = ntiles;
    ntiles += g.p[k].tiles;
    total += (int64_t)g.p[k].tiles * (nk(order[k]) + EPI);
  }
  g.n = g0.n;
  g.start[g.n] = ntiles;
  g.xstart[0] = 0;
  int x = 1, pi = 0;
  int64_t acc = 0;
  for (int tt = 0; tt < ntiles && x < 8; ++tt) {
    while (tt >= g.start[pi + 1]) ++pi;
    acc += nk(order[pi]) + EPI;
    if (acc * 8 >= total * x) g.xstart[x++] = tt + 1;
  }
  while (x <= 8) g.xstart[x++] = ntiles;
  int mx = 0;
  for (int k = 0; k < 8; ++k) mx = std::max(mx, g.xstart[k + 1] - g.xstart[k]);
  g.per_xcd = mx;
  constexpr int lds = lgxs::Cfg::LDS_STAGES;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)lgxs::s8f_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  if (g.per_xcd > 0) hipLaunchKernelGGL(lgxs::s8f_kernel, dim3(8 * g.per_xcd), dim3(lgxs::Cfg::NT), lds, s, g);
}

template <int KIND>
static void launch_gemm(const lgxs::Group& g, hipStream_t s) {
  constexpr int lds = lgxs::Cfg::LDS;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)lgxs::s8_gemm_kernel<KIND>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              lds);
    attr = true;
  }
  hipLaunchKernelGGL((lgxs::s8_gemm_kernel<KIND>), dim3(8 * g.per_xcd), dim3(lgxs::Cfg::NT), lds, s, g);
}

extern "C" {

int32_t lgx_s8_abi_version(void) { return LGX_S8_ABI_VERSION; }
#ifdef LGX_S8_CLOCK
int32_t lgx_s8_set_clock(void* dev_buf) {
  return hipMemcpyToSymbol(HIP_SYMBOL(lgxs::g_s8clk), &dev_buf, sizeof(void*)) == hipSuccess ? 0 : -1;
}
#endif
int32_t lgx_s8_sizeof_gemm_args(void) { return (int32_t)sizeof(lgx_s8_gemm_args); }
const char* lgx_s8_last_error(void) { return g_err; }

int32_t lgx_s8_pick_split(const int32_t* M, const int32_t* N, const int32_t* K, int32_t n, int32_t* out) {
  if (n < 0 || n > LGX_S8_GROUP_MAX) return fail("lgx_s8_pick_split: 0 <= n <= LGX_S8_GROUP_MAX");
  // one K chunk for every problem: the smallest that keeps the group within one residency
  // round of 2 blocks per CU (256 CUs)
  int64_t tiles = 0, kmax = 0;
  for (int i = 0; i < n; ++i) {
    if (M[i] <= 0 || N[i] <= 0 || K[i] < 0) return fail("lgx_s8_pick_split: bad shape");
    tiles += (int64_t)cdiv(M[i], lgxs::Cfg::BM) * cdiv(N[i], lgxs::BN);
    kmax = std::max<int64_t>(kmax, K[i]);
  }
  int64_t slots = 512;  // 2 blocks per CU x 256 CUs
  if (const char* e = LGX_DEV_KNOB("LGX_S8_DW_SLOTS")) slots = std::max(1, atoi(e));  // dev knob
  const int64_t s = std::max<int64_t>(1, tiles ? slots / tiles : 1);
  const int64_t chunk = ((kmax + s - 1) / s + lgxs::BK - 1) / lgxs::BK * lgxs::BK;
  for (int i = 0; i < n; ++i) out[i] = std::max(1, cdiv(K[i], (int)std::max<int64_t>(chunk, lgxs::BK)));
  return 0;
}

int32_t lgx_s8_gemm_group(const lgx_s8_gemm_args* a, int32_t n, int32_t kind, void* stream) {
  if (n < 0 || n > LGX_S8_GROUP_MAX) return fail("lgx_s8_gemm_group: 0 <= n <= LGX_S8_GROUP_MAX");
  if (kind < LGX_S8_FWD || kind > LGX_S8_DW) return fail("lgx_s8_gemm_group: unknown kind");
  lgxs::Group g;
  memset(&g, 0, sizeof g);
  int np = 0, acc = 0;
  for (int i = 0; i < n; ++i) {
    const lgx_s8_gemm_args& q = a[i];
    if (q.M < 0 || q.N < 0 || q.K < 0) return fail("lgx_s8_gemm_group: negative size");
    if (q.M == 0 || q.N == 0) continue;
    if (!q.A || !q.B) return fail("lgx_s8_gemm_group: null operand");
    if (q.lda % 8 || q.ldb % 8) return fail("lgx_s8_gemm_group: S8 pitches must be multiples of 8");
    if ((((uintptr_t)q.A) | ((uintptr_t)q.B)) & 15) return fail("lgx_s8_gemm_group: operands must be 16-B aligned");
    const bool atr = kind == LGX_S8_DW, btr = kind != LGX_S8_FWD;
    const int kp = cdiv(q.K, lgxs::BK) * lgxs::BK;
    // the source extent the DMA may touch (lane offsets are 32-bit)
    const int64_t abytes = atr ? (int64_t)kp * q.lda * 4 : (int64_t)q.M * q.lda * 4;
    const int64_t bbytes = btr ? (int64_t)kp * q.ldb * 4 : (int64_t)q.N * q.ldb * 4;
    if (abytes >= (1ll << 31) || bbytes >= (1ll << 31)) return fail("lgx_s8_gemm_group: operand spans >= 2 GB");
    if (!atr && q.lda < kp) return fail("lgx_s8_gemm_group: ROW operand A pitch < round_up(K, 32)");
    if (!btr && q.ldb < kp) return fail("lgx_s8_gemm_group: ROW operand B pitch < round_up(K, 32)");
    if (atr && q.lda < 8) return fail("lgx_s8_gemm_group: TR operand A pitch");
    lgxs::Prob& p = g.p[np];
    p.A = (const char*)q.A;
    p.B = (const char*)q.B;
    p.lda = q.lda * 4;
    p.ldb = q.ldb * 4;
    p.M = q.M;
    p.N = q.N;
    p.K = q.K;
    p.tiles_m = cdiv(q.M, lgxs::Cfg::BM);
    p.tiles_n = cdiv(q.N, lgxs::BN);
    p.epi = q.epilogue;
    p.C = (char*)q.C;
    p.ldc = q.ldc * 4;
    p.C32 = q.C32;
    p.ldc32 = q.ldc32;
    p.bias = q.bias;
    p.act = (const char*)q.act;
    p.ld_act = q.ld_act * 4;
    p.addend = q.addend;
    p.ld_add = q.ld_add;
    p.add_cols = q.addend ? q.add_cols : 0;
    p.colsum_ws = q.colsum_ws;
    int split = 1;
    if (kind == LGX_S8_DW) {
      split = std::max(1, q.split);
      if (!q.C32) return fail("lgx_s8_gemm_group: DW needs C32 (output or partial workspace)");
      if (split == 1 && q.ldc32 < q.N) return fail("lgx_s8_gemm_group: ldc32 < N");
    } else {
      if (!q.C && !q.C32) return fail("lgx_s8_gemm_group: no output");
      if (q.C && (q.ldc % 8 || (((uintptr_t)q.C) & 15))) return fail("lgx_s8_gemm_group: S8 output alignment");
      if ((q.epilogue & LGX_S8_EPI_BIAS) && !q.bias) return fail("lgx_s8_gemm_group: bias epilogue without bias");
      if ((q.epilogue & LGX_S8_EPI_DELU) && (!q.act || q.ld_act % 8 || (((uintptr_t)q.act) & 15)))
        return fail("lgx_s8_gemm_group: ELU' epilogue needs an aligned S8 act");
      if (q.C32 && q.ldc32 < q.N) return fail("lgx_s8_gemm_group: ldc32 < N");
    }
    const int ksteps = cdiv(q.K, lgxs::BK);
    const int per = std::max(1, cdiv(ksteps, split));
    p.kchunk = per * lgxs::BK;
    split = std::max(1, cdiv(ksteps, per));
    p.tiles = p.tiles_m * p.tiles_n * split;
    acc += cdiv(p.tiles, 8);
    g.start[++np] = acc;
  }
  g.n = np;
  g.per_xcd = acc;
  if (np == 0) return 0;
  if (kind == LGX_S8_DW && dw_xcd_units()) deal_units(g);
  hipStream_t s = (hipStream_t)stream;
  if (kind == LGX_S8_FWD && fwd_register_epilogue()) launch_fwd(g, s);
  else if (kind == LGX_S8_FWD) launch_gemm<LGX_S8_FWD>(g, s);
  else if (kind == LGX_S8_DX) launch_gemm<LGX_S8_DX>(g, s);
  else launch_gemm<LGX_S8_DW>(g, s);
  return launched("lgx_s8_gemm_group");
}

int32_t lgx_s8_split(const lgx_s8_split_args* a, int32_t n, void* stream) {
  if (n < 0 || n > LGX_S8_BATCH_MAX) return fail("lgx_s8_split: 0 <= n <= LGX_S8_BATCH_MAX");
  lgxs::SplitBatch b;
  memset(&b, 0, sizeof b);
  int blocks = 0, k = 0;
  for (int i = 0; i < n; ++i) {
    const lgx_s8_split_args& q = a[i];
    if (q.rows < 0 || q.cols < 0) return fail("lgx_s8_split: negative size");
    if (q.rows == 0 || q.cols == 0) continue;
    if (!q.src || !q.dst) return fail("lgx_s8_split: null pointer");
    if (q.packed_steps < 0 || (q.packed_steps && (q.packed_steps < cdiv(q.cols, 32) || q.colsum_ws || q.idx)) ||
        (q.transpose && !q.packed_steps))
      return fail("lgx_s8_split: packed_steps >= ceil(cols / 32), no column sums or gather; transpose packed only");
    if ((((uintptr_t)q.dst) & 15) || (!q.packed_steps && (q.ld_dst % 8 || q.ld_dst < cdiv(q.cols, 8) * 8)))
      return fail("lgx_s8_split: S8 destination alignment / pitch");
    if (q.colsum_ws && q.cols > 64) return fail("lgx_s8_split: column sums for <= 64 columns only");
    b.j[k] = lgxs::SplitJob{q.src, q.ld_src, (char*)q.dst, q.ld_dst * 4, q.rows, q.cols, q.colsum_ws, q.idx, blocks,
                            q.packed_steps, q.transpose != 0};
    const int64_t G = cdiv(q.cols, 8);
    blocks += G <= 8 ? cdiv(q.rows, LGX_S8_SPLIT_ROWS) : (int)((q.rows * G + LGX_S8_SPLIT_WIDE - 1) / LGX_S8_SPLIT_WIDE);
    ++k;
  }
  b.n = k;
  if (!k) return 0;
  hipLaunchKernelGGL(lgxs::s8_split_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, b);
  return launched("lgx_s8_split");
}

int32_t lgx_s8_reduce(const lgx_s8_reduce_args* a, int32_t n, void* stream) {
  if (n < 0 || n > LGX_S8_BATCH_MAX) return fail("lgx_s8_reduce: 0 <= n <= LGX_S8_BATCH_MAX");
  lgxs::ReduceBatch b;
  memset(&b, 0, sizeof b);
  int k = 0;
  b.start[0] = 0;
  for (int i = 0; i < n; ++i) {
    if (a[i].rows < 0 || a[i].cols < 0 || a[i].nsplit < 0) return fail("lgx_s8_reduce: negative size");
    if (a[i].rows == 0 || a[i].cols == 0) continue;
    if (!a[i].ws || !a[i].out) return fail("lgx_s8_reduce: null pointer");
    if (a[i].rows > 1 && (a[i].ld_ws < a[i].cols || a[i].ld_out < a[i].cols)) return fail("lgx_s8_reduce: pitch < cols");
    b.j[k] = a[i];
    b.wave[k] = a[i].nsplit >= 64 && (int64_t)a[i].rows * a[i].cols <= 4096;
    b.vec[k] = !b.wave[k] && a[i].rows == 1 && a[i].cols % 4 == 0 && a[i].stride % 4 == 0 &&
               ((((uintptr_t)a[i].ws) | ((uintptr_t)a[i].out)) & 15) == 0;
    b.start[k] = (b.start[k] + 255) / 256 * 256;  // one job per block (s8_reduce_kernel)
    b.start[k + 1] = b.start[k] + (b.vec[k] ? a[i].cols / 4 : (int64_t)a[i].rows * a[i].cols * (b.wave[k] ? 64 : 1));
    ++k;
  }
  b.n = k;
  if (!k) return 0;
  const int64_t tot = b.start[k];
  hipLaunchKernelGGL(lgxs::s8_reduce_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream, b);
  return launched("lgx_s8_reduce");
}

}  // extern "C"
