// lgx_s8chain.hip — the update's narrow forward chains in one launch, gfx950 (include/lgx_s8.h
// lgx_s8_chain).
//
// The privileged and scan encoders (support_networks.py:25-80) are 2-3 layers of <= 132 inputs:
// as grouped launches (one per depth, lgx_s8.hip) every level is a few-microsecond kernel bound
// by its launch and its 128-row tile fill, and the levels depend on each other. Here a block owns
// 32 rows of one chain and runs all of its layers: the activations stay in an LDS image (bf16 hi
// and lo planes, [32][IP], zero past K), the weights (S8, a few KB per layer, L2-resident) go
// from global memory straight into registers one K step ahead, and each layer's output is
// written once as S8 rows (32 B per 8-column group: the image's hi and lo slots side by side,
// the layout lgx_s8_gemm_group writes) and / or fp32.
//
// Arithmetic per output: lgx_s8.hip's — 32-deep K steps in order, lo*hi + hi*lo + hi*hi
// v_mfma_f32_16x16x32_bf16 into one fp32 accumulator, then bias, ELU, the S8 split (RN) and zero
// pad columns. Wave w owns the 16-column output tiles w, w + 4, ... of both 16-row tiles.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>

#include "../../include/lgx_s8.h"

int lgxs_fail(const char* msg);        // lgx_s8.hip: the library's last-error slot
int lgxs_launched(const char* what);

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

namespace lgxc {

constexpr int NT = 256;                        // 4 waves
constexpr int CMAX = LGX_S8_CHAIN_MAX;
#ifndef LGX_S8_CHAIN_D
#define LGX_S8_CHAIN_D 2
#endif
constexpr int D = LGX_S8_CHAIN_D;  // weight register sets in flight

struct Params {
  int n;
  int start[CMAX + 1];  // prefix sums of the chains' row blocks
  lgx_s8_chain_args c[CMAX];
};
static_assert(sizeof(Params) <= 4096, "kernel argument segment");

__device__ __forceinline__ float elu(float v) {  // lgx_s8.hip's ELU
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

template <int NJW>
struct BSet {
  u32x4 h[NJW], l[NJW];
};

// NJW = output tiles per wave (16 columns each): the launch's widest layer / 64, rounded up to
// 1, 2 or 4 (the registers of the narrow chains' launches stay few: 4 waves per SIMD). BR = rows
// per block. IPW = the image's width (its pitch IPW + 8 bf16: fragment reads conflict-free).
template <int NJW, int BR, int IPW, bool DX>  // DX: the input-gradient launches (ELU', column sums)
__global__ __launch_bounds__(NT) void chain_kernel(Params P) {
  constexpr int MI = BR / 16, IP = IPW + 8;
  __shared__ __align__(16) __bf16 ih[BR * IP];
  __shared__ __align__(16) __bf16 il[BR * IP];
  __shared__ float red[DX ? 4 : 1][DX ? IPW : 1];  // column-sum partials of the 4 lane groups
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fc = lane >> 4;
  const int blk = blockIdx.x;
  if (blk >= P.start[P.n]) return;
  int ci = 0;
  while (ci + 1 < P.n && blk >= P.start[ci + 1]) ++ci;
  const lgx_s8_chain_args& c = P.c[ci];
  const int rows = c.rows, r0 = (blk - P.start[ci]) * BR;

  {  // the input rows' S8 groups -> the image (clamped rows; zero past K: the input may be a
     // column span of a wider buffer)
    const int G = (c.layers[0].K + 31) / 32 * 4, GK = (c.layers[0].K + 7) / 8;
    const char* A = (const char*)c.A;
    for (int idx = tid; idx < BR * G; idx += NT) {
      const int r = idx / G, g = idx % G;
      const char* q = A + (int64_t)std::min(r0 + r, rows - 1) * c.lda * 4 + std::min(g, GK - 1) * 32;
      u32x4 h = reinterpret_cast<const u32x4*>(q)[0], l = reinterpret_cast<const u32x4*>(q)[1];
      if (g >= GK) h = l = u32x4{0u, 0u, 0u, 0u};
      *reinterpret_cast<u32x4*>(ih + r * IP + 8 * g) = h;
      *reinterpret_cast<u32x4*>(il + r * IP + 8 * g) = l;
    }
  }
  __syncthreads();

  for (int li = 0; li < c.nlayers; ++li) {
    const lgx_s8_chain_layer& L = c.layers[li];
    const int K = L.K, N = L.N;
    const int ns = (K + 31) / 32;
    const int nte = (N + 31) / 32 * 2;  // tiles up to the next K step's width (zeros past N)
    const char* W = (const char*)L.W;
    // B fragments: rows of the S8 weight (16 B of hi and of lo per lane: every load touches 16
    // half-used cache lines), or fragment-packed (1 KB contiguous per load: whole lines)
    const bool pk = L.packed != 0;
    const int64_t kstep = pk ? 2048 : 128, lo = pk ? 1024 : 16;
    int64_t wrow[NJW];
    bool tv[NJW];
#pragma unroll
    for (int j = 0; j < NJW; ++j) {
      const int t = wave + 4 * j;
      tv[j] = t < nte;
      wrow[j] = pk ? (int64_t)std::min(t, (N - 1) >> 4) * ns * 2048 + lane * 16
                   : (int64_t)std::min(16 * t + fr, N - 1) * L.ldw * 4 + fc * 32;
    }
    auto bload = [&](BSet<NJW>& S, int s) {
      const int64_t ko = (int64_t)std::min(s, ns - 1) * kstep;
#pragma unroll
      for (int j = 0; j < NJW; ++j) {
        if (!tv[j]) continue;  // wave-uniform
        const char* q = W + wrow[j] + ko;
        S.h[j] = *reinterpret_cast<const u32x4*>(q);
        S.l[j] = *reinterpret_cast<const u32x4*>(q + lo);
      }
    };
    // the ELU' epilogue's y values, requested before the K loop (their latency overlaps it)
    float yv[DX ? MI : 1][DX ? NJW : 1][4];
    if constexpr (DX) {
      const char* act = (const char*)L.act;
#pragma unroll
      for (int j = 0; j < NJW; ++j) {
        const int cc = std::min(16 * (wave + 4 * j) + fr, N - 1);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const unsigned short* q = reinterpret_cast<const unsigned short*>(
                act + (int64_t)std::min(r0 + 16 * i + 4 * fc + r, rows - 1) * L.ld_act * 4 + (cc >> 3) * 32 + (cc & 7) * 2);
            yv[i][j][r] = tv[j] ? __uint_as_float((unsigned)q[0] << 16) + __uint_as_float((unsigned)q[8] << 16) : 0.f;
          }
      }
    }
    f32x4 acc[MI][NJW];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto mma = [&](const BSet<NJW>& S, int s) {
      const bool live = s < ns;  // steps past the last multiply zeros (no branch around the loads)
      const bf16x8 z = {};
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int off = (16 * i + fr) * IP + 32 * std::min(s, ns - 1) + 8 * fc;
        const bf16x8 ah = live ? *reinterpret_cast<const bf16x8*>(ih + off) : z;
        const bf16x8 al = live ? *reinterpret_cast<const bf16x8*>(il + off) : z;
#pragma unroll
        for (int j = 0; j < NJW; ++j) {
          if (!tv[j]) continue;
          const bf16x8 bh = __builtin_bit_cast(bf16x8, S.h[j]), bl = __builtin_bit_cast(bf16x8, S.l[j]);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc[i][j], 0, 0, 0);
        }
      }
    };
    // weights D - 1 K steps ahead in a ring of D register sets; the loop is padded to whole
    // rings (no branch around the loads). Measured on the go2 encoders (tools/chain_bench.py):
    // D = 2 / 3 / 4: 24 / 26 / 27.5 us; 64-row blocks 29-34 us; row-layout weights 41.5 us.
    BSet<NJW> sets[D];
#pragma unroll
    for (int d = 0; d < D - 1; ++d) bload(sets[d], d);
    const int nsp = (ns + D - 1) / D * D;
    for (int s = 0; s < nsp; s += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        bload(sets[(d + D - 1) % D], s + d + D - 1);
        mma(sets[d], s + d);
      }
    }
    __syncthreads();  // every wave is done reading the image

    // epilogue: bias (+ ELU) or times ELU'(act), zero pad columns; fp32 rows out, the split back
    // into the image, the column sums of the block's valid rows
#pragma unroll
    for (int j = 0; j < NJW; ++j) {
      if (!tv[j]) continue;
      const int col = 16 * (wave + 4 * j) + fr;
      const float bias = col < N && L.bias != nullptr ? L.bias[col] : 0.f;
      float cs = 0.f;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * i + 4 * fc + r;
          float v = acc[i][j][r] + bias;
          if (!DX && L.elu == 1) {
            v = elu(v);
          } else if (DX && L.elu == 2) {  // y = hi + lo of the S8 ELU output (lgx_s8.hip load_s8)
            const float y = yv[DX ? i : 0][DX ? j : 0][r];
            v *= y > 0.f ? 1.f : y + 1.f;
          }
          v = col < N ? v : 0.f;
          if (DX && r0 + row < rows) cs += v;
          if (L.C32 != nullptr && col < N && r0 + row < rows) L.C32[(int64_t)(r0 + row) * L.ldc32 + col] = v;
          const __bf16 h = (__bf16)v;
          ih[row * IP + col] = h;
          il[row * IP + col] = (__bf16)(v - (float)h);
        }
      if constexpr (DX) red[fc][col] = cs;
    }
    __syncthreads();
    if (DX && L.colsum_ws != nullptr)  // the 4 lane groups' partials in order: the block's sums
      for (int n = tid; n < N; n += NT)
        L.colsum_ws[(int64_t)(r0 / BR) * N + n] = ((red[0][n] + red[1][n]) + red[2][n]) + red[3][n];
    if (L.C != nullptr) {  // the image's groups -> S8 rows (hi 16 B | lo 16 B)
      const int G = (N + 7) / 8;
      char* C = (char*)L.C;
      for (int idx = tid; idx < BR * G; idx += NT) {
        const int r = idx / G, g = idx % G;
        if (r0 + r >= rows) continue;
        char* q = C + (int64_t)(r0 + r) * L.ldc * 4 + g * 32;
        reinterpret_cast<u32x4*>(q)[0] = *reinterpret_cast<const u32x4*>(ih + r * IP + 8 * g);
        reinterpret_cast<u32x4*>(q)[1] = *reinterpret_cast<const u32x4*>(il + r * IP + 8 * g);
      }
    }
  }
}

}  // namespace lgxc

extern "C" {

int32_t lgx_s8_sizeof_chain_args(void) { return (int32_t)sizeof(lgx_s8_chain_args); }

int32_t lgx_s8_chain(const lgx_s8_chain_args* chains, int32_t n, void* stream) {
  if (n < 1 || n > LGX_S8_CHAIN_MAX || chains == nullptr) return lgxs_fail("lgx_s8_chain: 1 <= n <= LGX_S8_CHAIN_MAX");
  lgxc::Params P{};
  P.n = n;
  int tot = 0, wmax = 0, nmax = 0, ncs = 0, nl = 0;
  for (int i = 0; i < n; ++i) {
    const lgx_s8_chain_args& c = chains[i];
    if (c.A == nullptr || c.rows < 1 || c.nlayers < 1 || c.nlayers > LGX_S8_CHAIN_MAXL)
      return lgxs_fail("lgx_s8_chain: input, rows >= 1, 1 <= nlayers <= LGX_S8_CHAIN_MAXL");
    if ((reinterpret_cast<uintptr_t>(c.A) & 15) || c.lda < (c.layers[0].K + 31) / 32 * 32)
      return lgxs_fail("lgx_s8_chain: input pitch >= K rounded up to 32, 16-B aligned");
    for (int l = 0; l < c.nlayers; ++l) {
      const lgx_s8_chain_layer& L = c.layers[l];
      if (L.K < 1 || L.N < 1 || L.K > LGX_S8_CHAIN_MAXW || L.N > LGX_S8_CHAIN_MAXW)
        return lgxs_fail("lgx_s8_chain: 1 <= K, N <= LGX_S8_CHAIN_MAXW");
      if (l > 0 && L.K != c.layers[l - 1].N) return lgxs_fail("lgx_s8_chain: K_l must equal N_{l-1}");
      if (L.W == nullptr || (reinterpret_cast<uintptr_t>(L.W) & 15) || (!L.packed && L.ldw < (L.K + 31) / 32 * 32))
        return lgxs_fail("lgx_s8_chain: weight pitch >= K rounded up to 32, 16-B aligned");
      if (L.C != nullptr && ((reinterpret_cast<uintptr_t>(L.C) & 15) || L.ldc % 8 || L.ldc < (L.N + 7) / 8 * 8))
        return lgxs_fail("lgx_s8_chain: S8 output pitch a multiple of 8, >= N, 16-B aligned");
      if (L.C32 != nullptr && L.ldc32 < L.N) return lgxs_fail("lgx_s8_chain: fp32 output pitch >= N");
      if (L.elu < 0 || L.elu > 2 || (L.elu == 2 && (L.act == nullptr || L.ld_act < (L.N + 7) / 8 * 8)))
        return lgxs_fail("lgx_s8_chain: elu 0 / 1 / 2 (2: the S8 activation, pitch >= N)");
      if ((L.elu == 2) != (L.colsum_ws != nullptr))
        return lgxs_fail("lgx_s8_chain: column sums exactly on the ELU' (input-gradient) layers");
      nmax = std::max(nmax, (L.N + 31) / 32 * 32);  // output tiles per wave
      wmax = std::max(wmax, std::max((L.N + 31) / 32 * 32, (L.K + 31) / 32 * 32));  // the image
      ncs += L.colsum_ws != nullptr;
      ++nl;
    }
    P.c[i] = c;
  }
  if (ncs && ncs != nl) return lgxs_fail("lgx_s8_chain: column sums on every layer or none");
  const int br = 32;
  for (int i = 0; i < n; ++i) {
    P.start[i] = tot;
    tot += (chains[i].rows + br - 1) / br;
  }
  P.start[n] = tot;
  const hipStream_t s = (hipStream_t)stream;
  const dim3 g(tot), b(lgxc::NT);
  if (ncs) {
    if (nmax <= 64) hipLaunchKernelGGL((lgxc::chain_kernel<1, 32, 256, true>), g, b, 0, s, P);
    else if (nmax <= 128) hipLaunchKernelGGL((lgxc::chain_kernel<2, 32, 256, true>), g, b, 0, s, P);
    else hipLaunchKernelGGL((lgxc::chain_kernel<4, 32, 256, true>), g, b, 0, s, P);
  } else {
    if (nmax <= 64) hipLaunchKernelGGL((lgxc::chain_kernel<1, 32, 256, false>), g, b, 0, s, P);
    else if (nmax <= 128) hipLaunchKernelGGL((lgxc::chain_kernel<2, 32, 256, false>), g, b, 0, s, P);
    else hipLaunchKernelGGL((lgxc::chain_kernel<4, 32, 256, false>), g, b, 0, s, P);
  }
  return lgxs_launched("lgx_s8_chain");
}

}  // extern "C"
