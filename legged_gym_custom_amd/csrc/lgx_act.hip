// lgx_act.hip — the rollout's act networks in ONE launch (include/lgx_s8.h, lgx_s8_act):
// PPO.act's estimator, scan encoder, privileged encoder, actor and critic (ppo.py:129-153,
// actor_critic.py:79-107 / 190-226, support_networks.py:25-80) on S8 weights, gfx950.
//
// Block = 32 rows (envs) x 512 threads (8 waves, 2 per SIMD: 10 % faster than 4); one block
// per CU (149 KB of LDS). Half of the
// blocks ("actor blocks", on XCDs 0-3) run estimator -> scan encoder -> privileged encoder ->
// actor for their rows, the other half ("critic blocks", XCDs 4-7) the critic, so each XCD's L2
// holds one network's weights (≈2.4 MB). Activations stay in LDS (fp32, row pitch = 4 mod 64
// floats: the 16 rows a fragment read touches fall on 16 distinct bank quads); the actor input
// is assembled in place in the S8 update's segmented layout [obs | priv latent | scan latent |
// est] (each part at a multiple of 8 columns, zero gaps), which is the layout of its S8 weights.
//
// A layer: out[32, N] = act(in[32, K] W^T + b), 3 x bf16 MFMAs (lo*hi + hi*lo + hi*hi, fp32
// accumulation; lgx_s8.hip's order) per 16 x 16 x 32 tile. Wave w owns the 16-column tiles
// w, w + 8, ...; each K step's weight fragments are loaded two steps ahead into registers — with
// 32 rows per block the weights are the streamed operand (each block reads all of its network's
// weights once): the weight-streaming pattern of a small-M GEMM, not a staged tile. The weights
// are act-packed (lgx_s8_act_pack): a fragment is 1 KB contiguous, so each load instruction
// fetches 8 whole cache lines (row-major S8 rows would cost 16 half-used lines per instruction,
// twice: measured 2.4 us per 512-wide K step, L1-miss bound). The activation fragments are read
// from LDS (the critic's first layer: from the input rows, 32 B per lane) and split into hi / lo
// in registers; columns k >= K are zeroed by select (the packed pad columns are zero too).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

#include "../../include/lgx_mlp.h"  // LGX_ACT_NOISE_STREAM
#include "../../include/lgx_s8.h"
#include "lgx_device.h"  // philox4x32_10 / u01: the env's counter RNG (the act head's noise)

namespace lgxa {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
#define GAS __attribute__((address_space(1)))  // global: the layers are separate functions, so
                                               // their pointer arguments are cast back to it

constexpr int R = LGX_S8_ACT_ROWS;          // rows per block (32)
constexpr int NT = 512;                      // threads per block: 8 waves, 2 per SIMD
constexpr int NWV = NT / 64;
constexpr int XP = LGX_S8_ACT_MAXIN + 4;     // actor-input image pitch (floats, = 4 mod 64)
constexpr int YP = LGX_S8_ACT_MAXH + 4;      // hidden-layer image pitch
constexpr int SP = LGX_S8_ACT_MAXENC + 4;    // encoder scratch pitch (two images inside Y)
static_assert(XP % 64 == 4 && YP % 64 == 4 && SP % 64 == 4, "pitches: 4 mod 64 floats");
constexpr int XF = R * XP;                              // floats
constexpr int YF = R * YP > 2 * R * SP ? R * YP : 2 * R * SP;
constexpr int LDS_BYTES = (XF + YF) * 4;
static_assert(LDS_BYTES <= 160 * 1024, "LDS");

__device__ __forceinline__ float elu(float v) {  // lgx_mlp.hip's / lgx_s8.hip's ELU
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

// 8 fp32 (k >= K already zero) -> hi / lo bf16 fragments
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 h = (__bf16)v[e];
    hi[e] = h;
    lo[e] = (__bf16)(v[e] - (float)h);
  }
}

// the dynamic LDS (the layers are separate functions: they address it by float offsets, so
// their accesses stay LDS instructions)
extern __shared__ __align__(16) float act_lds[];

struct Src {  // a layer input: global rows (g, ld) or an LDS image (float offset of its first column, pitch ld)
  const float* g;
  int64_t ld;
  int off;
};
struct Dst {  // a layer output: global rows (g, ld) or an LDS image
  float* g;
  int64_t ld;
  int off;
};

// Register sets in the weight pipeline per tile count: the narrower layers' sets are smaller,
// so they keep more K steps in flight (a step's loads are L2 round trips)
#ifndef ACT_D4
#define ACT_D4 3
#endif
#ifndef ACT_D2
#define ACT_D2 3
#endif
#ifndef ACT_D1
#define ACT_D1 3
#endif
constexpr int act_depth(int tpw) { return tpw >= 4 ? ACT_D4 : tpw == 2 ? ACT_D2 : ACT_D1; }

// One layer for the block's 32 rows. TPW = 16-column tiles per wave (N <= 128 TPW); GIN: the
// input is global rows (else an LDS image). The K loop has no branches around its loads (steps
// past the last one read clamped addresses and multiply zeros), so hipcc counts the loads in
// flight instead of draining them every step.
template <int TPW, bool GIN>
__device__ __forceinline__ void layer(const lgx_s8_act_layer& L, const Src& in, const Dst& out, int rows) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, c = lane & 15;
  const int K = L.K, N = L.N;
  const int ns = (K + 31) / 32;
  const int nt = (N + 15) / 16;
  const GAS char* W = (const GAS char*)L.W + lane * 16;
  const int steps = (int)L.ldw;  // packed K steps per tile
  // this wave's tiles' packed blocks; tiles past N re-read the last tile (discarded)
  int64_t wtile[TPW];
  bool tv[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int t = wave + NWV * j;
    tv[j] = t < nt;
    wtile[j] = (int64_t)std::min(t, nt - 1) * steps * 2048;
  }
  // a global input: this lane's two rows (row tiles 0, 1), clamped into the block
  const GAS float* arow[2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
    arow[rt] = (const GAS float*)in.g + (int64_t)std::min(16 * rt + c, rows - 1) * in.ld;

  struct Set {
    u32x4 h[TPW], l[TPW];
    float a[2][8];  // a global input's values for this step
  };
  constexpr int D = act_depth(TPW);
  Set sets[D];
  // weights (and a global input) D - 1 steps ahead, D register sets in rotation
  auto load = [&](Set& S, int s) {
    const int sc = std::min(s, ns - 1);
    const int64_t ko = (int64_t)sc * 2048;
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const GAS char* q = W + wtile[j] + ko;
      S.h[j] = *(const GAS u32x4*)q;
      S.l[j] = *(const GAS u32x4*)(q + 1024);
    }
    if constexpr (GIN) {  // K % 32 == 0 and 16-B aligned rows (host-checked): 32 B per lane
      const int k0 = sc * 32 + 8 * g;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const f32x4 x = *(const GAS f32x4*)(arow[rt] + k0), y = *(const GAS f32x4*)(arow[rt] + k0 + 4);
        S.a[rt][0] = x[0]; S.a[rt][1] = x[1]; S.a[rt][2] = x[2]; S.a[rt][3] = x[3];
        S.a[rt][4] = y[0]; S.a[rt][5] = y[1]; S.a[rt][6] = y[2]; S.a[rt][7] = y[3];
      }
    }
  };
  f32x4 acc[2][TPW];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int j = 0; j < TPW; ++j) acc[rt][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto step = [&](const Set& S, int s) {
    bf16x8 ah[2], al[2];
    const int k0 = s * 32 + 8 * g;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      float v[8];
      if constexpr (GIN) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = S.a[rt][e];
      } else {
        const int kc = std::min(s, ns - 1) * 32 + 8 * g;  // in the image (zeroed below past K)
        const float* q = act_lds + in.off + (16 * rt + c) * (int)in.ld + kc;
        const f32x4 x = *reinterpret_cast<const f32x4*>(q), y = *reinterpret_cast<const f32x4*>(q + 4);
        v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3]; v[4] = y[0]; v[5] = y[1]; v[6] = y[2]; v[7] = y[3];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = k0 + e < K ? v[e] : 0.f;
      split8(v, ah[rt], al[rt]);
    }
    // the three products of every tile in turn (lo*hi, hi*lo, hi*hi: each accumulator's chain
    // in lgx_s8.hip's order), so dependent MFMAs are 2 TPW instructions apart
#pragma unroll
    for (int pr = 0; pr < 3; ++pr)
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        if (!tv[j]) continue;
        const bf16x8 bh = __builtin_bit_cast(bf16x8, S.h[j]), bl = __builtin_bit_cast(bf16x8, S.l[j]);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
          const bf16x8 x = pr == 0 ? al[rt] : ah[rt], y = pr == 1 ? bl : bh;
          acc[rt][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, acc[rt][j], 0, 0, 0);
        }
      }
  };

#pragma unroll
  for (int d = 0; d < D - 1; ++d) load(sets[d], d);
  const int nsp = (ns + D - 1) / D * D;  // steps past ns multiply zeros (A is zero for k >= K)
  for (int s = 0; s < nsp; s += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      load(sets[(d + D - 1) % D], s + d + D - 1);
      step(sets[d], s + d);
    }
  }

  // epilogue: bias (+ ELU); MFMA C map: col = lane & 15, row = 4 (lane >> 4) + r
#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    if (!tv[j]) continue;
    const int col = 16 * (wave + NWV * j) + c;
    if (col >= N) continue;
    const float bias = ((const GAS float*)L.b)[col];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * rt + 4 * g + r;
        float v = acc[rt][j][r] + bias;
        if (L.elu) v = elu(v);
        if (out.g) {
          if (row < rows) ((GAS float*)out.g)[(int64_t)row * out.ld + col] = v;
        } else {
          act_lds[out.off + row * (int)out.ld + col] = v;
        }
      }
  }
  __syncthreads();
}

// rows [r0, r0 + rows) x n columns of src (row stride ld) into the LDS image (lds_off >= 0,
// pitch lds_ld) and / or a contiguous global [.., n] destination: the block's rows x columns as
// one flat range, 16 loads per thread in flight per pass (a load per row would pay a round
// trip each)
__device__ __forceinline__ void copy_rows(const float* src, int64_t ld, int n, int r0, int rows, int lds_off, int lds_ld,
                                          float* st) {
  constexpr int U = 16;
  const int tid = threadIdx.x;
  const int total = rows * n;
  for (int base = 0; base < total; base += NT * U) {
    float v[U];
    int rr[U], kk[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int idx = std::min(base + tid + NT * u, total - 1);
      rr[u] = idx / n;
      kk[u] = idx - rr[u] * n;
      v[u] = src[(int64_t)(r0 + rr[u]) * ld + kk[u]];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (base + tid + NT * u >= total) continue;
      if (lds_off >= 0) act_lds[lds_off + rr[u] * lds_ld + kk[u]] = v[u];
      if (st) st[(int64_t)(r0 + rr[u]) * n + kk[u]] = v[u];
    }
  }
}

// Layer i of this block's chain sequence — critic blocks: the critic; actor blocks: estimator,
// scan encoder, privileged encoder, actor — with its input and output (LDS images: X the actor
// input [R][XP], Y the hidden layers [R][YP] or two encoder scratch images [R][SP])
__device__ __forceinline__ void job(const lgx_s8_act_args& a, bool critic, int i, int r0, lgx_s8_act_layer& L, Src& in,
                                    Dst& out) {
  constexpr int X = 0, Y = XF, S1 = XF, S2 = XF + R * SP;
  auto hidden = [&](int pos, int& off, int64_t& ld) {  // the wide chains' images: Y, X, Y, ...
    off = (pos & 1) ? X : Y;
    ld = (pos & 1) ? XP : YP;
  };
  if (critic) {
    L = a.critic[i];
    if (i == 0) in = Src{a.critic_obs + (int64_t)r0 * a.ld_critic, a.ld_critic, 0};
    else { in.g = nullptr; hidden(i - 1, in.off, in.ld); }
    if (i == a.n_critic - 1) out = Dst{a.value + r0, 1, 0};
    else { out.g = nullptr; hidden(i, out.off, out.ld); }
    return;
  }
  const lgx_s8_act_layer* ch;
  int n, p;
  Src first;
  Dst last;
  if (i < a.n_est) {
    ch = a.est; n = a.n_est; p = i;
    first = Src{nullptr, XP, X + a.seg[0] + a.est_c0};
    last = Dst{nullptr, XP, X + a.seg[3]};
  } else if (i < a.n_est + a.n_scan) {  // its input staged in S2 (act_kernel)
    ch = a.scan; n = a.n_scan; p = i - a.n_est;
    first = Src{nullptr, SP, S2};
    last = Dst{nullptr, XP, X + a.seg[2]};
  } else if (i < a.n_est + a.n_scan + a.n_priv) {
    ch = a.priv; n = a.n_priv; p = i - a.n_est - a.n_scan;
    first = Src{nullptr, SP, S2};
    last = Dst{nullptr, XP, X + a.seg[1]};
  } else {
    p = i - a.n_est - a.n_scan - a.n_priv;
    L = a.actor[p];
    if (p == 0) in = Src{nullptr, XP, X};
    else { in.g = nullptr; hidden(p - 1, in.off, in.ld); }
    if (p == a.n_actor - 1) {
      // mu: to the act head's LDS image (the free half of the hidden images), or to global
      if (a.actions) { out.g = nullptr; out.off = (p & 1) ? X : Y; out.ld = 16; }
      else out = Dst{a.mu + (int64_t)r0 * a.ld_mu, a.ld_mu, 0};
    } else { out.g = nullptr; hidden(p, out.off, out.ld); }
    return;
  }
  // encoder chains: scratch images S1, S2, S1, ...
  L = ch[p];
  in = p == 0 ? first : Src{nullptr, SP, ((p - 1) & 1) ? S2 : S1};
  out = p == n - 1 ? last : Dst{nullptr, SP, (p & 1) ? S2 : S1};
}

// Every layer of this block type's chains, loaded once by all of the type's blocks on this XCD
// together (wave gw of 256 takes every 256th KB): the weights come back from HBM / the
// Infinity Cache in one round trip at the start instead of at each of the 13 layer starts
// (the env step in between evicts them from L2). The values are summed into `sink`, which the
// caller keeps alive.
__device__ __forceinline__ void warm_l2(const lgx_s8_act_layer* Ls, int n, int gw, int nslot, float& sink) {
  constexpr int U = 8;  // loads in flight per pass
  const int lane = threadIdx.x & 63;
  for (int i = 0; i < n; ++i) {
    const int64_t bytes = (int64_t)((Ls[i].N + 15) / 16) * Ls[i].ldw * 2048;
    const GAS char* W = (const GAS char*)Ls[i].W;
    const int64_t stride = (int64_t)nslot * NWV * 1024;
    for (int64_t off0 = (int64_t)gw * 1024 + lane * 16; off0 < bytes; off0 += U * stride) {
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = *(const GAS float*)(W + std::min(off0 + u * stride, bytes - 4));
#pragma unroll
      for (int u = 0; u < U; ++u) sink += v[u];
    }
  }
}

// The act head for the block's rows (lgx_mlp.hip act_head_kernel, the same arithmetic): mu in
// the LDS image at `mu_off` [R][16]; four lanes per row, lane q takes actions 4q..4q+3 (one
// Philox call), the row's log-prob terms summed in action order by its lane 0.
__device__ __forceinline__ void act_head(const lgx_s8_act_args& a, int mu_off, int r0, int rows, int A) {
  const int t = threadIdx.x;
  const int i = t >> 2, q = t & 3;
  if (i >= R) return;
  const bool row = i < rows, on = row && 4 * q < A;
  const float cst = 0.91893853320467274178f;  // log(sqrt(2 pi))
  float term[4] = {0.f, 0.f, 0.f, 0.f};
  const int gi = r0 + i;
  if (on) {
    float e4[4];
    if (a.eps == nullptr) {
      const uint64_t step = (uint64_t)*a.step_dev;
      const uint32_t gid = (uint32_t)(a.env_offset + gi);
      uint32_t o[4];
      philox4x32_10(gid, (uint32_t)step, (uint32_t)q | ((uint32_t)LGX_ACT_NOISE_STREAM << 16), (uint32_t)(step >> 32),
                    (uint32_t)a.seed, (uint32_t)(a.seed >> 32), o);
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
      for (int jj = 0; jj < 4; ++jj) e4[jj] = 4 * q + jj < A ? a.eps[(size_t)gi * A + 4 * q + jj] : 0.f;
    }
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = 4 * q + jj;
      if (j >= A) break;
      const size_t k = (size_t)gi * A + j;
      const float m = act_lds[mu_off + i * 16 + j], sd = a.std[j];
      const float x = m + sd * e4[jj];
      const float d = x - m;
      term[jj] = -(d * d) / (2.0f * (sd * sd)) - logf(sd) - cst;
      a.actions[k] = x;
      if (a.actions_copy) a.actions_copy[k] = x;
      a.mu_st[k] = m;
      a.sigma_st[k] = sd;
    }
  }
  float all[16];
#pragma unroll
  for (int qq = 0; qq < 4; ++qq)
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) all[4 * qq + jj] = __shfl(term[jj], (threadIdx.x & ~3) + qq, 64);
  if (row && q == 0) {
    float lp = 0.0f;
    for (int j = 0; j < A; ++j) lp += all[j];
    a.logp_st[gi] = lp;
  }
}

__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2, 2))) void act_kernel(lgx_s8_act_args a) {
  // both networks: actor blocks on XCDs 0-3, critic blocks on 4-7; one network: block = row block
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, nslot = (gridDim.x + 7) >> 3;
  const bool critic = a.nets == 0 ? xcd >= 4 : a.nets == 2;
  const int rb = a.nets == 0 ? slot * 4 + (xcd & 3) : blockIdx.x;
  const int nrb = (a.B + R - 1) / R;
  if (rb >= nrb) return;
  const int r0 = rb * R, rows = std::min(R, a.B - r0);
  const int tid = threadIdx.x;
  float sink = 0.f;
  {
    const int gw = slot * NWV + (tid >> 6);  // this XCD's blocks x 8 waves
    if (critic) {
      warm_l2(a.critic, a.n_critic, gw, nslot, sink);
    } else {
      if (a.n_est) {
        warm_l2(a.est, a.n_est, gw, nslot, sink);
        warm_l2(a.scan, a.n_scan, gw, nslot, sink);
        warm_l2(a.priv, a.n_priv, gw, nslot, sink);
      }
      warm_l2(a.actor, a.n_actor, gw, nslot, sink);
    }
  }
  // this step's storage rows (optional): contiguous [rows, n] copies of the inputs
  if (critic) {
    if (a.critic_st) copy_rows(a.critic_obs, a.ld_critic, a.n_critic_in, r0, rows, -1, 0, a.critic_st);
  } else {
    // the actor-input image: zero (its gaps between parts stay zero), then obs (and its row)
    for (int i = tid; i < XF; i += NT) act_lds[i] = 0.f;
    __syncthreads();
    copy_rows(a.obs, a.ld_obs, a.n_obs, r0, rows, a.seg[0], XP, a.obs_st);
    if (a.n_est == 0)  // the encoders ran elsewhere: their outputs into the actor-input parts
      for (int q = 0; q < 3; ++q) copy_rows(a.part_src[q], a.part_ld[q], a.part_w[q], r0, rows, a.seg[q + 1], XP, nullptr);
    if (a.priv_st) copy_rows(a.priv_obs, a.ld_priv, a.n_priv_in, r0, rows, -1, 0, a.priv_st);
    if (a.scan_st) copy_rows(a.scan_obs, a.ld_scan, a.n_scan_in, r0, rows, -1, 0, a.scan_st);
    if (a.est_st) copy_rows(a.est_obs, a.ld_est, a.n_est_obs, r0, rows, -1, 0, a.est_st);
    __syncthreads();
  }
  const int njobs = critic ? a.n_critic : a.n_est + a.n_scan + a.n_priv + a.n_actor;
  for (int i = 0; i < njobs; ++i) {
    lgx_s8_act_layer L;
    Src in;
    Dst out;
    job(a, critic, i, r0, L, in, out);
    if (!critic && a.n_scan > 0 && (i == a.n_est || i == a.n_est + a.n_scan)) {
      // the scan / privileged encoder's input rows into S2 (free between chains)
      const bool sc = i == a.n_est;
      copy_rows(sc ? a.scan_obs : a.priv_obs, sc ? a.ld_scan : a.ld_priv, sc ? a.n_scan_in : a.n_priv_in, r0, rows,
                XF + R * SP, SP, nullptr);
      __syncthreads();
    }
    const int nt = (L.N + 15) / 16;  // one call site per width class and input kind
    if (in.g) {
      if (nt > 2 * NWV) layer<4, true>(L, in, out, rows);
      else if (nt > NWV) layer<2, true>(L, in, out, rows);
      else layer<1, true>(L, in, out, rows);
    } else {
      if (nt > 2 * NWV) layer<4, false>(L, in, out, rows);
      else if (nt > NWV) layer<2, false>(L, in, out, rows);
      else layer<1, false>(L, in, out, rows);
    }
  }
  if (!critic && a.actions) act_head(a, ((a.n_actor - 1) & 1) ? 0 : XF, r0, rows, a.actor[a.n_actor - 1].N);
  if (sink == 1.2345e-38f && a.B < 0) a.value[0] = sink;  // keeps the warm-up loads (never true)
}

// the act-packed weights: thread = one (tile, step, lane) fragment (hi and lo, 32 B)
struct PackBatch {
  int n;
  int64_t start[LGX_S8_BATCH_MAX + 1];  // prefix sums of fragments
  lgx_s8_act_pack_args j[LGX_S8_BATCH_MAX];
};

__global__ __launch_bounds__(256) void pack_kernel(PackBatch b) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= b.start[b.n]) return;
  int ji = 0;
  while (ji + 1 < b.n && i >= b.start[ji + 1]) ++ji;
  const lgx_s8_act_pack_args& J = b.j[ji];
  const int64_t f = i - b.start[ji];
  const int lane = (int)(f & 63);
  const int64_t ts = f >> 6;  // t * steps + s
  const int t = (int)(ts / J.steps), s = (int)(ts - (int64_t)t * J.steps);
  const int n = 16 * t + (lane & 15), k0 = 32 * s + 8 * (lane >> 4);
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int k = k0 + e;
    float x = 0.f;
    for (int q = 0; q < J.nspans; ++q)
      if (n < J.N && k >= J.span_p0[q] && k < J.span_p0[q] + J.span_w[q]) x = J.W[(int64_t)n * J.ld + J.span_c0[q] + (k - J.span_p0[q])];
    v[e] = x;
  }
  bf16x8 hi, lo;
  split8(v, hi, lo);
  char* d = static_cast<char*>(J.dst) + ts * 2048 + lane * 16;
  *reinterpret_cast<bf16x8*>(d) = hi;
  *reinterpret_cast<bf16x8*>(d + 1024) = lo;
}

}  // namespace lgxa

static thread_local char a_err[256] = "";
static int afail(const char* m) {
  snprintf(a_err, sizeof a_err, "%s", m);
  return -1;
}

static int check_chain(const lgx_s8_act_layer* L, int n, int k_in, int maxh, const char* what) {
  if (n < 1 || n > LGX_S8_ACT_MAXL) return afail(what);
  int k = k_in;
  for (int i = 0; i < n; ++i) {
    if (!L[i].W || !L[i].b || L[i].K != k || L[i].N < 1 || L[i].ldw != (L[i].K + 31) / 32 ||
        (((uintptr_t)L[i].W) & 15))
      return afail(what);
    if (i < n - 1 && L[i].N > maxh) return afail(what);
    k = L[i].N;
  }
  return 0;
}

extern "C" {

const char* lgx_s8_act_last_error(void) { return a_err; }
int32_t lgx_s8_sizeof_act_args(void) { return (int32_t)sizeof(lgx_s8_act_args); }
int32_t lgx_s8_sizeof_act_pack_args(void) { return (int32_t)sizeof(lgx_s8_act_pack_args); }

int32_t lgx_s8_act_pack(const lgx_s8_act_pack_args* args, int32_t n, void* stream) {
  if (n < 0 || n > LGX_S8_BATCH_MAX || (n && !args)) return afail("lgx_s8_act_pack: 0 <= n <= LGX_S8_BATCH_MAX");
  lgxa::PackBatch b;
  memset(&b, 0, sizeof b);
  int k = 0;
  for (int i = 0; i < n; ++i) {
    const lgx_s8_act_pack_args& q = args[i];
    if (!q.W || !q.dst || q.N < 1 || q.steps < 1 || q.nspans < 1 || q.nspans > 4 || (((uintptr_t)q.dst) & 15))
      return afail("lgx_s8_act_pack: bad layer");
    for (int s = 0; s < q.nspans; ++s)
      if (q.span_w[s] < 0 || q.span_p0[s] < 0 || q.span_p0[s] + q.span_w[s] > 32 * q.steps || q.span_c0[s] < 0 ||
          q.span_c0[s] + q.span_w[s] > q.ld)
        return afail("lgx_s8_act_pack: span outside the layer");
    b.j[k] = q;
    b.start[k + 1] = b.start[k] + (int64_t)((q.N + 15) / 16) * q.steps * 64;
    ++k;
  }
  b.n = k;
  if (!k) return 0;
  hipLaunchKernelGGL(lgxa::pack_kernel, dim3((unsigned)((b.start[k] + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     b);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(a_err, sizeof a_err, "lgx_s8_act_pack: %s", hipGetErrorString(e));
    return -2;
  }
  return 0;
}

int32_t lgx_s8_act(const lgx_s8_act_args* a, void* stream) {
  if (!a || a->B < 0) return afail("lgx_s8_act: bad arguments");
  if (a->B == 0) return 0;
  if (!a->obs || !a->scan_obs || !a->priv_obs || !a->critic_obs || !a->mu || !a->value)
    return afail("lgx_s8_act: null input / output");
  if (a->width > LGX_S8_ACT_MAXIN || a->width % 32 || a->seg[0] != 0 || a->n_obs + a->seg[0] > a->seg[1] ||
      a->seg[1] > a->seg[2] || a->seg[2] > a->seg[3] || a->seg[3] > a->width || (a->seg[1] | a->seg[2] | a->seg[3]) % 4 ||
      a->est_c0 % 4 || a->est_c0 < 0)
    return afail("lgx_s8_act: actor-input layout (parts at multiples of 4 columns, width <= MAXIN, multiple of 32)");
  const bool enc = a->n_est > 0;
  if (!enc) {
    if (a->n_scan || a->n_priv) return afail("lgx_s8_act: encoders all in the kernel or none");
    const int pw[3] = {a->seg[2] - a->seg[1], a->seg[3] - a->seg[2], a->width - a->seg[3]};
    for (int q = 0; q < 3; ++q)
      if (!a->part_src[q] || a->part_w[q] < 1 || a->part_w[q] > pw[q] || a->part_ld[q] < a->part_w[q])
        return afail("lgx_s8_act: actor-input part sources");
  }
  if ((enc && (check_chain(a->est, a->n_est, a->est->K, LGX_S8_ACT_MAXENC, "lgx_s8_act: estimator chain") ||
               check_chain(a->scan, a->n_scan, a->scan->K, LGX_S8_ACT_MAXENC, "lgx_s8_act: scan-encoder chain") ||
               check_chain(a->priv, a->n_priv, a->priv->K, LGX_S8_ACT_MAXENC,
                           "lgx_s8_act: privileged-encoder chain"))) ||
      check_chain(a->actor, a->n_actor, a->width, LGX_S8_ACT_MAXH, "lgx_s8_act: actor chain") ||
      check_chain(a->critic, a->n_critic, a->critic->K, LGX_S8_ACT_MAXH, "lgx_s8_act: critic chain"))
    return -1;
  if (a->est_st && (!a->est_obs || a->n_est_obs < 1 || a->ld_est < a->n_est_obs))
    return afail("lgx_s8_act: est storage row without its source");
  if (a->actions && (!a->std || !a->mu_st || !a->sigma_st || !a->logp_st || (!a->eps && !a->step_dev) ||
                     a->actor[a->n_actor - 1].N > 16))
    return afail("lgx_s8_act: act head arguments (A <= 16)");
  if (a->n_critic_in % 32 || a->ld_critic % 4 || (((uintptr_t)a->critic_obs) & 15))
    return afail("lgx_s8_act: critic input: width a multiple of 32, 16-B aligned rows");
  if (enc && (a->n_scan_in > LGX_S8_ACT_MAXENC || a->n_priv_in > LGX_S8_ACT_MAXENC))
    return afail("lgx_s8_act: scan / privileged inputs wider than LGX_S8_ACT_MAXENC");
  if ((enc && (a->est_c0 + a->est->K > a->n_obs || a->scan->K != a->n_scan_in || a->priv->K != a->n_priv_in)) ||
      a->critic->K != a->n_critic_in)
    return afail("lgx_s8_act: first-layer widths do not match the inputs");
  if ((enc && (a->est[a->n_est - 1].N > a->width - a->seg[3] || a->scan[a->n_scan - 1].N > a->seg[3] - a->seg[2] ||
               a->priv[a->n_priv - 1].N > a->seg[2] - a->seg[1])) ||
      a->critic[a->n_critic - 1].N != 1 || a->actor[a->n_actor - 1].N > a->ld_mu)
    return afail("lgx_s8_act: output widths do not fit their parts");
  if (a->nets < 0 || a->nets > 2) return afail("lgx_s8_act: nets must be 0, 1 or 2");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)lgxa::act_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              lgxa::LDS_BYTES);
    attr = true;
  }
  const int nrb = (a->B + lgxa::R - 1) / lgxa::R;
  hipLaunchKernelGGL(lgxa::act_kernel, dim3(a->nets == 0 ? 8 * ((nrb + 3) / 4) : nrb), dim3(lgxa::NT), lgxa::LDS_BYTES,
                     (hipStream_t)stream, *a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(a_err, sizeof a_err, "lgx_s8_act: %s", hipGetErrorString(e));
    return -2;
  }
  return 0;
}

}  // extern "C"
