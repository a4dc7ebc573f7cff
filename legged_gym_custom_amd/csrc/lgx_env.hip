// lgx_env.hip — MI355X (gfx950) env-step kernels behind include/lgx.h.
//
// One wavefront (64 lanes) per environment; the env's state lives in LDS for the whole
// step (decimation physics substeps + post-physics), so HBM sees each per-env row once
// in and once out, coalesced (rows are env-major, lanes sweep a row).
//
// Physics (replaces PhysX `gym.simulate`, legged_robot.py:79-85; spec in DESIGN.md):
//   lanes 0..11  PD torques (legged_robot.py:440-478)
//   lanes 0..12  kinematics, one lane per joint (lane 12 the base), parent state passed down
//                the chain by DPP; per-link COM wrench and the base sums about p0
//   lanes 0..39  mass matrix [A B; Bᵀ D] factored lane-parallel: joint bias and coupling,
//                leg blocks D_l, X = B D⁻¹, the 21 Schur sums, S⁻¹ by a register Cholesky
//   lanes 0..63  contact candidates (one sphere centre per lane) -> ballot-compacted rows
//   lanes 0..R-1 one constraint row each: Jacobian row, M⁻¹Jᵀ column (Schur solve), A_rr,
//                then projected Gauss-Seidel on A = J M⁻¹ Jᵀ (lane r holds row r's velocity
//                and impulse; A stored in LDS, or formed per row for a fallen robot's rows)
// Post-physics (Go2Robot.post_physics_step go2.py:345-387, LeggedRobot legged_robot.py:
//   103-138): uniform scalar control flow per env; vector outputs written lane-parallel.
#include <hip/hip_runtime.h>
#include "lgx_knobs.h"
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/lgx.h"
#include "lgx_device.h"
#include "lgx_host.h"

namespace lgx {

constexpr int NL = 13;  // dynamic links: base + 4 chains x 3 (checked by lgx_create)
constexpr int NJ = 12;
constexpr int NU = 18;
constexpr int MAXC = LGX_MAX_CONTACTS;
constexpr int MAXR = NJ + 3 * MAXC;
// Philox blocks per env per step: 9 fixed blocks (commands, push/terrain, dof, root, reset
// commands) + one per 4 observation-noise draws (oracle/philox.py num_blocks): Go2 22,
// ANYmal (235 proprio) 68
constexpr int NBLK_MAX = 9 + (LGX_MAX_PROPRIO + 3) / 4;
constexpr int NSLOT = NBLK_MAX * 4;
LGX_DEV int rng_blocks(const lgx_task_params* Pm) { return 9 + (Pm->num_proprio + 3) / 4; }
constexpr int MAXHIST = 1216;

enum Slot { S_CMD = 0, S_PUSH = 4, S_TERR = 6, S_DOF = 8, S_ROOT_XY = 20, S_ROOT_VEL = 24, S_RCMD = 32, S_NOISE = 36 };

struct Scratch {  // per-env post-physics scalars (go2.py:357-367, 279-328)
  float blv[3], bav[3], pg[3];
  float roll, pitch, yaw;
  float ph[4];  // fl fr bl br
  int contact[4];
  float feet_z[4];
  float jump;
};

// LDS arena (dynamic shared memory, sized per launch by arena_floats) time-shared by phase:
//   dynamics   Fw, Nw [NL][3], Dl [4][6], tot [16]
//   rows       ZG [MAXR][RW] at 0: z_r = S⁻¹ (J_b − X_l J_l) (6) | g_r = D_l⁻¹ J_l (3);
//              J9 [MAXR][RW] at MAXR*RW: sparse row r = [base part (6) | the 3 joints of leg
//              rleg[r]]; once J9 is in registers, the same region holds A = J M⁻¹ Jᵀ: square
//              [n][n] for n <= ASQ rows, packed lower triangle for ASQ < n <= AMAX (see substep)
//   post       U [4 rng_blocks] | cur [P] | hist [H*P] | heights [Hp] (stg_* below)
// Go2 needs 1116 floats (the rows), ANYmal's post-physics staging 1,924.
// Rows per env step: p50 9, p99 15, max 27 (tools/phase_clock.py, r02). The launch time is
// the slowest wave's, so the rare env above ASQ rows must not fall to the velocity-space sweep
// (a launch with one such env took 25-65 % longer): up to AMAX rows A is kept as a packed
// lower triangle in the same LDS.
constexpr int ASQ = 24;   // square A up to here
constexpr int AMAX = 33;  // packed-triangle A up to here (33 * 34 / 2 = 561 <= 24 * 24)
constexpr int RW = 9;     // sparse row width
constexpr int A_FLOATS = ASQ * ASQ > AMAX * (AMAX + 1) / 2 ? ASQ * ASQ : AMAX * (AMAX + 1) / 2;
constexpr int J9_FLOATS = MAXR * RW > A_FLOATS ? MAXR * RW : A_FLOATS;
constexpr int ROWS_FLOATS = MAXR * RW + J9_FLOATS;
extern __shared__ float lgx_dyn[];
struct DynTemps {
  float Fw[NL][3], Nw[NL][3];  // per-link COM wrench (bias)
  float Dl[4][6];              // leg blocks of the joint-space inertia (xx yy zz xy xz yz)
  float tot[16];               // base sums about p0: m, h(3), Ip(6), F(3), N(3)
  float Sp[21];                // Σ_j X_j B_jᵀ, packed lower
};
static_assert(sizeof(DynTemps) <= ROWS_FLOATS * sizeof(float), "dynamics temporaries fit the arena");
// Each env owns one arena (A below: lgx_dyn, or lgx_dyn + arena_floats for the second env of a
// paired wave, see env_step_kernel)
LGX_DEV DynTemps& dtmp(float* A) { return *reinterpret_cast<DynTemps*>(A); }
LGX_DEV float* stg_U(float* A) { return A; }
LGX_DEV float* stg_cur(float* A, const lgx_task_params* Pm) { return A + 4 * rng_blocks(Pm); }
// The old observation history is staged in LDS when it is short (Go2: 10 x 52 = 520); a long
// one (ANYmal: 5 x 235 = 1175, 4.7 KB) is shifted in place in HBM instead (post-physics below),
// which keeps ANYmal's arena at the Go2 size: 9.9 KB of LDS per env, 16 envs per CU.
constexpr int HIST_LDS_MAX = 640;
__host__ __device__ inline bool hist_in_lds(const lgx_task_params* Pm) {
  return Pm->history_len * Pm->num_proprio <= HIST_LDS_MAX || Pm->num_proprio < 64;
}
LGX_DEV float* stg_hist(float* A, const lgx_task_params* Pm) { return stg_cur(A, Pm) + Pm->num_proprio; }
LGX_DEV float* stg_heights(float* A, const lgx_task_params* Pm) {
  return stg_hist(A, Pm) + (hist_in_lds(Pm) ? Pm->history_len * Pm->num_proprio : 0);
}
__host__ __device__ inline int64_t arena_floats(const lgx_task_params& p) {
  const int64_t post = 4 * (9 + (p.num_proprio + 3) / 4) + p.num_proprio +
                       (hist_in_lds(&p) ? (int64_t)p.history_len * p.num_proprio : 0) + p.num_height_points;
  return post > ROWS_FLOATS ? post : ROWS_FLOATS;
}

struct Sh {
  // --- post-physics per-env scalars (written by lane 0, read by all lanes)
  Scratch x;
  float root[13], cmd[4], fat[4], lch[4];
  int lc[4];
  float rterm[64];
  float jsum[16];  // per-env joint / height-point sums the reward terms share (joint_sums)
  // post-physics inputs read at kernel start (their HBM latency hides behind the physics)
  long long ep_prev;
  int lc_prev[LGX_MAX_FEET];
  float lch_prev[LGX_MAX_FEET], fat_prev[LGX_MAX_FEET], jump_prev;
  float la_prev[NJ], lt_prev[NJ];     // last_actions / last_torques (reward joint sums)
  float es[LGX_MAX_REWARDS + 4];      // episode_sums row (updated by this step's terms)
  float fric;                         // raw friction coefficient (privileged obs)
  long long ep;
  int reset, tout;
  int blew;  // this step's physics went non-finite (NaN/Inf guard; the env is reset)
  // --- physics state (base velocity kept as the ORIGIN velocity inside the step)
  float qb[4], pb[3], vo[3], wb[3];
  float th[NJ], thd[NJ], tau[NJ], act[NJ], kpm[NJ], kdm[NJ], ldv[NJ];
  float madd, cadd[3], mu;
  // --- kinematics per dynamic link
  float R[NL][9], P[NL][3], Ax[NL][3], W[NL][3], V[NL][3], C[NL][3], I[NL][6], m[NL];
  // --- dynamics
  float Bc[NJ][6], Dinv[4][6], X[NJ][6], Sinv[6][6], us[NU], up[NU];
  // --- constraints (J, M⁻¹Jᵀ and A live in the arena below)
  float Arr[MAXR], tgt[MAXR], lam[MAXR];
  int rleg[MAXR];
  int cbody[MAXC];
  float cn[MAXC][3];  // contact normals (terrain); tangents follow from contact_tangents
  int nrows, nlim, ncon;
  float cf[LGX_MAX_BODIES][3];
  float rbz[LGX_MAX_BODIES];
#ifdef LGX_PHASE_CLOCK
  uint64_t phlast;
  uint32_t phacc[20];
#endif
};

// ---- per-phase cycle counters (dev builds only: -DLGX_PHASE_CLOCK, tools/phase_clock.py).
// Lane 0 accumulates s_memtime deltas per phase in LDS; the kernel's end writes them to
// g_phase_out[env][phase]. Compiled out of the product library.
#ifdef LGX_PHASE_CLOCK
constexpr int NPH = 20;  // 16 phases + [16] max constraint rows, [17] wide-path substeps, [18] HW_ID, [19] XCC_ID
__device__ uint32_t* g_phase_out = nullptr;
#define PH(k)                                              \
  do {                                                     \
    if (lane == 0) {                                       \
      const uint64_t _t = clock64();                       \
      s.phacc[k] += (uint32_t)(_t - s.phlast);             \
      s.phlast = _t;                                       \
    }                                                      \
  } while (0)
#else
#define PH(k) \
  do {        \
  } while (0)
#endif

// ============================================================== physics helpers
#pragma clang fp contract(fast)

// a pointer the compiler must treat as changed here (defeats loop-invariant hoisting)
template <class T>
LGX_DEV const T* opaque(const T* p) {
  __asm__ volatile("" : "+s"(p));
  return p;
}

// XCD-aware env order. The hardware deals consecutive blocks to the 8 XCDs in turn, and env e's
// rows ([N,13] root state, [N,24] dof state, ...) share 128-B lines with env e +- 1's, so neighbouring
// envs are given blocks of the same XCD (one L2 fetches the shared line once): XCD x = b % 8 runs
// the contiguous env range [x*q + min(x, r), ...) of q + (x < r) envs (N = 8q + r) — a bijection
// of [0, N).
LGX_DEV int env_of_block(int b, int n) {
  const int q = n >> 3, r = n & 7, x = b & 7, j = b >> 3;
  return x * q + min(x, r) + j;
}

#ifndef LGX_ROW_PRIO
#define LGX_ROW_PRIO 9  // 0: no priority
#endif
#ifndef LGX_SLOT_PRIO
#define LGX_SLOT_PRIO 0  // 1: issue priority by the wave's slot on its SIMD (see env_step_kernel)
#endif

// the wave's slot on its SIMD (HW_ID wave_id field)
LGX_DEV int wave_slot() { return __builtin_amdgcn_s_getreg(4 | (3 << 11)) & 15; }
// s_setprio(p) for a runtime p in 0..3
LGX_DEV void set_prio(int p) {
  if (p >= 3) __builtin_amdgcn_s_setprio(3);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
  else if (p == 1) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}

LGX_DEV int opaque_lane(int v) {
  __asm__ volatile("" : "+v"(v));
  return v;
}

// ---- lane groups. An env owns WL consecutive lanes of its wave: WL = 64 (one env per wave) or
// WL = 32 (two envs per wave, lanes 0..31 and 32..63: the phases that use a dozen to thirty
// lanes of an env then do two envs' work per instruction). The physics and post-physics
// functions below take `lane` = the lane within the group and the group's own Sh / arena; the
// helpers here are the cross-lane operations made group-local. (DPP row operations act on
// 16-lane rows and are group-local as they are.)
template <int WL>
LGX_DEV int grp_of_lane() {
  if constexpr (WL == 64) return 0;
  else return (int)(__lane_id() >> 5);
}
// this group's ballot, bit i = group lane i
template <int WL>
LGX_DEV uint64_t gballot(bool p) {
  const uint64_t m = __ballot(p);
  if constexpr (WL == 64) return m;
  else return (__lane_id() >> 5) ? (m >> 32) : (m & 0xffffffffull);
}
LGX_DEV float rdl(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
LGX_DEV int rdl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
// v of group lane r0 (group 0) / r1 (group 1), in every lane of the group (r0, r1 wave-uniform)
template <int WL>
LGX_DEV float gbcast(float v, int r0, int r1) {
  if constexpr (WL == 64) {
    return rdl(v, r0);
  } else {
    const float a = rdl(v, r0), b = rdl(v, 32 + r1);
    return (__lane_id() >> 5) ? b : a;
  }
}
template <int WL>
LGX_DEV float gbcast(float v, int r) { return gbcast<WL>(v, r, r); }
// a * b for a, b < 2^24 as one full-rate v_mul_u32_u24 (the compiler otherwise folds small
// index products into 64-bit multiply-adds)
LGX_DEV int mul24(int a, int b) {
  int r;
  __asm__("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// a group-uniform int of group 0 / group 1 as wave-uniform scalars
template <int WL>
LGX_DEV int gval(int v, int g) {
  if constexpr (WL == 64) return __builtin_amdgcn_readfirstlane(v);
  else return rdl(v, 32 * g);
}
// the largest of the groups' values of a group-uniform int (a wave-uniform loop bound)
template <int WL>
LGX_DEV int gmax(int v) {
  if constexpr (WL == 64) return __builtin_amdgcn_readfirstlane(v);
  else return max(rdl(v, 0), rdl(v, 32));
}
// sum over group lanes 0..15 (the group's first DPP row), returned to every lane of the group;
// lanes 0..15 of the group must be active
template <int WL>
LGX_DEV float grow_sum16(float x) {
  x += dpp_shr_t<0x111>(x);
  x += dpp_shr_t<0x112>(x);
  x += dpp_shr_t<0x114>(x);
  x += dpp_shr_t<0x118>(x);
  return gbcast<WL>(x, 15);
}

// symmetric 3x3 (xx yy zz xy xz yz) inverse
LGX_DEV void sym3_inv(const float* D, float* O) {
  float a = D[0], b = D[1], c = D[2], d = D[3], e = D[4], f = D[5];
  float A = b * c - f * f, Bm = -(d * c - e * f), Cm = d * f - b * e;
  float det = a * A + d * Bm + e * Cm;
  float inv = 1.0f / det;
  O[0] = A * inv;
  O[1] = (a * c - e * e) * inv;
  O[2] = (a * b - d * d) * inv;
  O[3] = Bm * inv;
  O[4] = Cm * inv;
  O[5] = -(a * f - d * e) * inv;
}
LGX_DEV float sym3(const float* S, int i, int j) {
  if (i == j) return S[i];
  int k = i + j;  // (0,1)->3 (0,2)->4 (1,2)->5
  return S[k == 1 ? 3 : (k == 2 ? 4 : 5)];
}
// packed symmetric 6x6 index (lower, row-major)
LGX_DEV int pk(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }

// lane i receives lane i-1's value (DPP row_shr:1; lanes 0..15 form one row)
LGX_DEV float from_prev_lane(float x) { return dpp_shr_t<0x111>(x); }

// Forward kinematics, velocities and bias accelerations, one lane per link: lane j < 12
// is joint j / link j+1 (leg j/3, chain position j%3), lane 12 the base. A chain is three
// deep: each of three rounds composes every lane with its parent's world state, then the
// parent state moves one lane down the chain by DPP, so no lane waits on LDS. Writes the
// link arrays the later phases read (R, P, Ax, W, V, C, I, m). With BIAS, the same lanes
// also form the per-link COM wrench (Fw, Nw) and return the 16 base sums about p0 (mass,
// first moment, inertia, wrench), reduced across lanes 0..15 by DPP (see dynamics).
template <bool BIAS>
LGX_DEV void kinematics(Sh& s, float* A, const lgx_model* M, const lgx_task_params* Pm, int lane) {
  const int j = lane < NJ ? lane : NJ - 1;
  const bool base = lane == NJ;  // the base rides the chain as a fixed joint at the root
  const int a = base ? 0 : j % 3;
  const int k = base ? 0 : j + 1;
  // per-lane model constants (vector loads, L1-resident); identity joint for the base lane
  const float bm = base ? 0.f : 1.f;
  const f3 orig = ld3(M->joint_origin[j + 1]) * bm, al = ld3(M->joint_axis[j + 1]) * bm;
  float Rj[9];
  {
    const float* Rjp = M->joint_rot[j + 1];
#pragma unroll
    for (int q = 0; q < 9; ++q) Rj[q] = base ? ((q & 3) == 0 ? 1.f : 0.f) : Rjp[q];
  }
  // local rotation of joint j: joint frame, then the axis-angle rotation
  const float th = base ? 0.f : s.th[j], thd = base ? 0.f : s.thd[j];
  float Rl[9];
  {
    const float ct = cosf(th), st = sinf(th), t1 = 1.f - ct;
    const float Ra[9] = {t1 * al.x * al.x + ct, t1 * al.x * al.y - st * al.z, t1 * al.x * al.z + st * al.y,
                         t1 * al.x * al.y + st * al.z, t1 * al.y * al.y + ct, t1 * al.y * al.z - st * al.x,
                         t1 * al.x * al.z - st * al.y, t1 * al.y * al.z + st * al.x, t1 * al.z * al.z + ct};
    mm(Rj, Ra, Rl);
  }
  const f3 axl = mv(Rj, al);
  // parent state, initially the base (uniform)
  float Rp[9];
  quat_to_R(s.qb, Rp);
  f3 Pp = ld3(s.pb), Wp = ld3(s.wb), Vp = ld3(s.vo), Alp = mk(0.f, 0.f, 0.f), Aop = mk(0.f, 0.f, 0.f);
  float R[9];
  f3 P, ax, W, V, Al, Ao;
#pragma unroll 1
  for (int d = 0; d < 3; ++d) {
    const f3 o = mv(Rp, orig);
    ax = mv(Rp, axl);
    mm(Rp, Rl, R);
    P = Pp + o;
    const f3 wa = ax * thd;
    W = Wp + wa;
    if constexpr (BIAS) {
      Al = Alp + cross(Wp, wa);
      Ao = Aop + cross(Alp, o) + cross(Wp, cross(Wp, o));
    } else {
      V = Vp + cross(Wp, o);
    }
    if (d < 2) {
      const bool take = a == d + 1;
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        const float v = from_prev_lane(R[q]);
        Rp[q] = take ? v : Rp[q];
      }
#define LGX_PASS(dst, src)                                                                          \
  {                                                                                                 \
    const float vx = from_prev_lane(src.x), vy = from_prev_lane(src.y), vz = from_prev_lane(src.z); \
    dst.x = take ? vx : dst.x;                                                                      \
    dst.y = take ? vy : dst.y;                                                                      \
    dst.z = take ? vz : dst.z;                                                                      \
  }
      LGX_PASS(Pp, P)
      LGX_PASS(Wp, W)
      if constexpr (BIAS) {
        LGX_PASS(Alp, Al)
        LGX_PASS(Aop, Ao)
      } else {
        LGX_PASS(Vp, V)
      }
#undef LGX_PASS
    }
  }
  const float* clp = M->link_com[k];
  const float cb = base ? 1.f : 0.f;
  const f3 cl = mk(clp[0] + cb * s.cadd[0], clp[1] + cb * s.cadd[1], clp[2] + cb * s.cadd[2]);
  const f3 C = P + mv(R, cl);
  if (lane <= NJ) {
#pragma unroll
    for (int q = 0; q < 9; ++q) s.R[k][q] = R[q];
    st3(s.P[k], P);
    st3(s.Ax[k], ax);
    st3(s.W[k], W);
    st3(s.C[k], C);
    if constexpr (!BIAS) st3(s.V[k], V);
  }
  if constexpr (BIAS) {
    const float m = M->link_mass[k] + cb * s.madd;
    // world inertia about the COM: R I Rᵀ
    float Iw[6];
    {
      const float* In = M->link_inertia[k];
      const float Il[9] = {In[0], In[3], In[4], In[3], In[1], In[5], In[4], In[5], In[2]};
      float T[9];
      mm(R, Il, T);
      Iw[0] = T[0] * R[0] + T[1] * R[1] + T[2] * R[2];
      Iw[1] = T[3] * R[3] + T[4] * R[4] + T[5] * R[5];
      Iw[2] = T[6] * R[6] + T[7] * R[7] + T[8] * R[8];
      Iw[3] = T[0] * R[3] + T[1] * R[4] + T[2] * R[5];
      Iw[4] = T[0] * R[6] + T[1] * R[7] + T[2] * R[8];
      Iw[5] = T[3] * R[6] + T[4] * R[7] + T[5] * R[8];
    }
    const f3 g = ld3(Pm->gravity);
    const f3 rl = C - P;
    const f3 acc = Ao + cross(Al, rl) + cross(W, cross(W, rl));
    const f3 F = (acc - g) * m;
    const f3 N = symv(Iw, Al) + cross(W, symv(Iw, W));
    if (lane <= NJ) {
#pragma unroll
      for (int q = 0; q < 6; ++q) s.I[k][q] = Iw[q];
      s.m[k] = m;
      st3(dtmp(A).Fw[k], F);
      st3(dtmp(A).Nw[k], N);
    }
    // the 16 base sums about p0, reduced over lanes 0..15 (row 0) by a DPP scan whose
    // total lands on lane 15
    const f3 r = C - ld3(s.pb);
    const float rr = dot(r, r);
    const f3 Nt = cross(r, F) + N;
    const float on = lane <= NJ ? 1.f : 0.f;
    const float rd[16] = {m, m * r.x, m * r.y, m * r.z,
                          Iw[0] + m * (rr - r.x * r.x), Iw[1] + m * (rr - r.y * r.y), Iw[2] + m * (rr - r.z * r.z),
                          Iw[3] - m * r.x * r.y, Iw[4] - m * r.x * r.z, Iw[5] - m * r.y * r.z,
                          F.x, F.y, F.z, Nt.x, Nt.y, Nt.z};
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      float x = rd[q] * on;
      x += dpp_shr_t<0x111>(x);
      x += dpp_shr_t<0x112>(x);
      x += dpp_shr_t<0x114>(x);
      x += dpp_shr_t<0x118>(x);
      if (lane == 15) dtmp(A).tot[q] = x;
    }
  }
  __syncthreads();
}

// Mass matrix M = [A B; Bᵀ D] over u = [base origin velocity, ω | 12 joint rates] (D block
// diagonal over the 4 chains) and bias h, factored so that every later product with M⁻¹ is
// a short lane-parallel chain instead of one lane's serial solve:
//   X = B D⁻¹ (s.X[j][r] = X[r][j]),  S = A − X Bᵀ (base Schur complement),  S⁻¹ (s.Sinv)
//   M⁻¹ f = [z ; D⁻¹ f_J − Xᵀ z]  with  z = S⁻¹ (f_B − X f_J)
//   J M⁻¹ Jᵀ = y_rᵀ S⁻¹ y_s + [leg_r = leg_s] J_r,Jᵀ D_l⁻¹ J_s,J  with  y = J_B − X J_J
// Lanes:
//   D1 (in kinematics<true>) per-link COM wrench; the 16 base sums about p0 by DPP
//   D2 lanes 0..11  joint bias h_j and coupling column B_j;  lanes 8..31 leg block D_l
//   D3 lanes 0..11  D_l⁻¹ (row a), X_j; the 21 Schur sums by DPP; every lane factors S in
//                   registers (Cholesky); lanes 0..5 write column `lane` of S⁻¹
struct DynOut {
  float hb[6];    // base bias (uniform)
  float hj;       // lane j < 12: joint bias
  float xj[6];    // lane j < 12: X_j
  float dinv[3];  // lane j < 12: row a of D_l⁻¹
};

LGX_DEV void dynamics(Sh& s, float* A, int lane, DynOut& o) {
  const f3 p0 = ld3(s.P[0]);
  const float* tot = dtmp(A).tot;
  const int j = lane < NJ ? lane : NJ - 1, l = j / 3, a = j % 3;
  if (lane < NJ) {  // ---- D2a: joint j (leg l, chain position a)
    const int kj = 1 + j;
    const f3 ax = ld3(s.Ax[kj]), pj = ld3(s.P[kj]);
    f3 acc = mk(0, 0, 0), hl = mk(0, 0, 0), bang = mk(0, 0, 0);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (i < a) continue;
      const int k = 1 + 3 * l + i;
      const f3 c = ld3(s.C[k]);
      const f3 d = c - pj;
      const float m = s.m[k];
      acc = acc + cross(d, ld3(dtmp(A).Fw[k])) + ld3(dtmp(A).Nw[k]);
      hl = hl + d * m;
      bang = bang + cross(c - p0, cross(ax, d)) * m + symv(s.I[k], ax);
    }
    o.hj = dot(ax, acc);
    const f3 blin = cross(ax, hl);
    float* Bj = s.Bc[j];
    Bj[0] = blin.x; Bj[1] = blin.y; Bj[2] = blin.z; Bj[3] = bang.x; Bj[4] = bang.y; Bj[5] = bang.z;
  }
  // (the two branches run one after the other in the wave either way; lanes 8..31 keep both
  // parts within one 32-lane group)
  if (lane >= 8 && lane < 32) {  // ---- D2b: leg block entry (xx yy zz xy xz yz)
    const int q = lane - 8, lq = q / 6, e = q % 6;
    const int j1 = e < 3 ? e : (e == 5 ? 1 : 0);
    const int j2 = e < 3 ? e : (e == 3 ? 1 : 2);
    const int k1 = 1 + 3 * lq + j1, k2 = 1 + 3 * lq + j2;
    const f3 a1 = ld3(s.Ax[k1]), a2 = ld3(s.Ax[k2]), p1 = ld3(s.P[k1]), p2 = ld3(s.P[k2]);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (i < j2) continue;
      const int k = 1 + 3 * lq + i;
      const f3 c = ld3(s.C[k]);
      acc += s.m[k] * dot(cross(a1, c - p1), cross(a2, c - p2)) + dot(a1, symv(s.I[k], a2));
    }
    dtmp(A).Dl[lq][e] = acc;
  }
  __syncthreads();
  // ---- D3
  float Di[6];
  sym3_inv(dtmp(A).Dl[l], Di);
#pragma unroll
  for (int c = 0; c < 3; ++c) o.dinv[c] = sym3(Di, a, c);
  if (lane < NJ && a == 0) {
#pragma unroll
    for (int q = 0; q < 6; ++q) s.Dinv[l][q] = Di[q];
  }
  float bj[6];
  {
    const float* B0 = s.Bc[3 * l];
    const float* B1 = s.Bc[3 * l + 1];
    const float* B2 = s.Bc[3 * l + 2];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const float b0 = B0[r], b1 = B1[r], b2 = B2[r];
      o.xj[r] = o.dinv[0] * b0 + o.dinv[1] * b1 + o.dinv[2] * b2;
      bj[r] = a == 0 ? b0 : (a == 1 ? b1 : b2);
    }
  }
  if (lane < NJ) {
#pragma unroll
    for (int r = 0; r < 6; ++r) s.X[j][r] = o.xj[r];
  }
  // the 21 Schur sums Σ_j X_j[r] B_j[c] (packed lower), one lane each over the 12 joints
  __syncthreads();
  if (lane < 21) {
    const int q = lane;
    const int r = (q >= 1) + (q >= 3) + (q >= 6) + (q >= 10) + (q >= 15), c = q - r * (r + 1) / 2;
    float acc = 0.f;
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj) acc += s.X[jj][r] * s.Bc[jj][c];
    dtmp(A).Sp[q] = acc;
  }
  __syncthreads();
  // S = A_bb − Σ_j X_j B_jᵀ; A_bb = [[M I, −[H]x], [[H]x, Ip]] (base origin velocity, ω),
  // [H]x = [[0,−Hz,Hy],[Hz,0,−Hx],[−Hy,Hx,0]]
  const float Mt = tot[0], Hx = tot[1], Hy = tot[2], Hz = tot[3];
  const float Ab[21] = {Mt, 0.f, Mt, 0.f, 0.f, Mt, 0.f, -Hz, Hy, tot[4], Hz, 0.f, -Hx, tot[7], tot[5],
                        -Hy, Hx, 0.f, tot[8], tot[9], tot[6]};
  float L[21];
#pragma unroll
  for (int q = 0; q < 21; ++q) L[q] = Ab[q] - dtmp(A).Sp[q];
  float inv[6];
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    float d = L[pk(c, c)];
#pragma unroll
    for (int k = 0; k < c; ++k) d -= L[pk(c, k)] * L[pk(c, k)];
    const float lcc = sqrtf(fmaxf(d, 1e-12f));
    inv[c] = 1.0f / lcc;
#pragma unroll
    for (int r = c + 1; r < 6; ++r) {
      float v = L[pk(r, c)];
#pragma unroll
      for (int k = 0; k < c; ++k) v -= L[pk(r, k)] * L[pk(c, k)];
      L[pk(r, c)] = v * inv[c];
    }
  }
  // column `lane` of S⁻¹ = L⁻ᵀ L⁻¹ e_lane
  float x[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) {
    float t = lane == r ? 1.f : 0.f;
#pragma unroll
    for (int k = 0; k < r; ++k) t -= L[pk(r, k)] * x[k];
    x[r] = t * inv[r];
  }
#pragma unroll
  for (int r = 5; r >= 0; --r) {
    float t = x[r];
#pragma unroll
    for (int k = r + 1; k < 6; ++k) t -= L[pk(k, r)] * x[k];
    x[r] = t * inv[r];
  }
  if (lane < 6) {
#pragma unroll
    for (int r = 0; r < 6; ++r) s.Sinv[lane][r] = x[r];
  }
#pragma unroll
  for (int q = 0; q < 6; ++q) o.hb[q] = tot[10 + q];
}

// ---- terrain contact (heightfield / trimesh)
// The reference collides against the triangle mesh convert_heightfield_to_trimesh builds
// (terrain_utils.py:382-465, legged_robot.py:788-802) or the PhysX heightfield
// (legged_robot.py:768-786). The mesh is never materialised: vertex (i, j) sits at
// ((i + dx) hs, (j + dy) hs, h vs) - border, where h (int16) and the slope-threshold
// shift (dx, dy in {-1, 0, 1}: steep steps become vertical walls) are packed in one 32-bit
// word per vertex (B.terrain_mesh, legged_gym_custom_amd/utils/terrain_utils.pack_mesh).
// Cell (i, j) holds the two triangles (v00, v11, v01), (v00, v10, v11). One lane queries
// one contact sphere: the closest mesh point over the cells whose (shifted) triangles can
// reach it, inside/outside from the surface height under the centre.
struct TerrainHit {
  float depth;  // sphere penetration (> 0: overlapping)
  f3 n;         // unit normal, terrain -> sphere
};

LGX_DEV f3 mesh_vertex(const uint32_t* mesh, int cols, int i, int j, int ci, int cj, float hs, float vs) {
  const uint32_t w = mesh[(size_t)i * cols + j];
  const float h = (float)(int16_t)(w & 0xffffu);
  const int dx = (int)((w >> 16) & 3u) - 1, dy = (int)((w >> 18) & 3u) - 1;
  return mk((float)(i - ci + dx) * hs, (float)(j - cj + dy) * hs, h * vs);
}

// closest point of triangle abc to p (Ericson, Real-Time Collision Detection 5.1.5),
// with guards for the zero-area triangles a wall shift can produce
LGX_DEV f3 closest_on_triangle(f3 p, f3 a, f3 b, f3 c) {
  const f3 ab = b - a, ac = c - a, ap = p - a;
  const float d1 = dot(ab, ap), d2 = dot(ac, ap);
  if (d1 <= 0.f && d2 <= 0.f) return a;
  const f3 bp = p - b;
  const float d3 = dot(ab, bp), d4 = dot(ac, bp);
  if (d3 >= 0.f && d4 <= d3) return b;
  const float vc = d1 * d4 - d3 * d2;
  if (vc <= 0.f && d1 >= 0.f && d3 <= 0.f) return a + ab * (d1 / fmaxf(d1 - d3, 1e-30f));
  const f3 cp = p - c;
  const float d5 = dot(ab, cp), d6 = dot(ac, cp);
  if (d6 >= 0.f && d5 <= d6) return c;
  const float vb = d5 * d2 - d1 * d6;
  if (vb <= 0.f && d2 >= 0.f && d6 <= 0.f) return a + ac * (d2 / fmaxf(d2 - d6, 1e-30f));
  const float va = d3 * d6 - d5 * d4;
  if (va <= 0.f && d4 - d3 >= 0.f && d5 - d6 >= 0.f)
    return b + (c - b) * ((d4 - d3) / fmaxf((d4 - d3) + (d5 - d6), 1e-30f));
  const float inv = 1.0f / fmaxf(va + vb + vc, 1e-30f);
  return a + ab * (vb * inv) + ac * (vc * inv);
}

// surface height of triangle abc above (p.x, p.y) if its xy projection contains it
LGX_DEV bool height_in_triangle(f3 p, f3 a, f3 b, f3 c, float& z) {
  const float e1x = b.x - a.x, e1y = b.y - a.y, e2x = c.x - a.x, e2y = c.y - a.y;
  const float det = e1x * e2y - e1y * e2x;
  if (fabsf(det) < 1e-10f) return false;  // vertical wall: no projection
  const float px = p.x - a.x, py = p.y - a.y;
  const float u = (px * e2y - py * e2x) / det, v = (e1x * py - e1y * px) / det;
  const float eps = -1e-6f;
  if (u < eps || v < eps || u + v > 1.0f - eps) return false;
  z = a.z + u * (b.z - a.z) + v * (c.z - a.z);
  return true;
}

// The trimesh contact query (closest point over the triangles of the cells a +-1 wall shift can
// reach; the host backend's / oracle's terrain_contact state it serially) for every contact
// candidate of the wave at once, the work spread over lanes:
// each candidate lane (cand) bounds its cell range, drops out when its sphere is above every
// vertex the range can reach (a conservative block maximum packed in the mesh words' bits
// 20-31, utils/terrain_utils.pack_mesh: such a sphere is farther than r + contact_margin from
// the surface, so it forms no row either way), and the remaining (candidate, cell) tasks run
// 64 per round, one per lane; each candidate lane then folds its tasks' closest points in the
// serial loop's (i, j, triangle) order with the same strict comparison, so the result equals
// the serial terrain_contact's exactly. One-candidate-per-lane made a wave as slow as its candidate with
// the most cells (25 cells x 2 triangles for a 0.1 m sphere) for all 22 (ANYmal) or 55 (Go2)
// lanes at once. Scratch: the LDS arena (rows are formed after detection).
constexpr int MESH_BLOCK = 8;  // vertices per block side of the packed block maxima
LGX_DEV float mesh_block_bound(uint32_t w) {  // block max height (raw units), or +inf if absent
  return (w >> 31) ? (float)((int)((w >> 20) & 0x7ffu) * 32 - 32768) : 3.0e38f;
}
template <int WL>
LGX_DEV TerrainHit terrain_contact_wave(const lgx_task_params* Pm, const lgx_buffers& B, float* A, f3 x, float r,
                                        bool cand, int lane) {
  const float hs = Pm->horizontal_scale, vs = Pm->vertical_scale;
  const int rows = Pm->hf_rows, cols = Pm->hf_cols;
  const uint32_t* mesh = B.terrain_mesh;
  int cnt = 0, ci = 0, cj = 0, i0 = 0, j0 = 0, w = 1;
  f3 p = mk(0.f, 0.f, 0.f);
  if (cand) {
    const float gx = x.x + Pm->border_size, gy = x.y + Pm->border_size;
    ci = (int)floorf(gx / hs);
    cj = (int)floorf(gy / hs);
    p = mk(gx - (float)ci * hs, gy - (float)cj * hs, x.z);
    i0 = max(ci + (int)ceilf((p.x - r) / hs) - 2, 0);
    const int i1 = min(ci + (int)floorf((p.x + r) / hs) + 1, rows - 2);
    j0 = max(cj + (int)ceilf((p.y - r) / hs) - 2, 0);
    const int j1 = min(cj + (int)floorf((p.y + r) / hs) + 1, cols - 2);
    if (i1 >= i0 && j1 >= j0) {
      w = j1 - j0 + 1;
      cnt = (i1 - i0 + 1) * w;
      if (i1 + 1 - i0 < MESH_BLOCK && j1 + 1 - j0 < MESH_BLOCK) {  // <= 2 blocks a side: the corners see them all
        const float hb = fmaxf(fmaxf(mesh_block_bound(mesh[(size_t)i0 * cols + j0]),
                                     mesh_block_bound(mesh[(size_t)i0 * cols + j1 + 1])),
                               fmaxf(mesh_block_bound(mesh[(size_t)(i1 + 1) * cols + j0]),
                                     mesh_block_bound(mesh[(size_t)(i1 + 1) * cols + j1 + 1])));
        if (hb < 1.0e38f && p.z - r - Pm->contact_margin > hb * vs + 1e-4f) cnt = 0;
      }
    }
  }
  // inclusive prefix of the task counts over the group's lanes
  int endp = cnt;
#pragma unroll
  for (int d = 1; d < WL; d <<= 1) {
    const int v = __shfl_up(endp, d, WL);
    if (lane >= d) endp += v;
  }
  const int total = __shfl(endp, WL - 1, WL);
  const int total_max = gmax<WL>(total);  // the groups' task lists run side by side
  int* const T_end = reinterpret_cast<int*>(A);
  int* const T_ci = T_end + 64;
  int* const T_cj = T_end + 128;
  int* const T_i0 = T_end + 192;
  int* const T_j0 = T_end + 256;
  int* const T_w = T_end + 320;
  float* const T_p = A + 384;        // [3][64]
  float* const R_ = A + 576;         // results [8][64]: d2, q(3), fn(3), zs
  T_end[lane] = endp; T_ci[lane] = ci; T_cj[lane] = cj; T_i0[lane] = i0; T_j0[lane] = j0; T_w[lane] = w;
  T_p[lane] = p.x; T_p[64 + lane] = p.y; T_p[128 + lane] = p.z;
  float best = 3.0e38f, zs = -3.0e38f;
  f3 q = mk(0.f, 0.f, -3.0e38f), fn = mk(0.f, 0.f, 1.f);
  const int mystart = endp - cnt;
  for (int base = 0; base < total_max; base += WL) {
    __syncthreads();  // the tables (first round) / the previous round's results are read
    const int t = base + lane;
    float td2 = 3.0e38f, tz = -3.0e38f;
    f3 tq = mk(0.f, 0.f, -3.0e38f), tfn = mk(0.f, 0.f, 1.f);
    if (t < total) {
      int lo = 0, hi = WL - 1;  // owner: the first lane whose inclusive end exceeds t
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (T_end[mid] > t) hi = mid; else lo = mid + 1;
      }
      const int c = lo;
      const int k = t - (c ? T_end[c - 1] : 0);  // task index within candidate c
      const int wc = T_w[c];
      const int i = T_i0[c] + k / wc, j = T_j0[c] + k % wc;
      const int cci = T_ci[c], ccj = T_cj[c];
      const f3 pc = mk(T_p[c], T_p[64 + c], T_p[128 + c]);
      const f3 v00 = mesh_vertex(mesh, cols, i, j, cci, ccj, hs, vs);
      const f3 v01 = mesh_vertex(mesh, cols, i, j + 1, cci, ccj, hs, vs);
      const f3 v10 = mesh_vertex(mesh, cols, i + 1, j, cci, ccj, hs, vs);
      const f3 v11 = mesh_vertex(mesh, cols, i + 1, j + 1, cci, ccj, hs, vs);
#pragma unroll
      for (int tri = 0; tri < 2; ++tri) {
        const f3 a = v00, b = tri == 0 ? v11 : v10, cc = tri == 0 ? v01 : v11;
        const f3 cpt = closest_on_triangle(pc, a, b, cc);
        const f3 dd = pc - cpt;
        const float d2 = dot(dd, dd);
        if (d2 < td2) { td2 = d2; tq = cpt; tfn = cross(b - a, cc - a); }
        float z;
        if (height_in_triangle(pc, a, b, cc, z)) tz = fmaxf(tz, z);
      }
    }
    R_[lane] = td2;
    R_[64 + lane] = tq.x; R_[128 + lane] = tq.y; R_[192 + lane] = tq.z;
    R_[256 + lane] = tfn.x; R_[320 + lane] = tfn.y; R_[384 + lane] = tfn.z;
    R_[448 + lane] = tz;
    __syncthreads();
    if (cnt > 0) {  // this candidate's tasks of the round, in order
      const int a0 = max(mystart, base) - base, a1 = min(endp, base + WL) - base;
      for (int sl = a0; sl < a1; ++sl) {
        const float d2 = R_[sl];
        if (d2 < best) {
          best = d2;
          q = mk(R_[64 + sl], R_[128 + sl], R_[192 + sl]);
          fn = mk(R_[256 + sl], R_[320 + sl], R_[384 + sl]);
        }
        zs = fmaxf(zs, R_[448 + sl]);
      }
    }
  }
  __syncthreads();  // the arena is the constraint rows' next
  TerrainHit h;
  if (best >= 3.0e38f) {  // culled, outside the field, or no candidate: nothing to touch
    h.depth = -3.0e38f;
    h.n = mk(0.f, 0.f, 1.f);
    return h;
  }
  const float dist = sqrtf(best);
  const bool below = p.z < zs;
  h.depth = below ? r + dist : r - dist;
  if (dist > 1e-6f) {
    h.n = (p - q) * ((below ? -1.0f : 1.0f) / dist);
  } else {
    h.n = fn * rsqrtf(fmaxf(dot(fn, fn), 1e-30f));
  }
  return h;
}

// tangent pair of a contact normal; (0,0,1) -> (1,0,0), (0,1,0) like the plane rows
LGX_DEV void contact_tangents(f3 n, f3& t1, f3& t2) {
  f3 a = mk(n.z, 0.f, -n.x);  // e_y x n
  float l2 = a.x * a.x + a.z * a.z;
  if (l2 < 1e-8f) {
    a = mk(0.f, n.z, -n.y);   // n x e_x (n close to +-e_y)
    l2 = a.y * a.y + a.z * a.z;
  }
  t1 = a * rsqrtf(l2);
  t2 = cross(n, t1);
}

// ---- ANYmal series-elastic actuator net (anymal.py:71-81): 2-layer
// LSTM(2 -> 8 -> 8) step + Linear(8 -> 1), torch.nn.LSTM gate order i f g o, state [2, N*D, 8] in
// HBM (read and written once per substep). The serial per-joint statement of it is the host
// backend's sea_torque (lgx_env_host.cpp) and the oracle's (oracle/lgx_oracle.c).
// The actuator net lane-parallel over hidden units (the kernel's form): lane L serves unit
// u = L & 7 of joint j = 8 * pass + (L >> 3) — joints 0..7, then 8..11 on lanes 0..31 — and holds
// only that unit's h and c of both layers. A gate row's dot product over the 8 units of a layer
// takes the joint's other units by ds_swizzle inside the 8-lane group; every sum runs in the order
// of the serial sea_torque (the host backend's and the oracle's), so the torques are the same. Weight
// rows are lane-indexed (vector loads of the params, L1-resident): 1/8 of the per-lane work and
// transcendentals of one-joint-per-lane, and 4 state values per lane instead of 32.
// The SEA net's weight block: lgx_task_params from sea_in_scale through sea_lin_w (972 floats),
// read from its LDS arena copy.
#define SEA_OFF(f) ((int)((offsetof(lgx_task_params, f) - offsetof(lgx_task_params, sea_in_scale)) / sizeof(float)))
constexpr int SEA_WN = (int)((offsetof(lgx_task_params, sea_lin_w) + sizeof(float) * 8 -
                              offsetof(lgx_task_params, sea_in_scale)) / sizeof(float));
static_assert(SEA_WN == 972, "the SEA weight block is contiguous in lgx_task_params");
static_assert(SEA_WN <= ROWS_FLOATS, "the SEA weights fit the arena");
struct SeaW {
  float* base;  // LDS
  LGX_DEV const float* w(int off) const { return base + off; }
};
template <int K>
LGX_DEV float unit_of(float v) {  // unit K of this lane's 8-lane group
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x18 | (K << 5)));
}
// One LSTM cell step for unit u with the k loop outermost: the other units' values are taken by ds_swizzle
// as each k is consumed and the four gates accumulate side by side, so neither an 8-value copy of
// the units (hall / the layer-1 input) nor a gate row of weights is ever live at once. Every sum
// keeps sea_lstm_layer's order (a and b each accumulate k = 0..NIN-1 / 0..7, then (a + b_ih) + (b + b_hh)).
// XSW: the layer input is the new layer-0 h of the group's units (swizzled from xs) instead of xin.
template <int NIN, bool XSW>
LGX_DEV void sea_unit_k(const float* __restrict__ w_ih, const float* __restrict__ w_hh,
                        const float* __restrict__ b_ih, const float* __restrict__ b_hh, int u, const float* xin,
                        float xs, float hold, float& h, float& c) {
  float a[4] = {0.0f, 0.0f, 0.0f, 0.0f}, b[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int k = 0; k < NIN; ++k) {
    float xk;
    if constexpr (XSW) {
      switch (k) {
        case 0: xk = unit_of<0>(xs); break; case 1: xk = unit_of<1>(xs); break;
        case 2: xk = unit_of<2>(xs); break; case 3: xk = unit_of<3>(xs); break;
        case 4: xk = unit_of<4>(xs); break; case 5: xk = unit_of<5>(xs); break;
        case 6: xk = unit_of<6>(xs); break; default: xk = unit_of<7>(xs); break;
      }
    } else {
      xk = xin[k];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) a[q] += w_ih[(q * 8 + u) * NIN + k] * xk;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float hk;
    switch (k) {
      case 0: hk = unit_of<0>(hold); break; case 1: hk = unit_of<1>(hold); break;
      case 2: hk = unit_of<2>(hold); break; case 3: hk = unit_of<3>(hold); break;
      case 4: hk = unit_of<4>(hold); break; case 5: hk = unit_of<5>(hold); break;
      case 6: hk = unit_of<6>(hold); break; default: hk = unit_of<7>(hold); break;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) b[q] += w_hh[(q * 8 + u) * 8 + k] * hk;
  }
  float g4[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) g4[q] = (a[q] + b_ih[q * 8 + u]) + (b[q] + b_hh[q * 8 + u]);
  // the gates on the hardware exp / rcp (v_exp_f32, v_rcp_f32, ~1 ulp each: sigmoid within
  // ~3e-7 relative, tanh(x) = 2 sigmoid(2x) - 1 within ~2e-7 absolute), ~40 instructions per
  // unit fewer than ocml expf / division / tanhf: C3 kernel 389 -> 372 us
  // (profiles/r03_sea_lds_fast.txt); ANYmal golden replay, SeaLSTM and oracle parity unchanged
  auto sg = [](float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); };
  const float ig = sg(g4[0]), fg = sg(g4[1]), gg = 2.0f * sg(2.0f * g4[2]) - 1.0f, og = sg(g4[3]);
  c = fg * c + ig * gg;
  h = og * (2.0f * sg(2.0f * c) - 1.0f);
}
// all 12 joints' SEA torques into s.tau (every lane of the wave takes part), one unit per lane
// over two passes. (Two units per lane in one pass measured 425-459 us vs 433 for C3's kernel,
// with 33-38 spilled VGPRs: not kept, profiles/r03_sea_spill_fix.txt.)
// inlined (54 VGPRs spill at the 4-waves-per-SIMD budget, yet C3's kernel is 589 us against 611
// as a call and 642 one joint per lane: profiles/r03_bench_anymal_c_rough_sea_waves.txt)
LGX_DEV void sea_torques_lanes(Sh& s, float* A, const lgx_task_params* Pm_, const lgx_buffers& B, int e, int lane) {
  const size_t NT = (size_t)Pm_->num_envs * Pm_->num_dof;
  const int u = lane & 7;
  // The net's 972 floats (sea_in_scale .. sea_lin_w, contiguous in lgx_task_params) are copied
  // into the LDS arena, idle at the top of a substep (the previous substep's constraint rows
  // are dead, this one's not yet formed): the ~120 lane-indexed weight reads of a pass become
  // LDS reads instead of vector-memory loads (8 distinct addresses per wave instruction).
  {
    const float* src = &Pm_->sea_in_scale[0];
    for (int i = lane; i < SEA_WN; i += 64) A[i] = src[i];
    __syncthreads();
  }
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    // the weights a lane reads do not depend on the pass: an opaque table pointer per pass keeps
    // them from being hoisted out of this loop (all ~130 live at once) and spilled
    const lgx_task_params* Pm = opaque(Pm_);
    int wb = 0;  // opaque per pass, as Pm
    __asm__ volatile("" : "+s"(wb));
    const SeaW W{A + wb};
    const int j = pass * 8 + (lane >> 3);
    const bool on = j < NJ;  // pass 1: lanes 0..31 (joints 8..11); lanes 32..63 follow along
    const int jj = on ? j : NJ - 1;
    const size_t r = (size_t)e * Pm->num_dof + jj;
    float h0 = B.sea_hidden[r * 8 + u], c0 = B.sea_cell[r * 8 + u];
    float h1 = B.sea_hidden[(NT + r) * 8 + u], c1 = B.sea_cell[(NT + r) * 8 + u];
    const float in0 = (s.act[jj] * Pm->action_scale + Pm->default_dof_pos[jj]) - s.th[jj];
    const float x[2] = {in0 * Pm->sea_in_scale[0], s.thd[jj] * Pm->sea_in_scale[1]};
    sea_unit_k<2, false>(W.w(SEA_OFF(sea_w_ih0)), W.w(SEA_OFF(sea_w_hh0)), W.w(SEA_OFF(sea_b_ih0)),
                         W.w(SEA_OFF(sea_b_hh0)), u, x, 0.0f, h0, h0, c0);
    sea_unit_k<8, true>(W.w(SEA_OFF(sea_w_ih1)), W.w(SEA_OFF(sea_w_hh1)), W.w(SEA_OFF(sea_b_ih1)),
                        W.w(SEA_OFF(sea_b_hh1)), u, nullptr, h0, h1, h1, c1);
    if (on) {
      B.sea_hidden[r * 8 + u] = h0; B.sea_cell[r * 8 + u] = c0;
      B.sea_hidden[(NT + r) * 8 + u] = h1; B.sea_cell[(NT + r) * 8 + u] = c1;
    }
    float y = 0.0f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float hk;
      switch (k) {
        case 0: hk = unit_of<0>(h1); break; case 1: hk = unit_of<1>(h1); break;
        case 2: hk = unit_of<2>(h1); break; case 3: hk = unit_of<3>(h1); break;
        case 4: hk = unit_of<4>(h1); break; case 5: hk = unit_of<5>(h1); break;
        case 6: hk = unit_of<6>(h1); break; default: hk = unit_of<7>(h1); break;
      }
      y += W.w(SEA_OFF(sea_lin_w))[k] * hk;
    }
    if (on && u == 0) s.tau[j] = Pm->sea_out_scale * (y + Pm->sea_lin_b);
  }
}

// ---- the constraint solve of one substep for one env (oracle_physics.c steps 3-4): per row
//      (one lane each) the Schur solves, A = J M⁻¹ Jᵀ, projected Gauss-Seidel -> s.lam; z_r, g_r
//      stay in the arena (ZG) for the velocity update. Input: the rows the detection wrote (J9,
//      s.rleg, s.tgt, s.nrows / nlim / ncon). WL = the env's lanes: 64, or 32 with both envs of
//      the wave at <= 32 rows (the groups' loops then run side by side to the larger count, each
//      group predicated on its own; the broadcasts read each group's own row lane).
template <int WL>
LGX_DEV void solve_rows(Sh& s, float* A, const lgx_task_params* Pm, int lane, int nrows, int nlim, int ncon) {
  float* const ZG = A;                // [nrows][RW]: z_r (6) | g_r (3)
  float* const J9 = A + MAXR * RW;    // [nrows][RW]: J_B (6) | J of leg rleg (3)
  float* const Am = J9;               // A [nrows][nrows] (A path, after J9 is consumed)
  // ---- per row (one lane each): y = J_B − X_l J_l, z = S⁻¹ y, g = D_l⁻¹ J_l,
  //      A_rr = y·z + J_l·g, w_r = J_r u*
  const bool row_lane = lane < nrows;
  float yr[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, jlr[3] = {0.f, 0.f, 0.f}, w0 = 0.f;
  int lr = -1;
  if (row_lane) {
    const float* jr = J9 + lane * RW;
    lr = s.rleg[lane];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      yr[q] = jr[q];
      w0 += yr[q] * s.us[q];
    }
    float g[3] = {0.f, 0.f, 0.f};
    if (lr >= 0) {
#pragma unroll
      for (int c = 0; c < 3; ++c) jlr[c] = jr[6 + c];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float* Xc = s.X[3 * lr + c];
#pragma unroll
        for (int q = 0; q < 6; ++q) yr[q] -= Xc[q] * jlr[c];
        w0 += jlr[c] * s.us[6 + 3 * lr + c];
      }
      const float* Di = s.Dinv[lr];
      g[0] = Di[0] * jlr[0] + Di[3] * jlr[1] + Di[4] * jlr[2];
      g[1] = Di[3] * jlr[0] + Di[1] * jlr[1] + Di[5] * jlr[2];
      g[2] = Di[4] * jlr[0] + Di[5] * jlr[1] + Di[2] * jlr[2];
    }
    float* zg = ZG + lane * RW;
    float arr = jlr[0] * g[0] + jlr[1] * g[1] + jlr[2] * g[2];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const float* Si = s.Sinv[q];
      const float zq = Si[0] * yr[0] + Si[1] * yr[1] + Si[2] * yr[2] + Si[3] * yr[3] + Si[4] * yr[4] + Si[5] * yr[5];
      zg[q] = zq;
      arr += yr[q] * zq;
    }
    zg[6] = g[0]; zg[7] = g[1]; zg[8] = g[2];
    s.Arr[lane] = arr;
    s.lam[lane] = 0.f;
  }
  __syncthreads();
  PH(6);
  // ---- A = J M⁻¹ Jᵀ: entry (q, r) = y_r·z_q + [leg_r = leg_q] J_l,r·g_q (J_l,r = 0 for rows
  //      without a leg part). Up to ASQ rows lane r stores column r of a square [q][r] image;
  //      up to AMAX the lower triangle q >= r packed at q (q + 1) / 2 + r; beyond (a fallen
  //      robot: up to 12 + 3 * MAXC rows) the PGS forms A[r][lane] from z_r, g_r (LDS) and the
  //      lane's own y, J_l (registers) each time it needs it — the same numbers, nothing stored.
  //      Two envs per wave (both <= 32 rows): each group its own form, read through a
  //      branch-free per-lane index (arow_mix below).
  const int NRm = gmax<WL>(nrows);
  const bool tri = nrows > ASQ, stored = nrows <= AMAX;
  if (stored && row_lane) {
#pragma unroll 4
    for (int q = 0; q < NRm; ++q) {
      if (q < nrows) {
        const float* zg = ZG + q * RW;
        const float v = yr[0] * zg[0] + yr[1] * zg[1] + yr[2] * zg[2] + yr[3] * zg[3] + yr[4] * zg[4] + yr[5] * zg[5];
        const float vl = jlr[0] * zg[6] + jlr[1] * zg[7] + jlr[2] * zg[8];
        const float a = v + (s.rleg[q] == lr ? vl : 0.f);
        if (!tri) Am[q * nrows + lane] = a;
        else if (q >= lane) Am[q * (q + 1) / 2 + lane] = a;
      }
    }
  }
  __syncthreads();
  PH(7);
  // ---- projected Gauss-Seidel on A (oracle_physics.c step 4). Rows are [nlim joint
  //      limits | ncon × (normal, tangent, tangent)]. Lane r keeps its row's velocity
  //      w_r = J_r u, λ_r and constants; every lane forms its own row's candidate update
  //      and only the row being swept keeps it (a select), so a row costs one readlane of
  //      its Δλ, broadcast into w += A[·][r] Δλ. The tangent pair trades its two candidates
  //      between neighbouring lanes by DPP for the friction-disk norm. A contact's three
  //      A columns are loaded one contact ahead.
  {
    float w = w0, lam = 0.f;
    const float mu = s.mu;
    auto wave_shl1 = [](float v) {  // lane x receives lane x + 1 (wave-wide shift)
      return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x130, 0xf, 0xf, false));
    };
    auto wave_shr1 = [](float v) {  // lane x receives lane x - 1
      return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x138, 0xf, 0xf, false));
    };
    const float tg = row_lane ? s.tgt[lane] : 0.f;
    const float ia = row_lane ? 1.0f / s.Arr[lane] : 0.f;
    const int rlast = max(nrows - 3, 0);      // first row of the last contact
    const int lc = max(min(lane, nrows - 1), 0);  // lanes past the rows read a valid (unused) entry
    // A[r][lane]: square, from the packed triangle (row r up to the diagonal, then column r),
    // or formed on the fly (lanes past the rows have y = J_l = 0 and read 0)
    const int tl = lc * (lc + 1) / 2;
    auto arow_sq = [&](int r) { return Am[r * nrows + lc]; };
    auto arow_tri = [&](int r) { return Am[lc <= r ? r * (r + 1) / 2 + lc : tl + r]; };
    // either form per lane, without a branch: the triangle index of (max, min) (24-bit products)
    auto arow_mix = [&](int r) {
      const int hi = max(r, lc), lo = min(r, lc);
      const int it = (mul24(hi, hi + 1) >> 1) + lo;
      const int is = mul24(r, nrows) + lc;
      return Am[tri ? it : is];
    };
    // keep a or take b where m, as a bitwise select (no branch)
    auto sel = [](bool m, float a, float b) {
      const int k = -(int)m;
      return __int_as_float((__float_as_int(b) & k) | (__float_as_int(a) & ~k));
    };
    auto arow_otf = [&](int r) {
      const float* zg = ZG + r * RW;
      const float v = yr[0] * zg[0] + yr[1] * zg[1] + yr[2] * zg[2] + yr[3] * zg[3] + yr[4] * zg[4] + yr[5] * zg[5];
      const float vl = jlr[0] * zg[6] + jlr[1] * zg[7] + jlr[2] * zg[8];
      return v + (s.rleg[r] == lr ? vl : 0.f);
    };
    // the groups' row counts as wave-uniform scalars (the loops run to the larger; a group past
    // its own count changes nothing)
    const int NLm = gmax<WL>(nlim), NCm = gmax<WL>(ncon);
    const int nl0 = gval<WL>(nlim, 0), nl1 = WL == 64 ? nl0 : gval<WL>(nlim, 1);
    // the sweeps, instantiated for each form of A (the square one carries no index selects)
    auto sweeps = [&](auto arow) {
      for (int it = 0; it < Pm->solver_iterations; ++it) {
        for (int r = 0; r < NLm; ++r) {
          const bool on = WL == 64 || r < nlim;
          const float a0 = on ? arow(r) : 0.f;
          const float cand = fmaxf(0.f, lam + (tg - w) * ia);
          const float d = gbcast<WL>(cand - lam, min(r, 31), min(r, 31));
          lam = sel(lane == r && on, lam, cand);
          w += on ? a0 * d : 0.f;
        }
        if (NCm == 0) continue;
        float n0 = arow(min(nlim, rlast)), n1 = arow(min(nlim + 1, rlast + 1)), n2 = arow(min(nlim + 2, rlast + 2));
        for (int c = 0; c < NCm; ++c) {
          const bool on = WL == 64 || c < ncon;
          const int r = nlim + 3 * c;                               // this group's row
          const int ra = nl0 + 3 * c, rb = nl1 + 3 * c;             // each group's, uniform
          const int ra_ = WL == 64 ? ra : min(ra, WL - 3), rb_ = WL == 64 ? rb : min(rb, WL - 3);
          const float a0 = on ? n0 : 0.f, a1 = on ? n1 : 0.f, a2 = on ? n2 : 0.f;
          const int rn = min(r + 3, rlast);
          n0 = arow(rn);
          n1 = arow(rn + 1);
          n2 = arow(rn + 2);
          // normal row
          const float cand = fmaxf(0.f, lam + (tg - w) * ia);
          const float d = gbcast<WL>(cand - lam, ra_, rb_);
          lam = sel(lane == r && on, lam, cand);
          w += a0 * d;
          // tangent pair, projected onto the friction disk |λ_t| <= μ λ_n
          const float lim = mu * gbcast<WL>(lam, ra_, rb_);
          const float l = lam - w * ia;
          // both shifts with every lane active (a DPP source lane outside EXEC reads 0), then
          // the select: lane r + 1 takes r + 2's candidate, lane r + 2 takes r + 1's (the pair
          // never straddles the two groups: r + 2 < WL)
          float from_next = wave_shl1(l), from_prev = wave_shr1(l);
          __asm__ volatile("" : "+v"(from_next), "+v"(from_prev));
          const float other = lane == r + 1 ? from_next : from_prev;
          const float nn = l * l + other * other;
          const float sc = nn > lim * lim ? lim * __builtin_amdgcn_rsqf(nn) : 1.0f;
          const float lt = l * sc;
          const float dl = lt - lam;
          const float d1 = gbcast<WL>(dl, ra_ + 1, rb_ + 1), d2 = gbcast<WL>(dl, ra_ + 2, rb_ + 2);
          lam = sel((unsigned)(lane - r - 1) < 2u && on, lam, lt);
          w += a1 * d1 + a2 * d2;
        }
      }
    };
    if constexpr (WL == 64) {
      if (!stored) sweeps(arow_otf);
      else if (tri) sweeps(arow_tri);
      else sweeps(arow_sq);
    } else {
      sweeps(arow_mix);
    }
    if (row_lane) s.lam[lane] = lam;
  }
  __syncthreads();
  PH(8);
}

// one physics substep (legged_robot.py:80-85 loop body) of the group's env. WL = the env's lanes
// (see grp_of_lane); with two envs per wave, S0 / A0 / astride locate both envs' Sh and arenas
// for the wide constraint solve (an env with more than 32 rows: each env in turn on all 64 lanes).
template <bool TERRAIN, bool ACTNET, int WL>
LGX_DEV void substep(Sh& s, float* A, Sh* S0, float* A0, int astride, const lgx_model* M_,
                     const lgx_task_params* Pm_, const lgx_buffers& B, int lane_, int e, bool last) {
  // The model and task tables are re-read each substep (L1 / scalar-cache hits) rather than
  // hoisted out of the decimation loop, where ~40 lane-indexed constants would otherwise stay
  // live in VGPRs across the whole step. Likewise the lane index, so that per-lane index and
  // LDS-address arithmetic is recomputed each substep instead of being hoisted and spilled.
  const lgx_model* M = opaque(M_);
  const lgx_task_params* Pm = opaque(Pm_);
  const int lane = opaque_lane(lane_);
  const float dt = Pm->sim_dt;
  // ---- PD torques: LeggedRobot._compute_torques legged_robot.py:440-478
  {
#pragma clang fp contract(off)
    if (ACTNET) {
      sea_torques_lanes(s, A, Pm, B, e, lane);
    } else if (lane < NJ) {
      const int j = lane;
      float as = s.act[j] * Pm->action_scale;
      float t;
      if (Pm->control_type == LGX_CONTROL_P) {
        float err = (as + Pm->default_dof_pos[j]) - s.th[j];
        if (Pm->randomize_kp_kd)
          t = (s.kpm[j] * Pm->p_gains[j]) * err - (s.kdm[j] * Pm->d_gains[j]) * s.thd[j];
        else
          t = Pm->p_gains[j] * err - Pm->d_gains[j] * s.thd[j];
      } else if (Pm->control_type == LGX_CONTROL_V) {
        t = Pm->p_gains[j] * (as - s.thd[j]) - Pm->d_gains[j] * ((s.thd[j] - s.ldv[j]) / Pm->sim_dt);
      } else {
        t = as;
      }
      s.tau[j] = fminf(fmaxf(t, -Pm->torque_limits[j]), Pm->torque_limits[j]);
    }
  }
  PH(1);
  kinematics<true>(s, A, M, Pm, lane);
  PH(2);
  DynOut dy;
  dynamics(s, A, lane, dy);
  const int jl_ = lane < NJ ? lane : NJ - 1, leg_ = jl_ / 3, pos_ = jl_ % 3;  // joint lanes' leg / chain position
  // ---- free velocity u* = u + dt M⁻¹ f, f = [−h_B ; τ − h_J] (factored form, see dynamics)
  const float fj = lane < NJ ? s.tau[lane] - dy.hj : 0.f;
  if (lane < NJ) s.up[lane] = fj;  // scratch: f_J, read by the leg's lanes below
  float vb[6];
#pragma unroll
  for (int r = 0; r < 6; ++r) vb[r] = -dy.hb[r] - grow_sum16<WL>(dy.xj[r] * fj);
  __syncthreads();  // S⁻¹ (dynamics) and f_J visible
  PH(3);
  {
    float zb[6];
#pragma unroll
    for (int r = 0; r < 6; ++r) {
      const float* Si = s.Sinv[r];
      zb[r] = Si[0] * vb[0] + Si[1] * vb[1] + Si[2] * vb[2] + Si[3] * vb[3] + Si[4] * vb[4] + Si[5] * vb[5];
    }
    if (lane < 6) {
      const float* Si = s.Sinv[lane];
      const float zl = Si[0] * vb[0] + Si[1] * vb[1] + Si[2] * vb[2] + Si[3] * vb[3] + Si[4] * vb[4] + Si[5] * vb[5];
      const float u0 = lane < 3 ? s.vo[lane] : s.wb[lane - 3];
      s.us[lane] = u0 + dt * zl;
    }
    if (lane < NJ) {
      const float* fl = s.up + 3 * leg_;
      float bot = dy.dinv[0] * fl[0] + dy.dinv[1] * fl[1] + dy.dinv[2] * fl[2];
#pragma unroll
      for (int r = 0; r < 6; ++r) bot -= dy.xj[r] * zb[r];
      s.us[6 + lane] = s.thd[lane] + dt * bot;
    }
  }
  PH(4);
  // ---- constraint detection: joint limits (lanes 0..11), contacts (one candidate per lane, in
  //      rounds of WL candidates: the rows keep the candidates' order)
  bool lim_lo = false, lim_hi = false;
  if (lane < NJ && M->joint_has_limits[lane + 1]) {
    lim_lo = s.th[lane] < M->joint_lower[lane + 1] + Pm->limit_margin;
    lim_hi = !lim_lo && s.th[lane] > M->joint_upper[lane + 1] - Pm->limit_margin;
  }
  const uint64_t lmask = gballot<WL>(lim_lo || lim_hi);
  const int nlim = __popcll(lmask);
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  auto target = [&](float d) {
    float tv;
    if (d > Pm->slop) tv = fminf(Pm->baumgarte * (d - Pm->slop) / dt, Pm->max_depenetration_vel);
    else if (d >= 0.f) tv = 0.f;
    else tv = d / dt;
    return tv;
  };
  float* const J9 = A + MAXR * RW;    // [nrows][RW]: J_B (6) | J of leg rleg (3)
  constexpr bool plane = !TERRAIN;  // the launch picks the variant from mesh_type
  // every candidate's contact query first (the trimesh query uses the arena the rows go to),
  // then the rows: limits, then contacts in candidate order
  constexpr int CR = (LGX_MAX_CANDIDATES + WL - 1) / WL;
  bool act[CR];
  f3 xc[CR], nrm[CR];
  float depth[CR];
  int ck[CR];
#pragma unroll
  for (int cr = 0; cr < CR; ++cr) {
    act[cr] = false;
    xc[cr] = mk(0, 0, 0);
    nrm[cr] = mk(0.f, 0.f, 1.f);
    depth[cr] = 0.f;
    ck[cr] = 0;
    if (cr * WL >= M->num_candidates) continue;  // uniform
    const int ci = cr * WL + lane;
    const bool cand = ci < M->num_candidates;
    if constexpr (plane) {
      if (cand) {
        ck[cr] = M->cand_link[ci];
        xc[cr] = ld3(s.P[ck[cr]]) + mv(s.R[ck[cr]], ld3(M->cand_pos[ci]));
        const float r = M->cand_radius[ci];
        depth[cr] = r - xc[cr].z;
        xc[cr].z -= r;
        act[cr] = depth[cr] > -Pm->contact_margin;
      }
    } else {
      float r = 0.f;
      if (cand) {
        ck[cr] = M->cand_link[ci];
        xc[cr] = ld3(s.P[ck[cr]]) + mv(s.R[ck[cr]], ld3(M->cand_pos[ci]));
        r = M->cand_radius[ci];
      }
      const TerrainHit th = terrain_contact_wave<WL>(Pm, B, A, xc[cr], r, cand, lane);
      if (cand) {
        depth[cr] = th.depth;
        nrm[cr] = th.n;
        xc[cr] = xc[cr] - nrm[cr] * r;  // deepest sphere point
        act[cr] = depth[cr] > -Pm->contact_margin;
      }
    }
  }
  if (lim_lo || lim_hi) {
    const int r = __popcll(lmask & below);
    float* jr = J9 + r * RW;
#pragma unroll
    for (int q = 0; q < RW; ++q) jr[q] = 0.f;
    jr[6 + pos_] = lim_lo ? 1.f : -1.f;
    const float d = lim_lo ? (M->joint_lower[lane + 1] - s.th[lane]) : (s.th[lane] - M->joint_upper[lane + 1]);
    s.tgt[r] = target(d);
    s.rleg[r] = leg_;
  }
  int nfound = 0;  // contacts of the earlier rounds (group-uniform)
#pragma unroll
  for (int cr = 0; cr < CR; ++cr) {
    if (cr * WL >= M->num_candidates) continue;  // uniform
    const int ci = cr * WL + lane;
    const uint64_t cmask = gballot<WL>(act[cr]);
    const int crank = nfound + __popcll(cmask & below);
    nfound += __popcll(cmask);
    if (act[cr] && crank < MAXC) {
      const int r0 = nlim + 3 * crank;
      const f3 p0 = ld3(s.P[0]);
      f3 dn = mk(0, 0, 1), dt1 = mk(1, 0, 0), dt2 = mk(0, 1, 0);
      if constexpr (!plane) {
        dn = nrm[cr];
        contact_tangents(nrm[cr], dt1, dt2);
      }
      st3(s.cn[crank], dn);
      const int leg = ck[cr] > 0 ? (ck[cr] - 1) / 3 : -1;
      const int pos = ck[cr] > 0 ? (ck[cr] - 1) % 3 : -1;
      const int kl = ck[cr] > 0 ? 1 + 3 * leg : 1;
      const f3 ax0 = ld3(s.Ax[kl]), ax1 = ld3(s.Ax[kl + 1]), ax2 = ld3(s.Ax[kl + 2]);
      const f3 r0p = xc[cr] - ld3(s.P[kl]), r1p = xc[cr] - ld3(s.P[kl + 1]), r2p = xc[cr] - ld3(s.P[kl + 2]);
      const f3 rb = xc[cr] - p0;
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int r = r0 + t;
        const f3 d = t == 0 ? dn : (t == 1 ? dt1 : dt2);
        const f3 ang = cross(rb, d);
        float* jr = J9 + r * RW;
        jr[0] = d.x; jr[1] = d.y; jr[2] = d.z;
        jr[3] = ang.x; jr[4] = ang.y; jr[5] = ang.z;
        jr[6] = pos >= 0 ? dot(ax0, cross(r0p, d)) : 0.f;
        jr[7] = pos >= 1 ? dot(ax1, cross(r1p, d)) : 0.f;
        jr[8] = pos >= 2 ? dot(ax2, cross(r2p, d)) : 0.f;
        s.rleg[r] = leg;
        s.tgt[r] = t == 0 ? target(depth[cr]) : 0.f;
      }
      s.cbody[crank] = M->cand_body[ci];
    }
  }
  const int ncon = min(nfound, MAXC);
  const int nrows = nlim + 3 * ncon;
  const int nrw = gmax<WL>(nrows);  // the wave's largest system
#if LGX_ROW_PRIO > 0
  // Issue priority by constraint-system size (s_setprio 0..3 above 0 / t / 2t / 3t rows): a
  // launch lasts as long as its slowest wave, and the waves with the largest systems are the
  // slow ones; the SIMD's other waves have the slack (profiles/r03_wave_priority.txt).
  {
    const int rp = nrw > LGX_ROW_PRIO * 3 ? 3 : nrw > LGX_ROW_PRIO * 2 ? 2 : nrw > LGX_ROW_PRIO ? 1 : 0;
    set_prio(LGX_SLOT_PRIO ? max(rp, min(wave_slot(), 3)) : rp);
  }
#endif
  if (lane == 0) { s.nrows = nrows; s.nlim = nlim; s.ncon = ncon; }
#ifdef LGX_PHASE_CLOCK
  if (lane == 0) {
    s.phacc[16] = max(s.phacc[16], (uint32_t)nrows);
    s.phacc[17] += nrows > AMAX ? 1u : 0u;
  }
#endif
  __syncthreads();
  PH(5);
  if constexpr (WL == 64) {
    solve_rows<64>(s, A, Pm, lane, nrows, nlim, ncon);
  } else if (nrw <= WL) {
    solve_rows<WL>(s, A, Pm, lane, nrows, nlim, ncon);
  } else {
    // an env of this wave has more rows than its group has lanes (a fallen robot): each env's
    // solve in turn on the whole wave (its rows from LDS; the same numbers)
    const int wl = (int)__lane_id();
#pragma unroll 1
    for (int g = 0; g < 64 / WL; ++g) {
      Sh& sg = S0[g];
      const int nr = gval<WL>(nrows, g), nli = gval<WL>(nlim, g), nco = gval<WL>(ncon, g);
      solve_rows<64>(sg, A0 + (size_t)g * astride, Pm, wl, nr, nli, nco);
    }
  }
  // ---- u+ = u* + M⁻¹ Jᵀ λ = u* + [Z ; G_J − Xᵀ Z]:  Z = Σ_r λ_r z_r,
  //      G_j = Σ_{r on leg(j)} λ_r g_r[pos(j)]
  {
    const float* const ZG = A;
    float Z[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, G = 0.f;
#pragma unroll 4
    for (int r = 0; r < nrw; ++r) {
      if (WL == 64 || r < nrows) {
        const float lr_ = s.lam[r];
        const float* zg = ZG + r * RW;
#pragma unroll
        for (int q = 0; q < 6; ++q) Z[q] += lr_ * zg[q];
        const float gq = pos_ == 0 ? zg[6] : (pos_ == 1 ? zg[7] : zg[8]);
        G += s.rleg[r] == leg_ ? lr_ * gq : 0.f;
      }
    }
    if (lane < 6) {
      float zl = 0.f;
#pragma unroll
      for (int q = 0; q < 6; ++q) zl = lane == q ? Z[q] : zl;
      s.up[lane] = s.us[lane] + zl;
    }
    if (lane < NJ) {
      const float* Xj = s.X[lane];
      float v = s.us[6 + lane] + G;
#pragma unroll
      for (int q = 0; q < 6; ++q) v -= Xj[q] * Z[q];
      s.up[6 + lane] = v;
    }
  }
  __syncthreads();
  PH(9);
  // ---- contact forces of the last substep, per reported body (world frame)
  if (last && lane < LGX_MAX_BODIES) {
    float f[3] = {0.f, 0.f, 0.f};
    const int ncm = gmax<WL>(ncon);
    for (int c = 0; c < ncm; ++c) {
      if (c >= ncon || s.cbody[c] != lane) continue;
      const int r = nlim + 3 * c;
      if constexpr (!TERRAIN) {
        f[2] += s.lam[r]; f[0] += s.lam[r + 1]; f[1] += s.lam[r + 2];
      } else {
        f3 t1, t2;
        const f3 n = ld3(s.cn[c]);
        contact_tangents(n, t1, t2);
        const f3 fc = n * s.lam[r] + t1 * s.lam[r + 1] + t2 * s.lam[r + 2];
        f[0] += fc.x; f[1] += fc.y; f[2] += fc.z;
      }
    }
    s.cf[lane][0] = f[0] / dt; s.cf[lane][1] = f[1] / dt; s.cf[lane][2] = f[2] / dt;
  }
  // ---- semi-implicit Euler
  if (lane == 0) {
    f3 v = mk(s.up[0], s.up[1], s.up[2]), w = mk(s.up[3], s.up[4], s.up[5]);
#pragma unroll
    for (int i = 0; i < 3; ++i) s.pb[i] += dt * s.up[i];
    float wn = sqrtf(dot(w, w));
    float ang = wn * dt;
    float dq[4];
    if (ang > 1e-12f) {
      float sc = sinf(0.5f * ang) / wn;
      dq[0] = w.x * sc; dq[1] = w.y * sc; dq[2] = w.z * sc; dq[3] = cosf(0.5f * ang);
    } else {
      dq[0] = 0.5f * dt * w.x; dq[1] = 0.5f * dt * w.y; dq[2] = 0.5f * dt * w.z; dq[3] = 1.f;
    }
    const float* q = s.qb;
    float qn[4];
    qn[3] = dq[3] * q[3] - (dq[0] * q[0] + dq[1] * q[1] + dq[2] * q[2]);
    qn[0] = dq[3] * q[0] + q[3] * dq[0] + (dq[1] * q[2] - dq[2] * q[1]);
    qn[1] = dq[3] * q[1] + q[3] * dq[1] + (dq[2] * q[0] - dq[0] * q[2]);
    qn[2] = dq[3] * q[2] + q[3] * dq[2] + (dq[0] * q[1] - dq[1] * q[0]);
    float nq = rsqrtf(qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3]);
#pragma unroll
    for (int i = 0; i < 4; ++i) s.qb[i] = qn[i] * nq;
    st3(s.vo, v);
    st3(s.wb, w);
  }
  if (lane < NJ) {
    s.thd[lane] = s.up[6 + lane];
    s.th[lane] += dt * s.thd[lane];
  }
  __syncthreads();
  PH(10);
}

#pragma clang fp contract(off)

// ============================================================== post-physics helpers
// (fp32, no contraction: the reference evaluates these as separate eager torch ops)

LGX_DEV void quat_rotate_inverse(const float* q, const float* v, float* out) {
  float w = q[3];
  float sc = 2.0f * (w * w) - 1.0f;
  float cx = q[1] * v[2] - q[2] * v[1];
  float cy = q[2] * v[0] - q[0] * v[2];
  float cz = q[0] * v[1] - q[1] * v[0];
  float d = q[0] * v[0] + q[1] * v[1] + q[2] * v[2];
  out[0] = v[0] * sc - cx * w * 2.0f + q[0] * d * 2.0f;
  out[1] = v[1] * sc - cy * w * 2.0f + q[1] * d * 2.0f;
  out[2] = v[2] * sc - cz * w * 2.0f + q[2] * d * 2.0f;
}
LGX_DEV void quat_apply(const float* q, const float* b, float* out) {
  float t0 = (q[1] * b[2] - q[2] * b[1]) * 2.0f;
  float t1 = (q[2] * b[0] - q[0] * b[2]) * 2.0f;
  float t2 = (q[0] * b[1] - q[1] * b[0]) * 2.0f;
  out[0] = b[0] + q[3] * t0 + (q[1] * t2 - q[2] * t1);
  out[1] = b[1] + q[3] * t1 + (q[2] * t0 - q[0] * t2);
  out[2] = b[2] + q[3] * t2 + (q[0] * t1 - q[1] * t0);
}
LGX_DEV float trem(float a, float b) {
  float m = fmodf(a, b);
  if (m != 0.0f && ((m < 0.0f) != (b < 0.0f))) m += b;
  return m;
}
LGX_DEV float wrap_to_pi(float a) {
  const float two_pi = 6.283185307179586f, pi = 3.141592653589793f;
  float m = trem(a, two_pi);
  m -= two_pi * (float)(m > pi);
  return m;
}
LGX_DEV float clipf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
LGX_DEV float sq(float x) { return x * x; }
LGX_DEV float nrm3(float a, float b, float c) { return sqrtf(a * a + b * b + c * c); }
LGX_DEV float nrm2(float a, float b) { return sqrtf(a * a + b * b); }
LGX_DEV float rand_range(float lo, float hi, float u) {
  float span = (float)((double)hi - (double)lo);
  return span * u + lo;
}
// torch_rand_float(lo, hi) with the reference's Python-float (double) bounds: (hi - lo) and lo
// enter the fp32 tensor ops as fp32 scalars
LGX_DEV float rand_range_d(double lo, double hi, float u) { return (float)(hi - lo) * u + (float)lo; }

// Go2Robot._resample_commands go2.py:413-464 / LeggedRobot legged_robot.py:406-437
// R: the mutable command ranges (lgx_buffers.command_ranges, double [8]) or NULL (params' ranges)
LGX_DEV void resample_commands(const lgx_task_params* Pm, const double* R, float* cmd, const float* U, int slot0,
                               const float* quat) {
  if (Pm->has_user_command) {
    for (int i = 0; i < 4; ++i) cmd[i] = Pm->user_command[i];
    return;
  }
  if (R) {
    cmd[0] = rand_range_d(R[0], R[1], U[slot0 + 0]);
    cmd[1] = rand_range_d(R[2], R[3], U[slot0 + 1]);
    if (Pm->heading_command)
      cmd[3] = rand_range_d(R[6], R[7], U[slot0 + 2]);
    else
      cmd[2] = rand_range_d(R[4], R[5], U[slot0 + 2]);
  } else {
    cmd[0] = rand_range(Pm->cmd_lin_vel_x[0], Pm->cmd_lin_vel_x[1], U[slot0 + 0]);
    cmd[1] = rand_range(Pm->cmd_lin_vel_y[0], Pm->cmd_lin_vel_y[1], U[slot0 + 1]);
    if (Pm->heading_command)
      cmd[3] = rand_range(Pm->cmd_heading[0], Pm->cmd_heading[1], U[slot0 + 2]);
    else
      cmd[2] = rand_range(Pm->cmd_ang_vel_yaw[0], Pm->cmd_ang_vel_yaw[1], U[slot0 + 2]);
  }
  float keep = (float)(nrm2(cmd[0], cmd[1]) > 0.2f);
  cmd[0] = cmd[0] * keep;
  cmd[1] = cmd[1] * keep;
  if (Pm->zero_command && U[slot0 + 3] < Pm->zero_command_prob) {
    if (Pm->task_kind == LGX_TASK_GO2) {
      cmd[0] = cmd[0] * 0.0f; cmd[1] = cmd[1] * 0.0f; cmd[2] = cmd[2] * 0.0f;
      if (Pm->heading_command) {
        const float fwd[3] = {1.f, 0.f, 0.f};
        float f[3];
        quat_apply(quat, fwd, f);
        cmd[3] = atan2f(f[1], f[0]);
      }
    } else {
      for (int i = 0; i < 4; ++i) cmd[i] = cmd[i] * 0.0f;
    }
  }
}

// reset_idx for one env (go2.py:207-263 / legged_robot.py:157-213). The env's root/dof/
// command state is in LDS (s.root, s.th, s.thd, s.cmd, s.ep): lane 0 does the scalar part,
// lanes write the per-env buffer rows. Called under a uniform branch.
template <int WL>
LGX_DEV void reset_env(const lgx_task_params* Pm, const lgx_buffers& B, Sh& s, float* A, int e, int lane,
                       bool after_init, bool zero_carried, bool sums_in_lds) {
  const int D = Pm->num_dof;
  const float* U = stg_U(A);
  if (lane == 0) {
    float* root = s.root;
    float* cmd = s.cmd;
    // terrain curriculum legged_robot.py:543-574
    if (Pm->curriculum && after_init && B.terrain_levels) {
      float dx = root[0] - B.env_origins[e * 3 + 0], dy = root[1] - B.env_origins[e * 3 + 1];
      float dist = nrm2(dx, dy);
      int up = dist > Pm->terrain_length * Pm->promote_threshold;
      float expct = nrm2(cmd[0], cmd[1]) * Pm->max_episode_length_s;
      int down = dist < expct * Pm->demote_threshold;
      int64_t lvl = B.terrain_levels[e] + up - down;
      if (lvl >= Pm->max_terrain_level) {
        lvl = (int64_t)(U[S_TERR] * (float)Pm->max_terrain_level);
        if (lvl >= Pm->max_terrain_level) lvl = Pm->max_terrain_level - 1;
      } else if (lvl < 0) {
        lvl = 0;
      }
      B.terrain_levels[e] = lvl;
      const float* o = B.terrain_origins + ((size_t)lvl * Pm->num_terrain_cols + B.terrain_types[e]) * 3;
      for (int i = 0; i < 3; ++i) B.env_origins[e * 3 + i] = o[i];
    }
    // _reset_root_states legged_robot.py:509-532
    for (int i = 0; i < 13; ++i) root[i] = Pm->base_init_state[i];
    for (int i = 0; i < 3; ++i) root[i] = root[i] + B.env_origins[e * 3 + i];
    if (Pm->custom_origins) {
      root[0] = root[0] + rand_range(-1.0f, 1.0f, U[S_ROOT_XY + 0]);
      root[1] = root[1] + rand_range(-1.0f, 1.0f, U[S_ROOT_XY + 1]);
    }
    for (int i = 0; i < 6; ++i) root[7 + i] = rand_range(-0.5f, 0.5f, U[S_ROOT_VEL + i]);
    resample_commands(Pm, B.command_ranges, cmd, U, S_RCMD, root + 3);
    s.ep = 0;
  }
  // _reset_dofs legged_robot.py:481-506: q = q0 + U(0, 0.9), qd = 0
  if (lane < D) {
    s.th[lane] = Pm->default_dof_pos[lane] + rand_range(0.0f, 0.9f, U[S_DOF + lane]);
    s.thd[lane] = 0.0f;
  }
  // buffer zeroing. Inside a step the last_* buffers and the history are rewritten at the
  // end of post_physics_step anyway (go2.py:380-384, 570-574); only an external reset
  // has to zero them.
  if (zero_carried) {
    const int A = Pm->num_actions, H = Pm->history_len * Pm->num_proprio;
    if (lane < A) B.last_actions[(size_t)e * A + lane] = 0.f;
    if (lane < D) { B.last_dof_vel[(size_t)e * D + lane] = 0.f; B.last_torques[(size_t)e * D + lane] = 0.f; }
    if (lane < 6) B.last_root_vel[e * 6 + lane] = 0.f;
    if (lane < 3) B.last_base_lin_vel[e * 3 + lane] = 0.f;
    for (int i = lane; i < H; i += WL) B.obs_history[(size_t)e * H + i] = 0.f;
  }
  if (Pm->actuator_net && lane < 2 * D) {  // Anymal.reset_idx anymal.py:56-60: zero h, c
    const size_t NT = (size_t)Pm->num_envs * D;
    const int l = lane / D, j = lane % D;
    float4* hp = reinterpret_cast<float4*>(B.sea_hidden + (l * NT + (size_t)e * D + j) * 8);
    float4* cp = reinterpret_cast<float4*>(B.sea_cell + (l * NT + (size_t)e * D + j) * 8);
    hp[0] = hp[1] = cp[0] = cp[1] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (Pm->task_kind == LGX_TASK_GO2 && lane < Pm->num_feet) {
    if (B.feet_air_time) B.feet_air_time[e * Pm->num_feet + lane] = 0.f;
    B.last_contacts[e * Pm->num_feet + lane] = 0;
    B.last_contact_heights[e * Pm->num_feet + lane] = 0.f;
  }
  const int K = Pm->num_reward_terms + (Pm->has_termination_reward ? 1 : 0);
  for (int k = lane; k < K; k += WL) {
    float* es = B.episode_sums + (size_t)e * K + k;
    const float sum = sums_in_lds ? s.es[k] : *es;  // in a step: this step's updated row, staged in LDS
    if (B.episode_stats) atomicAdd(B.episode_stats + k, sum);
    // the command curriculum's input (go2.py:87): this env's tracking_lin_vel sum at its reset
    if (sums_in_lds && B.curriculum_vals && k == Pm->curriculum_term) B.curriculum_vals[e] = sum;
    *es = 0.f;
  }
  if (lane == 0 && B.episode_stats) atomicAdd(B.episode_stats + K, 1.0f);
  __syncthreads();
}

template <int WL>
LGX_DEV void fill_uniforms(float* A, uint64_t seed, uint32_t gid, uint64_t step, uint32_t stream, int lane, int nblk) {
  for (int b = lane; b < nblk; b += WL) {
    uint32_t o[4];
    philox4x32_10(gid, (uint32_t)step, (uint32_t)b | (stream << 16), (uint32_t)(step >> 32), (uint32_t)seed,
                  (uint32_t)(seed >> 32), o);
    float* U = stg_U(A);
    U[4 * b + 0] = u01(o[0]); U[4 * b + 1] = u01(o[1]);
    U[4 * b + 2] = u01(o[2]); U[4 * b + 3] = u01(o[3]);
  }
  __syncthreads();
}

// The sums over joints (and height points) that reward terms use, formed lane-parallel
// (lane j = joint j, reduced over lanes 0..15 by a DPP scan; lane 15 writes them), so the
// per-term lanes below do no joint loops. Summation order differs from torch's sum over a
// dim by ~1 ulp of the sum (golden tests: 1e-5).
enum JSum { J_ACTION_RATE, J_DELTA_TORQUES, J_DOF_ACC, J_DOF_ERROR, J_DOF_POS_LIMITS, J_DOF_VEL, J_DOF_VEL_LIMITS,
            J_STAND_ABS, J_TORQUE_LIMITS, J_TORQUES, J_HIP_POS, J_THIGH_POS, J_CALF_POS, J_HEIGHT, J_N };
LGX_DEV void joint_sums(const lgx_task_params* Pm, const lgx_buffers& B, Sh& s, float* A, int e, int lane) {
  const int D = Pm->num_dof;
  const int j = lane < D ? lane : 0;
  const float on = lane < D ? 1.0f : 0.0f;
  const float la = s.la_prev[j], lt = s.lt_prev[j];  // prefetched at kernel start
  const float q = s.th[j], qd = s.thd[j], tau = s.tau[j], q0 = Pm->default_dof_pos[j];
  const float dq = q - q0;
  float v[J_N];
  v[J_ACTION_RATE] = sq(la - s.act[j]);
  v[J_DELTA_TORQUES] = sq(tau - lt);
  v[J_DOF_ACC] = sq((s.ldv[j] - qd) / Pm->dt);
  v[J_DOF_ERROR] = sq(dq);
  {
    const float lo = q - Pm->dof_pos_limits[j][0], hi = q - Pm->dof_pos_limits[j][1];
    float o = -(lo < 0.0f ? lo : 0.0f);
    o += (hi > 0.0f ? hi : 0.0f);
    v[J_DOF_POS_LIMITS] = o;
  }
  v[J_DOF_VEL] = sq(qd);
  v[J_DOF_VEL_LIMITS] = clipf(fabsf(qd) - Pm->dof_vel_limits[j] * Pm->soft_dof_vel_limit, 0.0f, 1.0f);
  v[J_STAND_ABS] = fabsf(dq);
  {
    const float t = fabsf(tau) - Pm->torque_limits[j] * Pm->soft_torque_limit;
    v[J_TORQUE_LIMITS] = t > 0.0f ? t : 0.0f;
  }
  v[J_TORQUES] = sq(tau);
  float hip = 0.f, thigh = 0.f, calf = 0.f;
  for (int i = 0; i < 4; ++i) {
    hip += Pm->hip_joint_idx[i] == j ? 1.f : 0.f;
    thigh += Pm->thigh_joint_idx[i] == j ? 1.f : 0.f;
    calf += Pm->calf_joint_idx[i] == j ? 1.f : 0.f;
  }
  v[J_HIP_POS] = hip * v[J_DOF_ERROR];
  v[J_THIGH_POS] = thigh * v[J_DOF_ERROR];
  v[J_CALF_POS] = calf * v[J_DOF_ERROR];
  // height points: lane i < 16 sums points i, i + 16, ...
  float hsum = 0.f;
  if (lane < 16) {
    const float* hts = stg_heights(A, Pm);
    for (int i = lane; i < Pm->num_height_points; i += 16) hsum += s.root[2] - hts[i];
  }
#pragma unroll
  for (int k = 0; k < J_N; ++k) {
    float x = k == J_HEIGHT ? (lane < 16 ? hsum : 0.f) : v[k] * on;
    x += dpp_shr_t<0x111>(x);
    x += dpp_shr_t<0x112>(x);
    x += dpp_shr_t<0x114>(x);
    x += dpp_shr_t<0x118>(x);
    if (lane == 15) s.jsum[k] = x;
  }
}

// one reward term (lane k computes term k); mirrors oracle/lgx_oracle.c reward_term.
// Side effects (kept from the reference): feet_air_time (go2.py:827-830) and the in-place
// wrap of commands[:, 3] (go2.py:744, Q7) are written back to LDS by the owning lane.
LGX_DEV float reward_term(const lgx_task_params* Pm, const lgx_buffers& B, Sh& s, int e, int id) {
  const Scratch& x = s.x;
  const float* root = s.root;
  float* cmd = s.cmd;
  const float* lch = s.lch;
  float* fat = s.fat;
  const int* lc = s.lc;
  float r = 0.0f;
  switch (id) {
    case LGX_REW_ACTION_RATE: return s.jsum[J_ACTION_RATE];
    case LGX_REW_ANG_VEL_XY: return sq(x.bav[0]) + sq(x.bav[1]);
    case LGX_REW_BASE_HEIGHT:
      return sq(s.jsum[J_HEIGHT] / (float)Pm->num_height_points - Pm->base_height_target);
    case LGX_REW_CALF_COLLISION:
      for (int i = 0; i < 4; ++i) { const float* c = s.cf[Pm->calf_idx[i]]; r += (float)(nrm3(c[0], c[1], c[2]) > 0.1f); }
      return r;
    case LGX_REW_CALF_POS: return s.jsum[J_CALF_POS];
    case LGX_REW_CALF_SYMMETRY: {
      const int* c = Pm->calf_joint_idx;
      return fabsf(s.th[c[0]] - s.th[c[1]]) + fabsf(s.th[c[2]] - s.th[c[3]]);
    }
    case LGX_REW_COLLISION:
      for (int i = 0; i < Pm->n_penalised; ++i) {
        const float* c = s.cf[Pm->penalised_idx[i]];
        r += (float)(nrm3(c[0], c[1], c[2]) > 0.1f);
      }
      return r;
    case LGX_REW_DELTA_TORQUES: return s.jsum[J_DELTA_TORQUES];
    case LGX_REW_DOF_ACC: return s.jsum[J_DOF_ACC];
    case LGX_REW_DOF_ERROR: return s.jsum[J_DOF_ERROR];
    case LGX_REW_DOF_POS_LIMITS: return s.jsum[J_DOF_POS_LIMITS];
    case LGX_REW_DOF_VEL: return s.jsum[J_DOF_VEL];
    case LGX_REW_DOF_VEL_LIMITS: return s.jsum[J_DOF_VEL_LIMITS];
    case LGX_REW_FEET_AIR_TIME: {
      float rew = 0.0f;
      for (int f = 0; f < Pm->num_feet; ++f) {
        int cfl = (s.cf[Pm->feet_idx[f]][2] > 1.0f) || lc[f];
        float first = (float)((fat[f] > 0.0f) && cfl);
        fat[f] = fat[f] + Pm->dt;
        rew += (fat[f] - 0.5f) * first;
      }
      rew = rew * (float)(nrm2(cmd[0], cmd[1]) > 0.1f);
      for (int f = 0; f < Pm->num_feet; ++f) {
        int cfl = (s.cf[Pm->feet_idx[f]][2] > 1.0f) || lc[f];
        fat[f] = fat[f] * (float)(!cfl);
      }
      return rew;
    }
    case LGX_REW_FEET_CONTACT_FORCES:
      for (int f = 0; f < Pm->num_feet; ++f) {
        const float* c = s.cf[Pm->feet_idx[f]];
        float v = nrm3(c[0], c[1], c[2]) - Pm->max_contact_force;
        r += v > 0.0f ? v : 0.0f;
      }
      return r;
    case LGX_REW_HEADING_ALIGNMENT: {
      const float fwd[3] = {1.f, 0.f, 0.f};
      float f[3];
      quat_apply(root + 3, fwd, f);
      float heading = atan2f(f[1], f[0]);
      float desired = 0.0f;
      if (Pm->heading_command) {
        cmd[3] = wrap_to_pi(cmd[3]);  // wrap_to_pi mutates commands[:, 3] (Q7)
        desired = cmd[3];
      }
      float err = wrap_to_pi(desired - heading);
      return sq(err) * (float)(nrm3(cmd[0], cmd[1], cmd[2]) >= 0.2f);
    }
    case LGX_REW_HIP_POS: return s.jsum[J_HIP_POS];
    case LGX_REW_JUMP_ZONE_FORWARD_VEL: {
      float fr = root[7] > 0.0f ? root[7] : 0.0f;
      return fr * (float)(x.jump > 0.0f) * (float)(nrm3(cmd[0], cmd[1], cmd[2]) >= 0.2f);
    }
    case LGX_REW_JUMP_ZONE_UPWARD_VEL: {
      float up = root[9] > 0.0f ? root[9] : 0.0f;
      return up * (float)(x.jump > 0.0f) * (float)(nrm3(cmd[0], cmd[1], cmd[2]) >= 0.2f);
    }
    case LGX_REW_LIN_VEL_Z: return sq(x.blv[2]);
    case LGX_REW_MIN_HEIGHT: {
      float ze = clipf(Pm->base_height_target - root[2], 0.0f, Pm->base_height_target);
      return ze * (float)(x.jump > 0.0f);
    }
    case LGX_REW_ORIENTATION: return sq(x.pg[0]) + sq(x.pg[1]);
    case LGX_REW_PHASE_CONTACT_MATCH: {
      float thr = 2.0f * Pm->percent_time_on_ground - 1.0f;
      float rew = 0.0f;
      for (int f = 0; f < 4; ++f) {
        int stance = sinf(6.283185307179586f * x.ph[f]) <= thr;
        rew += (x.contact[f] == stance) ? 0.25f : -0.25f;
      }
      return rew;
    }
    case LGX_REW_PHASE_FOOT_LIFTING: {
      float thr = 2.0f * Pm->percent_time_on_ground - 1.0f;
      float rew = 0.0f;
      for (int f = 0; f < 4; ++f) {
        int stance = sinf(6.283185307179586f * x.ph[f]) <= thr;
        float h = clipf(x.feet_z[f] - lch[f], 0.0f, Pm->max_foot_height);
        float nh = h / Pm->max_foot_height;
        rew += stance ? -nh : nh;
      }
      return rew / 2.0f;
    }
    case LGX_REW_REVERSE_PENALTY: return -(root[7] < 0.0f ? root[7] : 0.0f);
    case LGX_REW_STAND_STILL: return s.jsum[J_STAND_ABS] * (float)(nrm2(cmd[0], cmd[1]) < 0.1f);
    case LGX_REW_STUMBLE_CALVES: {
      int any = 0;
      for (int i = 0; i < 4; ++i) { const float* c = s.cf[Pm->calf_idx[i]]; any |= nrm2(c[0], c[1]) > 5.0f * fabsf(c[2]); }
      return (float)any;
    }
    case LGX_REW_STUMBLE_FEET: {
      int any = 0;
      for (int f = 0; f < Pm->num_feet; ++f) { const float* c = s.cf[Pm->feet_idx[f]]; any |= nrm2(c[0], c[1]) > 5.0f * fabsf(c[2]); }
      return (float)any;
    }
    case LGX_REW_THIGH_POS: return s.jsum[J_THIGH_POS];
    case LGX_REW_THIGH_SYMMETRY: {
      const int* c = Pm->thigh_joint_idx;
      return fabsf(s.th[c[0]] - s.th[c[1]]) + fabsf(s.th[c[2]] - s.th[c[3]]);
    }
    case LGX_REW_TORQUE_LIMITS: return s.jsum[J_TORQUE_LIMITS];
    case LGX_REW_TORQUES: return s.jsum[J_TORQUES];
    case LGX_REW_TRACKING_ANG_VEL: return expf(-sq(cmd[2] - x.bav[2]) / Pm->tracking_sigma);
    case LGX_REW_TRACKING_LIN_VEL: return expf(-(sq(cmd[0] - x.blv[0]) + sq(cmd[1] - x.blv[1])) / Pm->tracking_sigma);
    case LGX_REW_TRACKING_PITCH: {
      float deg = x.pitch * 57.29577951308232f;
      return expf(-sq(deg - Pm->pitch_deg_target) / Pm->tracking_sigma);
    }
    case LGX_REW_TRACKING_ROLL: {
      float deg = x.roll * 57.29577951308232f;
      return expf(-sq(deg - Pm->roll_deg_target) / Pm->tracking_sigma);
    }
    case LGX_REW_ZERO_CMD_DOF_ERROR:
      return s.jsum[J_DOF_ERROR] * (float)(nrm3(cmd[0], cmd[1], cmd[2]) < 0.2f);
    default: return 0.0f;
  }
}

template <int WL>
LGX_DEV void get_heights(const lgx_task_params* Pm, const lgx_buffers& B, Sh& s, float* A, int lane) {
  const int NP = Pm->num_height_points;
  const float* root = s.root;
  if (Pm->mesh_type == LGX_MESH_PLANE || B.height_samples == nullptr) {
    for (int i = lane; i < NP; i += WL) stg_heights(A, Pm)[i] = 0.0f;
    return;
  }
  float qz = root[5], qw = root[6];
  float n = sqrtf(qz * qz + qw * qw);
  n = n < 1e-9f ? 1e-9f : n;
  float qy[4] = {0.f, 0.f, qz / n, qw / n};
  for (int i = lane; i < NP; i += WL) {
    float p[3] = {Pm->height_points[i][0], Pm->height_points[i][1], 0.f}, w[3];
    quat_apply(qy, p, w);
    float px = (w[0] + root[0]) + Pm->border_size, py = (w[1] + root[1]) + Pm->border_size;
    long ix = (long)(px / Pm->horizontal_scale), iy = (long)(py / Pm->horizontal_scale);
    ix = ix < 0 ? 0 : (ix > Pm->hf_rows - 2 ? Pm->hf_rows - 2 : ix);
    iy = iy < 0 ? 0 : (iy > Pm->hf_cols - 2 ? Pm->hf_cols - 2 : iy);
    int16_t h1 = B.height_samples[ix * Pm->hf_cols + iy];
    int16_t h2 = B.height_samples[(ix + 1) * Pm->hf_cols + iy];
    int16_t h3 = B.height_samples[ix * Pm->hf_cols + iy + 1];
    int16_t h = h1 < h2 ? h1 : h2;
    h = h < h3 ? h : h3;
    stg_heights(A, Pm)[i] = (float)h * Pm->vertical_scale;
  }
}

// ============================================================== kernels
// Occupancy target: 4 waves per SIMD (<= 128 VGPRs; the Go2 LDS image is 9.6 KB, so 4096
// envs are one residency round on 256 CUs). The SEA-LSTM variant keeps its hidden states in
// registers (fewer waves per SIMD; ANYmal's LDS image is 13 KB).
#ifndef LGX_SEA_WAVES
#define LGX_SEA_WAVES 4
#endif
// EPW envs per wave (1, or 2: each env on a 32-lane group, grp_of_lane; blocks = N / 2, envs 2b'
// and 2b' + 1 of the XCD-aware pair order b' = env_of_block). Each env has its own Sh and LDS arena.
// Two envs per wave: LDS holds 2 x (Sh + arena) per block, so 8 blocks per CU (2 waves per
// SIMD) are resident — the register budget is that of 2 waves per SIMD.
template <bool PHYSICS, bool TERRAIN, bool ACTNET, int EPW>
__global__ __launch_bounds__(64, ACTNET ? LGX_SEA_WAVES : (EPW == 2 ? 2 : 4)) void env_step_kernel(const lgx_model* __restrict__ M,
                                                      const lgx_task_params* __restrict__ Pm,
                                                      const lgx_buffers* __restrict__ Bp, uint64_t seed,
                                                      uint64_t step_arg, const uint64_t* __restrict__ step_dev) {
  constexpr int WL = 64 / EPW;  // lanes per env
  __shared__ Sh S_[EPW];
  const int grp = grp_of_lane<WL>();
  Sh& s = S_[grp];
  const int astride = (int)arena_floats(*Pm);
  float* const AR = lgx_dyn + (EPW == 1 ? 0 : grp * astride);  // this env's arena
  // buffer pointers are read from device memory (scalar loads) when used, not held in SGPRs
  const lgx_buffers& B = *Bp;
  // graph-replayable form: the step counter is read from device memory (lgx_step_dev)
  const uint64_t step = step_dev ? *step_dev : step_arg;
  const int e = EPW * env_of_block(blockIdx.x, gridDim.x) + grp;
  const int lane = EPW == 1 ? (int)threadIdx.x : (int)(threadIdx.x & (WL - 1));
#if LGX_SLOT_PRIO
  // the SIMD's arbiter favours its older waves; a launch ends with its slowest wave, so the
  // younger slots get the higher issue priority
  set_prio(min(wave_slot(), 3));
#endif
  const int D = Pm->num_dof, A = Pm->num_actions, NB = Pm->num_bodies;
  const uint32_t gid = (uint32_t)(Pm->env_id_offset + e);

  // ---------------------------------------------------------------- load + clip
  float* root_g = B.root_states + (size_t)e * 13;
  if (lane < A) {
    float a = B.actions_in[(size_t)e * A + lane];
    a = clipf(a, -Pm->clip_actions, Pm->clip_actions);  // legged_robot.py:74-75
    s.act[lane] = a;
    B.actions[(size_t)e * A + lane] = a;
  }
  if (lane < D) {
    s.th[lane] = B.dof_state[((size_t)e * D + lane) * 2];
    s.thd[lane] = B.dof_state[((size_t)e * D + lane) * 2 + 1];
    s.kpm[lane] = B.kp_kd ? B.kp_kd[(size_t)e * D + lane] : 1.f;
    s.kdm[lane] = B.kp_kd ? B.kp_kd[((size_t)Pm->num_envs + e) * D + lane] : 1.f;
    s.ldv[lane] = B.last_dof_vel[(size_t)e * D + lane];
  }
  if (lane < 13) s.root[lane] = root_g[lane];
  if (lane == 0) {
    s.madd = B.mass_params ? B.mass_params[e * 4] : 0.f;
    s.mu = 0.5f * ((B.friction ? B.friction[e] : 1.f) + Pm->ground_friction);
  }
  if (lane < 3) s.cadd[lane] = B.mass_params ? B.mass_params[e * 4 + 1 + lane] : 0.f;
  if (lane < 4) s.cmd[lane] = B.commands[e * 4 + lane];
  if (lane == 0) {
    s.blew = 0;
    s.ep_prev = B.episode_length[e];
    s.jump_prev = B.rpy_phase ? B.rpy_phase[e * 8 + 7] : 0.f;
    s.fric = B.friction ? B.friction[e] : 1.f;
  }
  // inputs the post-physics phase reads (their latency hides behind the physics)
  if (lane < A) s.la_prev[lane] = B.last_actions[(size_t)e * A + lane];
  if (lane < D) s.lt_prev[lane] = B.last_torques[(size_t)e * D + lane];
  {
    const int KS0 = Pm->num_reward_terms + (Pm->has_termination_reward ? 1 : 0);
    for (int k = lane; k < KS0; k += WL) s.es[k] = B.episode_sums[(size_t)e * KS0 + k];
  }
  if (Pm->task_kind == LGX_TASK_GO2 && lane < Pm->num_feet) {
    s.lc_prev[lane] = B.last_contacts[e * Pm->num_feet + lane];
    s.lch_prev[lane] = B.last_contact_heights[e * Pm->num_feet + lane];
    s.fat_prev[lane] = B.feet_air_time ? B.feet_air_time[e * Pm->num_feet + lane] : 0.f;
  }
#ifdef LGX_PHASE_CLOCK
  if (lane < 20) s.phacc[lane] = 0u;
  if (lane == 0) s.phlast = clock64();
#endif
  __syncthreads();

  if (PHYSICS) {
    if (lane == 0) {
      float q[4] = {s.root[3], s.root[4], s.root[5], s.root[6]};
      float n = rsqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
      for (int i = 0; i < 4; ++i) s.qb[i] = q[i] * n;
      for (int i = 0; i < 3; ++i) { s.pb[i] = s.root[i]; s.wb[i] = s.root[10 + i]; }
      float R[9];
      quat_to_R(s.qb, R);
      f3 rc = mv(R, mk(M->link_com[0][0] + s.cadd[0], M->link_com[0][1] + s.cadd[1], M->link_com[0][2] + s.cadd[2]));
      f3 vo = ld3(s.root + 7) - cross(ld3(s.wb), rc);  // COM velocity -> origin velocity
      st3(s.vo, vo);
    }
    __syncthreads();
    PH(0);
    for (int sub = 0; sub < Pm->decimation; ++sub)
      substep<TERRAIN, ACTNET, WL>(s, AR, S_, lgx_dyn, astride, M, Pm, B, lane, e, sub == Pm->decimation - 1);
    __syncthreads();
    // NaN/Inf guard (SURVEY.md §5 "Failure detection"; the reference has none): a state that
    // went non-finite in any substep stays non-finite, so one check after the substeps sees it.
    // Such an env gets a finite stand-in state (default joint pose at its start position, at
    // rest, no torques / contact forces / actions), is flagged in blew_up, counted, and reset
    // below by the normal masked path, so no NaN reaches its observations, rewards or the
    // learner. Other envs are untouched.
    {
      bool bad = false;
      if (lane < D) bad = !(isfinite(s.th[lane]) && isfinite(s.thd[lane]) && isfinite(s.tau[lane]));
      if (lane < A) bad = bad || !isfinite(s.act[lane]);
      if (lane < 3) bad = bad || !(isfinite(s.pb[lane]) && isfinite(s.vo[lane]) && isfinite(s.wb[lane]));
      if (lane < 4) bad = bad || !isfinite(s.qb[lane]);
      if (lane < NB) bad = bad || !(isfinite(s.cf[lane][0]) && isfinite(s.cf[lane][1]) && isfinite(s.cf[lane][2]));
      if (gballot<WL>(bad) != 0ull) {
        if (lane < D) { s.th[lane] = Pm->default_dof_pos[lane]; s.thd[lane] = 0.f; s.tau[lane] = 0.f; }
        if (lane < A) { s.act[lane] = 0.f; B.actions[(size_t)e * A + lane] = 0.f; }
        if (lane < 3) { s.pb[lane] = isfinite(s.root[lane]) ? s.root[lane] : 0.f; s.vo[lane] = 0.f; s.wb[lane] = 0.f; }
        if (lane < 4) s.qb[lane] = lane == 3 ? 1.f : 0.f;
        if (lane < NB) { s.cf[lane][0] = 0.f; s.cf[lane][1] = 0.f; s.cf[lane][2] = 0.f; }
        if (lane == 0) {
          s.blew = 1;
          if (B.blowup_count) atomicAdd(B.blowup_count, 1u);
        }
      }
      __syncthreads();
    }
    // final kinematics for the rigid-body state tensor
    kinematics<false>(s, AR, M, Pm, lane);
    float root[13];
    {
      float R[9];
      quat_to_R(s.qb, R);
      f3 rc = mv(R, mk(M->link_com[0][0] + s.cadd[0], M->link_com[0][1] + s.cadd[1], M->link_com[0][2] + s.cadd[2]));
      f3 vc = ld3(s.vo) + cross(ld3(s.wb), rc);
      root[0] = s.pb[0]; root[1] = s.pb[1]; root[2] = s.pb[2];
      root[3] = s.qb[0]; root[4] = s.qb[1]; root[5] = s.qb[2]; root[6] = s.qb[3];
      root[7] = vc.x; root[8] = vc.y; root[9] = vc.z;
      root[10] = s.wb[0]; root[11] = s.wb[1]; root[12] = s.wb[2];
    }
    __syncthreads();
    if (lane < 13) s.root[lane] = root[lane];
    // rigid body states, contact forces, torques -> HBM
    if (lane < NB) {
      const int k = M->body_link[lane];
      f3 off = ld3(M->body_offset[lane]);
      f3 o = mv(s.R[k], off);
      f3 pos = ld3(s.P[k]) + o;
      bool primary = off.x == 0.f && off.y == 0.f && off.z == 0.f;
      f3 lv = ld3(s.V[k]) + cross(ld3(s.W[k]), primary ? (ld3(s.C[k]) - ld3(s.P[k])) : o);
      float Rb[9];
      mm(s.R[k], M->body_rot[lane], Rb);
      float tr = Rb[0] + Rb[4] + Rb[8], qq[4];
      if (tr > 0.f) {
        float sc = sqrtf(tr + 1.f) * 2.f;
        qq[3] = 0.25f * sc; qq[0] = (Rb[7] - Rb[5]) / sc; qq[1] = (Rb[2] - Rb[6]) / sc; qq[2] = (Rb[3] - Rb[1]) / sc;
      } else if (Rb[0] > Rb[4] && Rb[0] > Rb[8]) {
        float sc = sqrtf(1.f + Rb[0] - Rb[4] - Rb[8]) * 2.f;
        qq[3] = (Rb[7] - Rb[5]) / sc; qq[0] = 0.25f * sc; qq[1] = (Rb[1] + Rb[3]) / sc; qq[2] = (Rb[2] + Rb[6]) / sc;
      } else if (Rb[4] > Rb[8]) {
        float sc = sqrtf(1.f + Rb[4] - Rb[0] - Rb[8]) * 2.f;
        qq[3] = (Rb[2] - Rb[6]) / sc; qq[0] = (Rb[1] + Rb[3]) / sc; qq[1] = 0.25f * sc; qq[2] = (Rb[5] + Rb[7]) / sc;
      } else {
        float sc = sqrtf(1.f + Rb[8] - Rb[0] - Rb[4]) * 2.f;
        qq[3] = (Rb[3] - Rb[1]) / sc; qq[0] = (Rb[2] + Rb[6]) / sc; qq[1] = (Rb[5] + Rb[7]) / sc; qq[2] = 0.25f * sc;
      }
      if (qq[3] < 0.f) for (int i = 0; i < 4; ++i) qq[i] = -qq[i];
      float* rb = B.rigid_body_states + ((size_t)e * NB + lane) * 13;
      rb[0] = pos.x; rb[1] = pos.y; rb[2] = pos.z;
      rb[3] = qq[0]; rb[4] = qq[1]; rb[5] = qq[2]; rb[6] = qq[3];
      rb[7] = lv.x; rb[8] = lv.y; rb[9] = lv.z;
      const float* w = s.W[k];
      rb[10] = w[0]; rb[11] = w[1]; rb[12] = w[2];
      s.rbz[lane] = pos.z;
      float* cfo = B.contact_forces + ((size_t)e * NB + lane) * 3;
      cfo[0] = s.cf[lane][0]; cfo[1] = s.cf[lane][1]; cfo[2] = s.cf[lane][2];
    }
    if (lane < D) B.torques[(size_t)e * D + lane] = s.tau[lane];
    __syncthreads();
    PH(11);
  } else {
    // post-physics only: physics state supplied by the caller
    if (lane < NB) {
      const float* cfi = B.contact_forces + ((size_t)e * NB + lane) * 3;
      s.cf[lane][0] = cfi[0]; s.cf[lane][1] = cfi[1]; s.cf[lane][2] = cfi[2];
      s.rbz[lane] = B.rigid_body_states[((size_t)e * NB + lane) * 13 + 2];
    }
    if (lane < D) s.tau[lane] = B.torques[(size_t)e * D + lane];
    __syncthreads();
  }

  // ================================================================ post-physics
  // Go2Robot.post_physics_step go2.py:345-387 / LeggedRobot legged_robot.py:103-138.
  // Per-env scalars: lane 0, into LDS. Vectors: lane-parallel from LDS.
  // the old observation history (read back at the end of the step) in flight from here on:
  // the first HV x 64 entries into registers (all of Go2's 5 x 52)
  constexpr int HV = 320 / WL;
  float hv[HV];
  {
    const int HPn = Pm->history_len * Pm->num_proprio;
    const float* hsrc = B.obs_history + (size_t)e * HPn;
#pragma unroll
    for (int t = 0; t < HV; ++t) {
      const int i = lane + WL * t;
      hv[t] = i < HPn ? hsrc[i] : 0.f;
    }
  }
  fill_uniforms<WL>(AR, seed, gid, step, 0, lane, rng_blocks(Pm));
  PH(12);
  const bool go2 = Pm->task_kind == LGX_TASK_GO2;
  if (lane == 0) {
    Scratch& x = s.x;
    float* root = s.root;
    float* cmd = s.cmd;
    const long long ep = s.ep_prev + 1;
    s.ep = ep;
    const float g[3] = {0.f, 0.f, -1.f};
    quat_rotate_inverse(root + 3, root + 7, x.blv);
    quat_rotate_inverse(root + 3, root + 10, x.bav);
    quat_rotate_inverse(root + 3, g, x.pg);
    x.roll = x.pitch = x.yaw = 0.f;
    x.ph[0] = x.ph[1] = x.ph[2] = x.ph[3] = 0.f;
    for (int f = 0; f < 4; ++f) { x.contact[f] = 0; x.feet_z[f] = 0.f; s.lc[f] = 0; s.lch[f] = 0.f; s.fat[f] = 0.f; }
    if (go2) {
      // update_feet_states go2.py:266-328
      float phase = trem((float)ep * Pm->dt, Pm->period) / Pm->period;
      float pfr = trem(phase + Pm->offset_fr, 1.0f), pbl = trem(phase + Pm->offset_bl, 1.0f);
      float pfl = trem(phase + Pm->offset_fl, 1.0f), pbr = trem(phase + Pm->offset_br, 1.0f);
      float msk = (nrm3(cmd[0], cmd[1], cmd[2]) < 0.2f) ? 0.0f : 1.0f;
      x.ph[0] = pfl * msk; x.ph[1] = pfr * msk; x.ph[2] = pbl * msk; x.ph[3] = pbr * msk;
      for (int f = 0; f < 4; ++f) {
        int lcf = s.lc_prev[f];
        float lch = s.lch_prev[f];
        int curc = s.cf[Pm->feet_idx[f]][2] > 1.0f;
        x.contact[f] = curc || lcf;
        s.lc[f] = curc;
        x.feet_z[f] = s.rbz[Pm->feet_idx[f]];
        s.lch[f] = x.contact[f] ? x.feet_z[f] : lch;
        if (B.feet_air_time) s.fat[f] = s.fat_prev[f];
      }
      // quaternion_to_euler go2.py:11-31
      float qx = root[3], qy = root[4], qz = root[5], qw = root[6];
      x.roll = atan2f(2.0f * (qw * qx + qy * qz), 1.0f - 2.0f * (qx * qx + qy * qy));
      x.pitch = asinf(clipf(2.0f * (qw * qy - qz * qx), -1.0f, 1.0f));
      x.yaw = atan2f(2.0f * (qw * qz + qx * qy), 1.0f - 2.0f * (qy * qy + qz * qz));
    }
    // _post_physics_step_callback go2.py:390-410
    if (ep % Pm->resample_interval == 0) resample_commands(Pm, B.command_ranges, cmd, stg_U(AR), S_CMD, root + 3);
    if (Pm->heading_command) {
      const float fwd[3] = {1.f, 0.f, 0.f};
      float f[3];
      quat_apply(root + 3, fwd, f);
      float heading = atan2f(f[1], f[0]);
      float gain = go2 ? Pm->heading_error_gain : 0.5f;
      cmd[2] = clipf(wrap_to_pi(cmd[3] - heading) * gain, -1.0f, 1.0f);
    }
    if (Pm->push_robots && (step % (uint64_t)Pm->push_interval == 0)) {
      root[7] = rand_range(-Pm->max_push_vel_xy, Pm->max_push_vel_xy, stg_U(AR)[S_PUSH + 0]);
      root[8] = rand_range(-Pm->max_push_vel_xy, Pm->max_push_vel_xy, stg_U(AR)[S_PUSH + 1]);
    }
    // check_termination go2.py:186-204
    int reset = 0;
    for (int i = 0; i < Pm->n_termination; ++i) {
      const float* c = s.cf[Pm->termination_idx[i]];
      reset |= nrm3(c[0], c[1], c[2]) > 1.0f;
    }
    // a blown-up env (NaN/Inf guard) ends as a termination, never a time-out: its step is not
    // bootstrapped (ppo.py:166-167) and earns no reward (the stand-in state is not a real one)
    int tout = ep > Pm->max_episode_length && !s.blew;
    reset |= tout;
    reset |= x.pg[2] > 0.0f;
    if (Pm->parkour) reset |= root[2] < -1.0f;
    reset |= s.blew;  // NaN/Inf guard
    s.reset = reset;
    s.tout = tout;
    x.jump = s.jump_prev;  // set by the previous step's observations
  }
  __syncthreads();
  PH(13);
  get_heights<WL>(Pm, B, s, AR, lane);
  __syncthreads();
  joint_sums(Pm, B, s, AR, e, lane);
  __syncthreads();
  // compute_reward legged_robot.py:216-237: lane k evaluates term k (alphabetical order)
  const int K = Pm->num_reward_terms;
  const int KS = K + (Pm->has_termination_reward ? 1 : 0);
  for (int k = lane; k < K; k += WL)
    s.rterm[k] = s.blew ? 0.0f : reward_term(Pm, B, s, e, Pm->reward_ids[k]) * Pm->reward_scales[k];
  __syncthreads();
  const int reset = s.reset;
  if (lane == 0) {
    float rew = 0.0f;
    for (int k = 0; k < K; ++k) rew += s.rterm[k];  // sequential, the reference's order
    if (Pm->only_positive_rewards) rew = rew < 0.0f ? 0.0f : rew;
    if (Pm->has_termination_reward) {
      float v = (float)(reset && !s.tout && !s.blew) * Pm->termination_scale;
      rew += v;
      s.rterm[K] = v;
    }
    B.rew[e] = rew;
    B.reset[e] = (uint8_t)reset;
    B.time_out[e] = (uint8_t)s.tout;
    if (B.blew_up) B.blew_up[e] = (uint8_t)s.blew;
  }
  __syncthreads();
  for (int k = lane; k < KS; k += WL) {
    const float v = s.es[k] + s.rterm[k];
    s.es[k] = v;
    B.episode_sums[(size_t)e * KS + k] = v;
  }
  __syncthreads();
  PH(14);
  // reset_idx (go2.py:207-263)
  if (reset) reset_env<WL>(Pm, B, s, AR, e, lane, true, false, true);

  // compute_observations go2.py:467-574 / legged_robot.py:240-273
  const int Pp = Pm->num_proprio, H = Pm->history_len;
  const Scratch& x = s.x;
  if (go2 && Pm->parkour && lane == 0) {
    int outl = 0;
    for (int i = 0; i < Pm->num_height_points; ++i) outl += fabsf(stg_heights(AR, Pm)[i]) > 0.1f;
    s.x.jump = (float)(outl >= 8);
  }
  for (int i = lane; i < Pp; i += WL) {
    float v;
    if (go2) {
      if (i < 3) v = x.bav[i] * Pm->obs_scale_ang_vel;
      else if (i == 3) v = x.roll;
      else if (i == 4) v = x.pitch;
      else if (i < 8) v = s.cmd[i - 5] * Pm->commands_scale[i - 5];
      else if (i < 8 + D) v = (s.th[i - 8] - Pm->default_dof_pos[i - 8]) * Pm->obs_scale_dof_pos;
      else if (i < 8 + 2 * D) v = s.thd[i - 8 - D] * Pm->obs_scale_dof_vel;
      else if (i < 8 + 2 * D + A) v = s.act[i - 8 - 2 * D];
      else {
        int q = i - (8 + 2 * D + A);  // sin/cos of FR, FL, BL, BR
        int leg = (q >> 1) == 0 ? 1 : ((q >> 1) == 1 ? 0 : (q >> 1));
        float p = 6.283185307179586f * x.ph[leg];
        v = (q & 1) ? cosf(p) : sinf(p);
      }
    } else {
      if (i < 3) v = x.blv[i] * Pm->obs_scale_lin_vel;
      else if (i < 6) v = x.bav[i - 3] * Pm->obs_scale_ang_vel;
      else if (i < 9) v = x.pg[i - 6];
      else if (i < 12) v = s.cmd[i - 9] * Pm->commands_scale[i - 9];
      else if (i < 12 + D) v = (s.th[i - 12] - Pm->default_dof_pos[i - 12]) * Pm->obs_scale_dof_pos;
      else if (i < 12 + 2 * D) v = s.thd[i - 12 - D] * Pm->obs_scale_dof_vel;
      else if (i < 12 + 2 * D + A) v = s.act[i - 12 - 2 * D];
      else v = clipf(s.root[2] - 0.5f - stg_heights(AR, Pm)[i - (12 + 2 * D + A)], -1.0f, 1.0f) * Pm->obs_scale_height;
    }
    if (Pm->add_noise) v = v + (2.0f * stg_U(AR)[S_NOISE + i] - 1.0f) * Pm->noise_vec[i];
    stg_cur(AR, Pm)[i] = v;
  }
  // stage the old history (obs[0:H*P]) in LDS; a reset env's history was zeroed (go2.py:238)
  float* hist_g = B.obs_history + (size_t)e * H * Pp;
  float* const hist = stg_hist(AR, Pm);
  const float* const cur = stg_cur(AR, Pm);
  const bool hl = hist_in_lds(Pm);
  const long long ep = s.ep;
  const float co = Pm->clip_obs;
  float* obs = B.obs + (size_t)e * Pm->num_obs;
  float* cr = B.critic ? B.critic + (size_t)e * Pm->num_critic : nullptr;
  if (hl) {
#pragma unroll
    for (int t = 0; t < HV; ++t) {
      const int i = lane + WL * t;
      if (i < H * Pp) hist[i] = reset ? 0.f : hv[t];
    }
    for (int i = lane + WL * HV; i < H * Pp; i += WL) hist[i] = reset ? 0.f : hist_g[i];
  }
  __syncthreads();
  if (hl) {
    for (int i = lane; i < H * Pp; i += WL) {
      float v = clipf(hist[i], -co, co);
      obs[i] = v;
      if (go2 && cr) cr[i] = v;
    }
  } else {
    // long history, shifted in place: entry i of the old history goes to obs[i], and the new
    // history's entry i is old entry i + P (or the current observation, go2.py:570-574).
    // Chunks of 64 in increasing i: a chunk reads old entries >= its own first index (P >= 64)
    // and writes only its own 64, after its reads are consumed — no entry is overwritten
    // before it is read.
    const int HP = H * Pp, HP1 = (H - 1) * Pp;
#pragma unroll
    for (int t = 0; t < (MAXHIST + WL - 1) / WL; ++t) {
      const int i = lane + WL * t;
      if (WL * t >= HP) break;
      if (i < HP) {
        const float old = reset ? 0.f : (t < HV ? hv[t < HV ? t : 0] : hist_g[i]);
        const float v = clipf(old, -co, co);
        obs[i] = v;
        if (go2 && cr) cr[i] = v;
        const float nv = (ep <= 1) ? cur[i % Pp] : (i < HP1 ? hist_g[i + Pp] : cur[i - HP1]);
        hist_g[i] = nv;
      }
    }
  }
  for (int i = lane; i < Pp; i += WL) {
    float v = clipf(cur[i], -co, co);
    obs[H * Pp + i] = v;
    if (go2 && cr) cr[H * Pp + i] = v;
  }
  if (go2) {
    const int NO = Pm->num_obs;
    // priv = [mass params (4), friction, kp-1 (D), kd-1 (D)]
    for (int i = lane; i < Pm->num_priv; i += WL) {
      float v;
      if (i < 4) v = i == 0 ? s.madd : s.cadd[i - 1];  // mass_params row, staged at kernel start
      else if (i == 4) v = s.fric;
      else if (i < 5 + D) v = s.kpm[i - 5] - 1.0f;
      else v = s.kdm[i - 5 - D] - 1.0f;
      v = clipf(v, -co, co);
      B.priv[(size_t)e * Pm->num_priv + i] = v;
      if (cr) cr[NO + i] = v;
    }
    if (lane < 3) {
      float v = clipf(x.blv[lane] * Pm->obs_scale_lin_vel, -co, co);
      B.est[(size_t)e * Pm->num_est + lane] = v;
      if (cr) cr[NO + Pm->num_priv + lane] = v;
    }
    for (int i = lane; i < Pm->num_scan; i += WL) {
      float v = clipf(s.root[2] - 0.3f - stg_heights(AR, Pm)[i], -1.0f, 1.0f);
      B.scan[(size_t)e * Pm->num_scan + i] = v;
      if (cr) cr[NO + Pm->num_priv + 3 + i] = clipf(v, -co, co);
    }
  }
  // history update go2.py:570-574 (the long-history path wrote it above)
  if (hl)
    for (int i = lane; i < H * Pp; i += WL) {
      float v = (ep <= 1) ? cur[i % Pp] : (i < (H - 1) * Pp ? hist[i + Pp] : cur[i - (H - 1) * Pp]);
      hist_g[i] = v;
    }
  // last_* copies go2.py:380-384 and state write-back
  if (lane < A) B.last_actions[(size_t)e * A + lane] = s.act[lane];
  if (lane < D) {
    B.last_dof_vel[(size_t)e * D + lane] = s.thd[lane];
    B.last_torques[(size_t)e * D + lane] = s.tau[lane];
    B.dof_state[((size_t)e * D + lane) * 2] = s.th[lane];
    B.dof_state[((size_t)e * D + lane) * 2 + 1] = s.thd[lane];
  }
  if (lane < 6) B.last_root_vel[e * 6 + lane] = s.root[7 + lane];
  if (lane < 3) {
    B.last_base_lin_vel[e * 3 + lane] = x.blv[lane];
    if (B.base_lin_vel) B.base_lin_vel[e * 3 + lane] = x.blv[lane];
    if (B.base_ang_vel) B.base_ang_vel[e * 3 + lane] = x.bav[lane];
    if (B.projected_gravity) B.projected_gravity[e * 3 + lane] = x.pg[lane];
  }
  if (lane < 13) root_g[lane] = s.root[lane];
  if (lane < 4) B.commands[e * 4 + lane] = s.cmd[lane];
  if (go2 && lane < Pm->num_feet && !reset) {
    B.last_contacts[e * Pm->num_feet + lane] = (uint8_t)s.lc[lane];
    B.last_contact_heights[e * Pm->num_feet + lane] = s.lch[lane];
    if (B.feet_air_time) B.feet_air_time[e * Pm->num_feet + lane] = s.fat[lane];
  }
  if (lane == 0) B.episode_length[e] = ep;
  if (B.rpy_phase && lane < 8) {
    float v = lane == 0 ? x.roll : lane == 1 ? x.pitch : lane == 2 ? x.yaw : lane < 7 ? x.ph[lane - 3] : x.jump;
    B.rpy_phase[e * 8 + lane] = v;
  }
  if (B.measured_heights)
    for (int i = lane; i < Pm->num_height_points; i += WL)
      B.measured_heights[(size_t)e * Pm->num_height_points + i] = stg_heights(AR, Pm)[i];
#ifdef LGX_PHASE_CLOCK
  __syncthreads();
  PH(15);
  __syncthreads();
  if (lane == 0) {  // where the wave ran: HW_ID (wave, SIMD, CU, SE fields) and XCC_ID
    s.phacc[18] = __builtin_amdgcn_s_getreg(4 | (31 << 11));
    s.phacc[19] = __builtin_amdgcn_s_getreg(20 | (31 << 11));
  }
  __syncthreads();
  if (g_phase_out && lane < NPH) g_phase_out[(size_t)e * NPH + lane] = s.phacc[lane];
#endif
}

// BaseTask.reset -> reset_idx(env_ids) outside a step (RNG stream 1)
__global__ __launch_bounds__(64) void reset_kernel(const lgx_task_params* __restrict__ Pm,
                                                   const lgx_buffers* __restrict__ Bp,
                                                   const uint8_t* __restrict__ mask, uint64_t seed, uint64_t call) {
  __shared__ Sh s;
  const lgx_buffers& B = *Bp;
  const int e = blockIdx.x;
  const int lane = threadIdx.x;
  if (!mask[e]) return;
  const int D = Pm->num_dof;
  fill_uniforms<64>(lgx_dyn, seed, (uint32_t)(Pm->env_id_offset + e), call, 1, lane, rng_blocks(Pm));
  if (lane < 13) s.root[lane] = B.root_states[(size_t)e * 13 + lane];
  if (lane < 4) s.cmd[lane] = B.commands[e * 4 + lane];
  __syncthreads();
  // an external reset (BaseTask.reset -> reset_idx) only exists once the env is built,
  // i.e. with init_done set: the terrain curriculum applies (legged_robot.py:551-552)
  reset_env<64>(Pm, B, s, lgx_dyn, e, lane, true, true, false);
  if (lane < 13) B.root_states[(size_t)e * 13 + lane] = s.root[lane];
  if (lane < D) {
    B.dof_state[((size_t)e * D + lane) * 2] = s.th[lane];
    B.dof_state[((size_t)e * D + lane) * 2 + 1] = s.thd[lane];
  }
  if (lane < 4) B.commands[e * 4 + lane] = s.cmd[lane];
  if (lane == 0) { B.episode_length[e] = s.ep; B.reset[e] = 1; }
}

}  // namespace lgx

// ============================================================== C ABI
#include <stdio.h>

#include <string>

struct lgx_env {
  lgx_model model;
  lgx_task_params params;
  lgx_buffers buffers;
  lgx_model* d_model = nullptr;
  lgx_task_params* d_params = nullptr;
  lgx_buffers* d_buffers = nullptr;  // device copy of `buffers` (kernels read pointers from it)
  int device = 0;
  bool host = false;         // device < 0: the host backend (lgx_env_host.cpp), host buffers
  bool bound = false;
  bool stats_clean = false;  // episode_stats zeroed by lgx_episode_extras and not written since
  int epw = 0;               // envs per wave (lgx_set_envs_per_wave; 0: default)
  std::string err;
};

static int fail(lgx_env* env, const std::string& msg) {
  if (env) env->err = msg;
  return -1;
}

#define HIP_OK(call)                                                                   \
  do {                                                                                 \
    hipError_t _e = (call);                                                            \
    if (_e != hipSuccess) return fail(env, std::string(#call ": ") + hipGetErrorString(_e)); \
  } while (0)

extern "C" {

int32_t lgx_abi_version(void) { return LGX_ABI_VERSION; }
int64_t lgx_sizeof_model(void) { return (int64_t)sizeof(lgx_model); }
int64_t lgx_sizeof_task_params(void) { return (int64_t)sizeof(lgx_task_params); }
int64_t lgx_sizeof_buffers(void) { return (int64_t)sizeof(lgx_buffers); }

int lgx_create(const lgx_model* model, const lgx_task_params* params, int32_t device, lgx_env** out) {
  if (!model || !params || !out) return -2;
  lgx_env* env = new lgx_env();
  *out = env;
  env->model = *model;
  env->params = *params;
  env->device = device;
  if (params->abi_version != LGX_ABI_VERSION) return fail(env, "ABI version mismatch");
  // the kernel's structured solver assumes base + 4 chains of 3 revolute joints
  if (model->num_links != lgx::NL || params->num_dof != lgx::NJ)
    return fail(env, "model must be a floating base with 4 chains of 3 joints (13 links, 12 dof)");
  for (int l = 0; l < 4; ++l)
    for (int i = 0; i < 3; ++i) {
      int k = 1 + 3 * l + i;
      int expect = i == 0 ? 0 : k - 1;
      if (model->link_parent[k] != expect) return fail(env, "link tree is not 4 serial chains of 3");
    }
  if (model->num_candidates > LGX_MAX_CANDIDATES || model->num_bodies > LGX_MAX_BODIES)
    return fail(env, "too many contact candidates or bodies");
  if (params->history_len * params->num_proprio > lgx::MAXHIST) return fail(env, "history too long");
  if (params->num_proprio > LGX_MAX_PROPRIO || params->num_height_points > LGX_MAX_HEIGHT_POINTS)
    return fail(env, "observation too large");
  if (params->num_reward_terms + 1 > 64) return fail(env, "too many reward terms");
  // observation layout the step writes (go2.py:467-574 / legged_robot.py:240-273): obs =
  // [history (H x P) | current (P)]; Go2 critic = [obs | priv | est (3) | scan]. A config whose
  // declared sizes disagree (the reference's anymal_c_flat: 48-wide obs, 235-wide proprio)
  // fails here — the reference fails at its first compute_observations (torch.cat shapes).
  {
    const lgx_task_params& p = *params;
    const int D = p.num_dof, A = p.num_actions;
    const int want_p = p.task_kind == LGX_TASK_GO2 ? 8 + 2 * D + A + 8
                                                   : 12 + 2 * D + A + (p.measure_heights ? p.num_height_points : 0);
    char msg[256];
    if (p.num_proprio != want_p) {
      snprintf(msg, sizeof msg, "num_proprio %d != %d (the observation terms of this task)", p.num_proprio, want_p);
      return fail(env, msg);
    }
    if (p.num_obs != (p.history_len + 1) * p.num_proprio) {
      snprintf(msg, sizeof msg, "num_observations %d != (history_buffer_length + 1) * num_proprio = %d", p.num_obs,
               (p.history_len + 1) * p.num_proprio);
      return fail(env, msg);
    }
    if (p.task_kind == LGX_TASK_GO2 &&
        (p.num_priv != 5 + 2 * D || p.num_est != 3 || p.num_scan > p.num_height_points ||
         p.num_critic != p.num_obs + p.num_priv + p.num_est + p.num_scan))
      return fail(env, "Go2 privileged/estimated/scan/critic observation sizes do not match the step's layout");
    if (p.num_feet > LGX_MAX_FEET) return fail(env, "too many feet");
  }
  if (device < 0) {  // host backend: no device state; every buffer is host memory
    env->host = true;
    return 0;
  }
  HIP_OK(hipSetDevice(device));
  HIP_OK(hipMalloc(&env->d_model, sizeof(lgx_model)));
  HIP_OK(hipMalloc(&env->d_params, sizeof(lgx_task_params)));
  HIP_OK(hipMalloc(&env->d_buffers, sizeof(lgx_buffers)));
  HIP_OK(hipMemcpy(env->d_model, model, sizeof(lgx_model), hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(env->d_params, params, sizeof(lgx_task_params), hipMemcpyHostToDevice));
  return 0;
}

int lgx_bind(lgx_env* env, const lgx_buffers* b) {
  if (!env || !b) return -2;
  static const char* required[] = {"root_states", "dof_state", "contact_forces", "rigid_body_states", "actions_in",
                                   "actions", "torques", "last_actions", "last_dof_vel", "last_root_vel",
                                   "last_base_lin_vel", "last_torques", "commands", "episode_length",
                                   "episode_sums", "obs_history", "obs", "rew", "reset", "time_out", "env_origins"};
  const void* ptrs[] = {b->root_states, b->dof_state, b->contact_forces, b->rigid_body_states, b->actions_in,
                        b->actions, b->torques, b->last_actions, b->last_dof_vel, b->last_root_vel,
                        b->last_base_lin_vel, b->last_torques, b->commands, b->episode_length,
                        b->episode_sums, b->obs_history, b->obs, b->rew, b->reset, b->time_out, b->env_origins};
  for (size_t i = 0; i < sizeof(ptrs) / sizeof(ptrs[0]); ++i)
    if (!ptrs[i]) return fail(env, std::string("lgx_bind: required buffer missing: ") + required[i]);
  if (env->params.task_kind == LGX_TASK_GO2) {
    if (!b->priv || !b->est || !b->scan || !b->critic || !b->last_contacts || !b->last_contact_heights ||
        !b->mass_params || !b->friction)
      return fail(env, "lgx_bind: Go2 task needs priv/est/scan/critic/last_contacts/last_contact_heights/mass_params/friction");
  }
  if (env->params.mesh_type != LGX_MESH_PLANE) {
    if (!b->height_samples || !b->terrain_mesh)
      return fail(env, "lgx_bind: heightfield/trimesh terrain needs height_samples and terrain_mesh");
    if (env->params.hf_rows < 2 || env->params.hf_cols < 2) return fail(env, "lgx_bind: terrain smaller than 2x2");
  }
  if (env->params.actuator_net && (!b->sea_hidden || !b->sea_cell))
    return fail(env, "lgx_bind: the actuator network needs sea_hidden/sea_cell [2, N*D, 8]");
  if (env->params.actuator_net &&
      ((reinterpret_cast<uintptr_t>(b->sea_hidden) | reinterpret_cast<uintptr_t>(b->sea_cell)) & 15))
    return fail(env, "lgx_bind: sea_hidden/sea_cell must be 16-byte aligned");
  if (env->params.curriculum && (!b->terrain_levels || !b->terrain_types || !b->terrain_origins))
    return fail(env, "lgx_bind: terrain curriculum needs terrain_levels/terrain_types/terrain_origins");
  env->buffers = *b;
  if (env->host) {
    env->bound = true;
    env->stats_clean = false;
    return 0;
  }
  HIP_OK(hipSetDevice(env->device));
  HIP_OK(hipMemcpy(env->d_buffers, b, sizeof(lgx_buffers), hipMemcpyHostToDevice));
  env->bound = true;
  env->stats_clean = false;
  return 0;
}

static int launch_step(lgx_env* env, uint64_t seed, uint64_t step, const uint64_t* step_dev, void* stream,
                       bool physics) {
  if (!env) return -2;
  if (!env->bound) return fail(env, "lgx_step before lgx_bind");
  hipStream_t st = (hipStream_t)stream;
  const int N = env->params.num_envs;
  const int KS = env->params.num_reward_terms + (env->params.has_termination_reward ? 1 : 0);
  if (env->host) {
    if (env->buffers.episode_stats && !env->stats_clean)
      for (int k = 0; k <= KS; ++k) env->buffers.episode_stats[k] = 0.f;
    env->stats_clean = false;
    lgxh::step(&env->model, &env->params, &env->buffers, seed, step_dev ? *step_dev : step, physics);
    return 0;
  }
  if (env->buffers.episode_stats && !env->stats_clean)
    HIP_OK(hipMemsetAsync(env->buffers.episode_stats, 0, sizeof(float) * (KS + 1), st));
  env->stats_clean = false;
  // compiled variants: the plane/PD path (the benchmark) carries no terrain or LSTM code. Two
  // envs per wave (EPW 2: 32 lanes each, lgx_env.hip grp_of_lane) by default on the plane with an
  // even env count (measured: Go2 4096 envs 184 -> 177 us); on a trimesh the one-env kernel is
  // faster (go2_parkour 8192 envs: 423 vs 491 us), so there EPW 2 only when asked for
  // (lgx_set_envs_per_wave); never with the actuator net (its LSTM lanes need the whole wave).
  // LGX_ENVS_PER_WAVE=1 selects one env per wave (A/B, tests)
  const bool terrain = env->params.mesh_type != LGX_MESH_PLANE, actnet = env->params.actuator_net != 0;
  static const int epw_env = [] {
    const char* v = LGX_DEV_KNOB("LGX_ENVS_PER_WAVE");
    return v && atoi(v) == 1 ? 1 : 2;
  }();
  const int want = env->epw ? env->epw : (terrain ? 1 : epw_env);
  const int epw = (!actnet && N % 2 == 0 && want == 2) ? 2 : 1;
  auto kern = epw == 2 ? (!physics ? lgx::env_step_kernel<false, false, false, 2>
                                   : (terrain ? lgx::env_step_kernel<true, true, false, 2>
                                              : lgx::env_step_kernel<true, false, false, 2>))
            : !physics ? lgx::env_step_kernel<false, false, false, 1>
            : actnet   ? (terrain ? lgx::env_step_kernel<true, true, true, 1> : lgx::env_step_kernel<true, false, true, 1>)
                       : (terrain ? lgx::env_step_kernel<true, true, false, 1> : lgx::env_step_kernel<true, false, false, 1>);
  const size_t dyn = sizeof(float) * (size_t)lgx::arena_floats(env->params) * epw;
  hipLaunchKernelGGL(kern, dim3(N / epw), dim3(64), dyn, st, env->d_model, env->d_params, env->d_buffers, seed, step,
                     step_dev);
  HIP_OK(hipGetLastError());
  return 0;
}

int lgx_set_envs_per_wave(lgx_env* env, int32_t envs_per_wave) {
  if (!env) return -2;
  if (envs_per_wave < 0 || envs_per_wave > 2) return fail(env, "lgx_set_envs_per_wave: 0, 1 or 2");
  env->epw = envs_per_wave;
  return 0;
}

int lgx_step(lgx_env* env, uint64_t seed, uint64_t step_counter, void* hip_stream) {
  return launch_step(env, seed, step_counter, nullptr, hip_stream, true);
}

int lgx_step_dev(lgx_env* env, uint64_t seed, const uint64_t* d_step_counter, void* hip_stream) {
  if (!d_step_counter) return fail(env, "lgx_step_dev: null step counter");
  return launch_step(env, seed, 0, d_step_counter, hip_stream, true);
}

int lgx_post_physics(lgx_env* env, uint64_t seed, uint64_t step_counter, void* hip_stream) {
  return launch_step(env, seed, step_counter, nullptr, hip_stream, false);
}

int lgx_physics(lgx_env* env, void* hip_stream) {
  (void)hip_stream;
  return fail(env, "lgx_physics: use lgx_step (physics is fused with the post-physics pass)");
}

int lgx_reset_envs(lgx_env* env, const uint8_t* env_mask, uint64_t seed, uint64_t reset_call, void* hip_stream) {
  if (!env) return -2;
  if (!env->bound) return fail(env, "lgx_reset_envs before lgx_bind");
  if (!env_mask) return fail(env, "lgx_reset_envs: env_mask is NULL");
  hipStream_t st = (hipStream_t)hip_stream;
  const int KS = env->params.num_reward_terms + (env->params.has_termination_reward ? 1 : 0);
  if (env->host) {
    if (env->buffers.episode_stats && !env->stats_clean)
      for (int k = 0; k <= KS; ++k) env->buffers.episode_stats[k] = 0.f;
    env->stats_clean = false;
    lgxh::reset(&env->params, &env->buffers, env_mask, seed, reset_call);
    return 0;
  }
  if (env->buffers.episode_stats && !env->stats_clean)
    HIP_OK(hipMemsetAsync(env->buffers.episode_stats, 0, sizeof(float) * (KS + 1), st));
  env->stats_clean = false;
  const size_t dyn = sizeof(float) * (size_t)lgx::arena_floats(env->params);
  hipLaunchKernelGGL(lgx::reset_kernel, dim3(env->params.num_envs), dim3(64), dyn, st, env->d_params,
                     env->d_buffers, env_mask, seed, reset_call);
  HIP_OK(hipGetLastError());
  return 0;
}

namespace lgx {
// extras['episode'] / extras['time_outs'] (go2.py:246-263, Appendix B Q5 stale values):
// one block; thread k < K forms the episode mean of reward term k, the block reduces
// any(reset) and the mean terrain level, then time_outs is refreshed when any env reset.
// The statistics are consumed (zeroed for the next step, which then needs no memset) and
// the device step counter, if given, advances for the next lgx_step_dev.
__global__ __launch_bounds__(1024) void extras_kernel(float* __restrict__ stats, uint64_t* __restrict__ step_dev,
                                                      int K, float inv_T, int N,
                                                      const uint8_t* __restrict__ reset,
                                                      const uint8_t* __restrict__ time_out,
                                                      const int64_t* __restrict__ levels, float* __restrict__ means,
                                                      float* __restrict__ level_mean, uint8_t* __restrict__ time_outs) {
  __shared__ int any_s;
  __shared__ double lsum[16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) any_s = 0;
  __syncthreads();
  const float cnt = stats[K];
  if (tid < K && cnt > 0.f) means[tid] = stats[tid] / cnt * inv_T;
  int any = 0;
  double ls = 0.0;
  for (int i = tid; i < N; i += blockDim.x) {
    if (reset) any |= reset[i];
    if (levels) ls += (double)levels[i];
  }
  if (reset && __any(any)) {
    if (lane == 0) atomicOr(&any_s, 1);
  }
  if (levels) {
    for (int o = 32; o > 0; o >>= 1) ls += __shfl_down(ls, o, 64);
    if (lane == 0) lsum[wv] = ls;
  }
  __syncthreads();
  if (tid <= K) stats[tid] = 0.f;  // every thread read cnt before the barrier
  if (tid == 0 && step_dev) *step_dev += 1;
  if (levels && tid == 0 && cnt > 0.f) {
    double t = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += lsum[w];
    *level_mean = (float)(t / N);
  }
  if (time_outs && any_s)
    for (int i = tid; i < N; i += blockDim.x) time_outs[i] = time_out[i];
}
}  // namespace lgx

int lgx_episode_extras(lgx_env* env, float* means, float* level_mean, uint8_t* time_outs, uint64_t* step_dev,
                       void* hip_stream) {
  if (!env) return -2;
  if (!env->bound) return fail(env, "lgx_episode_extras before lgx_bind");
  const lgx_buffers& b = env->buffers;
  if (!b.episode_stats || !means) return fail(env, "lgx_episode_extras: episode_stats and means are required");
  if (level_mean && !b.terrain_levels) return fail(env, "lgx_episode_extras: level_mean needs terrain_levels");
  if (time_outs && (!b.reset || !b.time_out)) return fail(env, "lgx_episode_extras: time_outs needs reset/time_out");
  const int KS = env->params.num_reward_terms + (env->params.has_termination_reward ? 1 : 0);
  if (KS + 1 > 1024) return fail(env, "lgx_episode_extras: too many reward terms");
  if (env->host) {
    lgxh::episode_extras(&env->params, &b, means, level_mean, time_outs, step_dev);
    env->stats_clean = true;
    return 0;
  }
  hipStream_t st = (hipStream_t)hip_stream;
  // torch divides a tensor by a Python scalar as a multiply by the fp32 reciprocal
  hipLaunchKernelGGL(lgx::extras_kernel, dim3(1), dim3(1024), 0, st, b.episode_stats, step_dev, KS,
                     1.0f / env->params.max_episode_length_s, env->params.num_envs, time_outs ? b.reset : nullptr,
                     b.time_out, level_mean ? b.terrain_levels : nullptr, means, level_mean, time_outs);
  HIP_OK(hipGetLastError());
  env->stats_clean = true;
  return 0;
}

namespace lgx {
// One uniform of the env step's Philox table (fill_uniforms: slot = 4 * block + word).
LGX_DEV float step_uniform(uint64_t seed, uint32_t gid, uint64_t step, int slot) {
  uint32_t o[4];
  philox4x32_10(gid, (uint32_t)step, (uint32_t)(slot >> 2), (uint32_t)(step >> 32), (uint32_t)seed,
                (uint32_t)(seed >> 32), o);
  return u01(o[slot & 3]);
}

// update_command_curriculum (go2.py:80-107 / legged_robot.py:580-591) after a step: one block.
// The mean runs over the envs reset in this step (reset_idx's env_ids); their pre-reset
// tracking_lin_vel sums were left in curriculum_vals by the step kernel. When the range
// changes, the reset envs' commands are resampled again from the same uniforms with the new
// range (reset_idx resamples after the curriculum, go2.py:222-230) and the command entries of
// their observation rows are rewritten (a reset env's history is zero in obs and all copies of
// the current observation in obs_history, go2.py:570-574).
__global__ __launch_bounds__(1024) void curriculum_kernel(const lgx_task_params* __restrict__ Pm,
                                                          const lgx_buffers* __restrict__ Bp, uint64_t seed,
                                                          uint64_t step_arg, const uint64_t* __restrict__ step_dev,
                                                          const double* __restrict__ global_sc) {
  const lgx_buffers& B = *Bp;
  const uint64_t step = step_dev ? *step_dev : step_arg;
  if (step % (uint64_t)Pm->max_episode_length != 0) return;
  __shared__ double red_s[16], red_c[16];
  __shared__ int changed;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, N = Pm->num_envs;
  double sm = 0.0, ct = 0.0;
  if (!global_sc)
    for (int i = tid; i < N; i += blockDim.x)
      if (B.reset[i]) { sm += (double)B.curriculum_vals[i]; ct += 1.0; }
  for (int o = 32; o > 0; o >>= 1) { sm += __shfl_down(sm, o, 64); ct += __shfl_down(ct, o, 64); }
  if (lane == 0) { red_s[wv] = sm; red_c[wv] = ct; }
  __syncthreads();
  if (tid == 0) {
    double S = 0.0, Cn = 0.0;
    if (global_sc) { S = global_sc[0]; Cn = global_sc[1]; }
    else
      for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { S += red_s[w]; Cn += red_c[w]; }
    int ch = 0;
    // torch.mean (fp32) / max_episode_length, compared in fp32 (no reset: reset_idx returns early)
    const float mean = Cn > 0.0 ? ((float)S / (float)Cn) / (float)Pm->max_episode_length : 0.f;
    if (Cn > 0.0 && mean > Pm->curriculum_threshold) {
      double* R = B.command_ranges;
      const double lo = R[0], hi = R[1], d = Pm->curriculum_delta;
      const double lo_max = Pm->curriculum_lo_free ? lo - d : Pm->curriculum_lo_max;
      const double nlo = fmin(fmax(lo - d, Pm->curriculum_lo_min), lo_max);  // np.clip
      const double nhi = fmin(fmax(hi + d, 0.0), Pm->curriculum_hi_max);
      ch = (nlo != lo) || (nhi != hi);
      R[0] = nlo;
      R[1] = nhi;
      float* L = B.command_range_log;
      if (L) {
        if (Pm->command_curriculum == 1) { L[0] = (float)nhi; L[1] = (float)nlo; L[2] = (float)R[3]; L[3] = (float)R[5]; }
        else { L[0] = (float)nhi; L[1] = (float)R[3]; L[2] = (float)R[5]; }
      }
    }
    changed = ch;
  }
  __syncthreads();
  if (!changed) return;
  const bool go2 = Pm->task_kind == LGX_TASK_GO2;
  const int Pp = Pm->num_proprio, H = Pm->history_len, c0 = go2 ? 5 : 9;
  const float co = Pm->clip_obs;
  for (int e = tid; e < N; e += blockDim.x) {
    if (!B.reset[e]) continue;
    const uint32_t gid = (uint32_t)(Pm->env_id_offset + e);
    float U[4];  // the reset's command draws (slots S_RCMD..+3)
    for (int k = 0; k < 4; ++k) U[k] = step_uniform(seed, gid, step, S_RCMD + k);
    float cmd[4];
    for (int k = 0; k < 4; ++k) cmd[k] = B.commands[e * 4 + k];
    const float* quat = B.root_states + (size_t)e * 13 + 3;
    resample_commands(Pm, B.command_ranges, cmd, U, 0, quat);
    for (int k = 0; k < 4; ++k) B.commands[e * 4 + k] = cmd[k];
    float* obs = B.obs + (size_t)e * Pm->num_obs;
    float* cr = (go2 && B.critic) ? B.critic + (size_t)e * Pm->num_critic : nullptr;
    float* hist = B.obs_history + (size_t)e * H * Pp;
    for (int j = 0; j < 3; ++j) {
      const int i = c0 + j;
      float v = cmd[j] * Pm->commands_scale[j];
      if (Pm->add_noise) v = v + (2.0f * step_uniform(seed, gid, step, S_NOISE + i) - 1.0f) * Pm->noise_vec[i];
      const float vc = clipf(v, -co, co);
      obs[H * Pp + i] = vc;
      if (cr) cr[H * Pp + i] = vc;
      for (int t = 0; t < H; ++t) hist[t * Pp + i] = v;  // reset env: every history row = current obs
    }
  }
}
}  // namespace lgx

int lgx_command_curriculum(lgx_env* env, uint64_t seed, uint64_t step_counter, const uint64_t* d_step_counter,
                           const double* global_sum_count, void* hip_stream) {
  if (!env) return -2;
  if (!env->bound) return fail(env, "lgx_command_curriculum before lgx_bind");
  const lgx_buffers& b = env->buffers;
  if (!env->params.command_curriculum) return fail(env, "lgx_command_curriculum: params.command_curriculum is 0");
  if (!b.command_ranges || !b.curriculum_vals || !b.reset || !b.commands || !b.obs || !b.obs_history)
    return fail(env, "lgx_command_curriculum: command_ranges, curriculum_vals, reset, commands, obs, obs_history "
                     "must be bound");
  if (env->host) {
    lgxh::command_curriculum(&env->params, &b, seed, d_step_counter ? *d_step_counter : step_counter,
                             global_sum_count);
    return 0;
  }
  hipLaunchKernelGGL(lgx::curriculum_kernel, dim3(1), dim3(1024), 0, (hipStream_t)hip_stream, env->d_params,
                     env->d_buffers, seed, step_counter, d_step_counter, global_sum_count);
  HIP_OK(hipGetLastError());
  return 0;
}

#ifdef LGX_PHASE_CLOCK
// dev builds only: per-env phase cycle counters ([num_envs][16] uint32, device memory)
int lgx_debug_phase_buffer(uint32_t* dev_ptr) {
  return hipMemcpyToSymbol(HIP_SYMBOL(lgx::g_phase_out), &dev_ptr, sizeof(dev_ptr)) == hipSuccess ? 0 : -1;
}
#endif

const char* lgx_last_error(const lgx_env* env) { return env ? env->err.c_str() : "null env"; }

void lgx_destroy(lgx_env* env) {
  if (!env) return;
  if (env->host) {
    delete env;
    return;
  }
  if (env->d_model) (void)hipFree(env->d_model);
  if (env->d_params) (void)hipFree(env->d_params);
  if (env->d_buffers) (void)hipFree(env->d_buffers);
  delete env;
}

}  // extern "C"
