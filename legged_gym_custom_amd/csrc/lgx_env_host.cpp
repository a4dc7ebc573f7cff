// lgx_env_host.cpp — host (CPU) backend of the env step behind include/lgx.h
// (lgx_create(device = -1); the reference's `--sim_device=cpu`, helpers.py:174-177, config
// C1). Same entry points, buffers and semantics as the HIP kernels of lgx_env.hip; the
// algorithm is the kernel's (DESIGN.md §3 physics spec), laid out for a CPU core:
//   * one OpenMP thread steps one env at a time (dynamic schedule: contact counts vary);
//   * the env's working set (`Env`, ~25 KB with the dense constraint matrix) stays in the
//     thread's L1/L2 for the whole step, as the kernel keeps it in LDS;
//   * the kernel's lane-parallel phases become short loops in the kernel's order: links
//     base-to-tip, joints 0..11, constraint rows [joint limits | 3 per contact];
//   * the constraint solve always uses the dense A = J M⁻¹ Jᵀ (the kernel switches to a
//     velocity-space sweep above 24 rows to bound LDS; both are the same Gauss-Seidel).
// Post-physics follows legged_robot.py / go2.py statement order with no fp contraction
// (built with -ffp-contract=off), like the kernel's golden-pinned tail.
#include <math.h>
#include <cmath>
#include <omp.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "lgx_host.h"

namespace lgxh {

constexpr int NL = 13, NJ = 12, NU = 18;
constexpr int MAXC = LGX_MAX_CONTACTS;
constexpr int MAXR = NJ + 3 * MAXC;
constexpr int NBLK_MAX = 9 + (LGX_MAX_PROPRIO + 3) / 4;
constexpr int MAXHIST = 1216;
enum Slot { S_CMD = 0, S_PUSH = 4, S_TERR = 6, S_DOF = 8, S_ROOT_XY = 20, S_ROOT_VEL = 24, S_RCMD = 32, S_NOISE = 36 };

// ------------------------------------------------------------------ small math
struct v3 {
  float x, y, z;
};
static inline v3 V(float x, float y, float z) { return v3{x, y, z}; }
static inline v3 L3(const float* p) { return v3{p[0], p[1], p[2]}; }
static inline void S3(float* p, v3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }
static inline v3 operator+(v3 a, v3 b) { return v3{a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline v3 operator-(v3 a, v3 b) { return v3{a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline v3 operator*(v3 a, float s) { return v3{a.x * s, a.y * s, a.z * s}; }
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 cross(v3 a, v3 b) { return v3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
static inline v3 rot(const float* R, v3 v) {  // row-major 3x3 times v
  return v3{R[0] * v.x + R[1] * v.y + R[2] * v.z, R[3] * v.x + R[4] * v.y + R[5] * v.z,
            R[6] * v.x + R[7] * v.y + R[8] * v.z};
}
static inline void matmul3(const float* A, const float* B, float* O) {
  float T[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T[i * 3 + j] = A[i * 3] * B[j] + A[i * 3 + 1] * B[3 + j] + A[i * 3 + 2] * B[6 + j];
  memcpy(O, T, sizeof(T));
}
static inline v3 symmul(const float* I, v3 v) {  // symmetric (xx yy zz xy xz yz) times v
  return v3{I[0] * v.x + I[3] * v.y + I[4] * v.z, I[3] * v.x + I[1] * v.y + I[5] * v.z,
            I[4] * v.x + I[5] * v.y + I[2] * v.z};
}
static inline void quat_R(const float* q, float* R) {
  const float x = q[0], y = q[1], z = q[2], w = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - z * w); R[2] = 2 * (x * z + y * w);
  R[3] = 2 * (x * y + z * w); R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - x * w);
  R[6] = 2 * (x * z - y * w); R[7] = 2 * (y * z + x * w); R[8] = 1 - 2 * (x * x + y * y);
}
static inline void sym3_inverse(const float* D, float* O) {
  const float a = D[0], b = D[1], c = D[2], d = D[3], e = D[4], f = D[5];
  const float A = b * c - f * f, Bm = -(d * c - e * f), Cm = d * f - b * e;
  const float inv = 1.0f / (a * A + d * Bm + e * Cm);
  O[0] = A * inv; O[1] = (a * c - e * e) * inv; O[2] = (a * b - d * d) * inv;
  O[3] = Bm * inv; O[4] = Cm * inv; O[5] = -(a * f - d * e) * inv;
}
static inline float sym3_at(const float* S, int i, int j) {
  if (i == j) return S[i];
  const int k = i + j;
  return S[k == 1 ? 3 : (k == 2 ? 4 : 5)];
}
static inline int pk6(int i, int j) { return i >= j ? i * (i + 1) / 2 + j : j * (j + 1) / 2 + i; }

// Philox4x32-10 (oracle/philox.py layout: c0 = global env id, c1/c3 = step lo/hi,
// c2 = block | stream << 16, key = seed)
static inline void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                          uint32_t out[4]) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0, p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c0 = n0; c1 = (uint32_t)p1; c2 = n2; c3 = (uint32_t)p0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}
static inline float unit(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// ------------------------------------------------------------------ per-env state
struct Link {
  float R[9], P[3], ax[3], W[3], V[3], C[3], I[6], m, F[3], N[3];
};
struct Env {
  // physics (base velocity held as the ORIGIN velocity inside the step)
  float qb[4], pb[3], vo[3], wb[3];
  float th[NJ], thd[NJ], tau[NJ], act[NJ], kpm[NJ], kdm[NJ], ldv[NJ];
  float madd, cadd[3], mu;
  Link lk[NL];
  float tot[16];                               // base sums about p0: m, h(3), Ip(6), F(3), N(3)
  float hj[NJ], Bc[NJ][6], Dl[4][6], Dinv[4][6], X[NJ][6], Sinv[6][6], hb[6];
  float us[NU], up[NU];
  int nrows, nlim, ncon;
  float J[MAXR][9], ZG[MAXR][9];               // sparse rows [base 6 | leg 3]; z_r (6) | g_r (3)
  float Arr[MAXR], tgt[MAXR], lam[MAXR], w[MAXR];
  int rleg[MAXR];
  int cbody[MAXC];
  float cn[MAXC][3];
  float A[MAXR * MAXR];
  float cf[LGX_MAX_BODIES][3], rbz[LGX_MAX_BODIES];
  // post-physics
  float root[13], cmd[4], U[4 * NBLK_MAX];
  float blv[3], bav[3], pg[3], roll, pitch, yaw, ph[4], feet_z[4], jump;
  int contact[4], lc[4];
  float lch[4], fat[4];
  float cur[LGX_MAX_PROPRIO], hist[MAXHIST], heights[LGX_MAX_HEIGHT_POINTS];
  float jsum[16], rterm[64];
  long long ep;
  int reset, tout;
};

// ------------------------------------------------------------------ kinematics
// Links base to tip (chain position 0..2 of each leg after the base): world rotation,
// origin, joint axis, angular velocity, COM; with BIAS the velocity-product accelerations
// and per-link COM wrench plus the 16 base sums about p0; without, the origin velocities.
template <bool BIAS>
static void kinematics(Env& s, const lgx_model* M, const lgx_task_params* P) {
  float Al[NL][3], Ao[NL][3];
  {
    Link& b = s.lk[0];
    quat_R(s.qb, b.R);
    S3(b.P, L3(s.pb)); S3(b.ax, V(0, 0, 0)); S3(b.W, L3(s.wb)); S3(b.V, L3(s.vo));
    S3(Al[0], V(0, 0, 0)); S3(Ao[0], V(0, 0, 0));
  }
  for (int j = 0; j < NJ; ++j) {
    const int k = j + 1, par = (j % 3 == 0) ? 0 : j;
    const Link& p = s.lk[par];
    Link& c = s.lk[k];
    const v3 orig = L3(M->joint_origin[k]), al = L3(M->joint_axis[k]);
    const float* Rj = M->joint_rot[k];
    const float th = s.th[j], ct = cosf(th), st = sinf(th), t1 = 1.f - ct;
    const float Ra[9] = {t1 * al.x * al.x + ct, t1 * al.x * al.y - st * al.z, t1 * al.x * al.z + st * al.y,
                         t1 * al.x * al.y + st * al.z, t1 * al.y * al.y + ct, t1 * al.y * al.z - st * al.x,
                         t1 * al.x * al.z - st * al.y, t1 * al.y * al.z + st * al.x, t1 * al.z * al.z + ct};
    float Rl[9];
    matmul3(Rj, Ra, Rl);
    const v3 o = rot(p.R, orig), ax = rot(p.R, rot(Rj, al));
    matmul3(p.R, Rl, c.R);
    const v3 Wp = L3(p.W), wa = ax * s.thd[j];
    S3(c.P, L3(p.P) + o);
    S3(c.ax, ax);
    S3(c.W, Wp + wa);
    if constexpr (BIAS) {
      S3(Al[k], L3(Al[par]) + cross(Wp, wa));
      S3(Ao[k], L3(Ao[par]) + cross(L3(Al[par]), o) + cross(Wp, cross(Wp, o)));
    } else {
      S3(c.V, L3(p.V) + cross(Wp, o));
    }
  }
  const v3 g = L3(P->gravity), p0 = L3(s.pb);
  if constexpr (BIAS) memset(s.tot, 0, sizeof(s.tot));
  for (int k = 0; k < NL; ++k) {
    Link& c = s.lk[k];
    const float cb = k == 0 ? 1.f : 0.f;
    const float* cl = M->link_com[k];
    const v3 C = L3(c.P) + rot(c.R, V(cl[0] + cb * s.cadd[0], cl[1] + cb * s.cadd[1], cl[2] + cb * s.cadd[2]));
    S3(c.C, C);
    if constexpr (BIAS) {
      const float m = M->link_mass[k] + cb * s.madd;
      const float* In = M->link_inertia[k];
      const float Il[9] = {In[0], In[3], In[4], In[3], In[1], In[5], In[4], In[5], In[2]};
      const float* R = c.R;
      float T[9];
      matmul3(R, Il, T);
      float* Iw = c.I;
      Iw[0] = T[0] * R[0] + T[1] * R[1] + T[2] * R[2];
      Iw[1] = T[3] * R[3] + T[4] * R[4] + T[5] * R[5];
      Iw[2] = T[6] * R[6] + T[7] * R[7] + T[8] * R[8];
      Iw[3] = T[0] * R[3] + T[1] * R[4] + T[2] * R[5];
      Iw[4] = T[0] * R[6] + T[1] * R[7] + T[2] * R[8];
      Iw[5] = T[3] * R[6] + T[4] * R[7] + T[5] * R[8];
      c.m = m;
      const v3 W = L3(c.W), al = L3(Al[k]), rl = C - L3(c.P);
      const v3 acc = L3(Ao[k]) + cross(al, rl) + cross(W, cross(W, rl));
      const v3 F = (acc - g) * m, N = symmul(Iw, al) + cross(W, symmul(Iw, W));
      S3(c.F, F);
      S3(c.N, N);
      const v3 r = C - p0;
      const float rr = dot(r, r);
      const v3 Nt = cross(r, F) + N;
      const float rd[16] = {m, m * r.x, m * r.y, m * r.z,
                            Iw[0] + m * (rr - r.x * r.x), Iw[1] + m * (rr - r.y * r.y), Iw[2] + m * (rr - r.z * r.z),
                            Iw[3] - m * r.x * r.y, Iw[4] - m * r.x * r.z, Iw[5] - m * r.y * r.z,
                            F.x, F.y, F.z, Nt.x, Nt.y, Nt.z};
      for (int q = 0; q < 16; ++q) s.tot[q] += rd[q];
    }
  }
}

// Mass matrix M = [A B; Bᵀ D] (D block diagonal over the legs) and bias h, factored:
// X = B D⁻¹, S = A − X Bᵀ (base Schur complement), S⁻¹ — lgx_env.hip `dynamics`.
static void dynamics(Env& s) {
  const v3 p0 = L3(s.lk[0].P);
  for (int j = 0; j < NJ; ++j) {
    const int l = j / 3, a = j % 3;
    const Link& lj = s.lk[1 + j];
    const v3 ax = L3(lj.ax), pj = L3(lj.P);
    v3 acc = V(0, 0, 0), hl = V(0, 0, 0), bang = V(0, 0, 0);
    for (int i = a; i < 3; ++i) {
      const Link& c = s.lk[1 + 3 * l + i];
      const v3 C = L3(c.C), d = C - pj;
      acc = acc + cross(d, L3(c.F)) + L3(c.N);
      hl = hl + d * c.m;
      bang = bang + cross(C - p0, cross(ax, d)) * c.m + symmul(c.I, ax);
    }
    s.hj[j] = dot(ax, acc);
    const v3 blin = cross(ax, hl);
    float* Bj = s.Bc[j];
    Bj[0] = blin.x; Bj[1] = blin.y; Bj[2] = blin.z; Bj[3] = bang.x; Bj[4] = bang.y; Bj[5] = bang.z;
  }
  for (int l = 0; l < 4; ++l) {
    for (int e = 0; e < 6; ++e) {
      const int j1 = e < 3 ? e : (e == 5 ? 1 : 0), j2 = e < 3 ? e : (e == 3 ? 1 : 2);
      const Link& k1 = s.lk[1 + 3 * l + j1];
      const Link& k2 = s.lk[1 + 3 * l + j2];
      const v3 a1 = L3(k1.ax), a2 = L3(k2.ax), q1 = L3(k1.P), q2 = L3(k2.P);
      float acc = 0.f;
      for (int i = j2; i < 3; ++i) {
        const Link& c = s.lk[1 + 3 * l + i];
        const v3 C = L3(c.C);
        acc += c.m * dot(cross(a1, C - q1), cross(a2, C - q2)) + dot(a1, symmul(c.I, a2));
      }
      s.Dl[l][e] = acc;
    }
    sym3_inverse(s.Dl[l], s.Dinv[l]);
  }
  for (int j = 0; j < NJ; ++j) {
    const int l = j / 3, a = j % 3;
    const float d0 = sym3_at(s.Dinv[l], a, 0), d1 = sym3_at(s.Dinv[l], a, 1), d2 = sym3_at(s.Dinv[l], a, 2);
    for (int r = 0; r < 6; ++r) s.X[j][r] = d0 * s.Bc[3 * l][r] + d1 * s.Bc[3 * l + 1][r] + d2 * s.Bc[3 * l + 2][r];
  }
  const float* t = s.tot;
  const float Mt = t[0], Hx = t[1], Hy = t[2], Hz = t[3];
  const float Ab[21] = {Mt, 0.f, Mt, 0.f, 0.f, Mt, 0.f, -Hz, Hy, t[4], Hz, 0.f, -Hx, t[7], t[5],
                        -Hy, Hx, 0.f, t[8], t[9], t[6]};
  float L[21];
  for (int q = 0; q < 21; ++q) {
    const int r = (q >= 1) + (q >= 3) + (q >= 6) + (q >= 10) + (q >= 15), c = q - r * (r + 1) / 2;
    float acc = 0.f;
    for (int j = 0; j < NJ; ++j) acc += s.X[j][r] * s.Bc[j][c];
    L[q] = Ab[q] - acc;
  }
  float inv[6];
  for (int c = 0; c < 6; ++c) {  // Cholesky S = L Lᵀ (packed lower)
    float d = L[pk6(c, c)];
    for (int k = 0; k < c; ++k) d -= L[pk6(c, k)] * L[pk6(c, k)];
    inv[c] = 1.0f / sqrtf(fmaxf(d, 1e-12f));
    for (int r = c + 1; r < 6; ++r) {
      float v = L[pk6(r, c)];
      for (int k = 0; k < c; ++k) v -= L[pk6(r, k)] * L[pk6(c, k)];
      L[pk6(r, c)] = v * inv[c];
    }
  }
  for (int col = 0; col < 6; ++col) {  // S⁻¹ e_col
    float x[6];
    for (int r = 0; r < 6; ++r) {
      float v = r == col ? 1.f : 0.f;
      for (int k = 0; k < r; ++k) v -= L[pk6(r, k)] * x[k];
      x[r] = v * inv[r];
    }
    for (int r = 5; r >= 0; --r) {
      float v = x[r];
      for (int k = r + 1; k < 6; ++k) v -= L[pk6(k, r)] * x[k];
      x[r] = v * inv[r];
    }
    for (int r = 0; r < 6; ++r) s.Sinv[col][r] = x[r];
  }
  for (int q = 0; q < 6; ++q) s.hb[q] = t[10 + q];
}

// ------------------------------------------------------------------ terrain contact
// The reference's trimesh (terrain_utils.py:382-465) rebuilt per query from the packed
// per-vertex words (height | wall shift), as lgx_env.hip terrain_contact.
static inline v3 mesh_vertex(const uint32_t* mesh, int cols, int i, int j, int ci, int cj, float hs, float vs) {
  const uint32_t w = mesh[(size_t)i * cols + j];
  const float h = (float)(int16_t)(w & 0xffffu);
  const int dx = (int)((w >> 16) & 3u) - 1, dy = (int)((w >> 18) & 3u) - 1;
  return V((float)(i - ci + dx) * hs, (float)(j - cj + dy) * hs, h * vs);
}
static v3 closest_on_triangle(v3 p, v3 a, v3 b, v3 c) {  // Ericson 5.1.5
  const v3 ab = b - a, ac = c - a, ap = p - a;
  const float d1 = dot(ab, ap), d2 = dot(ac, ap);
  if (d1 <= 0.f && d2 <= 0.f) return a;
  const v3 bp = p - b;
  const float d3 = dot(ab, bp), d4 = dot(ac, bp);
  if (d3 >= 0.f && d4 <= d3) return b;
  const float vc = d1 * d4 - d3 * d2;
  if (vc <= 0.f && d1 >= 0.f && d3 <= 0.f) return a + ab * (d1 / fmaxf(d1 - d3, 1e-30f));
  const v3 cp = p - c;
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
static bool height_in_triangle(v3 p, v3 a, v3 b, v3 c, float& z) {
  const float e1x = b.x - a.x, e1y = b.y - a.y, e2x = c.x - a.x, e2y = c.y - a.y;
  const float det = e1x * e2y - e1y * e2x;
  if (fabsf(det) < 1e-10f) return false;
  const float px = p.x - a.x, py = p.y - a.y;
  const float u = (px * e2y - py * e2x) / det, v = (e1x * py - e1y * px) / det;
  const float eps = -1e-6f;
  if (u < eps || v < eps || u + v > 1.0f - eps) return false;
  z = a.z + u * (b.z - a.z) + v * (c.z - a.z);
  return true;
}
// penetration depth (> 0 overlapping) and unit normal (terrain -> sphere) at x, radius r
static float terrain_contact(const lgx_task_params* P, const lgx_buffers* B, v3 x, float r, v3& n) {
  const float hs = P->horizontal_scale, vs = P->vertical_scale;
  const int rows = P->hf_rows, cols = P->hf_cols;
  const float gx = x.x + P->border_size, gy = x.y + P->border_size;
  const int ci = (int)floorf(gx / hs), cj = (int)floorf(gy / hs);
  const v3 p = V(gx - (float)ci * hs, gy - (float)cj * hs, x.z);
  const int i0 = std::max(ci + (int)ceilf((p.x - r) / hs) - 2, 0), i1 = std::min(ci + (int)floorf((p.x + r) / hs) + 1, rows - 2);
  const int j0 = std::max(cj + (int)ceilf((p.y - r) / hs) - 2, 0), j1 = std::min(cj + (int)floorf((p.y + r) / hs) + 1, cols - 2);
  float best = 3.0e38f, zs = -3.0e38f;
  v3 q = V(0.f, 0.f, -3.0e38f), fn = V(0.f, 0.f, 1.f);
  for (int i = i0; i <= i1; ++i)
    for (int j = j0; j <= j1; ++j) {
      const v3 v00 = mesh_vertex(B->terrain_mesh, cols, i, j, ci, cj, hs, vs);
      const v3 v01 = mesh_vertex(B->terrain_mesh, cols, i, j + 1, ci, cj, hs, vs);
      const v3 v10 = mesh_vertex(B->terrain_mesh, cols, i + 1, j, ci, cj, hs, vs);
      const v3 v11 = mesh_vertex(B->terrain_mesh, cols, i + 1, j + 1, ci, cj, hs, vs);
      for (int t = 0; t < 2; ++t) {
        const v3 a = v00, b = t == 0 ? v11 : v10, c = t == 0 ? v01 : v11;
        const v3 cp = closest_on_triangle(p, a, b, c), d = p - cp;
        const float d2 = dot(d, d);
        if (d2 < best) { best = d2; q = cp; fn = cross(b - a, c - a); }
        float z;
        if (height_in_triangle(p, a, b, c, z)) zs = fmaxf(zs, z);
      }
    }
  if (best >= 3.0e38f) {
    n = V(0.f, 0.f, 1.f);
    return -3.0e38f;
  }
  const float dist = sqrtf(best);
  const bool below = p.z < zs;
  n = dist > 1e-6f ? (p - q) * ((below ? -1.0f : 1.0f) / dist) : fn * (1.0f / sqrtf(fmaxf(dot(fn, fn), 1e-30f)));
  return below ? r + dist : r - dist;
}
static void tangents(v3 n, v3& t1, v3& t2) {
  v3 a = V(n.z, 0.f, -n.x);
  float l2 = a.x * a.x + a.z * a.z;
  if (l2 < 1e-8f) {
    a = V(0.f, n.z, -n.y);
    l2 = a.y * a.y + a.z * a.z;
  }
  t1 = a * (1.0f / sqrtf(l2));
  t2 = cross(n, t1);
}

// ------------------------------------------------------------------ SEA actuator net
// anymal.py:71-81: 2-layer LSTM(2 -> 8 -> 8) (gates i f g o), Linear(8 -> 1); state
// [2, N*D, 8] in the caller's buffers.
static inline float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }
static void lstm_cell(const float* w_ih, int nin, const float* w_hh, const float* b_ih, const float* b_hh,
                      const float* x, float* h, float* c) {
  float hn[8];
  for (int u = 0; u < 8; ++u) {
    float g4[4];
    for (int q = 0; q < 4; ++q) {
      const int g = q * 8 + u;
      float a = 0.0f, b = 0.0f;
      for (int k = 0; k < nin; ++k) a += w_ih[g * nin + k] * x[k];
      for (int k = 0; k < 8; ++k) b += w_hh[g * 8 + k] * h[k];
      g4[q] = (a + b_ih[g]) + (b + b_hh[g]);
    }
    c[u] = sigm(g4[1]) * c[u] + sigm(g4[0]) * tanhf(g4[2]);
    hn[u] = sigm(g4[3]) * tanhf(c[u]);
  }
  memcpy(h, hn, sizeof(hn));
}
static float sea_torque(const lgx_task_params* P, const lgx_buffers* B, int e, int j, float in0, float in1) {
  const size_t NT = (size_t)P->num_envs * P->num_dof, r = (size_t)e * P->num_dof + j;
  float* h0 = B->sea_hidden + r * 8;
  float* c0 = B->sea_cell + r * 8;
  float* h1 = B->sea_hidden + (NT + r) * 8;
  float* c1 = B->sea_cell + (NT + r) * 8;
  const float x[2] = {in0 * P->sea_in_scale[0], in1 * P->sea_in_scale[1]};
  lstm_cell(P->sea_w_ih0, 2, P->sea_w_hh0, P->sea_b_ih0, P->sea_b_hh0, x, h0, c0);
  lstm_cell(P->sea_w_ih1, 8, P->sea_w_hh1, P->sea_b_ih1, P->sea_b_hh1, h0, h1, c1);
  float y = 0.0f;
  for (int k = 0; k < 8; ++k) y += P->sea_lin_w[k] * h1[k];
  return P->sea_out_scale * (y + P->sea_lin_b);
}

// ------------------------------------------------------------------ one physics substep
static void substep(Env& s, const lgx_model* M, const lgx_task_params* P, const lgx_buffers* B, int e, bool last) {
  const float dt = P->sim_dt;
  const bool terrain = P->mesh_type != LGX_MESH_PLANE;
  // PD torques: LeggedRobot._compute_torques legged_robot.py:440-478 (or the SEA net)
  for (int j = 0; j < NJ; ++j) {
    const float as = s.act[j] * P->action_scale;
    if (P->actuator_net) {
      s.tau[j] = sea_torque(P, B, e, j, (as + P->default_dof_pos[j]) - s.th[j], s.thd[j]);
      continue;
    }
    float t;
    if (P->control_type == LGX_CONTROL_P) {
      const float err = (as + P->default_dof_pos[j]) - s.th[j];
      t = P->randomize_kp_kd ? (s.kpm[j] * P->p_gains[j]) * err - (s.kdm[j] * P->d_gains[j]) * s.thd[j]
                             : P->p_gains[j] * err - P->d_gains[j] * s.thd[j];
    } else if (P->control_type == LGX_CONTROL_V) {
      t = P->p_gains[j] * (as - s.thd[j]) - P->d_gains[j] * ((s.thd[j] - s.ldv[j]) / P->sim_dt);
    } else {
      t = as;
    }
    s.tau[j] = fminf(fmaxf(t, -P->torque_limits[j]), P->torque_limits[j]);
  }
  kinematics<true>(s, M, P);
  dynamics(s);
  // free velocity u* = u + dt M⁻¹ [−h_B ; τ − h_J]
  float fj[NJ], vb[6], zb[6];
  for (int j = 0; j < NJ; ++j) fj[j] = s.tau[j] - s.hj[j];
  for (int r = 0; r < 6; ++r) {
    float acc = 0.f;
    for (int j = 0; j < NJ; ++j) acc += s.X[j][r] * fj[j];
    vb[r] = -s.hb[r] - acc;
  }
  for (int r = 0; r < 6; ++r) {
    const float* Si = s.Sinv[r];
    zb[r] = Si[0] * vb[0] + Si[1] * vb[1] + Si[2] * vb[2] + Si[3] * vb[3] + Si[4] * vb[4] + Si[5] * vb[5];
  }
  for (int r = 0; r < 3; ++r) { s.us[r] = s.vo[r] + dt * zb[r]; s.us[3 + r] = s.wb[r] + dt * zb[3 + r]; }
  for (int j = 0; j < NJ; ++j) {
    const int l = j / 3, a = j % 3;
    const float* Di = s.Dinv[l];
    float bot = sym3_at(Di, a, 0) * fj[3 * l] + sym3_at(Di, a, 1) * fj[3 * l + 1] + sym3_at(Di, a, 2) * fj[3 * l + 2];
    for (int r = 0; r < 6; ++r) bot -= s.X[j][r] * zb[r];
    s.us[6 + j] = s.thd[j] + dt * bot;
  }
  // constraint rows: joint limits (joint order), then contacts (candidate order, <= MAXC)
  auto target = [&](float d) {
    if (d > P->slop) return fminf(P->baumgarte * (d - P->slop) / dt, P->max_depenetration_vel);
    return d >= 0.f ? 0.f : d / dt;
  };
  int n = 0;
  for (int j = 0; j < NJ; ++j) {
    if (!M->joint_has_limits[j + 1]) continue;
    const float lo = M->joint_lower[j + 1], hi = M->joint_upper[j + 1];
    const bool llo = s.th[j] < lo + P->limit_margin, lhi = !llo && s.th[j] > hi - P->limit_margin;
    if (!llo && !lhi) continue;
    float* jr = s.J[n];
    memset(jr, 0, sizeof(float) * 9);
    jr[6 + j % 3] = llo ? 1.f : -1.f;
    s.tgt[n] = target(llo ? lo - s.th[j] : s.th[j] - hi);
    s.rleg[n] = j / 3;
    ++n;
  }
  s.nlim = n;
  int nc = 0;
  const v3 p0 = L3(s.lk[0].P);
  for (int c = 0; c < M->num_candidates && nc < MAXC; ++c) {
    const int ck = M->cand_link[c];
    const Link& lc = s.lk[ck];
    v3 xc = L3(lc.P) + rot(lc.R, L3(M->cand_pos[c]));
    const float r = M->cand_radius[c];
    float depth;
    v3 dn = V(0, 0, 1), d1 = V(1, 0, 0), d2 = V(0, 1, 0);
    if (!terrain) {
      depth = r - xc.z;
      xc.z -= r;
    } else {
      depth = terrain_contact(P, B, xc, r, dn);
      xc = xc - dn * r;
      tangents(dn, d1, d2);
    }
    if (!(depth > -P->contact_margin)) continue;
    S3(s.cn[nc], dn);
    const int leg = ck > 0 ? (ck - 1) / 3 : -1, pos = ck > 0 ? (ck - 1) % 3 : -1;
    const int kl = ck > 0 ? 1 + 3 * leg : 1;
    const v3 a0 = L3(s.lk[kl].ax), a1 = L3(s.lk[kl + 1].ax), a2 = L3(s.lk[kl + 2].ax);
    const v3 r0 = xc - L3(s.lk[kl].P), r1 = xc - L3(s.lk[kl + 1].P), r2 = xc - L3(s.lk[kl + 2].P), rb = xc - p0;
    for (int t = 0; t < 3; ++t) {
      const v3 d = t == 0 ? dn : (t == 1 ? d1 : d2), ang = cross(rb, d);
      float* jr = s.J[n];
      jr[0] = d.x; jr[1] = d.y; jr[2] = d.z; jr[3] = ang.x; jr[4] = ang.y; jr[5] = ang.z;
      jr[6] = pos >= 0 ? dot(a0, cross(r0, d)) : 0.f;
      jr[7] = pos >= 1 ? dot(a1, cross(r1, d)) : 0.f;
      jr[8] = pos >= 2 ? dot(a2, cross(r2, d)) : 0.f;
      s.rleg[n] = leg;
      s.tgt[n] = t == 0 ? target(depth) : 0.f;
      ++n;
    }
    s.cbody[nc++] = M->cand_body[c];
  }
  s.ncon = nc;
  s.nrows = n;
  // per row: y = J_B − X_l J_l, z = S⁻¹ y, g = D_l⁻¹ J_l, A_rr, w_r = J_r u*
  float Y[MAXR][6];
  for (int r = 0; r < n; ++r) {
    const float* jr = s.J[r];
    const int lr = s.rleg[r];
    float* y = Y[r];
    float w = 0.f;
    for (int q = 0; q < 6; ++q) { y[q] = jr[q]; w += jr[q] * s.us[q]; }
    float g[3] = {0.f, 0.f, 0.f}, arr = 0.f;
    if (lr >= 0) {
      for (int c = 0; c < 3; ++c) {
        const float* Xc = s.X[3 * lr + c];
        for (int q = 0; q < 6; ++q) y[q] -= Xc[q] * jr[6 + c];
        w += jr[6 + c] * s.us[6 + 3 * lr + c];
      }
      const float* Di = s.Dinv[lr];
      g[0] = Di[0] * jr[6] + Di[3] * jr[7] + Di[4] * jr[8];
      g[1] = Di[3] * jr[6] + Di[1] * jr[7] + Di[5] * jr[8];
      g[2] = Di[4] * jr[6] + Di[5] * jr[7] + Di[2] * jr[8];
      arr = jr[6] * g[0] + jr[7] * g[1] + jr[8] * g[2];
    }
    float* zg = s.ZG[r];
    for (int q = 0; q < 6; ++q) {
      const float* Si = s.Sinv[q];
      zg[q] = Si[0] * y[0] + Si[1] * y[1] + Si[2] * y[2] + Si[3] * y[3] + Si[4] * y[4] + Si[5] * y[5];
      arr += y[q] * zg[q];
    }
    zg[6] = g[0]; zg[7] = g[1]; zg[8] = g[2];
    s.Arr[r] = arr;
    s.lam[r] = 0.f;
    s.w[r] = w;
  }
  // A = J M⁻¹ Jᵀ: A[q][r] = y_r·z_q + [leg_r = leg_q] J_l,r·g_q
  for (int q = 0; q < n; ++q) {
    const float* zg = s.ZG[q];
    for (int r = 0; r < n; ++r) {
      const float* y = Y[r];
      const float* jr = s.J[r];
      const float v = y[0] * zg[0] + y[1] * zg[1] + y[2] * zg[2] + y[3] * zg[3] + y[4] * zg[4] + y[5] * zg[5];
      const float vl = jr[6] * zg[6] + jr[7] * zg[7] + jr[8] * zg[8];
      s.A[q * n + r] = v + (s.rleg[q] == s.rleg[r] ? vl : 0.f);
    }
  }
  // projected Gauss-Seidel: [limits | (normal, tangent pair on the friction disk) per contact]
  float* w = s.w;
  float* lam = s.lam;
  auto apply = [&](int r, float d) {
    const float* Ar = s.A + r * n;
    for (int q = 0; q < n; ++q) w[q] += Ar[q] * d;
  };
  for (int it = 0; it < P->solver_iterations; ++it) {
    for (int r = 0; r < s.nlim; ++r) {
      const float cand = fmaxf(0.f, lam[r] + (s.tgt[r] - w[r]) / s.Arr[r]);
      const float d = cand - lam[r];
      lam[r] = cand;
      apply(r, d);
    }
    for (int r = s.nlim; r < n; r += 3) {
      const float cand = fmaxf(0.f, lam[r] + (s.tgt[r] - w[r]) / s.Arr[r]);
      const float d = cand - lam[r];
      lam[r] = cand;
      apply(r, d);
      const float lim = s.mu * lam[r];
      float l1 = lam[r + 1] - w[r + 1] / s.Arr[r + 1], l2 = lam[r + 2] - w[r + 2] / s.Arr[r + 2];
      const float nn = l1 * l1 + l2 * l2;
      if (nn > lim * lim) {
        const float sc = lim / sqrtf(nn);
        l1 *= sc;
        l2 *= sc;
      }
      const float e1 = l1 - lam[r + 1], e2 = l2 - lam[r + 2];
      lam[r + 1] = l1;
      lam[r + 2] = l2;
      const float* A1 = s.A + (r + 1) * n;
      const float* A2 = s.A + (r + 2) * n;
      for (int q = 0; q < n; ++q) w[q] += A1[q] * e1 + A2[q] * e2;
    }
  }
  // u+ = u* + M⁻¹ Jᵀ λ = u* + [Z ; G_J − Xᵀ Z]
  float Z[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, G[NJ] = {0.f};
  for (int r = 0; r < n; ++r) {
    const float* zg = s.ZG[r];
    for (int q = 0; q < 6; ++q) Z[q] += lam[r] * zg[q];
    if (s.rleg[r] >= 0)
      for (int c = 0; c < 3; ++c) G[3 * s.rleg[r] + c] += lam[r] * zg[6 + c];
  }
  for (int q = 0; q < 6; ++q) s.up[q] = s.us[q] + Z[q];
  for (int j = 0; j < NJ; ++j) {
    float v = s.us[6 + j] + G[j];
    for (int q = 0; q < 6; ++q) v -= s.X[j][q] * Z[q];
    s.up[6 + j] = v;
  }
  // contact forces of the last substep per reported body (world frame)
  if (last) {
    memset(s.cf, 0, sizeof(s.cf));
    for (int c = 0; c < nc; ++c) {
      const int r = s.nlim + 3 * c;
      float* f = s.cf[s.cbody[c]];
      if (!terrain) {
        f[2] += lam[r]; f[0] += lam[r + 1]; f[1] += lam[r + 2];
      } else {
        v3 t1, t2;
        const v3 nrm = L3(s.cn[c]);
        tangents(nrm, t1, t2);
        const v3 fc = nrm * lam[r] + t1 * lam[r + 1] + t2 * lam[r + 2];
        f[0] += fc.x; f[1] += fc.y; f[2] += fc.z;
      }
    }
    for (int b = 0; b < LGX_MAX_BODIES; ++b)
      for (int i = 0; i < 3; ++i) s.cf[b][i] = s.cf[b][i] / dt;
  }
  // semi-implicit Euler
  const v3 wv = V(s.up[3], s.up[4], s.up[5]);
  for (int i = 0; i < 3; ++i) s.pb[i] += dt * s.up[i];
  const float wn = sqrtf(dot(wv, wv)), ang = wn * dt;
  float dq[4];
  if (ang > 1e-12f) {
    const float sc = sinf(0.5f * ang) / wn;
    dq[0] = wv.x * sc; dq[1] = wv.y * sc; dq[2] = wv.z * sc; dq[3] = cosf(0.5f * ang);
  } else {
    dq[0] = 0.5f * dt * wv.x; dq[1] = 0.5f * dt * wv.y; dq[2] = 0.5f * dt * wv.z; dq[3] = 1.f;
  }
  const float* q = s.qb;
  float qn[4];
  qn[3] = dq[3] * q[3] - (dq[0] * q[0] + dq[1] * q[1] + dq[2] * q[2]);
  qn[0] = dq[3] * q[0] + q[3] * dq[0] + (dq[1] * q[2] - dq[2] * q[1]);
  qn[1] = dq[3] * q[1] + q[3] * dq[1] + (dq[2] * q[0] - dq[0] * q[2]);
  qn[2] = dq[3] * q[2] + q[3] * dq[2] + (dq[0] * q[1] - dq[1] * q[0]);
  const float nq = 1.0f / sqrtf(qn[0] * qn[0] + qn[1] * qn[1] + qn[2] * qn[2] + qn[3] * qn[3]);
  for (int i = 0; i < 4; ++i) s.qb[i] = qn[i] * nq;
  for (int i = 0; i < 3; ++i) { s.vo[i] = s.up[i]; s.wb[i] = s.up[3 + i]; }
  for (int j = 0; j < NJ; ++j) {
    s.thd[j] = s.up[6 + j];
    s.th[j] += dt * s.thd[j];
  }
}

// ------------------------------------------------------------------ post-physics helpers
// (isaacgym torch_utils / legged_gym math, fp32, the reference's op order)
static void quat_rotate_inverse(const float* q, const float* v, float* out) {
  const float w = q[3], sc = 2.0f * (w * w) - 1.0f;
  const float cx = q[1] * v[2] - q[2] * v[1], cy = q[2] * v[0] - q[0] * v[2], cz = q[0] * v[1] - q[1] * v[0];
  const float d = q[0] * v[0] + q[1] * v[1] + q[2] * v[2];
  out[0] = v[0] * sc - cx * w * 2.0f + q[0] * d * 2.0f;
  out[1] = v[1] * sc - cy * w * 2.0f + q[1] * d * 2.0f;
  out[2] = v[2] * sc - cz * w * 2.0f + q[2] * d * 2.0f;
}
static void quat_apply(const float* q, const float* b, float* out) {
  const float t0 = (q[1] * b[2] - q[2] * b[1]) * 2.0f, t1 = (q[2] * b[0] - q[0] * b[2]) * 2.0f,
              t2 = (q[0] * b[1] - q[1] * b[0]) * 2.0f;
  out[0] = b[0] + q[3] * t0 + (q[1] * t2 - q[2] * t1);
  out[1] = b[1] + q[3] * t1 + (q[2] * t0 - q[0] * t2);
  out[2] = b[2] + q[3] * t2 + (q[0] * t1 - q[1] * t0);
}
static float torch_rem(float a, float b) {
  float m = fmodf(a, b);
  if (m != 0.0f && ((m < 0.0f) != (b < 0.0f))) m += b;
  return m;
}
static float wrap_pi(float a) {
  const float two_pi = 6.283185307179586f, pi = 3.141592653589793f;
  float m = torch_rem(a, two_pi);
  m -= two_pi * (float)(m > pi);
  return m;
}
static inline float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
static inline float sqr(float x) { return x * x; }
static inline float len3(float a, float b, float c) { return sqrtf(a * a + b * b + c * c); }
static inline float len2(float a, float b) { return sqrtf(a * a + b * b); }
static inline float urange(float lo, float hi, float u) { return (float)((double)hi - (double)lo) * u + lo; }
// with the reference's Python-float (double) bounds (lgx_buffers.command_ranges)
static inline float urange_d(double lo, double hi, float u) { return (float)(hi - lo) * u + (float)lo; }

static int rng_blocks(const lgx_task_params* P) { return 9 + (P->num_proprio + 3) / 4; }
static void fill_uniforms(Env& s, const lgx_task_params* P, uint64_t seed, uint32_t gid, uint64_t step,
                          uint32_t stream) {
  for (int b = 0; b < rng_blocks(P); ++b) {
    uint32_t o[4];
    philox(gid, (uint32_t)step, (uint32_t)b | (stream << 16), (uint32_t)(step >> 32), (uint32_t)seed,
           (uint32_t)(seed >> 32), o);
    for (int i = 0; i < 4; ++i) s.U[4 * b + i] = unit(o[i]);
  }
}

// Go2Robot._resample_commands go2.py:413-464 / LeggedRobot legged_robot.py:406-437
// R: lgx_buffers.command_ranges (mutable, double [8]) or NULL (the params' ranges)
static void resample_commands(const lgx_task_params* P, const double* R, float* cmd, const float* U, int slot0,
                              const float* quat) {
  if (P->has_user_command) {
    for (int i = 0; i < 4; ++i) cmd[i] = P->user_command[i];
    return;
  }
  if (R) {
    cmd[0] = urange_d(R[0], R[1], U[slot0 + 0]);
    cmd[1] = urange_d(R[2], R[3], U[slot0 + 1]);
    if (P->heading_command)
      cmd[3] = urange_d(R[6], R[7], U[slot0 + 2]);
    else
      cmd[2] = urange_d(R[4], R[5], U[slot0 + 2]);
  } else {
    cmd[0] = urange(P->cmd_lin_vel_x[0], P->cmd_lin_vel_x[1], U[slot0 + 0]);
    cmd[1] = urange(P->cmd_lin_vel_y[0], P->cmd_lin_vel_y[1], U[slot0 + 1]);
    if (P->heading_command)
      cmd[3] = urange(P->cmd_heading[0], P->cmd_heading[1], U[slot0 + 2]);
    else
      cmd[2] = urange(P->cmd_ang_vel_yaw[0], P->cmd_ang_vel_yaw[1], U[slot0 + 2]);
  }
  const float keep = (float)(len2(cmd[0], cmd[1]) > 0.2f);
  cmd[0] = cmd[0] * keep;
  cmd[1] = cmd[1] * keep;
  if (P->zero_command && U[slot0 + 3] < P->zero_command_prob) {
    if (P->task_kind == LGX_TASK_GO2) {
      cmd[0] = cmd[0] * 0.0f; cmd[1] = cmd[1] * 0.0f; cmd[2] = cmd[2] * 0.0f;
      if (P->heading_command) {
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

// reset_idx for env e (go2.py:207-263 / legged_robot.py:157-213) on the env's staged root,
// dof and command state. `stats` (K + 1 floats) receives the episode sums and the count.
static void reset_env(const lgx_task_params* P, const lgx_buffers* B, Env& s, int e, bool zero_carried, float* stats) {
  const int D = P->num_dof;
  const float* U = s.U;
  float* root = s.root;
  if (P->curriculum && B->terrain_levels) {  // legged_robot.py:543-574
    const float dist = len2(root[0] - B->env_origins[e * 3 + 0], root[1] - B->env_origins[e * 3 + 1]);
    const int up = dist > P->terrain_length * P->promote_threshold;
    const int down = dist < len2(s.cmd[0], s.cmd[1]) * P->max_episode_length_s * P->demote_threshold;
    int64_t lvl = B->terrain_levels[e] + up - down;
    if (lvl >= P->max_terrain_level) {
      lvl = (int64_t)(U[S_TERR] * (float)P->max_terrain_level);
      if (lvl >= P->max_terrain_level) lvl = P->max_terrain_level - 1;
    } else if (lvl < 0) {
      lvl = 0;
    }
    B->terrain_levels[e] = lvl;
    const float* o = B->terrain_origins + ((size_t)lvl * P->num_terrain_cols + B->terrain_types[e]) * 3;
    for (int i = 0; i < 3; ++i) B->env_origins[e * 3 + i] = o[i];
  }
  for (int i = 0; i < 13; ++i) root[i] = P->base_init_state[i];  // legged_robot.py:509-532
  for (int i = 0; i < 3; ++i) root[i] = root[i] + B->env_origins[e * 3 + i];
  if (P->custom_origins) {
    root[0] = root[0] + urange(-1.0f, 1.0f, U[S_ROOT_XY + 0]);
    root[1] = root[1] + urange(-1.0f, 1.0f, U[S_ROOT_XY + 1]);
  }
  for (int i = 0; i < 6; ++i) root[7 + i] = urange(-0.5f, 0.5f, U[S_ROOT_VEL + i]);
  resample_commands(P, B->command_ranges, s.cmd, U, S_RCMD, root + 3);
  s.ep = 0;
  for (int j = 0; j < D; ++j) {  // legged_robot.py:481-506
    s.th[j] = P->default_dof_pos[j] + urange(0.0f, 0.9f, U[S_DOF + j]);
    s.thd[j] = 0.0f;
  }
  if (zero_carried) {
    const int A = P->num_actions, H = P->history_len * P->num_proprio;
    memset(B->last_actions + (size_t)e * A, 0, sizeof(float) * A);
    memset(B->last_dof_vel + (size_t)e * D, 0, sizeof(float) * D);
    memset(B->last_torques + (size_t)e * D, 0, sizeof(float) * D);
    memset(B->last_root_vel + (size_t)e * 6, 0, sizeof(float) * 6);
    memset(B->last_base_lin_vel + (size_t)e * 3, 0, sizeof(float) * 3);
    memset(B->obs_history + (size_t)e * H, 0, sizeof(float) * H);
  }
  if (P->actuator_net) {  // anymal.py:56-60
    const size_t NT = (size_t)P->num_envs * D;
    for (int l = 0; l < 2; ++l) {
      memset(B->sea_hidden + (l * NT + (size_t)e * D) * 8, 0, sizeof(float) * 8 * D);
      memset(B->sea_cell + (l * NT + (size_t)e * D) * 8, 0, sizeof(float) * 8 * D);
    }
  }
  if (P->task_kind == LGX_TASK_GO2)
    for (int f = 0; f < P->num_feet; ++f) {
      if (B->feet_air_time) B->feet_air_time[e * P->num_feet + f] = 0.f;
      B->last_contacts[e * P->num_feet + f] = 0;
      B->last_contact_heights[e * P->num_feet + f] = 0.f;
    }
  const int K = P->num_reward_terms + (P->has_termination_reward ? 1 : 0);
  float* es = B->episode_sums + (size_t)e * K;
  // the command curriculum's input (go2.py:87): the tracking_lin_vel sum at an in-step reset
  if (!zero_carried && B->curriculum_vals) B->curriculum_vals[e] = es[P->curriculum_term];
  for (int k = 0; k < K; ++k) {
    stats[k] = es[k];
    es[k] = 0.f;
  }
  stats[K] = 1.0f;
}

// LeggedRobot._get_heights legged_robot.py:997-1032
static void get_heights(const lgx_task_params* P, const lgx_buffers* B, Env& s) {
  const int NP = P->num_height_points;
  if (P->mesh_type == LGX_MESH_PLANE || B->height_samples == nullptr) {
    for (int i = 0; i < NP; ++i) s.heights[i] = 0.0f;
    return;
  }
  const float* root = s.root;
  const float qz = root[5], qw = root[6];
  float n = sqrtf(qz * qz + qw * qw);
  n = n < 1e-9f ? 1e-9f : n;
  const float qy[4] = {0.f, 0.f, qz / n, qw / n};
  for (int i = 0; i < NP; ++i) {
    const float p[3] = {P->height_points[i][0], P->height_points[i][1], 0.f};
    float w[3];
    quat_apply(qy, p, w);
    const float px = (w[0] + root[0]) + P->border_size, py = (w[1] + root[1]) + P->border_size;
    long ix = (long)(px / P->horizontal_scale), iy = (long)(py / P->horizontal_scale);
    ix = ix < 0 ? 0 : (ix > P->hf_rows - 2 ? P->hf_rows - 2 : ix);
    iy = iy < 0 ? 0 : (iy > P->hf_cols - 2 ? P->hf_cols - 2 : iy);
    const int16_t* hsm = B->height_samples;
    int16_t h = std::min(std::min(hsm[ix * P->hf_cols + iy], hsm[(ix + 1) * P->hf_cols + iy]), hsm[ix * P->hf_cols + iy + 1]);
    s.heights[i] = (float)h * P->vertical_scale;
  }
}

// sums over joints / height points shared by the reward terms (lgx_env.hip joint_sums)
enum JSum { J_ACTION_RATE, J_DELTA_TORQUES, J_DOF_ACC, J_DOF_ERROR, J_DOF_POS_LIMITS, J_DOF_VEL, J_DOF_VEL_LIMITS,
            J_STAND_ABS, J_TORQUE_LIMITS, J_TORQUES, J_HIP_POS, J_THIGH_POS, J_CALF_POS, J_HEIGHT, J_N };
static void joint_sums(const lgx_task_params* P, const lgx_buffers* B, Env& s, int e) {
  const int D = P->num_dof, A = P->num_actions;
  for (int k = 0; k < J_N; ++k) s.jsum[k] = 0.f;
  for (int j = 0; j < D; ++j) {
    const float la = B->last_actions[(size_t)e * A + j], lt = B->last_torques[(size_t)e * D + j];
    const float q = s.th[j], qd = s.thd[j], tau = s.tau[j], dq = q - P->default_dof_pos[j];
    s.jsum[J_ACTION_RATE] += sqr(la - s.act[j]);
    s.jsum[J_DELTA_TORQUES] += sqr(tau - lt);
    s.jsum[J_DOF_ACC] += sqr((s.ldv[j] - qd) / P->dt);
    s.jsum[J_DOF_ERROR] += sqr(dq);
    const float lo = q - P->dof_pos_limits[j][0], hi = q - P->dof_pos_limits[j][1];
    float o = -(lo < 0.0f ? lo : 0.0f);
    o += (hi > 0.0f ? hi : 0.0f);
    s.jsum[J_DOF_POS_LIMITS] += o;
    s.jsum[J_DOF_VEL] += sqr(qd);
    s.jsum[J_DOF_VEL_LIMITS] += clampf(fabsf(qd) - P->dof_vel_limits[j] * P->soft_dof_vel_limit, 0.0f, 1.0f);
    s.jsum[J_STAND_ABS] += fabsf(dq);
    const float t = fabsf(tau) - P->torque_limits[j] * P->soft_torque_limit;
    s.jsum[J_TORQUE_LIMITS] += t > 0.0f ? t : 0.0f;
    s.jsum[J_TORQUES] += sqr(tau);
    for (int i = 0; i < 4; ++i) {
      if (P->hip_joint_idx[i] == j) s.jsum[J_HIP_POS] += sqr(dq);
      if (P->thigh_joint_idx[i] == j) s.jsum[J_THIGH_POS] += sqr(dq);
      if (P->calf_joint_idx[i] == j) s.jsum[J_CALF_POS] += sqr(dq);
    }
  }
  for (int i = 0; i < P->num_height_points; ++i) s.jsum[J_HEIGHT] += s.root[2] - s.heights[i];
}

static inline float fnorm(const float* c) { return len3(c[0], c[1], c[2]); }

// one reward term (the `_reward_<name>` methods; ids in include/lgx.h)
static float reward_term(const lgx_task_params* P, Env& s, int id) {
  const float* root = s.root;
  float* cmd = s.cmd;
  float r = 0.0f;
  switch (id) {
    case LGX_REW_ACTION_RATE: return s.jsum[J_ACTION_RATE];
    case LGX_REW_ANG_VEL_XY: return sqr(s.bav[0]) + sqr(s.bav[1]);
    case LGX_REW_BASE_HEIGHT: return sqr(s.jsum[J_HEIGHT] / (float)P->num_height_points - P->base_height_target);
    case LGX_REW_CALF_COLLISION:
      for (int i = 0; i < 4; ++i) r += (float)(fnorm(s.cf[P->calf_idx[i]]) > 0.1f);
      return r;
    case LGX_REW_CALF_POS: return s.jsum[J_CALF_POS];
    case LGX_REW_CALF_SYMMETRY: {
      const int* c = P->calf_joint_idx;
      return fabsf(s.th[c[0]] - s.th[c[1]]) + fabsf(s.th[c[2]] - s.th[c[3]]);
    }
    case LGX_REW_COLLISION:
      for (int i = 0; i < P->n_penalised; ++i) r += (float)(fnorm(s.cf[P->penalised_idx[i]]) > 0.1f);
      return r;
    case LGX_REW_DELTA_TORQUES: return s.jsum[J_DELTA_TORQUES];
    case LGX_REW_DOF_ACC: return s.jsum[J_DOF_ACC];
    case LGX_REW_DOF_ERROR: return s.jsum[J_DOF_ERROR];
    case LGX_REW_DOF_POS_LIMITS: return s.jsum[J_DOF_POS_LIMITS];
    case LGX_REW_DOF_VEL: return s.jsum[J_DOF_VEL];
    case LGX_REW_DOF_VEL_LIMITS: return s.jsum[J_DOF_VEL_LIMITS];
    case LGX_REW_FEET_AIR_TIME: {  // go2.py:819-832 (updates feet_air_time)
      float rew = 0.0f;
      for (int f = 0; f < P->num_feet; ++f) {
        const int cfl = (s.cf[P->feet_idx[f]][2] > 1.0f) || s.lc[f];
        const float first = (float)((s.fat[f] > 0.0f) && cfl);
        s.fat[f] = s.fat[f] + P->dt;
        rew += (s.fat[f] - 0.5f) * first;
      }
      rew = rew * (float)(len2(cmd[0], cmd[1]) > 0.1f);
      for (int f = 0; f < P->num_feet; ++f) {
        const int cfl = (s.cf[P->feet_idx[f]][2] > 1.0f) || s.lc[f];
        s.fat[f] = s.fat[f] * (float)(!cfl);
      }
      return rew;
    }
    case LGX_REW_FEET_CONTACT_FORCES:
      for (int f = 0; f < P->num_feet; ++f) {
        const float v = fnorm(s.cf[P->feet_idx[f]]) - P->max_contact_force;
        r += v > 0.0f ? v : 0.0f;
      }
      return r;
    case LGX_REW_HEADING_ALIGNMENT: {
      const float fwd[3] = {1.f, 0.f, 0.f};
      float f[3];
      quat_apply(root + 3, fwd, f);
      const float heading = atan2f(f[1], f[0]);
      float desired = 0.0f;
      if (P->heading_command) {
        cmd[3] = wrap_pi(cmd[3]);  // the reference wraps commands[:, 3] in place (go2.py:744)
        desired = cmd[3];
      }
      return sqr(wrap_pi(desired - heading)) * (float)(len3(cmd[0], cmd[1], cmd[2]) >= 0.2f);
    }
    case LGX_REW_HIP_POS: return s.jsum[J_HIP_POS];
    case LGX_REW_JUMP_ZONE_FORWARD_VEL:
      return (root[7] > 0.0f ? root[7] : 0.0f) * (float)(s.jump > 0.0f) * (float)(len3(cmd[0], cmd[1], cmd[2]) >= 0.2f);
    case LGX_REW_JUMP_ZONE_UPWARD_VEL:
      return (root[9] > 0.0f ? root[9] : 0.0f) * (float)(s.jump > 0.0f) * (float)(len3(cmd[0], cmd[1], cmd[2]) >= 0.2f);
    case LGX_REW_LIN_VEL_Z: return sqr(s.blv[2]);
    case LGX_REW_MIN_HEIGHT:
      return clampf(P->base_height_target - root[2], 0.0f, P->base_height_target) * (float)(s.jump > 0.0f);
    case LGX_REW_ORIENTATION: return sqr(s.pg[0]) + sqr(s.pg[1]);
    case LGX_REW_PHASE_CONTACT_MATCH: {
      const float thr = 2.0f * P->percent_time_on_ground - 1.0f;
      float rew = 0.0f;
      for (int f = 0; f < 4; ++f) {
        const int stance = sinf(6.283185307179586f * s.ph[f]) <= thr;
        rew += (s.contact[f] == stance) ? 0.25f : -0.25f;
      }
      return rew;
    }
    case LGX_REW_PHASE_FOOT_LIFTING: {
      const float thr = 2.0f * P->percent_time_on_ground - 1.0f;
      float rew = 0.0f;
      for (int f = 0; f < 4; ++f) {
        const int stance = sinf(6.283185307179586f * s.ph[f]) <= thr;
        const float nh = clampf(s.feet_z[f] - s.lch[f], 0.0f, P->max_foot_height) / P->max_foot_height;
        rew += stance ? -nh : nh;
      }
      return rew / 2.0f;
    }
    case LGX_REW_REVERSE_PENALTY: return -(root[7] < 0.0f ? root[7] : 0.0f);
    case LGX_REW_STAND_STILL: return s.jsum[J_STAND_ABS] * (float)(len2(cmd[0], cmd[1]) < 0.1f);
    case LGX_REW_STUMBLE_CALVES: {
      int any = 0;
      for (int i = 0; i < 4; ++i) {
        const float* c = s.cf[P->calf_idx[i]];
        any |= len2(c[0], c[1]) > 5.0f * fabsf(c[2]);
      }
      return (float)any;
    }
    case LGX_REW_STUMBLE_FEET: {
      int any = 0;
      for (int f = 0; f < P->num_feet; ++f) {
        const float* c = s.cf[P->feet_idx[f]];
        any |= len2(c[0], c[1]) > 5.0f * fabsf(c[2]);
      }
      return (float)any;
    }
    case LGX_REW_THIGH_POS: return s.jsum[J_THIGH_POS];
    case LGX_REW_THIGH_SYMMETRY: {
      const int* c = P->thigh_joint_idx;
      return fabsf(s.th[c[0]] - s.th[c[1]]) + fabsf(s.th[c[2]] - s.th[c[3]]);
    }
    case LGX_REW_TORQUE_LIMITS: return s.jsum[J_TORQUE_LIMITS];
    case LGX_REW_TORQUES: return s.jsum[J_TORQUES];
    case LGX_REW_TRACKING_ANG_VEL: return expf(-sqr(cmd[2] - s.bav[2]) / P->tracking_sigma);
    case LGX_REW_TRACKING_LIN_VEL: return expf(-(sqr(cmd[0] - s.blv[0]) + sqr(cmd[1] - s.blv[1])) / P->tracking_sigma);
    case LGX_REW_TRACKING_PITCH: return expf(-sqr(s.pitch * 57.29577951308232f - P->pitch_deg_target) / P->tracking_sigma);
    case LGX_REW_TRACKING_ROLL: return expf(-sqr(s.roll * 57.29577951308232f - P->roll_deg_target) / P->tracking_sigma);
    case LGX_REW_ZERO_CMD_DOF_ERROR: return s.jsum[J_DOF_ERROR] * (float)(len3(cmd[0], cmd[1], cmd[2]) < 0.2f);
    default: return 0.0f;
  }
}

// rotation matrix -> quaternion xyzw with w >= 0 (rigid-body state tensor)
static void mat_quat(const float* Rb, float* qq) {
  const float tr = Rb[0] + Rb[4] + Rb[8];
  if (tr > 0.f) {
    const float sc = sqrtf(tr + 1.f) * 2.f;
    qq[3] = 0.25f * sc; qq[0] = (Rb[7] - Rb[5]) / sc; qq[1] = (Rb[2] - Rb[6]) / sc; qq[2] = (Rb[3] - Rb[1]) / sc;
  } else if (Rb[0] > Rb[4] && Rb[0] > Rb[8]) {
    const float sc = sqrtf(1.f + Rb[0] - Rb[4] - Rb[8]) * 2.f;
    qq[3] = (Rb[7] - Rb[5]) / sc; qq[0] = 0.25f * sc; qq[1] = (Rb[1] + Rb[3]) / sc; qq[2] = (Rb[2] + Rb[6]) / sc;
  } else if (Rb[4] > Rb[8]) {
    const float sc = sqrtf(1.f + Rb[4] - Rb[0] - Rb[8]) * 2.f;
    qq[3] = (Rb[2] - Rb[6]) / sc; qq[0] = (Rb[1] + Rb[3]) / sc; qq[1] = 0.25f * sc; qq[2] = (Rb[5] + Rb[7]) / sc;
  } else {
    const float sc = sqrtf(1.f + Rb[8] - Rb[0] - Rb[4]) * 2.f;
    qq[3] = (Rb[3] - Rb[1]) / sc; qq[0] = (Rb[2] + Rb[6]) / sc; qq[1] = (Rb[5] + Rb[7]) / sc; qq[2] = 0.25f * sc;
  }
  if (qq[3] < 0.f)
    for (int i = 0; i < 4; ++i) qq[i] = -qq[i];
}

// ------------------------------------------------------------------ one env step
// legged_robot.py:67-100 (+ Go2Robot.post_physics_step go2.py:345-387 / LeggedRobot
// legged_robot.py:103-138) for env e; `stats` receives its episode statistics when it resets.
static void env_step(Env& s, const lgx_model* M, const lgx_task_params* P, const lgx_buffers* B, uint64_t seed,
                     uint64_t step, bool physics, int e, float* stats) {
  const int D = P->num_dof, A = P->num_actions, NB = P->num_bodies, F = P->num_feet;
  const bool go2 = P->task_kind == LGX_TASK_GO2;
  float* root_g = B->root_states + (size_t)e * 13;
  for (int j = 0; j < A; ++j) {  // clip actions legged_robot.py:74-75
    const float a = clampf(B->actions_in[(size_t)e * A + j], -P->clip_actions, P->clip_actions);
    s.act[j] = a;
    B->actions[(size_t)e * A + j] = a;
  }
  for (int j = 0; j < D; ++j) {
    s.th[j] = B->dof_state[((size_t)e * D + j) * 2];
    s.thd[j] = B->dof_state[((size_t)e * D + j) * 2 + 1];
    s.kpm[j] = B->kp_kd ? B->kp_kd[(size_t)e * D + j] : 1.f;
    s.kdm[j] = B->kp_kd ? B->kp_kd[((size_t)P->num_envs + e) * D + j] : 1.f;
    s.ldv[j] = B->last_dof_vel[(size_t)e * D + j];
  }
  memcpy(s.root, root_g, sizeof(s.root));
  s.madd = B->mass_params ? B->mass_params[e * 4] : 0.f;
  for (int i = 0; i < 3; ++i) s.cadd[i] = B->mass_params ? B->mass_params[e * 4 + 1 + i] : 0.f;
  s.mu = 0.5f * ((B->friction ? B->friction[e] : 1.f) + P->ground_friction);
  memcpy(s.cmd, B->commands + e * 4, sizeof(s.cmd));
  const long long ep_prev = B->episode_length[e];
  const float jump_prev = B->rpy_phase ? B->rpy_phase[e * 8 + 7] : 0.f;
  int blew = 0;  // NaN/Inf guard

  if (physics) {
    const float* r0 = s.root;
    const float nq = 1.0f / sqrtf(r0[3] * r0[3] + r0[4] * r0[4] + r0[5] * r0[5] + r0[6] * r0[6]);
    for (int i = 0; i < 4; ++i) s.qb[i] = r0[3 + i] * nq;
    for (int i = 0; i < 3; ++i) { s.pb[i] = r0[i]; s.wb[i] = r0[10 + i]; }
    float R[9];
    quat_R(s.qb, R);
    const v3 rc = rot(R, V(M->link_com[0][0] + s.cadd[0], M->link_com[0][1] + s.cadd[1], M->link_com[0][2] + s.cadd[2]));
    S3(s.vo, L3(r0 + 7) - cross(L3(s.wb), rc));  // COM velocity -> origin velocity
    for (int sub = 0; sub < P->decimation; ++sub) substep(s, M, P, B, e, sub == P->decimation - 1);
    // NaN/Inf guard (the kernel's rule, lgx_env.hip): a non-finite state after the substeps
    // becomes a finite stand-in and the env is reset below
    bool bad = false;
    for (int j = 0; j < D; ++j) bad = bad || !(std::isfinite(s.th[j]) && std::isfinite(s.thd[j]) && std::isfinite(s.tau[j]));
    for (int j = 0; j < A; ++j) bad = bad || !std::isfinite(s.act[j]);
    for (int i = 0; i < 3; ++i) bad = bad || !(std::isfinite(s.pb[i]) && std::isfinite(s.vo[i]) && std::isfinite(s.wb[i]));
    for (int i = 0; i < 4; ++i) bad = bad || !std::isfinite(s.qb[i]);
    for (int b = 0; b < NB; ++b)
      for (int i = 0; i < 3; ++i) bad = bad || !std::isfinite(s.cf[b][i]);
    if (bad) {
      for (int j = 0; j < D; ++j) { s.th[j] = P->default_dof_pos[j]; s.thd[j] = 0.f; s.tau[j] = 0.f; }
      for (int j = 0; j < A; ++j) { s.act[j] = 0.f; B->actions[(size_t)e * A + j] = 0.f; }
      for (int i = 0; i < 3; ++i) { s.pb[i] = std::isfinite(s.root[i]) ? s.root[i] : 0.f; s.vo[i] = 0.f; s.wb[i] = 0.f; }
      for (int i = 0; i < 4; ++i) s.qb[i] = i == 3 ? 1.f : 0.f;
      for (int b = 0; b < NB; ++b) s.cf[b][0] = s.cf[b][1] = s.cf[b][2] = 0.f;
      blew = 1;
    }
    kinematics<false>(s, M, P);
    quat_R(s.qb, R);
    const v3 rc2 = rot(R, V(M->link_com[0][0] + s.cadd[0], M->link_com[0][1] + s.cadd[1], M->link_com[0][2] + s.cadd[2]));
    const v3 vc = L3(s.vo) + cross(L3(s.wb), rc2);
    float* root = s.root;
    for (int i = 0; i < 3; ++i) root[i] = s.pb[i];
    for (int i = 0; i < 4; ++i) root[3 + i] = s.qb[i];
    root[7] = vc.x; root[8] = vc.y; root[9] = vc.z;
    for (int i = 0; i < 3; ++i) root[10 + i] = s.wb[i];
    for (int b = 0; b < NB; ++b) {
      const Link& lk = s.lk[M->body_link[b]];
      const v3 off = L3(M->body_offset[b]), o = rot(lk.R, off), pos = L3(lk.P) + o;
      const bool primary = off.x == 0.f && off.y == 0.f && off.z == 0.f;
      const v3 lv = L3(lk.V) + cross(L3(lk.W), primary ? (L3(lk.C) - L3(lk.P)) : o);
      float Rb[9], qq[4];
      matmul3(lk.R, M->body_rot[b], Rb);
      mat_quat(Rb, qq);
      float* rb = B->rigid_body_states + ((size_t)e * NB + b) * 13;
      rb[0] = pos.x; rb[1] = pos.y; rb[2] = pos.z;
      for (int i = 0; i < 4; ++i) rb[3 + i] = qq[i];
      rb[7] = lv.x; rb[8] = lv.y; rb[9] = lv.z;
      for (int i = 0; i < 3; ++i) rb[10 + i] = lk.W[i];
      s.rbz[b] = pos.z;
      memcpy(B->contact_forces + ((size_t)e * NB + b) * 3, s.cf[b], sizeof(float) * 3);
    }
    memcpy(B->torques + (size_t)e * D, s.tau, sizeof(float) * D);
  } else {  // post-physics only: physics state supplied by the caller
    for (int b = 0; b < NB; ++b) {
      memcpy(s.cf[b], B->contact_forces + ((size_t)e * NB + b) * 3, sizeof(float) * 3);
      s.rbz[b] = B->rigid_body_states[((size_t)e * NB + b) * 13 + 2];
    }
    memcpy(s.tau, B->torques + (size_t)e * D, sizeof(float) * D);
  }

  // ---------------------------------------------------------------- post-physics
  fill_uniforms(s, P, seed, (uint32_t)(P->env_id_offset + e), step, 0);
  float* root = s.root;
  float* cmd = s.cmd;
  const long long ep = ep_prev + 1;
  s.ep = ep;
  const float g[3] = {0.f, 0.f, -1.f};
  quat_rotate_inverse(root + 3, root + 7, s.blv);
  quat_rotate_inverse(root + 3, root + 10, s.bav);
  quat_rotate_inverse(root + 3, g, s.pg);
  s.roll = s.pitch = s.yaw = 0.f;
  for (int f = 0; f < 4; ++f) { s.ph[f] = 0.f; s.contact[f] = 0; s.feet_z[f] = 0.f; s.lc[f] = 0; s.lch[f] = 0.f; s.fat[f] = 0.f; }
  if (go2) {  // update_feet_states go2.py:266-328
    const float phase = torch_rem((float)ep * P->dt, P->period) / P->period;
    const float pfr = torch_rem(phase + P->offset_fr, 1.0f), pbl = torch_rem(phase + P->offset_bl, 1.0f);
    const float pfl = torch_rem(phase + P->offset_fl, 1.0f), pbr = torch_rem(phase + P->offset_br, 1.0f);
    const float msk = (len3(cmd[0], cmd[1], cmd[2]) < 0.2f) ? 0.0f : 1.0f;
    s.ph[0] = pfl * msk; s.ph[1] = pfr * msk; s.ph[2] = pbl * msk; s.ph[3] = pbr * msk;
    for (int f = 0; f < F; ++f) {
      const int lcf = B->last_contacts[e * F + f];
      const float lch = B->last_contact_heights[e * F + f];
      const int curc = s.cf[P->feet_idx[f]][2] > 1.0f;
      s.contact[f] = curc || lcf;
      s.lc[f] = curc;
      s.feet_z[f] = s.rbz[P->feet_idx[f]];
      s.lch[f] = s.contact[f] ? s.feet_z[f] : lch;
      if (B->feet_air_time) s.fat[f] = B->feet_air_time[e * F + f];
    }
    const float qx = root[3], qy = root[4], qz = root[5], qw = root[6];  // go2.py:11-31
    s.roll = atan2f(2.0f * (qw * qx + qy * qz), 1.0f - 2.0f * (qx * qx + qy * qy));
    s.pitch = asinf(clampf(2.0f * (qw * qy - qz * qx), -1.0f, 1.0f));
    s.yaw = atan2f(2.0f * (qw * qz + qx * qy), 1.0f - 2.0f * (qy * qy + qz * qz));
  }
  // _post_physics_step_callback go2.py:390-410
  if (ep % P->resample_interval == 0) resample_commands(P, B->command_ranges, cmd, s.U, S_CMD, root + 3);
  if (P->heading_command) {
    const float fwd[3] = {1.f, 0.f, 0.f};
    float f[3];
    quat_apply(root + 3, fwd, f);
    cmd[2] = clampf(wrap_pi(cmd[3] - atan2f(f[1], f[0])) * (go2 ? P->heading_error_gain : 0.5f), -1.0f, 1.0f);
  }
  if (P->push_robots && (step % (uint64_t)P->push_interval == 0)) {
    root[7] = urange(-P->max_push_vel_xy, P->max_push_vel_xy, s.U[S_PUSH + 0]);
    root[8] = urange(-P->max_push_vel_xy, P->max_push_vel_xy, s.U[S_PUSH + 1]);
  }
  // check_termination go2.py:186-204
  int reset = 0;
  for (int i = 0; i < P->n_termination; ++i) reset |= fnorm(s.cf[P->termination_idx[i]]) > 1.0f;
  const int tout = ep > P->max_episode_length && !blew;  // a blow-up is a termination (kernel)
  reset |= tout;
  reset |= s.pg[2] > 0.0f;
  if (P->parkour) reset |= root[2] < -1.0f;
  reset |= blew;
  s.jump = jump_prev;
  get_heights(P, B, s);
  joint_sums(P, B, s, e);
  // compute_reward legged_robot.py:216-237: the terms in the reference's (alphabetical) order
  const int K = P->num_reward_terms, KS = K + (P->has_termination_reward ? 1 : 0);
  float rew = 0.0f;
  for (int k = 0; k < K; ++k) {
    s.rterm[k] = blew ? 0.0f : reward_term(P, s, P->reward_ids[k]) * P->reward_scales[k];
  }
  for (int k = 0; k < K; ++k) rew += s.rterm[k];
  if (P->only_positive_rewards) rew = rew < 0.0f ? 0.0f : rew;
  if (P->has_termination_reward) {
    const float v = (float)(reset && !tout && !blew) * P->termination_scale;
    rew += v;
    s.rterm[K] = v;
  }
  B->rew[e] = rew;
  B->reset[e] = (uint8_t)reset;
  B->time_out[e] = (uint8_t)tout;
  if (B->blew_up) B->blew_up[e] = (uint8_t)blew;
  if (blew && B->blowup_count) {
#pragma omp atomic
    *B->blowup_count += 1u;
  }
  for (int k = 0; k < KS; ++k) B->episode_sums[(size_t)e * KS + k] += s.rterm[k];
  if (reset) reset_env(P, B, s, e, false, stats);  // reset_idx go2.py:207-263

  // compute_observations go2.py:467-574 / legged_robot.py:240-273
  const int Pp = P->num_proprio, H = P->history_len;
  if (go2 && P->parkour) {
    int outl = 0;
    for (int i = 0; i < P->num_height_points; ++i) outl += fabsf(s.heights[i]) > 0.1f;
    s.jump = (float)(outl >= 8);
  }
  for (int i = 0; i < Pp; ++i) {
    float v;
    if (go2) {
      if (i < 3) v = s.bav[i] * P->obs_scale_ang_vel;
      else if (i == 3) v = s.roll;
      else if (i == 4) v = s.pitch;
      else if (i < 8) v = s.cmd[i - 5] * P->commands_scale[i - 5];
      else if (i < 8 + D) v = (s.th[i - 8] - P->default_dof_pos[i - 8]) * P->obs_scale_dof_pos;
      else if (i < 8 + 2 * D) v = s.thd[i - 8 - D] * P->obs_scale_dof_vel;
      else if (i < 8 + 2 * D + A) v = s.act[i - 8 - 2 * D];
      else {
        const int q = i - (8 + 2 * D + A);  // sin/cos of FR, FL, BL, BR
        const int leg = (q >> 1) == 0 ? 1 : ((q >> 1) == 1 ? 0 : (q >> 1));
        const float p = 6.283185307179586f * s.ph[leg];
        v = (q & 1) ? cosf(p) : sinf(p);
      }
    } else {
      if (i < 3) v = s.blv[i] * P->obs_scale_lin_vel;
      else if (i < 6) v = s.bav[i - 3] * P->obs_scale_ang_vel;
      else if (i < 9) v = s.pg[i - 6];
      else if (i < 12) v = s.cmd[i - 9] * P->commands_scale[i - 9];
      else if (i < 12 + D) v = (s.th[i - 12] - P->default_dof_pos[i - 12]) * P->obs_scale_dof_pos;
      else if (i < 12 + 2 * D) v = s.thd[i - 12 - D] * P->obs_scale_dof_vel;
      else if (i < 12 + 2 * D + A) v = s.act[i - 12 - 2 * D];
      else v = clampf(s.root[2] - 0.5f - s.heights[i - (12 + 2 * D + A)], -1.0f, 1.0f) * P->obs_scale_height;
    }
    if (P->add_noise) v = v + (2.0f * s.U[S_NOISE + i] - 1.0f) * P->noise_vec[i];
    s.cur[i] = v;
  }
  float* hist_g = B->obs_history + (size_t)e * H * Pp;
  for (int i = 0; i < H * Pp; ++i) s.hist[i] = reset ? 0.f : hist_g[i];  // go2.py:238
  const float co = P->clip_obs;
  float* obs = B->obs + (size_t)e * P->num_obs;
  float* cr = B->critic ? B->critic + (size_t)e * P->num_critic : nullptr;
  for (int i = 0; i < H * Pp; ++i) {
    const float v = clampf(s.hist[i], -co, co);
    obs[i] = v;
    if (go2 && cr) cr[i] = v;
  }
  for (int i = 0; i < Pp; ++i) {
    const float v = clampf(s.cur[i], -co, co);
    obs[H * Pp + i] = v;
    if (go2 && cr) cr[H * Pp + i] = v;
  }
  if (go2) {
    const int NO = P->num_obs;
    for (int i = 0; i < P->num_priv; ++i) {  // [mass params (4), friction, kp-1 (D), kd-1 (D)]
      float v;
      if (i < 4) v = B->mass_params[e * 4 + i];
      else if (i == 4) v = B->friction[e];
      else if (i < 5 + D) v = s.kpm[i - 5] - 1.0f;
      else v = s.kdm[i - 5 - D] - 1.0f;
      v = clampf(v, -co, co);
      B->priv[(size_t)e * P->num_priv + i] = v;
      if (cr) cr[NO + i] = v;
    }
    for (int i = 0; i < 3; ++i) {
      const float v = clampf(s.blv[i] * P->obs_scale_lin_vel, -co, co);
      B->est[(size_t)e * P->num_est + i] = v;
      if (cr) cr[NO + P->num_priv + i] = v;
    }
    for (int i = 0; i < P->num_scan; ++i) {
      const float v = clampf(s.root[2] - 0.3f - s.heights[i], -1.0f, 1.0f);
      B->scan[(size_t)e * P->num_scan + i] = v;
      if (cr) cr[NO + P->num_priv + 3 + i] = clampf(v, -co, co);
    }
  }
  for (int i = 0; i < H * Pp; ++i)  // history update go2.py:570-574
    hist_g[i] = (s.ep <= 1) ? s.cur[i % Pp] : (i < (H - 1) * Pp ? s.hist[i + Pp] : s.cur[i - (H - 1) * Pp]);
  // last_* copies go2.py:380-384 and state write-back
  memcpy(B->last_actions + (size_t)e * A, s.act, sizeof(float) * A);
  for (int j = 0; j < D; ++j) {
    B->last_dof_vel[(size_t)e * D + j] = s.thd[j];
    B->last_torques[(size_t)e * D + j] = s.tau[j];
    B->dof_state[((size_t)e * D + j) * 2] = s.th[j];
    B->dof_state[((size_t)e * D + j) * 2 + 1] = s.thd[j];
  }
  memcpy(B->last_root_vel + e * 6, s.root + 7, sizeof(float) * 6);
  memcpy(B->last_base_lin_vel + e * 3, s.blv, sizeof(float) * 3);
  if (B->base_lin_vel) memcpy(B->base_lin_vel + e * 3, s.blv, sizeof(float) * 3);
  if (B->base_ang_vel) memcpy(B->base_ang_vel + e * 3, s.bav, sizeof(float) * 3);
  if (B->projected_gravity) memcpy(B->projected_gravity + e * 3, s.pg, sizeof(float) * 3);
  memcpy(root_g, s.root, sizeof(float) * 13);
  memcpy(B->commands + e * 4, s.cmd, sizeof(float) * 4);
  if (go2 && !reset)
    for (int f = 0; f < F; ++f) {
      B->last_contacts[e * F + f] = (uint8_t)s.lc[f];
      B->last_contact_heights[e * F + f] = s.lch[f];
      if (B->feet_air_time) B->feet_air_time[e * F + f] = s.fat[f];
    }
  B->episode_length[e] = s.ep;
  if (B->rpy_phase) {
    const float v[8] = {s.roll, s.pitch, s.yaw, s.ph[0], s.ph[1], s.ph[2], s.ph[3], s.jump};
    memcpy(B->rpy_phase + e * 8, v, sizeof(v));
  }
  if (B->measured_heights)
    memcpy(B->measured_heights + (size_t)e * P->num_height_points, s.heights, sizeof(float) * P->num_height_points);
}

// Episode statistics (extras['episode'] numerators and the reset count): per-env rows of
// the envs that reset, summed in env order after the parallel loop (deterministic).
static void fold_stats(const lgx_buffers* B, int N, int KS, const std::vector<float>& rows,
                       const std::vector<uint8_t>& hit) {
  if (!B->episode_stats) return;
  for (int e = 0; e < N; ++e)
    if (hit[e])
      for (int k = 0; k <= KS; ++k) B->episode_stats[k] += rows[(size_t)e * (KS + 1) + k];
}

void step(const lgx_model* M, const lgx_task_params* P, const lgx_buffers* B, uint64_t seed, uint64_t stepn,
          bool physics) {
  const int N = P->num_envs, KS = P->num_reward_terms + (P->has_termination_reward ? 1 : 0);
  std::vector<float> rows((size_t)N * (KS + 1), 0.f);
  std::vector<uint8_t> hit(N, 0);
#pragma omp parallel
  {
    Env* s = new Env;
#pragma omp for schedule(dynamic, 4)
    for (int e = 0; e < N; ++e) {
      env_step(*s, M, P, B, seed, stepn, physics, e, &rows[(size_t)e * (KS + 1)]);
      hit[e] = B->reset[e];
    }
    delete s;
  }
  fold_stats(B, N, KS, rows, hit);
}

void reset(const lgx_task_params* P, const lgx_buffers* B, const uint8_t* mask, uint64_t seed, uint64_t call) {
  const int N = P->num_envs, D = P->num_dof, KS = P->num_reward_terms + (P->has_termination_reward ? 1 : 0);
  std::vector<float> rows((size_t)N * (KS + 1), 0.f);
  std::vector<uint8_t> hit(mask, mask + N);
#pragma omp parallel
  {
    Env* s = new Env;
#pragma omp for schedule(static)
    for (int e = 0; e < N; ++e) {
      if (!mask[e]) continue;
      fill_uniforms(*s, P, seed, (uint32_t)(P->env_id_offset + e), call, 1);
      memcpy(s->root, B->root_states + (size_t)e * 13, sizeof(s->root));
      memcpy(s->cmd, B->commands + e * 4, sizeof(s->cmd));
      // an external reset exists only once the env is built: the terrain curriculum applies
      reset_env(P, B, *s, e, true, &rows[(size_t)e * (KS + 1)]);
      memcpy(B->root_states + (size_t)e * 13, s->root, sizeof(s->root));
      for (int j = 0; j < D; ++j) {
        B->dof_state[((size_t)e * D + j) * 2] = s->th[j];
        B->dof_state[((size_t)e * D + j) * 2 + 1] = s->thd[j];
      }
      memcpy(B->commands + e * 4, s->cmd, sizeof(s->cmd));
      B->episode_length[e] = s->ep;
      B->reset[e] = 1;
    }
    delete s;
  }
  fold_stats(B, N, KS, rows, hit);
}

void episode_extras(const lgx_task_params* P, const lgx_buffers* B, float* means, float* level_mean,
                    uint8_t* time_outs, uint64_t* step_counter) {
  const int N = P->num_envs, KS = P->num_reward_terms + (P->has_termination_reward ? 1 : 0);
  float* st = B->episode_stats;
  const float cnt = st[KS];
  const float inv_T = 1.0f / P->max_episode_length_s;  // torch: tensor / python float
  if (cnt > 0.f) {
    for (int k = 0; k < KS; ++k) means[k] = st[k] / cnt * inv_T;
    if (level_mean) {
      double t = 0.0;
      for (int e = 0; e < N; ++e) t += (double)B->terrain_levels[e];
      *level_mean = (float)(t / N);
    }
  }
  if (time_outs) {
    int any = 0;
    for (int e = 0; e < N && !any; ++e) any |= B->reset[e];
    if (any) memcpy(time_outs, B->time_out, (size_t)N);
  }
  for (int k = 0; k <= KS; ++k) st[k] = 0.f;
  if (step_counter) *step_counter += 1;
}

// update_command_curriculum (go2.py:80-107 / legged_robot.py:580-591): the kernel's rule
// (lgx_env.hip curriculum_kernel), envs in order
void command_curriculum(const lgx_task_params* P, const lgx_buffers* B, uint64_t seed, uint64_t step,
                        const double* global_sum_count) {
  if (step % (uint64_t)P->max_episode_length != 0) return;
  const int N = P->num_envs;
  double S = 0.0, Cn = 0.0;
  if (global_sum_count) {
    S = global_sum_count[0];
    Cn = global_sum_count[1];
  } else {
    for (int e = 0; e < N; ++e)
      if (B->reset[e]) { S += (double)B->curriculum_vals[e]; Cn += 1.0; }
  }
  if (Cn <= 0.0) return;
  const float mean = ((float)S / (float)Cn) / (float)P->max_episode_length;
  if (!(mean > P->curriculum_threshold)) return;
  double* R = B->command_ranges;
  const double lo = R[0], hi = R[1], d = P->curriculum_delta;
  const double lo_max = P->curriculum_lo_free ? lo - d : P->curriculum_lo_max;
  const double nlo = std::min(std::max(lo - d, P->curriculum_lo_min), lo_max);  // np.clip
  const double nhi = std::min(std::max(hi + d, 0.0), P->curriculum_hi_max);
  const bool changed = nlo != lo || nhi != hi;
  R[0] = nlo;
  R[1] = nhi;
  if (float* L = B->command_range_log) {
    if (P->command_curriculum == 1) { L[0] = (float)nhi; L[1] = (float)nlo; L[2] = (float)R[3]; L[3] = (float)R[5]; }
    else { L[0] = (float)nhi; L[1] = (float)R[3]; L[2] = (float)R[5]; }
  }
  if (!changed) return;
  const bool go2 = P->task_kind == LGX_TASK_GO2;
  const int Pp = P->num_proprio, H = P->history_len, c0 = go2 ? 5 : 9;
  const float co = P->clip_obs;
  for (int e = 0; e < N; ++e) {
    if (!B->reset[e]) continue;
    const uint32_t gid = (uint32_t)(P->env_id_offset + e);
    auto uni = [&](int slot) {
      uint32_t o[4];
      philox(gid, (uint32_t)step, (uint32_t)(slot >> 2), (uint32_t)(step >> 32), (uint32_t)seed,
             (uint32_t)(seed >> 32), o);
      return unit(o[slot & 3]);
    };
    float U[4];
    for (int k = 0; k < 4; ++k) U[k] = uni(S_RCMD + k);
    float* cmd = B->commands + e * 4;
    resample_commands(P, R, cmd, U, 0, B->root_states + (size_t)e * 13 + 3);
    float* obs = B->obs + (size_t)e * P->num_obs;
    float* cr = (go2 && B->critic) ? B->critic + (size_t)e * P->num_critic : nullptr;
    float* hist = B->obs_history + (size_t)e * H * Pp;
    for (int j = 0; j < 3; ++j) {
      const int i = c0 + j;
      float v = cmd[j] * P->commands_scale[j];
      if (P->add_noise) v = v + (2.0f * uni(S_NOISE + i) - 1.0f) * P->noise_vec[i];
      const float vc = clampf(v, -co, co);
      obs[H * Pp + i] = vc;
      if (cr) cr[H * Pp + i] = vc;
      for (int t = 0; t < H; ++t) hist[t * Pp + i] = v;
    }
  }
}

int threads() { return omp_get_max_threads(); }

}  // namespace lgxh
