/*
 * lgx_oracle.c — CPU ORACLE (test infrastructure; never linked into the product).
 *
 * A plain-C, env-by-env restatement of the reference's env step, used only by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker:
 *
 *   post-physics  : Go2Robot.post_physics_step go2.py:345-387 and
 *                   LeggedRobot.post_physics_step legged_robot.py:103-138, statement by
 *                   statement, in the reference's fp32 operation order (compile with
 *                   -ffp-contract=off so a*b+c stays two roundings, like eager torch).
 *                   Pinned against tests/golden/ fixtures recorded from the reference's own
 *                   tensor code (tools/gen_golden.py, masked-RNG mode).
 *   actuator      : LeggedRobot._compute_torques legged_robot.py:440-478 (pinned).
 *   physics       : this build's articulated-body + contact solver (replaces the closed
 *                   PhysX binary, legged_robot.py:82). PARITY UNPINNED vs the reference
 *                   (no PhysX oracle exists); restated here densely
 *                   (18x18 mass matrix, dense Cholesky, double precision) as an independent
 *                   check of the HIP kernel's structured fp32 solver. See oracle_physics.c.
 *   RNG           : Philox4x32-10 (oracle/philox.py has the slot layout).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/lgx.h"
#include "lgx_oracle.h"

/* ------------------------------------------------------------------------- RNG */
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
    uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += PHILOX_W0; k1 += PHILOX_W1;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* uniform for slot s of env e at (step, stream) */
static float urand(uint64_t seed, uint32_t env, uint64_t step, uint32_t stream, int slot) {
  uint32_t ctr[4] = {env, (uint32_t)step, (uint32_t)((slot >> 2) | (stream << 16)), (uint32_t)(step >> 32)};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t o[4];
  oracle_philox4x32_10(ctr, key, o);
  return (float)(o[slot & 3] >> 8) * (1.0f / 16777216.0f);
}

/* torch_rand_float(lo, hi): (hi - lo) * u + lo  (isaacgym torch_utils; fp32) */
static float rand_range(float lo, float hi, float u) {
  float span = (float)((double)hi - (double)lo);
  float r = span * u;
  return r + lo;
}
/* the same with Python-float bounds: (hi - lo) in double, then an fp32 scalar in the tensor ops */
static float rand_range_d(double lo, double hi, float u) {
  float span = (float)(hi - lo);
  float r = span * u;
  return r + (float)lo;
}

/* ------------------------------------------------------------ small fp32 math */
/* isaacgym torch_utils.quat_rotate_inverse (xyzw): a - b + c */
static void quat_rotate_inverse(const float q[4], const float v[3], float out[3]) {
  float w = q[3];
  float s = 2.0f * (w * w) - 1.0f;
  float cx = q[1] * v[2] - q[2] * v[1];
  float cy = q[2] * v[0] - q[0] * v[2];
  float cz = q[0] * v[1] - q[1] * v[0];
  float d = q[0] * v[0] + q[1] * v[1] + q[2] * v[2];
  float a[3] = {v[0] * s, v[1] * s, v[2] * s};
  float b[3] = {cx * w * 2.0f, cy * w * 2.0f, cz * w * 2.0f};
  float c[3] = {q[0] * d * 2.0f, q[1] * d * 2.0f, q[2] * d * 2.0f};
  for (int i = 0; i < 3; ++i) out[i] = a[i] - b[i] + c[i];
}

/* isaacgym torch_utils.quat_apply: b + w*t + xyz x t, t = 2 xyz x b */
static void quat_apply(const float q[4], const float b[3], float out[3]) {
  float t0 = (q[1] * b[2] - q[2] * b[1]) * 2.0f;
  float t1 = (q[2] * b[0] - q[0] * b[2]) * 2.0f;
  float t2 = (q[0] * b[1] - q[1] * b[0]) * 2.0f;
  float x0 = q[1] * t2 - q[2] * t1;
  float x1 = q[2] * t0 - q[0] * t2;
  float x2 = q[0] * t1 - q[1] * t0;
  out[0] = b[0] + q[3] * t0 + x0;
  out[1] = b[1] + q[3] * t1 + x1;
  out[2] = b[2] + q[3] * t2 + x2;
}

/* legged_gym/utils/math.py:45-48 wrap_to_pi */
static float wrap_to_pi(float a) {
  const float two_pi = (float)(2.0 * M_PI);
  const float pi = (float)M_PI;
  /* torch remainder (python %): fmod then fix sign */
  float m = fmodf(a, two_pi);
  if (m != 0.0f && ((m < 0.0f) != (two_pi < 0.0f))) m += two_pi;
  m -= two_pi * (float)(m > pi);
  return m;
}

static float torch_remainder(float a, float b) {
  float m = fmodf(a, b);
  if (m != 0.0f && ((m < 0.0f) != (b < 0.0f))) m += b;
  return m;
}

static float clipf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
static float sq(float x) { return x * x; }
static float norm3(const float* v) { return sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }
static float norm2(float a, float b) { return sqrtf(a * a + b * b); }

/* --------------------------------------------------------- actuator (pinned) */
/* ANYmal SEA actuator network, Anymal._compute_torques anymal.py:71-81: one step of the
   2-layer LSTM (torch.nn.LSTM cell: gates = W_ih x + b_ih + W_hh h + b_hh, order i f g o;
   c' = f c + i g; h' = o tanh(c')) then Linear, per joint; state [2, N*D, 8] in place. */
static float sigm(float x) { return 1.0f / (1.0f + expf(-x)); }

static void lstm_layer(const float* w_ih, int nin, const float* w_hh, const float* b_ih, const float* b_hh,
                       const float* x, float* h, float* c) {
  float gates[32], hn[8];
  for (int g = 0; g < 32; ++g) {
    float a = 0.0f, b = 0.0f;
    for (int k = 0; k < nin; ++k) a += w_ih[g * nin + k] * x[k];
    for (int k = 0; k < 8; ++k) b += w_hh[g * 8 + k] * h[k];
    gates[g] = (a + b_ih[g]) + (b + b_hh[g]);
  }
  for (int u = 0; u < 8; ++u) {
    float i = sigm(gates[u]), f = sigm(gates[8 + u]), gg = tanhf(gates[16 + u]), o = sigm(gates[24 + u]);
    c[u] = f * c[u] + i * gg;
    hn[u] = o * tanhf(c[u]);
  }
  for (int u = 0; u < 8; ++u) h[u] = hn[u];
}

static float sea_torque(const lgx_task_params* P, const lgx_buffers* B, int e, int j, float in0, float in1) {
  const size_t NT = (size_t)P->num_envs * P->num_dof, r = (size_t)e * P->num_dof + j;
  float* h0 = B->sea_hidden + r * 8;
  float* c0 = B->sea_cell + r * 8;
  float* h1 = B->sea_hidden + (NT + r) * 8;
  float* c1 = B->sea_cell + (NT + r) * 8;
  float x[2] = {in0 * P->sea_in_scale[0], in1 * P->sea_in_scale[1]};
  lstm_layer(P->sea_w_ih0, 2, P->sea_w_hh0, P->sea_b_ih0, P->sea_b_hh0, x, h0, c0);
  lstm_layer(P->sea_w_ih1, 8, P->sea_w_hh1, P->sea_b_ih1, P->sea_b_hh1, h0, h1, c1);
  float y = 0.0f;
  for (int k = 0; k < 8; ++k) y += P->sea_lin_w[k] * h1[k];
  return P->sea_out_scale * (y + P->sea_lin_b);
}

/* LeggedRobot._compute_torques, legged_robot.py:440-478 (P control, kp/kd mult.) */
void oracle_compute_torques(const lgx_task_params* P, const lgx_buffers* B, int e) {
  const int D = P->num_dof, N = P->num_envs;
  if (P->actuator_net) {
    for (int j = 0; j < D; ++j) {
      float a = B->actions[e * P->num_actions + j];
      float q = B->dof_state[(e * D + j) * 2 + 0];
      float qd = B->dof_state[(e * D + j) * 2 + 1];
      B->torques[e * D + j] = sea_torque(P, B, e, j, (a * P->action_scale + P->default_dof_pos[j]) - q, qd);
    }
    return;
  }
  for (int j = 0; j < D; ++j) {
    float a = B->actions[e * P->num_actions + j];
    float q = B->dof_state[(e * D + j) * 2 + 0];
    float qd = B->dof_state[(e * D + j) * 2 + 1];
    float as = a * P->action_scale;
    float t;
    if (P->control_type == LGX_CONTROL_P) {
      float err = (as + P->default_dof_pos[j]) - q;
      if (P->randomize_kp_kd) {
        float kpm = B->kp_kd[(0 * N + e) * D + j], kdm = B->kp_kd[(1 * N + e) * D + j];
        t = (kpm * P->p_gains[j]) * err - (kdm * P->d_gains[j]) * qd;
      } else {
        t = P->p_gains[j] * err - P->d_gains[j] * qd;
      }
    } else if (P->control_type == LGX_CONTROL_V) {
      float lv = B->last_dof_vel[e * D + j];
      t = P->p_gains[j] * (as - qd) - P->d_gains[j] * ((qd - lv) / P->sim_dt);
    } else {
      t = as;
    }
    B->torques[e * D + j] = clipf(t, -P->torque_limits[j], P->torque_limits[j]);
  }
}

/* ------------------------------------------------------------ terrain heights */
/* LeggedRobot._get_heights legged_robot.py:997-1032 (+ quat_apply_yaw math.py:38-42) */
static void get_heights(const lgx_task_params* P, const lgx_buffers* B, int e, float* out) {
  const int NP = P->num_height_points;
  if (P->mesh_type == LGX_MESH_PLANE || B->height_samples == NULL) {
    for (int i = 0; i < NP; ++i) out[i] = 0.0f;
    return;
  }
  const float* root = B->root_states + e * 13;
  float qy[4] = {0.0f, 0.0f, root[5], root[6]};
  float n = sqrtf(qy[2] * qy[2] + qy[3] * qy[3]);
  if (n < 1e-9f) n = 1e-9f;
  qy[2] = qy[2] / n; qy[3] = qy[3] / n;
  for (int i = 0; i < NP; ++i) {
    float p[3] = {P->height_points[i][0], P->height_points[i][1], 0.0f}, w[3];
    quat_apply(qy, p, w);
    float px = w[0] + root[0], py = w[1] + root[1];
    px = px + P->border_size; py = py + P->border_size;
    long ix = (long)(px / P->horizontal_scale), iy = (long)(py / P->horizontal_scale);
    if (ix < 0) ix = 0;
    if (ix > P->hf_rows - 2) ix = P->hf_rows - 2;
    if (iy < 0) iy = 0;
    if (iy > P->hf_cols - 2) iy = P->hf_cols - 2;
    int16_t h1 = B->height_samples[ix * P->hf_cols + iy];
    int16_t h2 = B->height_samples[(ix + 1) * P->hf_cols + iy];
    int16_t h3 = B->height_samples[ix * P->hf_cols + iy + 1];
    int16_t h = h1 < h2 ? h1 : h2;
    h = h < h3 ? h : h3;
    out[i] = (float)h * P->vertical_scale;
  }
}

/* ------------------------------------------------------------ commands (RNG) */
/* Go2Robot._resample_commands go2.py:413-464 / LeggedRobot legged_robot.py:406-437 */
static void resample_commands(const lgx_task_params* P, lgx_buffers* B, int e, uint64_t seed, uint64_t step,
                              uint32_t stream, int slot0) {
  float* cmd = B->commands + e * 4;
  uint32_t gid = (uint32_t)(P->env_id_offset + e);
  if (P->has_user_command) {
    for (int i = 0; i < 4; ++i) cmd[i] = P->user_command[i];
    return;
  }
  const double* R = B->command_ranges; /* self.command_ranges (Python floats), when bound */
  if (R) {
    cmd[0] = rand_range_d(R[0], R[1], urand(seed, gid, step, stream, slot0 + 0));
    cmd[1] = rand_range_d(R[2], R[3], urand(seed, gid, step, stream, slot0 + 1));
    if (P->heading_command)
      cmd[3] = rand_range_d(R[6], R[7], urand(seed, gid, step, stream, slot0 + 2));
    else
      cmd[2] = rand_range_d(R[4], R[5], urand(seed, gid, step, stream, slot0 + 2));
  } else {
    cmd[0] = rand_range(P->cmd_lin_vel_x[0], P->cmd_lin_vel_x[1], urand(seed, gid, step, stream, slot0 + 0));
    cmd[1] = rand_range(P->cmd_lin_vel_y[0], P->cmd_lin_vel_y[1], urand(seed, gid, step, stream, slot0 + 1));
    if (P->heading_command)
      cmd[3] = rand_range(P->cmd_heading[0], P->cmd_heading[1], urand(seed, gid, step, stream, slot0 + 2));
    else
      cmd[2] = rand_range(P->cmd_ang_vel_yaw[0], P->cmd_ang_vel_yaw[1], urand(seed, gid, step, stream, slot0 + 2));
  }
  float keep = (float)(norm2(cmd[0], cmd[1]) > 0.2f);
  cmd[0] = cmd[0] * keep;
  cmd[1] = cmd[1] * keep;
  if (P->zero_command) {
    float u = urand(seed, gid, step, stream, slot0 + 3);
    if (u < P->zero_command_prob) {
      if (P->task_kind == LGX_TASK_GO2) {
        cmd[0] = cmd[0] * 0.0f; cmd[1] = cmd[1] * 0.0f; cmd[2] = cmd[2] * 0.0f;
        if (P->heading_command) {
          const float fwd[3] = {1.0f, 0.0f, 0.0f};
          float f[3];
          quat_apply(B->root_states + e * 13 + 3, fwd, f);
          cmd[3] = atan2f(f[1], f[0]);
        }
      } else {
        for (int i = 0; i < 4; ++i) cmd[i] = cmd[i] * 0.0f;
      }
    }
  }
}

/* ------------------------------------------------------------------ reset_idx */
/* go2.py:207-263 / legged_robot.py:157-213 for one env. Episode stats are
 * accumulated into B->episode_stats[K] sums + [K] count (caller divides). */
static void reset_env(const lgx_task_params* P, lgx_buffers* B, int e, uint64_t seed, uint64_t step,
                      uint32_t stream, int after_init) {
  const int D = P->num_dof, N = P->num_envs;
  uint32_t gid = (uint32_t)(P->env_id_offset + e);
  float* root = B->root_states + e * 13;
  (void)N;
  /* terrain curriculum legged_robot.py:543-574 (only when init_done) */
  if (P->curriculum && after_init && B->terrain_levels) {
    float dx = root[0] - B->env_origins[e * 3 + 0];
    float dy = root[1] - B->env_origins[e * 3 + 1];
    float dist = norm2(dx, dy);
    int up = dist > P->terrain_length * P->promote_threshold;
    float expct = norm2(B->commands[e * 4 + 0], B->commands[e * 4 + 1]) * P->max_episode_length_s;
    int down = dist < expct * P->demote_threshold;
    int64_t lvl = B->terrain_levels[e];
    if (up) lvl += 1;
    if (down) lvl -= 1;
    if (lvl >= P->max_terrain_level) {
      float u = urand(seed, gid, step, stream, 6); /* SLOT_PUSH + 2 */
      lvl = (int64_t)(u * (float)P->max_terrain_level);
      if (lvl >= P->max_terrain_level) lvl = P->max_terrain_level - 1;
    } else if (lvl < 0) {
      lvl = 0;
    }
    B->terrain_levels[e] = lvl;
    int64_t tt = B->terrain_types[e];
    const float* o = B->terrain_origins + ((size_t)lvl * P->num_terrain_cols + tt) * 3;
    B->env_origins[e * 3 + 0] = o[0];
    B->env_origins[e * 3 + 1] = o[1];
    B->env_origins[e * 3 + 2] = o[2];
  }
  /* _reset_dofs legged_robot.py:481-506: q = q0 + U(0, 0.9), qd = 0 */
  for (int j = 0; j < D; ++j) {
    float u = urand(seed, gid, step, stream, 8 + j);
    B->dof_state[(e * D + j) * 2 + 0] = P->default_dof_pos[j] + rand_range(0.0f, 0.9f, u);
    B->dof_state[(e * D + j) * 2 + 1] = 0.0f;
  }
  /* _reset_root_states legged_robot.py:509-532 */
  for (int i = 0; i < 13; ++i) root[i] = P->base_init_state[i];
  for (int i = 0; i < 3; ++i) root[i] = root[i] + B->env_origins[e * 3 + i];
  if (P->custom_origins) {
    root[0] = root[0] + rand_range(-1.0f, 1.0f, urand(seed, gid, step, stream, 20));
    root[1] = root[1] + rand_range(-1.0f, 1.0f, urand(seed, gid, step, stream, 21));
  }
  for (int i = 0; i < 6; ++i) root[7 + i] = rand_range(-0.5f, 0.5f, urand(seed, gid, step, stream, 24 + i));
  /* _resample_commands (reset slots) */
  resample_commands(P, B, e, seed, step, stream, 32);
  /* buffers */
  for (int j = 0; j < P->num_actions; ++j) B->last_actions[e * P->num_actions + j] = 0.0f;
  for (int j = 0; j < D; ++j) B->last_dof_vel[e * D + j] = 0.0f;
  for (int i = 0; i < 6; ++i) B->last_root_vel[e * 6 + i] = 0.0f;
  for (int i = 0; i < 3; ++i) B->last_base_lin_vel[e * 3 + i] = 0.0f;
  for (int j = 0; j < D; ++j) B->last_torques[e * D + j] = 0.0f;
  for (int i = 0; i < P->history_len * P->num_proprio; ++i) B->obs_history[(size_t)e * P->history_len * P->num_proprio + i] = 0.0f;
  B->episode_length[e] = 0;
  B->reset[e] = 1;
  if (P->actuator_net && B->sea_hidden) { /* Anymal.reset_idx anymal.py:56-60 */
    const size_t NT = (size_t)P->num_envs * D;
    for (int l = 0; l < 2; ++l)
      for (int k = 0; k < D * 8; ++k) {
        B->sea_hidden[(l * NT + (size_t)e * D) * 8 + k] = 0.0f;
        B->sea_cell[(l * NT + (size_t)e * D) * 8 + k] = 0.0f;
      }
  }
  if (P->task_kind == LGX_TASK_GO2) {
    for (int f = 0; f < P->num_feet; ++f) {
      if (B->feet_air_time) B->feet_air_time[e * P->num_feet + f] = 0.0f;
      B->last_contacts[e * P->num_feet + f] = 0;
      B->last_contact_heights[e * P->num_feet + f] = 0.0f;
    }
  }
  int K = P->num_reward_terms + (P->has_termination_reward ? 1 : 0);
  const int KS = K;
  for (int k = 0; k < K; ++k) {
    if (B->episode_stats) B->episode_stats[k] += B->episode_sums[(size_t)e * KS + k];
    B->episode_sums[(size_t)e * KS + k] = 0.0f;
  }
  if (B->episode_stats) B->episode_stats[K] += 1.0f;
}

/* ------------------------------------------------------------------ rewards */
typedef struct {
  float blv[3], bav[3], pg[3];
  float roll, pitch, yaw;
  float phase_fl, phase_fr, phase_bl, phase_br;
  int contact[4]; /* fl, fr, bl, br filtered contacts */
  float feet_z[4];
  float heights[LGX_MAX_HEIGHT_POINTS];
  float jump_flag;
} env_scratch;

static float cmd_norm3(const float* c) { return norm3(c); }

static float reward_term(const lgx_task_params* P, lgx_buffers* B, int e, int id, const env_scratch* s) {
  const int D = P->num_dof, A = P->num_actions, N = P->num_envs;
  const float* q = B->dof_state + (size_t)e * D * 2;
  const float* root = B->root_states + e * 13;
  const float* cmd = B->commands + e * 4;
  const float* cf = B->contact_forces + (size_t)e * P->num_bodies * 3;
  float r = 0.0f;
  (void)N;
  switch (id) {
    case LGX_REW_ACTION_RATE:
      for (int j = 0; j < A; ++j) r += sq(B->last_actions[e * A + j] - B->actions[e * A + j]);
      return r;
    case LGX_REW_ANG_VEL_XY: return sq(s->bav[0]) + sq(s->bav[1]);
    case LGX_REW_BASE_HEIGHT: {
      float acc = 0.0f;
      for (int i = 0; i < P->num_height_points; ++i) acc += root[2] - s->heights[i];
      float bh = acc / (float)P->num_height_points;
      return sq(bh - P->base_height_target);
    }
    case LGX_REW_CALF_COLLISION:
      for (int i = 0; i < 4; ++i) r += (float)(norm3(cf + P->calf_idx[i] * 3) > 0.1f);
      return r;
    case LGX_REW_CALF_POS:
      for (int i = 0; i < 4; ++i) { int j = P->calf_joint_idx[i]; r += sq(q[j * 2] - P->default_dof_pos[j]); }
      return r;
    case LGX_REW_CALF_SYMMETRY: {
      const int* c = P->calf_joint_idx;
      return fabsf(q[c[0] * 2] - q[c[1] * 2]) + fabsf(q[c[2] * 2] - q[c[3] * 2]);
    }
    case LGX_REW_COLLISION:
      for (int i = 0; i < P->n_penalised; ++i) r += (float)(norm3(cf + P->penalised_idx[i] * 3) > 0.1f);
      return r;
    case LGX_REW_DELTA_TORQUES:
      for (int j = 0; j < D; ++j) r += sq(B->torques[e * D + j] - B->last_torques[e * D + j]);
      return r;
    case LGX_REW_DOF_ACC:
      for (int j = 0; j < D; ++j) r += sq((B->last_dof_vel[e * D + j] - q[j * 2 + 1]) / P->dt);
      return r;
    case LGX_REW_DOF_ERROR:
      for (int j = 0; j < D; ++j) r += sq(q[j * 2] - P->default_dof_pos[j]);
      return r;
    case LGX_REW_DOF_POS_LIMITS:
      for (int j = 0; j < D; ++j) {
        float lo = q[j * 2] - P->dof_pos_limits[j][0];
        float hi = q[j * 2] - P->dof_pos_limits[j][1];
        float o = -(lo < 0.0f ? lo : 0.0f);
        o += (hi > 0.0f ? hi : 0.0f);
        r += o;
      }
      return r;
    case LGX_REW_DOF_VEL:
      for (int j = 0; j < D; ++j) r += sq(q[j * 2 + 1]);
      return r;
    case LGX_REW_DOF_VEL_LIMITS:
      for (int j = 0; j < D; ++j) r += clipf(fabsf(q[j * 2 + 1]) - P->dof_vel_limits[j] * P->soft_dof_vel_limit, 0.0f, 1.0f);
      return r;
    case LGX_REW_FEET_AIR_TIME: { /* go2.py:819-831 (mutates feet_air_time) */
      float* fat = B->feet_air_time + e * P->num_feet;
      uint8_t* lc = B->last_contacts + e * P->num_feet;
      float rew = 0.0f;
      for (int f = 0; f < P->num_feet; ++f) {
        int c = cf[P->feet_idx[f] * 3 + 2] > 1.0f;
        int cfilt = c || lc[f];
        float first = (float)((fat[f] > 0.0f) && cfilt);
        fat[f] = fat[f] + P->dt;
        rew += (fat[f] - 0.5f) * first;
      }
      rew = rew * (float)(norm2(cmd[0], cmd[1]) > 0.1f);
      for (int f = 0; f < P->num_feet; ++f) {
        int c = cf[P->feet_idx[f] * 3 + 2] > 1.0f;
        int cfilt = c || lc[f];
        fat[f] = fat[f] * (float)(!cfilt);
      }
      return rew;
    }
    case LGX_REW_FEET_CONTACT_FORCES:
      for (int f = 0; f < P->num_feet; ++f) {
        float v = norm3(cf + P->feet_idx[f] * 3) - P->max_contact_force;
        r += v > 0.0f ? v : 0.0f;
      }
      return r;
    case LGX_REW_HEADING_ALIGNMENT: {
      const float fwd[3] = {1.0f, 0.0f, 0.0f};
      float f[3];
      quat_apply(root + 3, fwd, f);
      float heading = atan2f(f[1], f[0]);
      float desired = 0.0f;
      if (P->heading_command) {
        /* wrap_to_pi mutates commands[:, 3] in place (Q7) */
        float w = wrap_to_pi(B->commands[e * 4 + 3]);
        B->commands[e * 4 + 3] = w;
        desired = w;
      }
      float err = wrap_to_pi(desired - heading);
      float nz = (float)(cmd_norm3(cmd) >= 0.2f);
      return sq(err) * nz;
    }
    case LGX_REW_HIP_POS:
      for (int i = 0; i < 4; ++i) { int j = P->hip_joint_idx[i]; r += sq(q[j * 2] - P->default_dof_pos[j]); }
      return r;
    case LGX_REW_JUMP_ZONE_FORWARD_VEL: {
      float fr = root[7] > 0.0f ? root[7] : 0.0f;
      return fr * (float)(s->jump_flag > 0.0f) * (float)(cmd_norm3(cmd) >= 0.2f);
    }
    case LGX_REW_JUMP_ZONE_UPWARD_VEL: {
      float up = root[9] > 0.0f ? root[9] : 0.0f;
      return up * (float)(s->jump_flag > 0.0f) * (float)(cmd_norm3(cmd) >= 0.2f);
    }
    case LGX_REW_LIN_VEL_Z: return sq(s->blv[2]);
    case LGX_REW_MIN_HEIGHT: {
      float ze = clipf(P->base_height_target - root[2], 0.0f, P->base_height_target);
      return ze * (float)(s->jump_flag > 0.0f);
    }
    case LGX_REW_ORIENTATION: return sq(s->pg[0]) + sq(s->pg[1]);
    case LGX_REW_PHASE_CONTACT_MATCH: {
      float thr = 2.0f * P->percent_time_on_ground - 1.0f;
      const float two_pi = (float)(2.0 * M_PI);
      float ph[4] = {s->phase_fl, s->phase_fr, s->phase_bl, s->phase_br};
      float rew = 0.0f;
      for (int f = 0; f < 4; ++f) {
        int stance = sinf(two_pi * ph[f]) <= thr;
        rew += (s->contact[f] == stance) ? 0.25f : -0.25f;
      }
      return rew;
    }
    case LGX_REW_PHASE_FOOT_LIFTING: {
      float thr = 2.0f * P->percent_time_on_ground - 1.0f;
      const float two_pi = (float)(2.0 * M_PI);
      float ph[4] = {s->phase_fl, s->phase_fr, s->phase_bl, s->phase_br};
      float rew = 0.0f;
      for (int f = 0; f < 4; ++f) {
        int stance = sinf(two_pi * ph[f]) <= thr;
        float h = s->feet_z[f] - B->last_contact_heights[e * P->num_feet + f];
        h = clipf(h, 0.0f, P->max_foot_height);
        float nh = h / P->max_foot_height;
        rew += stance ? -nh : nh;
      }
      return rew / 2.0f;
    }
    case LGX_REW_REVERSE_PENALTY: {
      float rv = root[7] < 0.0f ? root[7] : 0.0f;
      return -rv;
    }
    case LGX_REW_STAND_STILL: {
      for (int j = 0; j < D; ++j) r += fabsf(q[j * 2] - P->default_dof_pos[j]);
      return r * (float)(norm2(cmd[0], cmd[1]) < 0.1f);
    }
    case LGX_REW_STUMBLE_CALVES: {
      int any = 0;
      for (int i = 0; i < 4; ++i) {
        const float* c = cf + P->calf_idx[i] * 3;
        any |= norm2(c[0], c[1]) > 5.0f * fabsf(c[2]);
      }
      return (float)any;
    }
    case LGX_REW_STUMBLE_FEET: {
      int any = 0;
      for (int f = 0; f < P->num_feet; ++f) {
        const float* c = cf + P->feet_idx[f] * 3;
        any |= norm2(c[0], c[1]) > 5.0f * fabsf(c[2]);
      }
      return (float)any;
    }
    case LGX_REW_THIGH_POS:
      for (int i = 0; i < 4; ++i) { int j = P->thigh_joint_idx[i]; r += sq(q[j * 2] - P->default_dof_pos[j]); }
      return r;
    case LGX_REW_THIGH_SYMMETRY: {
      const int* c = P->thigh_joint_idx;
      return fabsf(q[c[0] * 2] - q[c[1] * 2]) + fabsf(q[c[2] * 2] - q[c[3] * 2]);
    }
    case LGX_REW_TORQUE_LIMITS:
      for (int j = 0; j < D; ++j) {
        float v = fabsf(B->torques[e * D + j]) - P->torque_limits[j] * P->soft_torque_limit;
        r += v > 0.0f ? v : 0.0f;
      }
      return r;
    case LGX_REW_TORQUES:
      for (int j = 0; j < D; ++j) r += sq(B->torques[e * D + j]);
      return r;
    case LGX_REW_TRACKING_ANG_VEL: {
      float err = sq(cmd[2] - s->bav[2]);
      return expf(-err / P->tracking_sigma);
    }
    case LGX_REW_TRACKING_LIN_VEL: {
      float err = sq(cmd[0] - s->blv[0]) + sq(cmd[1] - s->blv[1]);
      return expf(-err / P->tracking_sigma);
    }
    case LGX_REW_TRACKING_PITCH: {
      float deg = s->pitch * (float)(180.0 / M_PI);
      return expf(-sq(deg - P->pitch_deg_target) / P->tracking_sigma);
    }
    case LGX_REW_TRACKING_ROLL: {
      float deg = s->roll * (float)(180.0 / M_PI);
      return expf(-sq(deg - P->roll_deg_target) / P->tracking_sigma);
    }
    case LGX_REW_ZERO_CMD_DOF_ERROR: {
      float zm = (float)(cmd_norm3(cmd) < 0.2f);
      for (int j = 0; j < D; ++j) r += sq(q[j * 2] - P->default_dof_pos[j]);
      return r * zm;
    }
    default: return 0.0f;
  }
}

/* -------------------------------------------------------------- post-physics */
void oracle_post_physics(const lgx_task_params* P, lgx_buffers* B, uint64_t seed, uint64_t step) {
  const int N = P->num_envs, D = P->num_dof, A = P->num_actions;
  const int Pp = P->num_proprio, H = P->history_len;
  const int K = P->num_reward_terms;
  const int KS = K + (P->has_termination_reward ? 1 : 0);
  env_scratch* S = (env_scratch*)calloc((size_t)N, sizeof(env_scratch));
  int any_reset = 0;
  /* Pass 1 (per env, independent): everything up to and including reset_idx. */
  for (int e = 0; e < N; ++e) {
    env_scratch* s = &S[e];
    uint32_t gid = (uint32_t)(P->env_id_offset + e);
    float* root = B->root_states + e * 13;
    float* cmd = B->commands + e * 4;
    const float* cf = B->contact_forces + (size_t)e * P->num_bodies * 3;
    B->episode_length[e] += 1;
    int64_t ep = B->episode_length[e];
    /* base kinematics go2.py:358-361 */
    const float g[3] = {0.0f, 0.0f, -1.0f};
    quat_rotate_inverse(root + 3, root + 7, s->blv);
    quat_rotate_inverse(root + 3, root + 10, s->bav);
    quat_rotate_inverse(root + 3, g, s->pg);
    if (P->task_kind == LGX_TASK_GO2) {
      /* update_feet_states go2.py:266-328 */
      float ph = torch_remainder((float)ep * P->dt, P->period) / P->period;
      float pfr = torch_remainder(ph + P->offset_fr, 1.0f);
      float pbl = torch_remainder(ph + P->offset_bl, 1.0f);
      float pfl = torch_remainder(ph + P->offset_fl, 1.0f);
      float pbr = torch_remainder(ph + P->offset_br, 1.0f);
      float m = (cmd_norm3(cmd) < 0.2f) ? 0.0f : 1.0f;
      s->phase_fr = pfr * m; s->phase_fl = pfl * m; s->phase_bl = pbl * m; s->phase_br = pbr * m;
      uint8_t* lc = B->last_contacts + e * P->num_feet;
      for (int f = 0; f < 4; ++f) {
        int cur = cf[P->feet_idx[f] * 3 + 2] > 1.0f;
        s->contact[f] = cur || lc[f];
        lc[f] = (uint8_t)cur;
        const float* rb = B->rigid_body_states + ((size_t)e * P->num_bodies + P->feet_idx[f]) * 13;
        s->feet_z[f] = rb[2];
        if (s->contact[f]) B->last_contact_heights[e * P->num_feet + f] = rb[2];
      }
      /* quaternion_to_euler go2.py:11-31 */
      float x = root[3], y = root[4], z = root[5], w = root[6];
      float t0 = 2.0f * (w * x + y * z);
      float t1 = 1.0f - 2.0f * (x * x + y * y);
      s->roll = atan2f(t0, t1);
      float t2 = 2.0f * (w * y - z * x);
      t2 = clipf(t2, -1.0f, 1.0f);
      s->pitch = asinf(t2);
      float t3 = 2.0f * (w * z + x * y);
      float t4 = 1.0f - 2.0f * (y * y + z * z);
      s->yaw = atan2f(t3, t4);
    }
    /* _post_physics_step_callback go2.py:390-410 / legged_robot.py:383-403 */
    if (ep % P->resample_interval == 0) resample_commands(P, B, e, seed, step, 0, 0);
    if (P->heading_command) {
      const float fwd[3] = {1.0f, 0.0f, 0.0f};
      float f[3];
      quat_apply(root + 3, fwd, f);
      float heading = atan2f(f[1], f[0]);
      float gain = P->task_kind == LGX_TASK_GO2 ? P->heading_error_gain : 0.5f;
      float he = wrap_to_pi(cmd[3] - heading) * gain;
      if (P->task_kind != LGX_TASK_GO2) he = gain * wrap_to_pi(cmd[3] - heading);
      cmd[2] = clipf(he, -1.0f, 1.0f);
    }
    get_heights(P, B, e, s->heights);
    if (P->push_robots && (step % (uint64_t)P->push_interval == 0)) {
      root[7] = rand_range(-P->max_push_vel_xy, P->max_push_vel_xy, urand(seed, gid, step, 0, 4));
      root[8] = rand_range(-P->max_push_vel_xy, P->max_push_vel_xy, urand(seed, gid, step, 0, 5));
    }
    /* check_termination go2.py:186-204 */
    int reset = 0;
    for (int i = 0; i < P->n_termination; ++i) reset |= norm3(cf + P->termination_idx[i] * 3) > 1.0f;
    int tout = ep > P->max_episode_length;
    reset |= tout;
    reset |= s->pg[2] > 0.0f;
    if (P->parkour) reset |= root[2] < -1.0f;
    B->reset[e] = (uint8_t)reset;
    B->time_out[e] = (uint8_t)tout;
    /* jump flag (parkour) needs measured heights: go2.py:487-494 — computed before
     * rewards use it? No: jump_flags is set in compute_observations, i.e. AFTER the
     * rewards; rewards see the previous step's flag (carried in rpy_phase[7]). */
    s->jump_flag = B->rpy_phase ? B->rpy_phase[e * 8 + 7] : 0.0f;
    /* compute_reward legged_robot.py:216-237 */
    float rew = 0.0f;
    for (int k = 0; k < K; ++k) {
      float v = reward_term(P, B, e, P->reward_ids[k], s) * P->reward_scales[k];
      rew += v;
      B->episode_sums[(size_t)e * KS + k] += v;
    }
    if (P->only_positive_rewards) rew = rew < 0.0f ? 0.0f : rew;
    if (P->has_termination_reward) {
      float v = (float)(reset && !tout) * P->termination_scale;
      rew += v;
      B->episode_sums[(size_t)e * KS + K] += v;
    }
    B->rew[e] = rew;
    any_reset |= reset;
  }
  /* reset_idx: update_command_curriculum first (go2.py:221-223 / legged_robot.py:176-177),
     on steps where common_step_counter % max_episode_length == 0, over the resetting envs */
  if (P->command_curriculum && any_reset && step % (uint64_t)P->max_episode_length == 0) {
    float sum = 0.0f;
    int cnt = 0;
    for (int e = 0; e < N; ++e)
      if (B->reset[e]) { sum += B->episode_sums[(size_t)e * KS + P->curriculum_term]; ++cnt; }
    float mean = (sum / (float)cnt) / (float)P->max_episode_length; /* torch.mean (fp32) / max_episode_length */
    if (mean > P->curriculum_threshold) {
      double* R = B->command_ranges;
      double d = P->curriculum_delta, lo = R[0] - d, hi = R[1] + d;
      double lo_max = P->curriculum_lo_free ? R[0] - d : P->curriculum_lo_max;
      /* np.clip(x, a, b) = minimum(maximum(x, a), b) */
      lo = lo < P->curriculum_lo_min ? P->curriculum_lo_min : lo;
      lo = lo > lo_max ? lo_max : lo;
      hi = hi < 0.0 ? 0.0 : hi;
      hi = hi > P->curriculum_hi_max ? P->curriculum_hi_max : hi;
      R[0] = lo;
      R[1] = hi;
    }
  }
  /* per env (the terrain curriculum only reads per-env data) */
  for (int e = 0; e < N; ++e)
    if (B->reset[e]) reset_env(P, B, e, seed, step, 0, 1);
  (void)any_reset;
  /* compute_observations + last_* copies (per env) */
  for (int e = 0; e < N; ++e) {
    env_scratch* s = &S[e];
    uint32_t gid = (uint32_t)(P->env_id_offset + e);
    float* root = B->root_states + e * 13;
    const float* q = B->dof_state + (size_t)e * D * 2;
    float* hist = B->obs_history + (size_t)e * H * Pp;
    float cur[LGX_MAX_PROPRIO];
    int n = 0;
    if (P->task_kind == LGX_TASK_GO2) {
      const float two_pi = (float)(2.0 * M_PI);
      if (P->parkour) {
        int outl = 0;
        for (int i = 0; i < P->num_height_points; ++i) outl += fabsf(s->heights[i]) > 0.1f;
        s->jump_flag = (float)(outl >= 8);
      }
      for (int i = 0; i < 3; ++i) cur[n++] = s->bav[i] * P->obs_scale_ang_vel;
      cur[n++] = s->roll;
      cur[n++] = s->pitch;
      for (int i = 0; i < 3; ++i) cur[n++] = B->commands[e * 4 + i] * P->commands_scale[i];
      for (int j = 0; j < D; ++j) cur[n++] = (q[j * 2] - P->default_dof_pos[j]) * P->obs_scale_dof_pos;
      for (int j = 0; j < D; ++j) cur[n++] = q[j * 2 + 1] * P->obs_scale_dof_vel;
      for (int j = 0; j < A; ++j) cur[n++] = B->actions[e * A + j];
      float pf[4] = {s->phase_fr, s->phase_fl, s->phase_bl, s->phase_br};
      for (int f = 0; f < 4; ++f) {
        cur[n++] = sinf(two_pi * pf[f]);
        cur[n++] = cosf(two_pi * pf[f]);
      }
    } else {
      for (int i = 0; i < 3; ++i) cur[n++] = s->blv[i] * P->obs_scale_lin_vel;
      for (int i = 0; i < 3; ++i) cur[n++] = s->bav[i] * P->obs_scale_ang_vel;
      for (int i = 0; i < 3; ++i) cur[n++] = s->pg[i];
      for (int i = 0; i < 3; ++i) cur[n++] = B->commands[e * 4 + i] * P->commands_scale[i];
      for (int j = 0; j < D; ++j) cur[n++] = (q[j * 2] - P->default_dof_pos[j]) * P->obs_scale_dof_pos;
      for (int j = 0; j < D; ++j) cur[n++] = q[j * 2 + 1] * P->obs_scale_dof_vel;
      for (int j = 0; j < A; ++j) cur[n++] = B->actions[e * A + j];
      if (P->measure_heights)
        for (int i = 0; i < P->num_height_points; ++i)
          cur[n++] = clipf(root[2] - 0.5f - s->heights[i], -1.0f, 1.0f) * P->obs_scale_height;
    }
    if (P->add_noise)
      for (int i = 0; i < Pp; ++i) {
        float u = urand(seed, gid, step, 0, 36 + i);
        cur[i] = cur[i] + (2.0f * u - 1.0f) * P->noise_vec[i];
      }
    /* obs = [history ‖ cur], clip ±clip_obs (legged_robot.py:91-95) */
    float* obs = B->obs + (size_t)e * P->num_obs;
    for (int i = 0; i < H * Pp; ++i) obs[i] = clipf(hist[i], -P->clip_obs, P->clip_obs);
    for (int i = 0; i < Pp; ++i) obs[H * Pp + i] = clipf(cur[i], -P->clip_obs, P->clip_obs);
    if (P->task_kind == LGX_TASK_GO2) {
      float* pv = B->priv + (size_t)e * P->num_priv;
      int m = 0;
      for (int i = 0; i < 4; ++i) pv[m++] = B->mass_params[e * 4 + i];
      pv[m++] = B->friction[e];
      for (int j = 0; j < D; ++j) pv[m++] = B->kp_kd[(size_t)(0 * N + e) * D + j] - 1.0f;
      for (int j = 0; j < D; ++j) pv[m++] = B->kp_kd[(size_t)(1 * N + e) * D + j] - 1.0f;
      for (int i = 0; i < m; ++i) pv[i] = clipf(pv[i], -P->clip_obs, P->clip_obs);
      float* es = B->est + (size_t)e * P->num_est;
      for (int i = 0; i < 3; ++i) es[i] = clipf(s->blv[i] * P->obs_scale_lin_vel, -P->clip_obs, P->clip_obs);
      float* sc = B->scan + (size_t)e * P->num_scan;
      for (int i = 0; i < P->num_scan; ++i) sc[i] = clipf(root[2] - 0.3f - s->heights[i], -1.0f, 1.0f);
      /* critic = [obs ‖ priv ‖ est ‖ scan] (pre-clip values; clip applied after) */
      float* cr = B->critic + (size_t)e * P->num_critic;
      int c = 0;
      for (int i = 0; i < P->num_obs; ++i) cr[c++] = obs[i];
      for (int i = 0; i < P->num_priv; ++i) cr[c++] = pv[i];
      for (int i = 0; i < 3; ++i) cr[c++] = es[i];
      for (int i = 0; i < P->num_scan; ++i) cr[c++] = clipf(sc[i], -P->clip_obs, P->clip_obs);
    }
    /* history update go2.py:570-574 */
    if (B->episode_length[e] <= 1) {
      for (int h = 0; h < H; ++h)
        for (int i = 0; i < Pp; ++i) hist[h * Pp + i] = cur[i];
    } else {
      memmove(hist, hist + Pp, sizeof(float) * (size_t)(H - 1) * Pp);
      for (int i = 0; i < Pp; ++i) hist[(H - 1) * Pp + i] = cur[i];
    }
    /* last_* copies go2.py:380-384 */
    for (int j = 0; j < A; ++j) B->last_actions[e * A + j] = B->actions[e * A + j];
    for (int j = 0; j < D; ++j) B->last_dof_vel[e * D + j] = q[j * 2 + 1];
    for (int i = 0; i < 6; ++i) B->last_root_vel[e * 6 + i] = root[7 + i];
    for (int i = 0; i < 3; ++i) B->last_base_lin_vel[e * 3 + i] = s->blv[i];
    for (int j = 0; j < D; ++j) B->last_torques[e * D + j] = B->torques[e * D + j];
    /* exported per-env intermediates */
    if (B->base_lin_vel) for (int i = 0; i < 3; ++i) B->base_lin_vel[e * 3 + i] = s->blv[i];
    if (B->base_ang_vel) for (int i = 0; i < 3; ++i) B->base_ang_vel[e * 3 + i] = s->bav[i];
    if (B->projected_gravity) for (int i = 0; i < 3; ++i) B->projected_gravity[e * 3 + i] = s->pg[i];
    if (B->rpy_phase) {
      float* r = B->rpy_phase + e * 8;
      r[0] = s->roll; r[1] = s->pitch; r[2] = s->yaw;
      r[3] = s->phase_fl; r[4] = s->phase_fr; r[5] = s->phase_bl; r[6] = s->phase_br;
      r[7] = s->jump_flag;
    }
    if (B->measured_heights)
      for (int i = 0; i < P->num_height_points; ++i) B->measured_heights[(size_t)e * P->num_height_points + i] = s->heights[i];
  }
  free(S);
}

/* BaseTask.reset -> reset_idx(env_ids) outside a step (stream 1) */
void oracle_reset_envs(const lgx_task_params* P, lgx_buffers* B, const uint8_t* mask, uint64_t seed, uint64_t call,
                       int after_init) {
  for (int e = 0; e < P->num_envs; ++e)
    if (mask[e]) reset_env(P, B, e, seed, call, 1, after_init);
}

/* clip actions (legged_robot.py:74-75) */
void oracle_clip_actions(const lgx_task_params* P, lgx_buffers* B) {
  for (int i = 0; i < P->num_envs * P->num_actions; ++i)
    B->actions[i] = clipf(B->actions_in[i], -P->clip_actions, P->clip_actions);
}

/* full step: clip, decimation x (torques, physics substep), post-physics */
void oracle_step(const lgx_model* M, const lgx_task_params* P, lgx_buffers* B, uint64_t seed, uint64_t step) {
  oracle_clip_actions(P, B);
  /* envs are independent in the physics: OpenMP over envs (OMP_NUM_THREADS; 1 = serial) */
  for (int s = 0; s < P->decimation; ++s) {
#pragma omp parallel for schedule(static)
    for (int e = 0; e < P->num_envs; ++e) {
      oracle_compute_torques(P, B, e);
      oracle_physics_substep(M, P, B, e);
    }
  }
  oracle_post_physics(P, B, seed, step);
}

int64_t oracle_sizeof_params(void) { return (int64_t)sizeof(lgx_task_params); }
int64_t oracle_sizeof_model(void) { return (int64_t)sizeof(lgx_model); }
int64_t oracle_sizeof_buffers(void) { return (int64_t)sizeof(lgx_buffers); }
