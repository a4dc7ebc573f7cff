"""Config object -> lgx_task_params (the constants the HIP step and the oracle read).

Every derived constant is computed exactly as the reference derives it, in the same
precision (Python double, then rounded to fp32 where torch would store it):
  dt, max_episode_length, push_interval        legged_robot.py:946-955
  reward scale filtering and *dt, order          legged_robot.py:730-754 (alphabetical)
  soft dof limits (fp32 tensor ops)              legged_robot.py:344-357
  PD gains by joint-name substring               legged_robot.py:704-727
  noise vector                                   go2.py:110-129 / legged_robot.py:594-622
  height points meshgrid(x, y)                   legged_robot.py:980-994
  command resampling interval                    go2.py:393
"""
import math

import numpy as np

from . import _abi
from .utils.helpers import class_to_dict

F32 = np.float32


def reward_terms(cfg, dt):
    """(names, ids, scales_f32, termination_scale or None) in the reference's order."""
    scales = class_to_dict(cfg.rewards.scales)
    names, ids, vals = [], [], []
    term = None
    for key in list(scales.keys()):
        s = scales[key]
        if s == 0:
            continue
        s = s * dt
        if key == "termination":
            term = s
            continue
        if key not in _abi.REWARD_IDS:
            raise NotImplementedError(f"reward term '{key}' has no _reward_{key} implementation")
        names.append(key)
        ids.append(_abi.REWARD_IDS[key])
        vals.append(s)
    return names, ids, vals, term


def go2_proprio_layout(num_dof=12):
    """The Go2 current-observation vector (go2.py:506-515) as ordered (field, width) slots:
    the order the env kernel writes (lgx_env.hip compute_observations) and the deploy
    observation builder fills (deploy/base/deploy_base.py). Phase = sin/cos of the FR, FL,
    BL, BR gait phases (go2.py:497-504)."""
    return (("ang_vel", 3), ("roll_pitch", 2), ("command", 3), ("dof_pos", num_dof), ("dof_vel", num_dof),
            ("actions", num_dof), ("phase", 8))


GO2_PHASE_LEGS = ("fr", "fl", "bl", "br")


def noise_vector(cfg, go2):
    p = cfg.env.num_proprio
    v = np.zeros(p, dtype=np.float32)
    ns, lvl, sc = cfg.noise.noise_scales, cfg.noise.noise_level, cfg.normalization.obs_scales
    if go2:  # go2.py:120-127 — note the slot offsets (Appendix B Q1)
        v[0:3] = ns.ang_vel * lvl * sc.ang_vel
        v[3:5] = ns.imu * lvl
        v[5:8] = 0.0
        v[8:9] = 0.0
        v[9:21] = ns.dof_pos * lvl * sc.dof_pos
        v[21:33] = ns.dof_vel * lvl * sc.dof_vel
        v[33:45] = 0.0
        v[45:53] = 0.0
    else:  # legged_robot.py:611-621
        v[:3] = ns.lin_vel * lvl * sc.lin_vel
        v[3:6] = ns.ang_vel * lvl * sc.ang_vel
        v[6:9] = ns.gravity * lvl
        v[9:12] = 0.0
        v[12:24] = ns.dof_pos * lvl * sc.dof_pos
        v[24:36] = ns.dof_vel * lvl * sc.dof_vel
        v[36:48] = 0.0
        if cfg.terrain.measure_heights:
            v[48:235] = ns.height_measurements * lvl * sc.height_measurements
    return v


def soft_dof_limits(lower, upper, soft):
    lo = np.asarray(lower, dtype=F32)
    hi = np.asarray(upper, dtype=F32)
    m = (lo + hi) / F32(2)
    r = hi - lo
    return np.stack([m - (F32(0.5) * r) * F32(soft), m + (F32(0.5) * r) * F32(soft)], 1).astype(F32)


def build_task_params(cfg, model, num_envs, num_envs_total=None, env_id_offset=0, sim_dt=None, go2=True,
                      terrain_shape=None):
    P = _abi.TaskParams()
    P.abi_version = _abi.ABI_VERSION
    P.task_kind = _abi.TASK_GO2 if go2 else _abi.TASK_LEGGED
    P.num_envs = num_envs
    P.num_envs_total = num_envs_total or num_envs
    P.env_id_offset = env_id_offset
    D = len(model["dof_names"])
    names = model["body_names"]
    P.num_dof = D
    P.num_bodies = len(names)
    P.num_actions = cfg.env.num_actions
    P.num_proprio = cfg.env.num_proprio
    P.history_len = cfg.env.history_buffer_length
    P.num_obs = cfg.env.num_observations
    P.num_priv = cfg.env.num_privileged_obs
    P.num_est = cfg.env.num_estimated_obs
    P.num_scan = cfg.env.num_scan_obs
    P.num_critic = cfg.env.num_critic_obs
    P.decimation = cfg.control.decimation
    sdt = sim_dt if sim_dt is not None else cfg.sim.dt
    dt = cfg.control.decimation * sdt
    P.sim_dt = sdt
    P.dt = dt
    P.action_scale = cfg.control.action_scale
    P.clip_actions = cfg.normalization.clip_actions
    P.clip_obs = cfg.normalization.clip_observations
    P.control_type = _abi.CONTROL[cfg.control.control_type]
    dr = cfg.domain_rand
    P.randomize_kp_kd = int(getattr(dr, "randomize_kp_kd", False))
    links = model["links"][1:]
    for i, dn in enumerate(model["dof_names"]):
        P.default_dof_pos[i] = cfg.init_state.default_joint_angles[dn]
        kp = kd = 0.0
        for key in cfg.control.stiffness.keys():
            if key in dn:
                kp, kd = cfg.control.stiffness[key], cfg.control.damping[key]
        P.p_gains[i], P.d_gains[i] = kp, kd
        P.torque_limits[i] = links[i]["effort"]
        P.dof_vel_limits[i] = links[i]["velocity"]
    lim = soft_dof_limits([l["lower"] for l in links], [l["upper"] for l in links], cfg.rewards.soft_dof_pos_limit)
    for i in range(D):
        P.dof_pos_limits[i][0], P.dof_pos_limits[i][1] = float(lim[i, 0]), float(lim[i, 1])
    P.soft_dof_vel_limit = getattr(cfg.rewards, "soft_dof_vel_limit", 1.0)
    P.soft_torque_limit = getattr(cfg.rewards, "soft_torque_limit", 1.0)
    sc = cfg.normalization.obs_scales
    P.obs_scale_lin_vel, P.obs_scale_ang_vel = sc.lin_vel, sc.ang_vel
    P.obs_scale_dof_pos, P.obs_scale_dof_vel, P.obs_scale_height = sc.dof_pos, sc.dof_vel, sc.height_measurements
    P.add_noise = int(cfg.noise.add_noise)
    nv = noise_vector(cfg, go2)
    for i in range(len(nv)):
        P.noise_vec[i] = float(nv[i])
    P.measure_heights = int(cfg.terrain.measure_heights)
    xs, ys = cfg.terrain.measured_points_x, cfg.terrain.measured_points_y
    P.num_height_points = len(xs) * len(ys)
    for i, x in enumerate(xs):
        for j, y in enumerate(ys):
            P.height_points[i * len(ys) + j][0] = x
            P.height_points[i * len(ys) + j][1] = y
    # commands
    c = cfg.commands
    P.heading_command = int(c.heading_command)
    P.zero_command = int(getattr(c, "zero_command", False))
    P.zero_command_prob = getattr(c, "zero_command_prob", 0.0)
    P.resample_interval = int(c.resampling_time / dt)
    P.has_user_command = int(len(getattr(c, "user_command", [])) > 0)
    for i, v in enumerate(getattr(c, "user_command", [])[:4]):
        P.user_command[i] = v
    P.cmd_lin_vel_x[:] = c.ranges.lin_vel_x
    P.cmd_lin_vel_y[:] = c.ranges.lin_vel_y
    P.cmd_ang_vel_yaw[:] = c.ranges.ang_vel_yaw
    P.cmd_heading[:] = c.ranges.heading
    P.heading_error_gain = getattr(c, "heading_error_gain", 0.5)
    P.commands_scale[:] = [sc.lin_vel, sc.lin_vel, sc.ang_vel]
    e = cfg.env
    P.period = getattr(e, "period", 1.0)
    P.offset_fl, P.offset_fr = getattr(e, "fl_offset", 0.0), getattr(e, "fr_offset", 0.0)
    P.offset_bl, P.offset_br = getattr(e, "bl_offset", 0.0), getattr(e, "br_offset", 0.0)
    P.max_episode_length_s = e.episode_length_s
    P.max_episode_length = int(np.ceil(e.episode_length_s / dt))
    P.parkour = int(getattr(cfg.terrain, "parkour", False))
    # body index tables (legged_robot.py:846-894, go2.py:40-77)
    feet = [i for i, n in enumerate(names) if cfg.asset.foot_name in n]
    pen, term = [], []
    for key in cfg.asset.penalize_contacts_on:
        pen.extend([i for i, n in enumerate(names) if key in n])
    for key in cfg.asset.terminate_after_contacts_on:
        term.extend([i for i, n in enumerate(names) if key in n])
    P.num_feet = len(feet)
    P.n_termination, P.n_penalised = len(term), len(pen)
    for i, v in enumerate(term):
        P.termination_idx[i] = v
    for i, v in enumerate(pen):
        P.penalised_idx[i] = v
    for i, v in enumerate(feet[: _abi.MAX_FEET]):
        P.feet_idx[i] = v
    calves = [i for i, n in enumerate(names) if "calf" in n]
    for i, v in enumerate(calves[:4]):
        P.calf_idx[i] = v
    dn = model["dof_names"]
    for i, leg in enumerate(("FL", "FR", "RL", "RR")):
        for arr, j in ((P.hip_joint_idx, "hip"), (P.thigh_joint_idx, "thigh"), (P.calf_joint_idx, "calf")):
            name = f"{leg}_{j}_joint"
            arr[i] = dn.index(name) if name in dn else 0
    # rewards
    rn, rid, rs, term_scale = reward_terms(cfg, dt)
    P.num_reward_terms = len(rid)
    for i, (a, b) in enumerate(zip(rid, rs)):
        P.reward_ids[i] = a
        P.reward_scales[i] = b
    # command curriculum (go2.py:80-107 / legged_robot.py:580-591; lgx.h command_curriculum)
    c = cfg.commands
    if getattr(c, "curriculum", False):
        if "tracking_lin_vel" not in rn:
            # the reference indexes episode_sums['tracking_lin_vel'] (KeyError without the term)
            raise KeyError("commands.curriculum needs the tracking_lin_vel reward term")
        P.curriculum_term = rn.index("tracking_lin_vel")
        P.curriculum_threshold = float(np.float32(0.8 * rs[P.curriculum_term]))
        if go2:
            P.command_curriculum = 1
            P.curriculum_delta = float(c.vel_increment)
            P.curriculum_lo_min = float(c.max_reverse_vel)
            P.curriculum_lo_max = 0.0
            P.curriculum_lo_free = int(c.max_reverse_vel >= 0.0)
            P.curriculum_hi_max = float(c.max_forward_vel)
        else:
            P.command_curriculum = 2
            P.curriculum_delta = 0.05
            P.curriculum_lo_min = -float(c.max_curriculum)
            P.curriculum_lo_max = 0.0
            P.curriculum_hi_max = float(c.max_curriculum)
    P.only_positive_rewards = int(cfg.rewards.only_positive_rewards)
    P.has_termination_reward = int(term_scale is not None)
    P.termination_scale = term_scale or 0.0
    r = cfg.rewards
    P.tracking_sigma = r.tracking_sigma
    P.base_height_target = r.base_height_target
    P.max_foot_height = getattr(r, "max_foot_height", 0.0)
    P.percent_time_on_ground = getattr(r, "percent_time_on_ground", 0.5)
    P.max_contact_force = r.max_contact_force
    P.pitch_deg_target = getattr(r, "pitch_deg_target", 0.0)
    P.roll_deg_target = getattr(r, "roll_deg_target", 0.0)
    # events
    P.push_robots = int(getattr(dr, "push_robots", False))
    P.push_interval = int(np.ceil(getattr(dr, "push_interval_s", 15) / dt))
    P.max_push_vel_xy = getattr(dr, "max_push_vel_xy", 0.0)
    ist = cfg.init_state
    P.base_init_state[:] = list(ist.pos) + list(ist.rot) + list(ist.lin_vel) + list(ist.ang_vel)
    t = cfg.terrain
    P.mesh_type = {"plane": _abi.MESH_PLANE, "heightfield": _abi.MESH_HEIGHTFIELD,
                   "trimesh": _abi.MESH_TRIMESH}.get(t.mesh_type, _abi.MESH_PLANE)
    P.custom_origins = int(t.mesh_type in ("heightfield", "trimesh"))
    P.horizontal_scale, P.vertical_scale, P.border_size = t.horizontal_scale, t.vertical_scale, t.border_size
    P.curriculum = int(t.curriculum and t.mesh_type in ("heightfield", "trimesh"))
    P.terrain_length = t.terrain_length
    P.promote_threshold, P.demote_threshold = t.promote_threshold, t.demote_threshold
    P.num_terrain_rows, P.num_terrain_cols = t.num_rows, t.num_cols
    P.max_terrain_level = t.num_rows
    if terrain_shape is not None:  # Terrain.tot_rows, tot_cols (terrain.py:29-31)
        P.hf_rows, P.hf_cols = int(terrain_shape[0]), int(terrain_shape[1])
    # physics
    P.gravity[:] = cfg.sim.gravity
    P.ground_friction = t.static_friction
    P.solver_iterations = max(4, int(cfg.sim.physx.num_position_iterations) * 2)
    P.baumgarte = 0.2
    P.slop = 0.001
    P.max_depenetration_vel = cfg.sim.physx.max_depenetration_velocity
    P.contact_margin = cfg.sim.physx.contact_offset
    P.limit_margin = 0.01
    return P
