"""ctypes mirror of include/lgx.h (the C ABI of liblgx.so).

Field order and array sizes must match the header exactly; `check_layout()` compares
sizeof against the values the native library (and the oracle) report.
"""
import ctypes as C

ABI_VERSION = 6
MAX_DOF = 12
MAX_LINKS = 16
MAX_BODIES = 24
MAX_FEET = 4
MAX_PROPRIO = 240
MAX_HEIGHT_POINTS = 192
MAX_REWARDS = 40
MAX_CANDIDATES = 64
MAX_CONTACTS = 16
MAX_PENALISED = 24
MAX_TERMINATION = 8

TASK_LEGGED = 0
TASK_GO2 = 1
MESH_PLANE, MESH_HEIGHTFIELD, MESH_TRIMESH = 0, 1, 2
CONTROL = {"P": 0, "V": 1, "T": 2}

# enum lgx_reward_id (include/lgx.h) — name -> id
REWARD_IDS = {name: i for i, name in enumerate([
    "action_rate", "ang_vel_xy", "base_height", "calf_collision", "calf_pos", "calf_symmetry",
    "collision", "delta_torques", "dof_acc", "dof_error", "dof_pos_limits", "dof_vel",
    "dof_vel_limits", "feet_air_time", "feet_contact_forces", "heading_alignment", "hip_pos",
    "jump_zone_forward_vel", "jump_zone_upward_vel", "lin_vel_z", "min_height", "orientation",
    "phase_contact_match", "phase_foot_lifting", "reverse_penalty", "stand_still", "stumble_calves",
    "stumble_feet", "thigh_pos", "thigh_symmetry", "torque_limits", "torques", "tracking_ang_vel",
    "tracking_lin_vel", "tracking_pitch", "tracking_roll", "zero_cmd_dof_error",
])}

f32 = C.c_float
i32 = C.c_int32


class Model(C.Structure):
    _fields_ = [
        ("num_links", i32), ("num_bodies", i32), ("num_candidates", i32),
        ("link_parent", i32 * MAX_LINKS),
        ("joint_origin", (f32 * 3) * MAX_LINKS),
        ("joint_axis", (f32 * 3) * MAX_LINKS),
        ("joint_rot", (f32 * 9) * MAX_LINKS),
        ("joint_lower", f32 * MAX_LINKS),
        ("joint_upper", f32 * MAX_LINKS),
        ("joint_has_limits", i32 * MAX_LINKS),
        ("link_mass", f32 * MAX_LINKS),
        ("link_com", (f32 * 3) * MAX_LINKS),
        ("link_inertia", (f32 * 6) * MAX_LINKS),
        ("body_link", i32 * MAX_BODIES),
        ("body_offset", (f32 * 3) * MAX_BODIES),
        ("body_rot", (f32 * 9) * MAX_BODIES),
        ("cand_link", i32 * MAX_CANDIDATES),
        ("cand_body", i32 * MAX_CANDIDATES),
        ("cand_pos", (f32 * 3) * MAX_CANDIDATES),
        ("cand_radius", f32 * MAX_CANDIDATES),
    ]


class TaskParams(C.Structure):
    _fields_ = [
        ("abi_version", i32), ("task_kind", i32), ("num_envs", i32), ("num_envs_total", i32),
        ("env_id_offset", i32),
        ("num_dof", i32), ("num_bodies", i32), ("num_actions", i32), ("num_feet", i32),
        ("num_proprio", i32), ("history_len", i32), ("num_obs", i32), ("num_priv", i32), ("num_est", i32),
        ("num_scan", i32), ("num_critic", i32),
        ("num_height_points", i32), ("num_reward_terms", i32), ("decimation", i32),
        ("sim_dt", f32), ("dt", f32),
        ("action_scale", f32), ("clip_actions", f32), ("clip_obs", f32),
        ("control_type", i32), ("randomize_kp_kd", i32),
        ("p_gains", f32 * MAX_DOF), ("d_gains", f32 * MAX_DOF), ("default_dof_pos", f32 * MAX_DOF),
        ("torque_limits", f32 * MAX_DOF), ("dof_pos_limits", (f32 * 2) * MAX_DOF),
        ("dof_vel_limits", f32 * MAX_DOF),
        ("soft_dof_vel_limit", f32), ("soft_torque_limit", f32),
        ("obs_scale_lin_vel", f32), ("obs_scale_ang_vel", f32), ("obs_scale_dof_pos", f32),
        ("obs_scale_dof_vel", f32), ("obs_scale_height", f32),
        ("add_noise", i32), ("noise_vec", f32 * MAX_PROPRIO),
        ("measure_heights", i32), ("height_points", (f32 * 2) * MAX_HEIGHT_POINTS),
        ("heading_command", i32), ("zero_command", i32), ("resample_interval", i32), ("has_user_command", i32),
        ("cmd_lin_vel_x", f32 * 2), ("cmd_lin_vel_y", f32 * 2), ("cmd_ang_vel_yaw", f32 * 2),
        ("cmd_heading", f32 * 2),
        ("heading_error_gain", f32), ("zero_command_prob", f32),
        ("user_command", f32 * 4), ("commands_scale", f32 * 3),
        ("period", f32), ("offset_fl", f32), ("offset_fr", f32), ("offset_bl", f32), ("offset_br", f32),
        ("max_episode_length", i32), ("max_episode_length_s", f32), ("parkour", i32),
        ("n_termination", i32), ("termination_idx", i32 * MAX_TERMINATION),
        ("n_penalised", i32), ("penalised_idx", i32 * MAX_PENALISED),
        ("feet_idx", i32 * MAX_FEET), ("calf_idx", i32 * MAX_FEET),
        ("hip_joint_idx", i32 * MAX_FEET), ("thigh_joint_idx", i32 * MAX_FEET), ("calf_joint_idx", i32 * MAX_FEET),
        ("reward_ids", i32 * MAX_REWARDS), ("reward_scales", f32 * MAX_REWARDS),
        ("only_positive_rewards", i32), ("has_termination_reward", i32), ("termination_scale", f32),
        ("tracking_sigma", f32), ("base_height_target", f32), ("max_foot_height", f32),
        ("percent_time_on_ground", f32),
        ("max_contact_force", f32), ("pitch_deg_target", f32), ("roll_deg_target", f32),
        ("push_robots", i32), ("push_interval", i32), ("max_push_vel_xy", f32),
        ("base_init_state", f32 * 13), ("custom_origins", i32),
        ("mesh_type", i32), ("horizontal_scale", f32), ("vertical_scale", f32), ("border_size", f32),
        ("hf_rows", i32), ("hf_cols", i32),
        ("curriculum", i32), ("terrain_length", f32), ("promote_threshold", f32), ("demote_threshold", f32),
        ("max_terrain_level", i32), ("num_terrain_rows", i32), ("num_terrain_cols", i32),
        ("gravity", f32 * 3), ("ground_friction", f32), ("solver_iterations", i32),
        ("baumgarte", f32), ("slop", f32), ("max_depenetration_vel", f32), ("contact_margin", f32),
        ("limit_margin", f32),
        ("actuator_net", i32), ("sea_in_scale", f32 * 2), ("sea_out_scale", f32), ("sea_lin_b", f32),
        ("sea_w_ih0", f32 * 64), ("sea_w_hh0", f32 * 256), ("sea_b_ih0", f32 * 32), ("sea_b_hh0", f32 * 32),
        ("sea_w_ih1", f32 * 256), ("sea_w_hh1", f32 * 256), ("sea_b_ih1", f32 * 32), ("sea_b_hh1", f32 * 32),
        ("sea_lin_w", f32 * 8),
        ("command_curriculum", i32), ("curriculum_term", i32), ("curriculum_threshold", f32),
        ("curriculum_lo_free", i32), ("curriculum_delta", C.c_double), ("curriculum_lo_min", C.c_double),
        ("curriculum_lo_max", C.c_double), ("curriculum_hi_max", C.c_double),
    ]


P = C.c_void_p


class Buffers(C.Structure):
    _fields_ = [(name, P) for name in [
        "root_states", "dof_state", "contact_forces", "rigid_body_states",
        "actions_in", "actions", "torques",
        "last_actions", "last_dof_vel", "last_root_vel", "last_base_lin_vel", "last_torques",
        "commands", "episode_length", "episode_sums", "obs_history", "last_contacts",
        "last_contact_heights", "feet_air_time",
        "obs", "priv", "critic", "est", "scan", "rew", "reset", "time_out",
        "base_lin_vel", "base_ang_vel", "projected_gravity", "rpy_phase", "measured_heights",
        "friction", "mass_params", "kp_kd", "env_origins", "terrain_levels", "terrain_types",
        "terrain_origins", "height_samples", "terrain_mesh", "sea_hidden", "sea_cell", "episode_stats",
        "blew_up", "blowup_count", "command_ranges", "curriculum_vals", "command_range_log",
    ]]


BUFFER_FIELDS = [f[0] for f in Buffers._fields_]


def check_layout(lib, prefix):
    """Compare ctypes sizes with the native library's sizeof() exports."""
    for name, cls in (("model", Model), ("params", TaskParams), ("buffers", Buffers)):
        fn = getattr(lib, f"{prefix}{name}", None)
        if fn is None:
            continue
        fn.restype = C.c_int64
        n = fn()
        if n != C.sizeof(cls):
            raise RuntimeError(f"ABI layout mismatch for {name}: native {n} vs ctypes {C.sizeof(cls)}")
