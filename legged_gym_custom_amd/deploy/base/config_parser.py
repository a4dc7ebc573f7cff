"""ConfigParser — drop-in for deploy/base/config_parser.py:5-80: the unified MuJoCo/real
deploy YAML (network paths with {LEGGED_GYM_ROOT_DIR} and *model substitution, timing,
gains, default pose, scales, offsets, clipping, obs sizes, gait phase). Loaded with
yaml.safe_load (the reference uses FullLoader; the file is plain data)."""
import numpy as np
import yaml

from legged_gym_custom_amd import LEGGED_GYM_ROOT_DIR


def _path(cfg, key):
    return cfg[key].replace("{LEGGED_GYM_ROOT_DIR}", LEGGED_GYM_ROOT_DIR).replace("*model", cfg["model_name"])


class ConfigParser:
    def __init__(self, file_path) -> None:
        with open(file_path, "r") as f:
            cfg = yaml.safe_load(f)
        # real robot only
        self.msg_type = cfg["msg_type"]
        self.lowcmd_topic = cfg["lowcmd_topic"]
        self.lowstate_topic = cfg["lowstate_topic"]
        self.leg_joint2motor_idx = cfg["leg_joint2motor_idx"]
        self.weak_motor = cfg.get("weak_motor", [])
        # simulation only
        self.xml_path = cfg["xml_path"].replace("{LEGGED_GYM_ROOT_DIR}", LEGGED_GYM_ROOT_DIR)
        # networks
        self.policy_path = _path(cfg, "policy_path")
        self.adaptation_path = _path(cfg, "adaptation_path")
        self.estimator_path = _path(cfg, "estimator_path")
        self.scan_encoder_path = _path(cfg, "scan_encoder_path")
        # timing
        self.simulation_dt = cfg["simulation_dt"]
        self.control_decimation = cfg["control_decimation"]
        self.control_dt = self.simulation_dt * self.control_decimation
        # joints
        self.kps = cfg["kps"]
        self.kds = cfg["kds"]
        self.default_angles = np.array(cfg["default_angles"], dtype=np.float32)
        # scales / offsets
        self.lin_vel_scale = cfg["lin_vel_scale"]
        self.ang_vel_scale = cfg["ang_vel_scale"]
        self.dof_pos_scale = cfg["dof_pos_scale"]
        self.dof_vel_scale = cfg["dof_vel_scale"]
        self.action_scale = cfg["action_scale"]
        self.pitch_offset = cfg["pitch_offset"]
        self.roll_offset = cfg["roll_offset"]
        self.rc_scale = np.array(cfg["rc_scale"], dtype=np.float32)
        self.cmd_scale = np.array([self.lin_vel_scale, self.lin_vel_scale, self.ang_vel_scale], dtype=np.float32)
        # clipping
        self.clip_obs = cfg["clip_observations"]
        self.clip_actions = cfg["clip_actions"]
        # sizes
        self.num_actions = cfg["num_actions"]
        self.num_proprio = cfg["num_proprio"]
        self.buffer_length = cfg["buffer_length"]
        self.num_scan_obs = cfg["num_scan_obs"]
        self.num_obs = self.num_proprio + self.num_proprio * self.buffer_length
        # gait phase
        self.period = cfg["period"]
        self.fr_offset = cfg["fr_offset"]
        self.bl_offset = cfg["bl_offset"]
        self.fl_offset = cfg["fl_offset"]
        self.br_offset = cfg["br_offset"]
