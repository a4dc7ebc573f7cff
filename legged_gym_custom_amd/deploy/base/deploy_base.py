"""BaseController — drop-in for deploy/base/deploy_base.py:26-270 (the per-tick policy loop
a MuJoCo or real-robot subclass drives: it fills qj, dqj, ang_vel, base_quat (wxyz), cmd and
jump_button_pressed in _refresh_robot_states(), calls step(elapsed_s) and reads
target_dof_pos).

Built from three parts of this package instead of a monolithic tick:
  * `ProprioBuilder` fills the 52-wide Go2 current observation slot by slot from
    params.go2_proprio_layout() — the same table the env kernel's observation order follows
    (go2.py:506-515), evaluated without noise on a wxyz quaternion;
  * `ObsHistory` — the env's history rule for a single robot (filled with the first
    observation, then shifted; the network sees the history from BEFORE this tick);
  * `ScanReplay` — a recorded scan sequence replayed when armed and the gait phase reaches
    the recording's sync phase (deploy_base.py:110-147), zeros otherwise.
The networks are the four TorchScript files export_policy_as_jit writes.
"""
import logging
import re

import numpy as np
import torch

from legged_gym_custom_amd.deploy.base.config_parser import ConfigParser  # noqa: F401  (re-exported, as the reference)
from legged_gym_custom_amd.params import GO2_PHASE_LEGS, go2_proprio_layout

log = logging.getLogger(__name__)


def quaternion_to_euler(quat_angle):
    """(roll, pitch, yaw) of a wxyz quaternion; the xyzw form the env uses is go2.py:11-31."""
    w, x, y, z = quat_angle[0], quat_angle[1], quat_angle[2], quat_angle[3]
    return (np.arctan2(2.0 * (w * x + y * z), 1.0 - 2.0 * (x * x + y * y)),
            np.arcsin(np.clip(2.0 * (w * y - z * x), -1.0, 1.0)),
            np.arctan2(2.0 * (w * z + x * y), 1.0 - 2.0 * (y * y + z * z)))


def rotate_inverse_wxyz(q, v):
    """R(q)^T v for a wxyz quaternion (quat_rotate_inverse of isaacgym.torch_utils, wxyz order)."""
    w = float(q[0])
    u = np.asarray(q[1:4], dtype=np.float64)
    v = np.asarray(v, dtype=np.float64)
    return v * (2.0 * w * w - 1.0) - np.cross(u, v) * (2.0 * w) + u * (2.0 * np.dot(u, v))


def parse_scan_replay(text):
    """A scan recording: blank-line separated `[v v v ...]` blocks; the first block holds the
    sync phase, each further block one tick's scan observation. -> (sync phase, [vectors])."""
    vecs = []
    for block in re.split(r"\n\s*\n", text.strip()):
        body = block.strip()
        if body.startswith("["):
            body = body[1:]
        if body.endswith("]"):
            body = body[:-1]
        vecs.append([float(tok) for tok in body.split()])
    return vecs[0][0], vecs[1:]


class ScanReplay:
    """NORMAL -> (armed) WAITING -> (|phase - sync| < 0.005) REPLAY -> NORMAL. The replay stops
    one recording short of the end and rewinds (deploy_base.py:140-145)."""

    SYNC_TOL = 0.005

    def __init__(self, num_scan, sync_phase=-1.0, recording=()):
        self.num_scan = num_scan
        self.sync_phase = sync_phase
        self.recording = list(recording)
        self.mode = "NORMAL"
        self.index = 0

    @classmethod
    def from_file(cls, num_scan, path):
        with open(path) as f:
            sync, rec = parse_scan_replay(f.read())
        log.info("scan replay %s: %d recorded ticks, sync phase %.4f", path, len(rec), sync)
        return cls(num_scan, sync, rec)

    def next(self, phase, armed):
        """The (1, num_scan) scan observation for this tick."""
        if armed and self.mode == "NORMAL":
            self.mode = "WAITING"
        if self.mode == "WAITING" and abs(phase - self.sync_phase) < self.SYNC_TOL:
            self.mode = "REPLAY"
        if self.mode != "REPLAY":
            return torch.zeros((1, self.num_scan), dtype=torch.float32)
        out = torch.tensor(self.recording[self.index], dtype=torch.float32).reshape(1, -1)
        self.index += 1
        if self.index == len(self.recording) - 1:
            self.mode, self.index = "NORMAL", 0
        return out


class ObsHistory:
    """[length, width] history rows, oldest first."""

    def __init__(self, length, width):
        self.rows = np.zeros((length, width), dtype=np.float32)
        self.primed = False

    def push(self, cur):
        if not self.primed:
            self.rows[:] = cur
            self.primed = True
        else:
            self.rows[:-1] = self.rows[1:]
            self.rows[-1] = cur


class ProprioBuilder:
    """The Go2 current observation (go2.py:506-515) of one robot, noise-free."""

    def __init__(self, cfg):
        self.cfg = cfg
        self.layout = go2_proprio_layout(cfg.num_actions)
        self.offsets = {}
        off = 0
        for name, width in self.layout:
            self.offsets[name] = (off, off + width)
            off += width
        assert off == cfg.num_proprio, (off, cfg.num_proprio)

    def gait_phase(self, elapsed_s):
        c = self.cfg
        return (elapsed_s % c.period) / c.period

    def phase_features(self, phase, cmd):
        """sin/cos of each leg's phase (offset, wrapped), all zero phase under |cmd| < 0.2."""
        c = self.cfg
        offs = {"fr": c.fr_offset, "fl": c.fl_offset, "bl": c.bl_offset, "br": c.br_offset}
        moving = float(np.linalg.norm(cmd[:3]) >= 0.2)
        ang = np.array([2.0 * np.pi * (((phase + offs[leg]) % 1.0) * moving) for leg in GO2_PHASE_LEGS])
        return np.stack([np.sin(ang), np.cos(ang)], axis=1).reshape(-1)

    def build(self, state, phase):
        """state: dict of ang_vel, quat (wxyz), cmd, qj, dqj, actions."""
        c = self.cfg
        roll, pitch, _ = quaternion_to_euler(state["quat"])
        fields = {
            "ang_vel": np.asarray(state["ang_vel"], np.float32).reshape(-1) * c.ang_vel_scale,
            "roll_pitch": np.array([roll + c.roll_offset * (np.pi / 180), pitch + c.pitch_offset * (np.pi / 180)]),
            "command": state["cmd"] * c.cmd_scale * c.rc_scale,
            "dof_pos": (state["qj"] - c.default_angles) * c.dof_pos_scale,
            "dof_vel": state["dqj"] * c.dof_vel_scale,
            "actions": state["actions"],
            "phase": self.phase_features(phase, state["cmd"]),
        }
        cur = np.empty(c.num_proprio, dtype=np.float32)
        for name, (a, b) in self.offsets.items():
            cur[a:b] = fields[name]
        return cur


class BaseController:
    def __init__(self, cfg, scan_replay_path="SCAN_v12_ft_iii.txt", networks=None) -> None:
        """`networks`: optional (policy, adaptation, estimator, scan_encoder) callables; by
        default the cfg's TorchScript files (deploy_base.py:32-35). `scan_replay_path`: the
        scan recording (None: scans are always zero)."""
        self.cfg = cfg
        if networks is None:
            networks = tuple(torch.jit.load(p) for p in (cfg.policy_path, cfg.adaptation_path, cfg.estimator_path,
                                                         cfg.scan_encoder_path))
        self.policy, self.adaptation, self.estimator, self.scan_encoder = networks
        na = cfg.num_actions
        # robot state written by the subclass's _refresh_robot_states
        self.qj = np.zeros(na, dtype=np.float32)
        self.dqj = np.zeros(na, dtype=np.float32)
        self.ang_vel = np.zeros(3, dtype=np.float32)
        self.base_quat = np.zeros(4, dtype=np.float32)
        self.cmd = np.zeros(3, dtype=np.float32)
        self.jump_button_pressed = False
        # controller outputs / state
        self.actions = np.zeros(na, dtype=np.float32)
        self.target_dof_pos = cfg.default_angles.copy()
        self.smoothed_cmd = np.zeros(3, dtype=np.float32)
        self.projected_gravity = np.array([0.0, 0.0, -1.0], dtype=np.float32)
        self.phase = 0.0
        self.roll = self.pitch = self.yaw = 0.0  # last tick's IMU angles, offsets applied (deploy_base.py:184,219-220)
        self.obs = np.zeros(cfg.num_obs, dtype=np.float32)
        self._proprio = ProprioBuilder(cfg)
        self._history = ObsHistory(cfg.buffer_length, cfg.num_proprio)
        self._scan = (ScanReplay.from_file(cfg.num_scan_obs, scan_replay_path) if scan_replay_path is not None
                      else ScanReplay(cfg.num_scan_obs))

    # views the reference exposes as attributes
    @property
    def obs_history(self):
        return self._history.rows

    @property
    def first_step_ever(self):
        """True until the first observation fills the history (deploy_base.py:47,237-238)."""
        return not self._history.primed

    @property
    def mode(self):
        return self._scan.mode

    @property
    def scan_idx(self):
        return self._scan.index

    @property
    def fake_scan_obs(self):
        return self._scan.recording

    @property
    def phase_sync_point(self):
        return self._scan.sync_phase

    def _refresh_robot_states(self):
        """Subclass hook: fill qj, dqj, ang_vel (body frame), base_quat (wxyz), cmd and
        jump_button_pressed from the robot or simulator."""
        raise NotImplementedError(f"{type(self).__name__} must implement _refresh_robot_states()")

    def _get_gravity_orientation(self, quaternion):
        return rotate_inverse_wxyz(quaternion, (0.0, 0.0, -1.0))

    def _get_scan_obs(self):
        return self._scan.next(self.phase, self.jump_button_pressed)

    def get_smoothed_command(self, raw_cmd, smoothing_factor):
        """First-order low-pass of the operator command [vx, vy, wz]."""
        self.smoothed_cmd = self.smoothed_cmd + smoothing_factor * (raw_cmd - self.smoothed_cmd)
        return self.smoothed_cmd

    def build_observation(self, elapsed_time_s):
        """This tick's policy input, (1, num_obs) clipped: [history before this tick | current]."""
        self.projected_gravity = self._get_gravity_orientation(self.base_quat)
        c = self.cfg
        roll, pitch, self.yaw = quaternion_to_euler(self.base_quat)
        self.roll = roll + c.roll_offset * (np.pi / 180)
        self.pitch = pitch + c.pitch_offset * (np.pi / 180)
        self.phase = self._proprio.gait_phase(elapsed_time_s)
        state = {"ang_vel": self.ang_vel, "quat": self.base_quat, "cmd": self.cmd, "qj": self.qj, "dqj": self.dqj,
                 "actions": self.actions}
        cur = self._proprio.build(state, self.phase)
        nh = self.cfg.buffer_length * self.cfg.num_proprio
        self.obs[:nh] = self._history.rows.reshape(-1)
        self.obs[nh:] = cur
        self._history.push(cur)
        return torch.clamp(torch.from_numpy(self.obs.copy()).reshape(1, -1), -self.cfg.clip_obs, self.cfg.clip_obs)

    def infer(self, obs):
        """policy([obs | adaptation(history) | scan_encoder(scan) | estimator(obs)]) (actor_critic.py:79,
        with the adaptation latent, as act_inference in adaptation mode)."""
        c = self.cfg
        hist = obs[:, :c.buffer_length * c.num_proprio].reshape(1, c.buffer_length, c.num_proprio)
        with torch.no_grad():
            parts = (obs, self.adaptation(hist), self.scan_encoder(self._get_scan_obs()), self.estimator(obs))
            return self.policy(torch.cat(parts, dim=-1))

    def step(self, elapsed_time_s):
        """One control tick: robot state -> observation -> networks -> PD targets."""
        self._refresh_robot_states()
        c = self.cfg
        a = self.infer(self.build_observation(elapsed_time_s))
        self.actions = torch.clamp(a, -c.clip_actions, c.clip_actions).numpy().reshape(-1)
        self.target_dof_pos = self.actions * c.action_scale + c.default_angles
