"""BaseController — drop-in for deploy/base/deploy_base.py:6-270: the per-tick Go2 policy
loop of a deployed robot, as numpy.

Observation (52 = the env's Go2 proprio, go2.py:506-515, WITHOUT noise): body angular
velocity * 0.25, roll, pitch (+ configured offsets), command * cmd_scale * rc_scale,
(q - q0), qd * 0.05, previous actions, then sin/cos of the FR, FL, BL, BR gait phases
(zeroed under |cmd| < 0.2). The robot quaternion here is MuJoCo/Unitree **wxyz** (the env
uses xyzw). History: filled with the first observation, then rolled; the network input is
[history (before this tick) | current], clipped. Networks: the four TorchScript files
export_policy_as_jit writes (policy(cat(obs, adaptation(hist), scan_encoder(scan),
estimator(obs)))).

Scan replay (deploy_base.py:60-147): a recorded sequence of scan observations (text file:
a first block [sync_phase], then one [..132 values..] block per tick, blank-line
separated). NORMAL feeds zeros; the jump button arms WAITING; when the gait phase is
within 0.005 of the sync phase the recording is REPLAYed tick by tick, then NORMAL again.
"""
import re

import numpy as np
import torch


def quaternion_to_euler(quat_angle):
    """(roll, pitch, yaw) of a wxyz quaternion (pitch argument clipped to [-1, 1])."""
    w, x, y, z = quat_angle[0], quat_angle[1], quat_angle[2], quat_angle[3]
    roll = np.arctan2(+2.0 * (w * x + y * z), +1.0 - 2.0 * (x * x + y * y))
    pitch = np.arcsin(np.clip(+2.0 * (w * y - z * x), -1, 1))
    yaw = np.arctan2(+2.0 * (w * z + x * y), +1.0 - 2.0 * (y * y + z * z))
    return roll, pitch, yaw


def parse_scan_replay(text):
    """(sync phase, [scan vectors]) from a scan-replay recording."""
    blocks = re.split(r"\n\s*\n", text.strip())
    vecs = [[float(v) for v in b.strip().lstrip("[").rstrip("]").split()] for b in blocks]
    return vecs[0][0], vecs[1:]


class BaseController:
    def __init__(self, cfg, scan_replay_path="SCAN_v12_ft_iii.txt", networks=None) -> None:
        """`networks`: optional (policy, adaptation, estimator, scan_encoder) callables;
        by default the cfg's TorchScript files are loaded (deploy_base.py:32-35)."""
        self.cfg = cfg
        if networks is None:
            networks = [torch.jit.load(p) for p in (cfg.policy_path, cfg.adaptation_path, cfg.estimator_path,
                                                    cfg.scan_encoder_path)]
        self.policy, self.adaptation, self.estimator, self.scan_encoder = networks
        na = cfg.num_actions
        self.qj = np.zeros(na, dtype=np.float32)
        self.dqj = np.zeros(na, dtype=np.float32)
        self.ang_vel = np.zeros(3, dtype=np.float32)
        self.base_quat = np.zeros(4, dtype=np.float32)
        self.actions = np.zeros(na, dtype=np.float32)
        self.target_dof_pos = cfg.default_angles.copy()
        self.obs = np.zeros(cfg.num_obs, dtype=np.float32)
        self.obs_history = np.zeros((cfg.buffer_length, cfg.num_proprio), dtype=np.float32)
        self.cmd = np.array([0.0, 0.0, 0.0], dtype=np.float32)
        self.first_step_ever = True
        self.projected_gravity = np.array([0.0, 0.0, -1.0], dtype=np.float32)
        self.smoothed_cmd = np.zeros(3, dtype=np.float32)
        self.phase = 0.0
        # scan replay
        self.jump_button_pressed = False
        self.scan_idx = 0
        self.mode = "NORMAL"
        self.phase_sync_point, self.fake_scan_obs = -1, []
        if scan_replay_path is not None:
            with open(scan_replay_path) as f:
                self.phase_sync_point, self.fake_scan_obs = parse_scan_replay(f.read())
            print("Parsed fake scan observations of length: ", len(self.fake_scan_obs) + 1)
            print("Phase sync point: ", self.phase_sync_point)

    def _get_gravity_orientation(self, quaternion):
        """World gravity [0, 0, -1] in the body frame of a wxyz quaternion."""
        qw, qx, qy, qz = quaternion[0], quaternion[1], quaternion[2], quaternion[3]
        g = np.zeros(3)
        g[0] = 2 * (-qz * qx + qw * qy)
        g[1] = -2 * (qz * qy + qw * qx)
        g[2] = 1 - 2 * (qw * qw + qz * qz)
        return g

    def _get_scan_obs(self) -> torch.Tensor:
        """(1, num_scan_obs): zeros, or the next recorded scan while replaying."""
        scan = torch.zeros((1, self.cfg.num_scan_obs), dtype=torch.float32)
        if self.jump_button_pressed and self.mode == "NORMAL":
            self.mode = "WAITING"
        if self.mode == "WAITING" and np.abs(self.phase - self.phase_sync_point) < 0.005:
            self.mode = "REPLAY"
            print("Replay mode activated")
        if self.mode == "REPLAY":
            scan = torch.tensor(self.fake_scan_obs[self.scan_idx], dtype=torch.float32).view(1, -1)
            self.scan_idx += 1
            print(f"Feeding scan_obs[{self.scan_idx}]")
            if self.scan_idx == len(self.fake_scan_obs) - 1:
                self.mode = "NORMAL"
                print("Replay mode deactivated")
                self.scan_idx = 0
        return scan

    def _refresh_robot_states(self):
        """Fill qj, dqj, ang_vel (body frame), base_quat (wxyz), jump button."""
        raise NotImplementedError("_refresh_robot_states() not implemented")

    def get_smoothed_command(self, raw_cmd, smoothing_factor):
        """Exponential smoothing of the operator command [vx, vy, wz]."""
        self.smoothed_cmd = self.smoothed_cmd + smoothing_factor * (raw_cmd - self.smoothed_cmd)
        return self.smoothed_cmd

    def _phase_features(self, elapsed_time_s):
        c = self.cfg
        self.phase = (elapsed_time_s % c.period) / c.period
        ph = {k: (self.phase + off) % 1 for k, off in (("fr", c.fr_offset), ("bl", c.bl_offset), ("fl", c.fl_offset),
                                                       ("br", c.br_offset))}
        if np.linalg.norm(self.cmd[:3]) < 0.2:
            ph = {k: v * 0.0 for k, v in ph.items()}
        out = []
        for leg in ("fr", "fl", "bl", "br"):
            out += [np.sin(2 * np.pi * ph[leg]), np.cos(2 * np.pi * ph[leg])]
        return np.array(out, dtype=np.float32)

    def build_observation(self, elapsed_time_s):
        """The policy input for this tick ([1, num_obs] clipped tensor); updates history."""
        c = self.cfg
        na = c.num_actions
        self.projected_gravity = self._get_gravity_orientation(self.base_quat)
        self.roll, self.pitch, self.yaw = quaternion_to_euler(self.base_quat)
        phase_features = self._phase_features(elapsed_time_s)
        self.pitch += c.pitch_offset * (np.pi / 180)
        self.roll += c.roll_offset * (np.pi / 180)
        cur = np.zeros(c.num_proprio, dtype=np.float32)
        cur[:3] = self.ang_vel * c.ang_vel_scale
        cur[3:5] = np.stack([self.roll, self.pitch])
        cur[5:8] = self.cmd * c.cmd_scale * c.rc_scale
        cur[8:8 + na] = (self.qj - c.default_angles) * c.dof_pos_scale
        cur[8 + na:8 + 2 * na] = self.dqj * c.dof_vel_scale
        cur[8 + 2 * na:8 + 3 * na] = self.actions
        cur[8 + 3 * na:8 + 3 * na + 8] = phase_features
        self.obs[:] = np.concatenate([self.obs_history.flatten(), cur])
        if self.first_step_ever:
            self.first_step_ever = False
            self.obs_history = np.tile(cur, (c.buffer_length, 1))
        else:
            self.obs_history = np.roll(self.obs_history, -1, axis=0)
            self.obs_history[-1] = cur
        return torch.clip(torch.from_numpy(self.obs).unsqueeze(0), -c.clip_obs, c.clip_obs)

    def step(self, elapsed_time_s):
        """One control tick: refresh state, build the observation, run the networks,
        update actions and the PD targets (deploy_base.py:166-270)."""
        self._refresh_robot_states()
        c = self.cfg
        obs = self.build_observation(elapsed_time_s)
        n_hist = c.buffer_length * c.num_proprio
        with torch.no_grad():
            priv_latent = self.adaptation(obs[:, :n_hist].reshape(1, c.buffer_length, c.num_proprio))
            estimated = self.estimator(obs)
            scan_latent = self.scan_encoder(self._get_scan_obs())
            actions = self.policy(torch.cat((obs, priv_latent, scan_latent, estimated), dim=-1))
        self.actions = torch.clip(actions, -c.clip_actions, c.clip_actions).detach().numpy().squeeze()
        self.target_dof_pos = self.actions * c.action_scale + c.default_angles
