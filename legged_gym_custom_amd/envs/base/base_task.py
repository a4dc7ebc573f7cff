"""BaseTask — drop-in for legged_gym/envs/base/base_task.py:38-164.

Same attributes and getters the runner reads (num_envs, num_obs, num_proprio,
num_privileged_obs, num_critic_obs, num_estimated_obs, num_scan_obs,
history_buffer_length, num_actions; get_*_observations; reset(); step()).
The simulator handle is the MI355X env-step library (liblgx.so: HIP kernels for
sim_device=cuda:N, its host backend for sim_device=cpu); there is no viewer.
"""
import sys

import torch


class BaseTask:
    def __init__(self, cfg, sim_params, physics_engine, sim_device, headless):
        self.sim_params = sim_params
        self.physics_engine = physics_engine
        self.sim_device = sim_device
        dev = torch.device(sim_device)
        if dev.type == "cpu":
            # --sim_device=cpu (helpers.py:174-177): liblgx.so's host backend, OpenMP over envs
            self.sim_device_id = -1
            self.device = "cpu"
        elif dev.type == "cuda":
            if not torch.cuda.is_available():
                raise RuntimeError("no HIP device visible: --sim_device=cuda needs an MI355X (or use --sim_device=cpu)")
            self.sim_device_id = dev.index if dev.index is not None else torch.cuda.current_device()
            self.device = f"cuda:{self.sim_device_id}"
        else:
            raise RuntimeError(f"sim_device={sim_device}: use cuda:N (HIP kernels) or cpu (host backend)")
        self.headless = True  # rendering is out of scope (play/viewer)
        self.graphics_device_id = -1

        self.num_envs = cfg.env.num_envs
        self.num_proprio = cfg.env.num_proprio
        self.num_obs = cfg.env.num_observations
        self.num_privileged_obs = cfg.env.num_privileged_obs
        self.num_critic_obs = cfg.env.num_critic_obs
        self.num_estimated_obs = cfg.env.num_estimated_obs
        self.num_scan_obs = cfg.env.num_scan_obs
        self.history_buffer_length = cfg.env.history_buffer_length
        self.num_actions = cfg.env.num_actions

        z = lambda *s, dtype=torch.float: torch.zeros(*s, device=self.device, dtype=dtype)  # noqa: E731
        self.obs_buf = z(self.num_envs, self.num_obs)
        self.privileged_obs_buf = z(self.num_envs, self.num_privileged_obs)
        self.critic_obs_buf = z(self.num_envs, self.num_critic_obs)
        self.estimated_obs_buf = z(self.num_envs, self.num_estimated_obs)
        self.scan_obs_buf = z(self.num_envs, self.num_scan_obs)
        self.rew_buf = z(self.num_envs)
        self.reset_buf = torch.ones(self.num_envs, device=self.device, dtype=torch.bool)
        self._episode_length_buf = z(self.num_envs, dtype=torch.long)
        self.time_out_buf = z(self.num_envs, dtype=torch.bool)
        self.extras = {}

        self.create_sim()
        self.enable_viewer_sync = True
        self.viewer = None

    # the runner REASSIGNS this attribute (on_policy_runner.py:121-122): copy into the
    # buffer the native library is bound to instead of rebinding.
    @property
    def episode_length_buf(self):
        return self._episode_length_buf

    @episode_length_buf.setter
    def episode_length_buf(self, value):
        self._episode_length_buf.copy_(value.to(self._episode_length_buf.dtype))

    def get_observations(self):
        return self.obs_buf

    def get_privileged_observations(self):
        return self.privileged_obs_buf

    def get_critic_observations(self):
        return self.critic_obs_buf

    def get_estimated_observations(self):
        return self.estimated_obs_buf

    def get_scan_observations(self):
        return self.scan_obs_buf

    def reset_idx(self, env_ids):
        raise NotImplementedError

    def reset(self):
        """Reset all robots (base_task.py:131-135): reset_idx(all) then a zero-action step."""
        self.reset_idx(torch.arange(self.num_envs, device=self.device))
        obs, priv, critic, est, scan, _, _, _ = self.step(
            torch.zeros(self.num_envs, self.num_actions, device=self.device))
        return obs, priv, critic, est, scan

    def step(self, actions):
        raise NotImplementedError

    def render(self, sync_frame_time=True):
        if self.viewer is not None:  # pragma: no cover - no viewer in this build
            sys.exit()
