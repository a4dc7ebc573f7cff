"""LeggedRobot — drop-in for legged_gym/envs/base/legged_robot.py:21-1152.

The whole env step (legged_robot.py:67-100: clip, decimation x {PD torque, simulate},
post_physics_step, obs clip) is ONE HIP kernel launch of liblgx.so (lgx_step), one
wavefront per env (--sim_device=cpu: the same entry point on the library's host backend). This class owns the torch buffers (same names/shapes as the
reference, env-major), builds the model/params once, binds the buffers to the native
env, and keeps the reference's Python-visible surface: step/reset/reset_idx, the
8-tuple return, extras['time_outs'/'episode'], common_step_counter, buffer attributes.
"""
import os

import numpy as np
import torch

from legged_gym_custom_amd import LEGGED_GYM_ROOT_DIR, _abi, _native
from legged_gym_custom_amd import model as mdl
from legged_gym_custom_amd import params as prm
from legged_gym_custom_amd.envs.base.base_task import BaseTask
from legged_gym_custom_amd.utils import terrain_utils
from legged_gym_custom_amd.utils.helpers import class_to_dict
from legged_gym_custom_amd.utils.terrain import Terrain


class LeggedRobot(BaseTask):
    TASK_KIND = _abi.TASK_LEGGED

    def __init__(self, cfg, sim_params, physics_engine, sim_device, headless):
        self.cfg = cfg
        self.sim_params = sim_params
        self.height_samples = None
        self.debug_viz = False
        self.init_done = False
        self._parse_cfg(self.cfg)
        self.num_envs = self.cfg.env.num_envs
        self.seed = int(getattr(cfg, "seed", 1))
        if self.seed < 0:
            self.seed = 1
        # env sharding across ranks (one process per GPU): global env ids are used for
        # the RNG counter and terrain_types, so a sharded run draws what one GPU would.
        rank, world = 0, 1
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            rank, world = torch.distributed.get_rank(), torch.distributed.get_world_size()
        self.env_id_offset = rank * self.num_envs
        self.num_envs_total = world * self.num_envs
        super().__init__(self.cfg, sim_params, physics_engine, sim_device, headless)
        self._init_buffers()
        self._prepare_reward_function()
        self.init_done = True

    # ------------------------------------------------------------------ step
    def step(self, actions):
        """legged_robot.py:67-100 as one kernel launch; returns the reference's 8-tuple."""
        if actions.data_ptr() != self.actions_in.data_ptr():  # the PPO act head may write it in place
            self.actions_in.copy_(actions, non_blocking=True)
        # the counter the kernel reads lives on the device (lgx_step_dev; it holds the NEXT
        # step's number and lgx_episode_extras advances it), so a captured rollout replays with
        # the right step numbers; the host mirror follows
        self._csc += 1
        self._native.step_dev(self.seed, self._step_dev, self._stream())
        if self._cmd_curriculum:
            self._command_curriculum()
        self._update_extras(advance_step=True)
        return (self.obs_buf, self.privileged_obs_buf, self.critic_obs_buf, self.estimated_obs_buf, self.scan_obs_buf,
                self.rew_buf, self.reset_buf, self.extras)

    def _command_curriculum(self):
        """update_command_curriculum for the step just run (one launch; a no-op unless the
        step is a multiple of max_episode_length). Env shards: the mean runs over the reset
        envs of every rank — one all-reduce of {sum, count} on those steps (the host knows
        them: common_step_counter), so the rollout of such a run is not graph-captured."""
        gsc = None
        if self.num_envs_total > self.num_envs and self._csc % int(self.max_episode_length) == 0:
            m = self.reset_buf
            gsc = torch.stack([torch.where(m, self._curriculum_vals, 0.0).double().sum(), m.double().sum()])
            torch.distributed.all_reduce(gsc)
        self._native.command_curriculum(self.seed, self._step_dev, gsc, self._stream())

    @property
    def graph_capturable(self):
        """Whether the runner may capture the rollout as one graph (not with a sharded
        command curriculum: it all-reduces on host-known steps)."""
        return not (self._cmd_curriculum and self.num_envs_total > self.num_envs)

    def reset_idx(self, env_ids):
        """reset_idx outside a step (BaseTask.reset): masked reset on device (RNG stream 1)."""
        if isinstance(env_ids, torch.Tensor):
            env_ids = env_ids.to(self.device)
        mask = torch.zeros(self.num_envs, dtype=torch.uint8, device=self.device)
        mask[env_ids] = 1
        self._native.reset_envs(mask, self.seed, self._reset_calls, self._stream())
        self._reset_calls += 1
        self.reset_buf[env_ids] = True
        self._update_extras()

    def _update_extras(self, advance_step=False):
        """extras['episode'] / ['time_outs'] with the reference's stale-when-no-reset
        semantics (go2.py:246-263, Appendix B Q5): one lgx_episode_extras launch (no host
        sync); _update_extras_torch states the same in torch ops (tests compare them)."""
        cur, to = self.cfg.terrain.curriculum, self.cfg.env.send_timeouts
        self._native.episode_extras(self._episode_means, self._terrain_level_mean if cur else None,
                                    self._extras_time_outs if to else None,
                                    self._stream(),
                                    self._step_dev if advance_step else None)
        self._publish_extras()

    def _publish_extras(self):
        if "episode" not in self.extras:
            self.extras["episode"] = {"rew_" + k: self._episode_means[i] for i, k in enumerate(self._episode_keys)}
            if self.cfg.terrain.curriculum:
                self.extras["episode"]["terrain_level"] = self._terrain_level_mean
            if self._cmd_curriculum:  # go2.py:255-259 / legged_robot.py:206-209
                keys = (["max_command_x", "min_command_x", "max_command_y", "max_command_yaw"]
                        if self.TASK_KIND == _abi.TASK_GO2 else ["max_command_x", "max_command_y", "max_command_yaw"])
                for i, k in enumerate(keys):
                    self.extras["episode"][k] = self._command_range_log[i]
        if self.cfg.env.send_timeouts:
            self.extras["time_outs"] = self._extras_time_outs

    def _update_extras_torch(self):
        st = self.episode_stats
        cnt = st[-1]
        means = st[:-1] / torch.clamp(cnt, min=1.0) / self.max_episode_length_s
        # in place on static buffers: a captured rollout keeps the stale-value chain
        self._episode_means.copy_(torch.where(cnt > 0, means, self._episode_means))
        if self.cfg.terrain.curriculum:  # go2.py:252-253 (mean level, refreshed when envs reset)
            self._terrain_level_mean.copy_(torch.where(cnt > 0, self.terrain_levels.float().mean(),
                                                       self._terrain_level_mean))
        if self.cfg.env.send_timeouts:
            self._extras_time_outs.copy_(torch.where(self.reset_buf.any(), self.time_out_buf, self._extras_time_outs))
        self._publish_extras()

    def _stream(self):
        """The HIP stream the env's launches are ordered on (0 for the host backend)."""
        return torch.cuda.current_stream(self.device).cuda_stream if self.sim_device_id >= 0 else 0

    @property
    def common_step_counter(self):
        return self._csc

    @common_step_counter.setter
    def common_step_counter(self, value):
        self._csc = int(value)
        if hasattr(self, "_step_dev"):
            self._step_dev.fill_(self._csc + 1)  # the number the next step reads

    def advance_step_counter(self, k):
        """Host mirror after a replayed capture that already advanced the device counter k times."""
        self._csc += int(k)

    # ------------------------------------------------------------------ setup
    def create_sim(self):
        """legged_robot.py:278-293: terrain (heightfield / trimesh) or plane, then envs."""
        self.up_axis_idx = 2
        mesh_type = self.cfg.terrain.mesh_type
        if mesh_type in ("heightfield", "trimesh"):
            self.terrain = Terrain(self.cfg.terrain, self.num_envs)
        if mesh_type == "plane":
            self._create_ground_plane()
        elif mesh_type == "heightfield":
            self._create_heightfield()
        elif mesh_type == "trimesh":
            self._create_trimesh()
        elif mesh_type is not None:
            raise ValueError("Terrain mesh type not recognised. Allowed types are [None, plane, heightfield, trimesh]")
        self._create_envs()

    def _create_ground_plane(self):
        """legged_robot.py:757-765: the kernel's contact against z = 0 (no buffers)."""
        self._terrain_mesh = None

    def _upload_terrain(self, slope_threshold):
        t = self.terrain
        self.height_samples = torch.tensor(t.heightsamples).view(t.tot_rows, t.tot_cols).to(self.device)
        mesh = terrain_utils.pack_mesh(t.heightsamples, t.cfg.horizontal_scale, t.cfg.vertical_scale, slope_threshold)
        self._terrain_mesh = torch.from_numpy(mesh.view(np.int32)).to(self.device)

    def _create_heightfield(self):
        """legged_robot.py:768-786: heightfield collision (no wall correction) + samples."""
        self._upload_terrain(None)

    def _create_trimesh(self):
        """legged_robot.py:788-802: the slope-corrected triangle mesh + samples. The kernel
        collides against it through the packed per-vertex words (no index buffer)."""
        self._upload_terrain(self.cfg.terrain.slope_treshold)

    def _create_envs(self):
        """legged_robot.py:805-894: model, body/dof names, index tables, domain randomisation."""
        asset_cfg = self.cfg.asset
        self.model_dict = mdl.load_model(asset_cfg.file, asset_cfg.foot_name, LEGGED_GYM_ROOT_DIR)
        self.body_names = list(self.model_dict["body_names"])
        self.dof_names = list(self.model_dict["dof_names"])
        self.num_bodies = len(self.body_names)
        self.num_dof = self.num_dofs = len(self.dof_names)
        base = list(self.cfg.init_state.pos) + list(self.cfg.init_state.rot) + list(self.cfg.init_state.lin_vel) + \
            list(self.cfg.init_state.ang_vel)
        self.base_init_state = torch.tensor(base, dtype=torch.float, device=self.device)
        self._get_env_origins()
        # Setup-time randomisation is drawn for ALL global envs (the single-GPU draw order)
        # and this shard's slice kept, so env k gets the same friction / mass / gains on any
        # number of ranks.
        n, total = self.num_envs, self.num_envs_total
        sl = slice(self.env_id_offset, self.env_id_offset + n)
        dr = self.cfg.domain_rand
        # _process_rigid_shape_props legged_robot.py:318-329 (64 friction buckets, CPU RNG)
        if dr.randomize_friction:
            bucket_ids = torch.randint(0, 64, (total, 1))
            lo, hi = dr.friction_range
            buckets = (hi - lo) * torch.rand(64, 1) + lo
            self.friction_coeffs = buckets[bucket_ids][sl]
        mass = np.zeros((total, 4), dtype=np.float32)
        for i in range(total):
            torch.rand(2, 1)  # start-pose xy jitter draw (legged_robot.py:867), kept for RNG order
            if dr.randomize_base_mass:
                mass[i, 0] = np.random.uniform(dr.added_mass_range[0], dr.added_mass_range[1], size=(1,))[0]
            if getattr(dr, "randomize_center_of_mass", False):
                mass[i, 1:4] = np.random.uniform(dr.added_com_range[0], dr.added_com_range[1], size=(3,))
        self.privileged_mass_params = torch.from_numpy(mass[sl].copy()).to(self.device)
        names = self.body_names
        feet = [s for s in names if self.cfg.asset.foot_name in s]
        pen, term = [], []
        for key in self.cfg.asset.penalize_contacts_on:
            pen.extend([s for s in names if key in s])
        for key in self.cfg.asset.terminate_after_contacts_on:
            term.extend([s for s in names if key in s])
        idx = lambda lst: torch.tensor([names.index(s) for s in lst], dtype=torch.long, device=self.device)  # noqa: E731
        self.feet_indices = idx(feet)
        self.penalised_contact_indices = idx(pen)
        self.termination_contact_indices = idx(term)
        links = self.model_dict["links"][1:]
        self.dof_pos_limits = torch.from_numpy(prm.soft_dof_limits(
            [l["lower"] for l in links], [l["upper"] for l in links], self.cfg.rewards.soft_dof_pos_limit)).to(self.device)
        self.dof_vel_limits = torch.tensor([l["velocity"] for l in links], dtype=torch.float, device=self.device)
        self.torque_limits = torch.tensor([l["effort"] for l in links], dtype=torch.float, device=self.device)

    def _get_env_origins(self):
        """legged_robot.py:897-930. Rough terrain: origins from the terrain tiles
        (level = random up to max_init_terrain_level, type = global env index / (N / cols));
        plane: a grid with env_spacing. Both use the GLOBAL env index, and the level draw is
        made for all envs and sliced, so shards reproduce the single-GPU layout."""
        total, sl = self.num_envs_total, slice(self.env_id_offset, self.env_id_offset + self.num_envs)
        self.env_origins = torch.zeros(self.num_envs, 3, device=self.device)
        if self.cfg.terrain.mesh_type in ("heightfield", "trimesh"):
            self.custom_origins = True
            t = self.cfg.terrain
            max_init_level = t.max_init_terrain_level if t.curriculum else t.num_rows - 1
            if max_init_level >= t.num_rows:
                # the reference indexes terrain_origins out of bounds here (a device fault);
                # refuse the configuration up front instead
                raise ValueError(f"terrain.max_init_terrain_level ({max_init_level}) must be < terrain.num_rows "
                                 f"({t.num_rows})")
            self.max_terrain_level = t.num_rows
            self.terrain_levels = torch.randint(0, max_init_level + 1, (total,), device=self.device)[sl].contiguous()
            self.terrain_types = torch.div(torch.arange(total, device=self.device), (total / t.num_cols),
                                           rounding_mode="floor").to(torch.long)[sl].contiguous()
            self.terrain_origins = torch.from_numpy(self.terrain.env_origins).to(self.device).to(torch.float)
            self.env_origins[:] = self.terrain_origins[self.terrain_levels, self.terrain_types]
            return
        self.custom_origins = False
        num_cols = np.floor(np.sqrt(total))
        num_rows = np.ceil(total / num_cols)
        xx, yy = torch.meshgrid(torch.arange(num_rows), torch.arange(num_cols), indexing="ij")
        spacing = self.cfg.env.env_spacing
        self.env_origins[:, 0] = spacing * xx.flatten()[sl].to(self.device)
        self.env_origins[:, 1] = spacing * yy.flatten()[sl].to(self.device)

    def _parse_cfg(self, cfg):
        """legged_robot.py:933-955."""
        self.dt = self.cfg.control.decimation * self.sim_params.dt
        self.obs_scales = self.cfg.normalization.obs_scales
        self.reward_scales = class_to_dict(self.cfg.rewards.scales)
        self.command_ranges = class_to_dict(self.cfg.commands.ranges)
        if self.cfg.terrain.mesh_type not in ("heightfield", "trimesh"):
            self.cfg.terrain.curriculum = False
        self.max_episode_length_s = self.cfg.env.episode_length_s
        self.max_episode_length = np.ceil(self.max_episode_length_s / self.dt)
        self.cfg.domain_rand.push_interval = np.ceil(self.cfg.domain_rand.push_interval_s / self.dt)

    def _init_buffers(self):
        """legged_robot.py:625-727 (+ go2.py:132-177): torch-owned, env-major buffers,
        bound once to the native env."""
        n, d, nb, na = self.num_envs, self.num_dof, self.num_bodies, self.num_actions
        dev = self.device
        z = lambda *s, dtype=torch.float: torch.zeros(*s, device=dev, dtype=dtype)  # noqa: E731
        self.root_states = z(n, 13)
        self.root_states[:] = self.base_init_state
        self.root_states[:, :3] += self.env_origins
        self._dof_state3 = z(n, d, 2)
        self.dof_state = self._dof_state3.view(n * d, 2)
        self.dof_pos = self._dof_state3[..., 0]
        self.dof_vel = self._dof_state3[..., 1]
        self.base_quat = self.root_states[:, 3:7]
        self._contact3 = z(n, nb, 3)
        self.contact_forces = self._contact3
        self.rigid_body_states = z(n * nb, 13)
        self.rigid_body_states_view = self.rigid_body_states.view(n, nb, 13)
        self._step_dev = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.common_step_counter = 0
        self._reset_calls = 0
        self.extras = {}
        self.noise_scale_vec = torch.from_numpy(prm.noise_vector(self.cfg, self.TASK_KIND == _abi.TASK_GO2)).to(dev)
        self.add_noise = self.cfg.noise.add_noise
        self.gravity_vec = torch.tensor([0.0, 0.0, -1.0], device=dev).repeat((n, 1))
        self.forward_vec = torch.tensor([1.0, 0.0, 0.0], device=dev).repeat((n, 1))
        self.actions_in = z(n, na)
        self.actions = z(n, na)
        self.torques = z(n, na)
        self.last_actions = z(n, na)
        self.last_dof_vel = z(n, d)
        self.last_root_vel = z(n, 6)
        self.last_torques = z(n, na)
        self.commands = z(n, self.cfg.commands.num_commands)
        sc = self.obs_scales
        self.commands_scale = torch.tensor([sc.lin_vel, sc.lin_vel, sc.ang_vel], device=dev)
        self.base_lin_vel = z(n, 3)
        self.base_ang_vel = z(n, 3)
        self.projected_gravity = z(n, 3)
        self.projected_gravity[:, 2] = -1.0
        self.last_base_lin_vel = z(n, 3)
        xs, ys = self.cfg.terrain.measured_points_x, self.cfg.terrain.measured_points_y
        self.num_height_points = len(xs) * len(ys)
        self.measured_heights = z(n, self.num_height_points)
        self.obs_history_buf = z(n, self.cfg.env.history_buffer_length, self.cfg.env.num_proprio)
        self.rpy_phase = z(n, 8)
        self.roll, self.pitch, self.yaw = self.rpy_phase[:, 0], self.rpy_phase[:, 1], self.rpy_phase[:, 2]
        self.phase_fl, self.phase_fr = self.rpy_phase[:, 3], self.rpy_phase[:, 4]
        self.phase_bl, self.phase_br = self.rpy_phase[:, 5], self.rpy_phase[:, 6]
        self.jump_flags = self.rpy_phase[:, 7:8]
        nf = len(self.feet_indices)
        self.last_contacts = z(n, nf, dtype=torch.bool)
        self.last_contact_heights = z(n, nf)
        self.feet_air_time = z(n, nf)
        dr = self.cfg.domain_rand
        if dr.randomize_friction:
            self._friction = self.friction_coeffs.to(dev).to(torch.float).reshape(n).contiguous()
        else:
            self._friction = torch.ones(n, device=dev) * self.cfg.terrain.dynamic_friction
        self.privileged_friction_coeffs = self._friction.view(n, 1)
        lo, hi = getattr(dr, "kp_kd_range", [1.0, 1.0])
        self.kp_kd_multipliers = ((hi - lo) * torch.rand(2, self.num_envs_total, na, device=dev) + lo)[
            :, self.env_id_offset:self.env_id_offset + n].contiguous()
        if not getattr(dr, "randomize_kp_kd", False):
            self.kp_kd_multipliers.fill_(1.0)
        self.default_dof_pos = torch.tensor([self.cfg.init_state.default_joint_angles[nm] for nm in self.dof_names],
                                            device=dev).unsqueeze(0)
        self._dof_state3[..., 0] = self.default_dof_pos
        p_gains, d_gains = [], []
        for nm in self.dof_names:
            kp = kd = 0.0
            for key in self.cfg.control.stiffness.keys():
                if key in nm:
                    kp, kd = self.cfg.control.stiffness[key], self.cfg.control.damping[key]
            p_gains.append(kp)
            d_gains.append(kd)
        self.p_gains = torch.tensor(p_gains, device=dev)
        self.d_gains = torch.tensor(d_gains, device=dev)
        # ---- native env
        model_struct = mdl.to_struct(self.model_dict)
        terrain = getattr(self, "terrain", None)
        self.task_params = prm.build_task_params(self.cfg, self.model_dict, n, self.num_envs_total, self.env_id_offset,
                                                 sim_dt=self.sim_params.dt, go2=self.TASK_KIND == _abi.TASK_GO2,
                                                 terrain_shape=(terrain.tot_rows, terrain.tot_cols) if terrain else None)
        self._sea_buffers = self._setup_actuator(self.task_params)
        names, _, _, term = prm.reward_terms(self.cfg, self.dt)
        self._episode_keys = names + (["termination"] if term is not None else [])
        ks = len(self._episode_keys)
        self.episode_sums_buf = z(n, ks)
        self.episode_sums = {k: self.episode_sums_buf[:, i] for i, k in enumerate(self._episode_keys)}
        self.episode_stats = z(ks + 1)
        # extras['episode'] values in key order in one buffer (the runner's native episode
        # tracking reads them as contiguous runs): rew_* means | terrain_level | command range log
        self._extras_vals = z(ks + 1 + 4)
        self._episode_means = self._extras_vals[:ks]
        self._terrain_level_mean = self._extras_vals[ks]
        self._command_range_log = self._extras_vals[ks + 1:]
        self._extras_time_outs = z(n, dtype=torch.bool)
        # command curriculum (go2.py:80-107 / legged_robot.py:580-591): the ranges are device
        # state (double, the reference's Python floats) updated by lgx_command_curriculum
        self._cmd_curriculum = bool(getattr(self.cfg.commands, "curriculum", False))
        self._command_ranges_buf = self._curriculum_vals = None
        if self._cmd_curriculum:
            r = self.cfg.commands.ranges
            self._command_ranges_buf = torch.tensor(list(r.lin_vel_x) + list(r.lin_vel_y) + list(r.ang_vel_yaw) +
                                                    list(r.heading), dtype=torch.float64, device=dev)
            self._curriculum_vals = z(n)
            go2 = self.TASK_KIND == _abi.TASK_GO2
            log = ([r.lin_vel_x[1], r.lin_vel_x[0], r.lin_vel_y[1], r.ang_vel_yaw[1]] if go2
                   else [r.lin_vel_x[1], r.lin_vel_y[1], r.ang_vel_yaw[1], 0.0])
            self._command_range_log.copy_(torch.tensor(log, dtype=torch.float32))
            self.command_ranges = _DeviceCommandRanges(self._command_ranges_buf)
        # NaN/Inf guard outputs (lgx_buffers.blew_up / blowup_count): per step, the envs whose
        # physics state went non-finite (given a finite stand-in state and reset); the count
        self.blew_up_buf = z(n, dtype=torch.bool)
        self._blowup_count = torch.zeros(1, dtype=torch.int32, device=dev)
        self._native = _native.NativeEnv(model_struct, self.task_params, self.sim_device_id)
        self._bind()

    def _bind(self):
        self._native.bind({
            "root_states": self.root_states, "dof_state": self._dof_state3, "contact_forces": self._contact3,
            "rigid_body_states": self.rigid_body_states, "actions_in": self.actions_in, "actions": self.actions,
            "torques": self.torques, "last_actions": self.last_actions, "last_dof_vel": self.last_dof_vel,
            "last_root_vel": self.last_root_vel, "last_base_lin_vel": self.last_base_lin_vel,
            "last_torques": self.last_torques, "commands": self.commands,
            "episode_length": self._episode_length_buf, "episode_sums": self.episode_sums_buf,
            "obs_history": self.obs_history_buf, "last_contacts": self.last_contacts,
            "last_contact_heights": self.last_contact_heights, "feet_air_time": self.feet_air_time,
            "obs": self.obs_buf, "priv": self.privileged_obs_buf if self.num_privileged_obs else None,
            "critic": self.critic_obs_buf, "est": self.estimated_obs_buf if self.num_estimated_obs else None,
            "scan": self.scan_obs_buf if self.num_scan_obs else None, "rew": self.rew_buf, "reset": self.reset_buf,
            "time_out": self.time_out_buf, "base_lin_vel": self.base_lin_vel, "base_ang_vel": self.base_ang_vel,
            "projected_gravity": self.projected_gravity, "rpy_phase": self.rpy_phase,
            "measured_heights": self.measured_heights, "friction": self._friction,
            "mass_params": self.privileged_mass_params, "kp_kd": self.kp_kd_multipliers,
            "env_origins": self.env_origins, "episode_stats": self.episode_stats,
            "terrain_levels": getattr(self, "terrain_levels", None), "terrain_types": getattr(self, "terrain_types", None),
            "terrain_origins": getattr(self, "terrain_origins", None), "height_samples": self.height_samples,
            "terrain_mesh": self._terrain_mesh, "blew_up": self.blew_up_buf, "blowup_count": self._blowup_count,
            "command_ranges": self._command_ranges_buf, "curriculum_vals": self._curriculum_vals,
            "command_range_log": self._command_range_log if self._cmd_curriculum else None,
            **self._sea_buffers,
        })

    @property
    def physics_blowups(self):
        """Number of env steps whose physics went non-finite since creation (host sync)."""
        return int(self._blowup_count.item())

    def _setup_actuator(self, P):
        """PD control (legged_robot.py:440-478) lives in the kernel; subclasses with an
        actuator network fill P.sea_* and return its state buffers (anymal.py)."""
        return {}

    def _prepare_reward_function(self):
        """legged_robot.py:730-754: nonzero scales x dt, alphabetical; the terms run in
        the kernel (params.reward_terms validates that each one is implemented)."""
        for key in list(self.reward_scales.keys()):
            if self.reward_scales[key] == 0:
                self.reward_scales.pop(key)
            else:
                self.reward_scales[key] *= self.dt
        self.reward_names = [k for k in self.reward_scales if k != "termination"]


class _RangePair(list):
    """One [lo, hi] entry of _DeviceCommandRanges: item writes go through to the device ranges
    (the reference idiom `self.command_ranges["lin_vel_x"][1] = v`, go2.py:96-107)."""

    def __init__(self, owner, key, vals):
        super().__init__(vals)
        self._owner, self._key = owner, key

    def __setitem__(self, i, v):
        super().__setitem__(i, v)
        if len(self) != 2:
            raise ValueError("a command range is [lo, hi]")
        self._owner[self._key] = list(self)

    def __reduce__(self):  # a detached copy pickles as the plain [lo, hi] list
        return (list, (list(self),))


class _DeviceCommandRanges(dict):
    """self.command_ranges under the command curriculum: {'lin_vel_x': [lo, hi], ...} read
    from the device ranges the curriculum updates. Every read is a device-to-host copy (it
    synchronises with the stream); item writes, whole or per end, go to the device."""
    _KEYS = ("lin_vel_x", "lin_vel_y", "ang_vel_yaw", "heading")

    def __init__(self, buf):
        super().__init__()
        self._buf = buf
        for k in self._KEYS:
            dict.__setitem__(self, k, None)

    def __getitem__(self, key):
        i = self._KEYS.index(key)
        return _RangePair(self, key, [float(v) for v in self._buf[2 * i:2 * i + 2].tolist()])

    def __setitem__(self, key, value):
        i = self._KEYS.index(key)
        self._buf[2 * i:2 * i + 2] = torch.tensor([float(value[0]), float(value[1])], dtype=torch.float64)

    def values(self):
        return [self[k] for k in self._KEYS]

    def items(self):
        return [(k, self[k]) for k in self._KEYS]
