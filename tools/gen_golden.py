#!/usr/bin/env python3
"""Golden-vector generator: runs the REFERENCE's own tensor code (read-only at
/root/reference) in this container through the stub `isaacgym` in
tools/refharness/ and records inputs -> outputs as small .npz fixtures under
tests/golden/. Test infrastructure only; never shipped to the GPU box as code
(only the .npz data it writes travels).

Masked-RNG mode: every random draw of the reference post-physics
path is routed through a per-env Philox uniform table (oracle/philox.py), so the
oracle and the HIP kernel, which draw the same table, must reproduce it.

Usage:  python tools/gen_golden.py            (writes tests/golden/go2_flat_n64.npz, ...)
"""
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path[:0] = [os.path.join(HERE, "refharness"), REF, os.path.join(REF, "rsl_rl"), os.path.join(REPO, "oracle")]
sys.path.append(REPO)  # after the reference: only legged_gym_custom_amd.actuator is taken from the build

import numpy as np  # noqa: E402
import torch  # noqa: E402

# tensorboard is not installed: stub the writer (runner import only)
_tb = types.ModuleType("torch.utils.tensorboard")


class _SW:
    def __init__(self, *a, **k):
        pass

    def add_scalar(self, *a, **k):
        pass


_tb.SummaryWriter = _SW
sys.modules["torch.utils.tensorboard"] = _tb

import isaacgym  # noqa: E402,F401  (the stub)
from isaacgym import gymapi  # noqa: E402
import legged_gym.envs as lg_envs  # noqa: E402  (registers tasks; import order matters)
from legged_gym.envs.go2.go2 import Go2Robot  # noqa: E402
import legged_gym.envs.go2.go2 as go2_mod  # noqa: E402
import legged_gym.envs.base.legged_robot as lr_mod  # noqa: E402
from legged_gym.utils.task_registry import task_registry  # noqa: E402
from legged_gym.utils.helpers import class_to_dict  # noqa: E402

import philox  # noqa: E402

GO2_BODY_NAMES = ["base", "Head_upper", "Head_lower",
                  "FL_hip", "FL_thigh", "FL_calf", "FL_foot",
                  "FR_hip", "FR_thigh", "FR_calf", "FR_foot",
                  "RL_hip", "RL_thigh", "RL_calf", "RL_foot",
                  "RR_hip", "RR_thigh", "RR_calf", "RR_foot"]
GO2_DOF_NAMES = [f"{l}_{j}_joint" for l in ("FL", "FR", "RL", "RR") for j in ("hip", "thigh", "calf")]
# URDF limits (go2.urdf): lower, upper, effort, velocity
_LIM = {"hip": (-1.0472, 1.0472, 23.7, 30.1), "thigh_F": (-1.5708, 3.4907, 23.7, 30.1),
        "thigh_R": (-0.5236, 4.5379, 23.7, 30.1), "calf": (-2.7227, -0.83776, 35.55, 20.07)}


def go2_dof_props():
    rec = []
    for n in GO2_DOF_NAMES:
        leg, j = n.split("_")[0], n.split("_")[1]
        key = "thigh_" + leg[0] if j == "thigh" else j
        rec.append(_LIM[key])
    # numpy structured array, as gym.get_asset_dof_properties returns (len() = num dofs)
    return np.array([tuple(r) for r in rec], dtype=[("lower", "f4"), ("upper", "f4"), ("effort", "f4"), ("velocity", "f4")])


class FakeGym:
    """Returns host tensors for the acquire_* calls; every other call is a no-op."""

    def __init__(self, n, nb, nd):
        self.root = torch.zeros(n, 13)
        self.dof = torch.zeros(n * nd, 2)
        self.contact = torch.zeros(n * nb, 3)
        self.rb = torch.zeros(n * nb, 13)

    def acquire_actor_root_state_tensor(self, sim):
        return self.root

    def acquire_dof_state_tensor(self, sim):
        return self.dof

    def acquire_net_contact_force_tensor(self, sim):
        return self.contact

    def acquire_rigid_body_state_tensor(self, sim):
        return self.rb

    def __getattr__(self, name):
        return lambda *a, **k: None


class _Props(list):
    pass


class _Prop:
    def __init__(self):
        self.friction = 1.0
        self.mass = 6.921
        self.com = gymapi.Vec3(0, 0, 0)


class RNGRouter:
    """Routes the reference's random draws to Philox table columns."""

    def __init__(self, env, seed):
        self.env = env
        self.seed = seed
        self.table = None
        self.ctx = None  # (name, env_ids, cursor)
        self.stream = philox.STREAM_STEP
        self.reset_calls = 0

    def make_table(self, step, stream):
        self.table = torch.from_numpy(philox.uniform_table(self.seed, np.arange(self.env.num_envs), step, stream,
                                                           philox.num_blocks(self.env.cfg.env.num_proprio)))

    def take(self, n_rows, n_cols):
        name, env_ids, cur = self.ctx
        base = {"cmd": philox.SLOT_CMD, "rcmd": philox.SLOT_RCMD, "push": philox.SLOT_PUSH, "terr": philox.SLOT_TERR,
                "dof": philox.SLOT_DOF, "root_xy": philox.SLOT_ROOT_XY, "root_vel": philox.SLOT_ROOT_VEL,
                "noise": philox.SLOT_NOISE}[name]
        idx = env_ids if env_ids is not None else torch.arange(self.env.num_envs)
        assert n_rows == len(idx), (name, n_rows, len(idx))
        u = self.table[idx][:, base + cur: base + cur + n_cols]
        self.ctx = (name, env_ids, cur + n_cols)
        return u.clone()


def install_rng(router):
    def torch_rand_float(lower, upper, shape, device):
        if router.ctx is None:  # setup-time draws (domain randomisation): real RNG
            return (upper - lower) * real_rand(*shape, device=device) + lower
        u = router.take(shape[0], shape[1])
        return (upper - lower) * u + lower

    real_rand = torch.rand
    real_rand_like = torch.rand_like
    lr_mod.torch_rand_float = torch_rand_float
    go2_mod.torch_rand_float = torch_rand_float

    def rand(*shape, **kw):
        if router.ctx is None:
            return real_rand(*shape, **kw)
        if len(shape) == 1 and isinstance(shape[0], (tuple, list)):
            shape = tuple(shape[0])
        assert len(shape) == 1
        return router.take(shape[0], 1)[:, 0]

    def rand_like(t, **kw):
        if router.ctx is None:
            return real_rand_like(t, **kw)
        return router.take(t.shape[0], t.shape[1])

    real_randint_like = torch.randint_like

    def randint_like(t, *args, **kw):
        # torch.randint_like(t, high) in _update_terrain_curriculum (legged_robot.py:572):
        # floor(u * high) of the Philox uniform, as the kernel draws it
        if router.ctx is None:
            return real_randint_like(t, *args, **kw)
        high = args[-1]
        u = router.take(t.shape[0], 1)[:, 0]
        return (u * float(high)).to(torch.long)

    torch.rand = rand
    torch.rand_like = rand_like
    torch.randint_like = randint_like


ANYMAL_JSON = os.path.join(REPO, "legged_gym_custom_amd", "resources", "robots", "anymal_c.json")


def anymal_tables():
    """Body/dof names and URDF dof limits of ANYmal C (the build's model file, made from
    the reference URDF by tools/build_models.py)."""
    import json
    with open(ANYMAL_JSON) as f:
        d = json.load(f)
    links = d["links"][1:]
    props = np.array([(l["lower"], l["upper"], l["effort"], l["velocity"]) for l in links],
                     dtype=[("lower", "f4"), ("upper", "f4"), ("effort", "f4"), ("velocity", "f4")])
    return list(d["body_names"]), list(d["dof_names"]), props


def make_harness_class(base=None, robot="go2"):
    base = base or Go2Robot
    if robot == "go2":
        body_names, dof_names, dof_props = GO2_BODY_NAMES, GO2_DOF_NAMES, go2_dof_props()
    else:
        body_names, dof_names, dof_props = anymal_tables()

    class Harness(base):
        """The task class with the Isaac Gym actor creation replaced by a fixed body/dof
        table and RNG routed through Philox."""

        def _create_envs(self):
            self.num_dof = len(dof_names)
            self.num_dofs = len(dof_names)
            self.body_names = list(body_names)
            self.dof_names = list(dof_names)
            self.num_bodies = len(self.body_names)
            pen, term = [], []
            for name in self.cfg.asset.penalize_contacts_on:
                pen.extend([s for s in self.body_names if name in s])
            for name in self.cfg.asset.terminate_after_contacts_on:
                term.extend([s for s in self.body_names if name in s])
            from isaacgym.torch_utils import to_torch
            lst = self.cfg.init_state.pos + self.cfg.init_state.rot + self.cfg.init_state.lin_vel + self.cfg.init_state.ang_vel
            self.base_init_state = to_torch(lst, device=self.device)
            self._get_env_origins()
            if not hasattr(self, "privileged_mass_params"):
                self.privileged_mass_params = torch.zeros(self.num_envs, 4)
            for i in range(self.num_envs):
                self._process_rigid_shape_props([_Prop()], i)
                self._process_dof_props(dof_props, i)
                _, mp = self._process_rigid_body_props([_Prop()], i)
                self.privileged_mass_params[i, :] = torch.from_numpy(mp).to(torch.float)
            feet = [s for s in self.body_names if self.cfg.asset.foot_name in s]
            self.feet_indices = torch.tensor([self.body_names.index(s) for s in feet], dtype=torch.long)
            self.penalised_contact_indices = torch.tensor([self.body_names.index(s) for s in pen], dtype=torch.long)
            self.termination_contact_indices = torch.tensor([self.body_names.index(s) for s in term], dtype=torch.long)
            if robot == "go2":
                self.hip_indices = torch.tensor([i for i, s in enumerate(self.body_names) if "hip" in s])
                self.thigh_indices = torch.tensor([i for i, s in enumerate(self.body_names) if "thigh" in s])
                self.calf_indices = torch.tensor([i for i, s in enumerate(self.body_names) if "calf" in s])
                self.hip_joint_indices = torch.tensor([self.dof_names.index(f"{l}_hip_joint") for l in ("FL", "FR", "RL", "RR")])
                self.thigh_joint_indices = torch.tensor([self.dof_names.index(f"{l}_thigh_joint") for l in ("FL", "FR", "RL", "RR")])
                self.calf_joint_indices = torch.tensor([self.dof_names.index(f"{l}_calf_joint") for l in ("FL", "FR", "RL", "RR")])

        # --- RNG context routing -------------------------------------------------
        def _resample_commands(self, env_ids):
            r = self._router
            r.ctx = ("rcmd" if self._in_reset else "cmd", env_ids, 0)
            super()._resample_commands(env_ids)
            r.ctx = None

        def reset_idx(self, env_ids):
            self._in_reset = True
            super().reset_idx(env_ids)
            self._in_reset = False

        def _reset_dofs(self, env_ids):
            self._router.ctx = ("dof", env_ids, 0)
            super()._reset_dofs(env_ids)
            self._router.ctx = None

        def _reset_root_states(self, env_ids):
            r = self._router
            if self.custom_origins:
                r.ctx = ("root_xy", env_ids, 0)
                orig = lr_mod.torch_rand_float

                def two_phase(lower, upper, shape, device):
                    if shape[1] == 6:
                        r.ctx = ("root_vel", env_ids, 0)
                    return orig(lower, upper, shape, device)
                lr_mod.torch_rand_float = two_phase
                super()._reset_root_states(env_ids)
                lr_mod.torch_rand_float = orig
            else:
                r.ctx = ("root_vel", env_ids, 0)
                super()._reset_root_states(env_ids)
            r.ctx = None

        def _update_terrain_curriculum(self, env_ids):
            self._router.ctx = ("terr", env_ids, 0)
            super()._update_terrain_curriculum(env_ids)
            self._router.ctx = None

        def _push_robots(self):
            self._router.ctx = ("push", None, 0)
            super()._push_robots()
            self._router.ctx = None

        def compute_observations(self):
            self._router.ctx = ("noise", None, 0)
            super().compute_observations()
            self._router.ctx = None

        def post_physics_step(self):
            self._router.make_table(self.common_step_counter + 1, philox.STREAM_STEP)
            super().post_physics_step()

        def external_reset(self, env_ids):
            """BaseTask.reset() path: reset_idx outside step (stream 1)."""
            self._router.make_table(self._router.reset_calls, philox.STREAM_RESET)
            self._router.reset_calls += 1
            self.reset_idx(env_ids)

    return Harness


class _Interp2dLinear:
    """interp2d(x, y, z, kind='linear') (removed in SciPy 1.14; terrain_utils.py:42) via
    RegularGridInterpolator, as in tools/gen_terrain_golden.py."""

    def __init__(self, x, y, z, kind="linear"):
        import scipy.interpolate as si
        self._f = si.RegularGridInterpolator((np.asarray(y, float), np.asarray(x, float)), np.asarray(z, float))

    def __call__(self, xn, yn):
        yy, xx = np.meshgrid(np.asarray(yn, float), np.asarray(xn, float), indexing="ij")
        return self._f(np.stack([yy.ravel(), xx.ravel()], -1)).reshape(yy.shape)


def build_env(task, n, seed=1, overrides=None, sea_seed=None):
    import legged_gym.utils.terrain_utils as ref_tu
    ref_tu.interpolate.interp2d = _Interp2dLinear
    env_cfg, train_cfg = task_registry.get_cfgs(task)
    env_cfg.env.num_envs = n
    if overrides:
        overrides(env_cfg)
    torch.manual_seed(seed)
    np.random.seed(seed)
    sim_params = gymapi.SimParams()
    sim_params.dt = env_cfg.sim.dt
    sim_params.use_gpu_pipeline = False
    anymal = task.startswith("anymal")
    fake = FakeGym(n, 17 if anymal else 19, 12)
    gymapi.acquire_gym = lambda: fake
    if anymal:
        # the reference torch.jit.load()s its SEA archive (anymal.py:24): hand it the
        # build's torch restatement with synthetic weights instead (no archive is run)
        from legged_gym.envs.anymal_c.anymal import Anymal
        from legged_gym_custom_amd import actuator as act
        sea_w = act.random_sea_weights(sea_seed if sea_seed is not None else seed)
        torch.jit.load = lambda *a, **k: act.SeaLSTM(sea_w)
        cls = make_harness_class(Anymal, "anymal")
    else:
        sea_w = None
        cls = make_harness_class()
    cls._in_reset = False
    # the router is needed before __init__ (reset draws happen only later)
    env = cls.__new__(cls)
    env._router = RNGRouter(env, seed)
    env._in_reset = False
    install_rng(env._router)
    cls.__init__(env, env_cfg, sim_params, gymapi.SIM_PHYSX, "cpu", True)
    env._fake = fake
    env._sea_w = sea_w
    return env, env_cfg


def scripted_physics(env, rng, t):
    """Plausible post-simulate state written into the fake gym tensors."""
    n = env.num_envs
    root = env.root_states
    # keep positions near origins; tilt a little; a few flipped
    root[:, 0:2] = env.env_origins[:, 0:2] + torch.from_numpy(rng.uniform(-0.5, 0.5, (n, 2))).float()
    root[:, 2] = torch.from_numpy(rng.uniform(0.2, 0.4, n)).float()
    axis = rng.normal(size=(n, 3))
    axis /= np.linalg.norm(axis, axis=1, keepdims=True)
    ang = rng.uniform(0, 0.6, n)
    flip = rng.uniform(size=n) < 0.03
    ang[flip] = rng.uniform(2.0, 3.1, flip.sum())
    q = np.concatenate([axis * np.sin(ang / 2)[:, None], np.cos(ang / 2)[:, None]], 1)
    root[:, 3:7] = torch.from_numpy(q).float()
    root[:, 7:13] = torch.from_numpy(rng.normal(0, 0.5, (n, 6))).float()
    dof = env.dof_state.view(n, 12, 2)
    nb = env.num_bodies
    dof[:, :, 0] = env.default_dof_pos + torch.from_numpy(rng.normal(0, 0.2, (n, 12))).float()
    dof[:, :, 1] = torch.from_numpy(rng.normal(0, 2.0, (n, 12))).float()
    cf = env.contact_forces
    cf[:] = 0
    cf[:, env.feet_indices, :] = torch.from_numpy(rng.normal(0, 5, (n, 4, 3))).float()
    cf[:, env.feet_indices, 2] = torch.from_numpy(rng.uniform(-2, 40, (n, 4))).float()
    pen = torch.from_numpy(rng.uniform(size=(n, nb)) < 0.05)
    cf[pen] = torch.from_numpy(rng.normal(0, 3, (int(pen.sum()), 3))).float()
    if not hasattr(env, "rigid_body_states"):  # the base task never reads body states
        env.rigid_body_states = torch.zeros(n * nb, 13)
    rb = env.rigid_body_states.view(n, nb, 13)
    rb[:] = torch.from_numpy(rng.normal(0, 0.3, (n, nb, 13))).float()
    rb[:, env.feet_indices, 2] = torch.from_numpy(rng.uniform(-0.01, 0.12, (n, 4))).float()


def scripted_physics_course(env, rng, t):
    """Like scripted_physics, but robots spread along their terrain tile (parkour: x from
    the tile start), z set above the local ground, and a few fallen into gaps (z < -1)."""
    scripted_physics(env, rng, t)
    n = env.num_envs
    root = env.root_states
    tl = env.cfg.terrain
    x0 = 0.0 if getattr(tl, "parkour", False) else -0.5 * tl.terrain_length  # parkour origin = tile start
    root[:, 0] = env.env_origins[:, 0] + x0 + torch.from_numpy(rng.uniform(0.5, tl.terrain_length - 0.5, n)).float()
    root[:, 1] = env.env_origins[:, 1] + torch.from_numpy(rng.uniform(-0.45, 0.45, n) * tl.terrain_width).float()
    hs = env.height_samples
    ix = ((root[:, 0] + tl.border_size) / tl.horizontal_scale).long().clamp(0, hs.shape[0] - 1)
    iy = ((root[:, 1] + tl.border_size) / tl.horizontal_scale).long().clamp(0, hs.shape[1] - 1)
    ground = hs[ix, iy].float() * tl.vertical_scale
    root[:, 2] = ground + torch.from_numpy(rng.uniform(0.2, 0.45, n)).float()
    fell = torch.from_numpy(rng.uniform(size=n) < 0.06)
    root[fell, 2] = torch.from_numpy(rng.uniform(-1.8, -1.05, int(fell.sum()))).float()


STATE_KEYS = ["root_states", "dof_state", "contact_forces", "commands", "last_actions", "last_dof_vel",
              "last_root_vel", "last_base_lin_vel", "last_torques", "obs_history_buf", "episode_length_buf",
              "last_contacts", "last_contact_heights", "feet_air_time"]
OUT_KEYS = ["obs_buf", "privileged_obs_buf", "critic_obs_buf", "estimated_obs_buf", "scan_obs_buf", "rew_buf",
            "reset_buf", "time_out_buf", "torques", "actions", "base_lin_vel", "base_ang_vel", "projected_gravity"]


def snapshot(env, keys):
    out = {}
    for k in keys:
        v = getattr(env, k)
        out[k] = v.detach().clone().numpy().copy()
    out["roll"] = env.roll.numpy().copy() if hasattr(env, "roll") else None
    return out


def _ranges8(env):
    r = env.command_ranges
    return np.array(list(r["lin_vel_x"]) + list(r["lin_vel_y"]) + list(r["ang_vel_yaw"]) + list(r["heading"]),
                    dtype=np.float64)


def run_fixture(task, n, steps, seed, path, ep_init=None, csc0=0, overrides=None, physics=None, terrain=False,
                inject=None):
    """inject: optional {step t: {reward name: fp32 [n] episode sums}} written into the
    reference's episode_sums before step t (recorded; the replay writes the same)."""
    env, cfg = build_env(task, n, seed, overrides)
    physics = physics or scripted_physics
    state_keys = STATE_KEYS + (["terrain_levels", "env_origins"] if terrain else [])
    state_keys = [k for k in state_keys if hasattr(env, k)]  # the base task has no feet-state buffers
    rng = np.random.default_rng(seed + 100)
    rec = {"num_envs": n, "seed": seed, "task": task, "torch_version": torch.__version__}
    # static per-env setup-time params (inputs to the oracle/kernel)
    rec["friction"] = env.privileged_friction_coeffs.numpy().reshape(n).astype(np.float32)
    rec["mass_params"] = env.privileged_mass_params.numpy().astype(np.float32)
    rec["kp_kd_multipliers"] = env.kp_kd_multipliers.numpy().astype(np.float32)
    rec["env_origins"] = env.env_origins.numpy().astype(np.float32)
    rec["default_dof_pos"] = env.default_dof_pos.numpy().reshape(12).astype(np.float32)
    rec["dof_pos_limits"] = env.dof_pos_limits.numpy().astype(np.float32)
    rec["torque_limits"] = env.torque_limits.numpy().astype(np.float32)
    rec["p_gains"] = env.p_gains.numpy().astype(np.float32)
    rec["d_gains"] = env.d_gains.numpy().astype(np.float32)
    rec["noise_scale_vec"] = env.noise_scale_vec.numpy().astype(np.float32)
    rec["reward_names"] = np.array(list(env.reward_scales.keys()))
    rec["reward_scales"] = np.array([env.reward_scales[k] for k in env.reward_scales], dtype=np.float64)
    if terrain:
        import hashlib
        rec["terrain_levels"] = env.terrain_levels.numpy().copy()
        rec["terrain_types"] = env.terrain_types.numpy().copy()
        rec["terrain_origins"] = env.terrain_origins.numpy().astype(np.float32)
        rec["height_samples_sha1"] = np.array(hashlib.sha1(env.height_samples.numpy().tobytes()).hexdigest())
        rec["np_seed"] = np.array(seed)

    curriculum = bool(getattr(cfg.commands, "curriculum", False))
    if curriculum:
        rec["command_ranges0"] = _ranges8(env)
        c = cfg.commands
        rec["curriculum_cfg"] = np.array([getattr(c, k, np.nan) for k in
                                          ("vel_increment", "max_forward_vel", "max_reverse_vel", "max_curriculum")],
                                         dtype=np.float64)
    # ---- BaseTask.reset(): external reset_idx(all) then step(zeros) ------------
    env.external_reset(torch.arange(n))
    rec["reset0_state"] = {k: getattr(env, k).detach().clone().numpy() for k in state_keys}

    def one_step(actions):
        env.actions = torch.clip(actions, -cfg.normalization.clip_actions, cfg.normalization.clip_actions)
        physics(env, rng, None)
        pre = {k: getattr(env, k).detach().clone().numpy() for k in ["root_states", "dof_state", "contact_forces", "rigid_body_states"]}
        env.torques = env._compute_torques(env.actions).view(env.torques.shape)
        env.post_physics_step()
        clip = cfg.normalization.clip_observations
        env.obs_buf = torch.clip(env.obs_buf, -clip, clip)
        env.privileged_obs_buf = torch.clip(env.privileged_obs_buf, -clip, clip)
        env.critic_obs_buf = torch.clip(env.critic_obs_buf, -clip, clip)
        env.estimated_obs_buf = torch.clip(env.estimated_obs_buf, -clip, clip)
        return pre

    steps_rec = []
    # step 0 = the zero-action step of BaseTask.reset()
    env.common_step_counter = 0
    for t in range(steps):
        if t == 1:
            # init_at_random_ep_len (on_policy_runner.py:121-122) + place a few envs at edge cases
            ep = torch.randint(0, int(env.max_episode_length), (n,), generator=torch.Generator().manual_seed(seed))
            ep[: min(4, n)] = torch.tensor([998, 999, 1000, 499][: min(4, n)])
            env.episode_length_buf = ep
            env.common_step_counter = csc0
        acts = torch.from_numpy(rng.normal(0, 1.5, (n, 12))).float() if t > 0 else torch.zeros(n, 12)
        ep_in = env.episode_length_buf.clone().numpy()
        csc_in = env.common_step_counter
        inj = (inject or {}).get(t)
        for name, vals in (inj or {}).items():
            env.episode_sums[name][:] = torch.from_numpy(np.asarray(vals, np.float32))
        pre = one_step(acts)
        o = {}
        o["obs_cur"] = env.obs_buf[:, -env.num_proprio:].numpy().copy()
        for k in ["privileged_obs_buf", "estimated_obs_buf", "scan_obs_buf", "rew_buf", "reset_buf",
                  "time_out_buf", "torques"]:
            o[k] = getattr(env, k).detach().clone().numpy()
        if t < 3:
            o["obs_buf"] = env.obs_buf.numpy().copy()
            o["critic_obs_buf"] = env.critic_obs_buf.numpy().copy()
        o["state_out"] = {k: getattr(env, k).detach().clone().numpy() for k in state_keys if k != "obs_history_buf"}
        if terrain:
            o["measured_heights"] = env.measured_heights.numpy().copy()
            if hasattr(env, "jump_flags"):
                o["jump_flags"] = env.jump_flags.numpy().copy()
        o["episode_sums"] = np.stack([env.episode_sums[k].numpy() for k in env.reward_scales]).astype(np.float32)
        o["extras_time_outs"] = env.extras["time_outs"].numpy().copy() if "time_outs" in env.extras else None
        if "episode" in env.extras:
            o["extras_episode"] = np.array([float(env.extras["episode"]["rew_" + k]) for k in env.reward_scales],
                                           dtype=np.float64)
        if hasattr(env, "roll"):
            o["roll"] = env.roll.numpy().copy(); o["pitch"] = env.pitch.numpy().copy()
        if curriculum:
            o["command_ranges"] = _ranges8(env)
            ep = env.extras.get("episode", {})
            o["extras_command"] = np.array([float(ep.get(k, np.nan)) for k in
                                            ("max_command_x", "min_command_x", "max_command_y", "max_command_yaw")])
        phys = {"root_states": pre["root_states"], "dof_state": pre["dof_state"],
                "contact_forces": pre["contact_forces"],
                "feet_pos": pre["rigid_body_states"].reshape(n, env.num_bodies, 13)[:, env.feet_indices.numpy(), 0:3].copy()}
        st = {"csc_in": csc_in, "ep_in": ep_in, "actions_raw": acts.numpy(), "physics": phys, "out": o}
        if inj:
            st["inject"] = {name: np.asarray(v, np.float32) for name, v in inj.items()}
        steps_rec.append(st)
    rec["final_obs_history"] = env.obs_history_buf.numpy().copy()
    if env._sea_w is not None:
        rec["sea_seed"] = np.array(seed)
        rec["final_sea_hidden"] = env.sea_hidden_state.numpy().copy()
        rec["final_sea_cell"] = env.sea_cell_state.numpy().copy()
    rec["steps"] = steps_rec
    flat = flatten(rec)
    np.savez_compressed(path, **flat)
    print("wrote", path, "keys", len(flat), "bytes", os.path.getsize(path))


def flatten(d, prefix=""):
    out = {}
    for k, v in d.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict):
            out.update(flatten(v, key + "."))
        elif isinstance(v, list):
            for i, item in enumerate(v):
                out.update(flatten(item, f"{key}.{i}."))
        elif v is None:
            continue
        else:
            out[key] = np.asarray(v)
    return out


if __name__ == "__main__":
    os.makedirs(os.path.join(REPO, "tests", "golden"), exist_ok=True)
    which = sys.argv[1:] or ["go2", "go2_parkour", "anymal_c_rough"]
    if "go2" in which:
        run_fixture("go2", 64, 30, 1, os.path.join(REPO, "tests", "golden", "go2_flat_n64.npz"), csc0=390)
    if "anymal_c_rough" in which:
        # C3: base LeggedRobot obs (235 = 48 + 187 heights, history 5) on the rough
        # curriculum trimesh, SEA actuator net (synthetic weights) for the torques
        run_fixture("anymal_c_rough", 64, 20, 1, os.path.join(REPO, "tests", "golden", "anymal_c_rough_n64.npz"),
                    csc0=390, physics=scripted_physics_course, terrain=True)
    if "curriculum" in which:
        # the command curriculum (go2.py:80-107 / legged_robot.py:580-591) on the step whose
        # common_step_counter is 1000: every env's tracking_lin_vel episode sum is set before
        # it to 0.9 x the episode maximum, so the envs resetting there (time-outs placed at
        # ep 999, flipped robots) pass the 0.8 threshold and the range grows by delta
        def cur(rev, lo=-0.5):
            def ov(c):
                c.commands.curriculum = True
                c.commands.ranges.lin_vel_x = [lo, 0.6]
                if hasattr(c.commands, "max_reverse_vel"):
                    c.commands.max_reverse_vel = rev
            return ov

        def full(task, n, frac=0.9):
            cfg_, _ = task_registry.get_cfgs(task)
            dt = cfg_.control.decimation * cfg_.sim.dt
            scale = cfg_.rewards.scales.tracking_lin_vel * dt
            ml = int(np.ceil(cfg_.env.episode_length_s / dt))
            return {2: {"tracking_lin_vel": np.full(n, frac * scale * ml, np.float32)}}
        gd = os.path.join(REPO, "tests", "golden")
        run_fixture("go2", 64, 6, 2, os.path.join(gd, "go2_cmd_curriculum_n64.npz"), csc0=998,
                    overrides=cur(-1.0), inject=full("go2", 64))
        # max_reverse_vel >= 0 (go2_parkour's sprint setting): the lower bound's np.clip has
        # a_max = lo - delta, so it moves down by delta without a floor
        run_fixture("go2", 64, 6, 3, os.path.join(gd, "go2_cmd_curriculum_rev_n64.npz"), csc0=998,
                    overrides=cur(0.5, lo=0.1), inject=full("go2", 64))
        # LeggedRobot.update_command_curriculum (+-0.05 within max_curriculum) on ANYmal rough
        run_fixture("anymal_c_rough", 64, 5, 4, os.path.join(gd, "anymal_cmd_curriculum_n64.npz"), csc0=998,
                    overrides=cur(None), inject=full("anymal_c_rough", 64), physics=scripted_physics_course,
                    terrain=True)
    if "go2_parkour" in which:
        # C4 task on its full terrain (12 x 20 gap courses); robots spread along the
        # courses so the scan, jump flags, hole termination and curriculum all fire
        run_fixture("go2_parkour", 64, 24, 1, os.path.join(REPO, "tests", "golden", "go2_parkour_n64.npz"),
                    csc0=390, physics=scripted_physics_course, terrain=True)
