"""ctypes driver for the CPU oracle (TEST INFRASTRUCTURE ONLY: imported by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg).

Allocates numpy buffers for every lgx_buffers field and runs the oracle entry points.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("LGX_ORACLE_LIB") or os.path.join(HERE, "build", "liblgx_oracle.so")  # (sanitizer builds)

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        from legged_gym_custom_amd import _abi
        _abi.check_layout(_lib, "oracle_sizeof_")
        vp, u64, i32 = C.c_void_p, C.c_uint64, C.c_int
        _lib.oracle_post_physics.argtypes = [vp, vp, u64, u64]
        _lib.oracle_reset_envs.argtypes = [vp, vp, vp, u64, u64, i32]
        _lib.oracle_step.argtypes = [vp, vp, vp, u64, u64]
        _lib.oracle_clip_actions.argtypes = [vp, vp]
        _lib.oracle_compute_torques.argtypes = [vp, vp, i32]
        _lib.oracle_physics_substep.argtypes = [vp, vp, vp, i32]
        _lib.oracle_energy.argtypes = [vp, vp, vp, i32]
        _lib.oracle_energy.restype = C.c_double
        _lib.oracle_debug_rows.argtypes = [i32]
        _lib.oracle_debug_rows.restype = i32
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class OracleEnv:
    """numpy-owned buffers + params/model structs for one oracle instance."""

    def __init__(self, params, model_struct, num_reward_slots):
        from legged_gym_custom_amd import _abi
        P = params
        self.P, self.M = P, model_struct
        N, D, B = P.num_envs, P.num_dof, P.num_bodies
        f = lambda *s: np.zeros(s, dtype=np.float32)
        self.a = {
            "root_states": f(N, 13), "dof_state": f(N, D, 2), "contact_forces": f(N, B, 3),
            "rigid_body_states": f(N, B, 13), "actions_in": f(N, P.num_actions), "actions": f(N, P.num_actions),
            "torques": f(N, D), "last_actions": f(N, P.num_actions), "last_dof_vel": f(N, D),
            "last_root_vel": f(N, 6), "last_base_lin_vel": f(N, 3), "last_torques": f(N, D), "commands": f(N, 4),
            "episode_length": np.zeros(N, dtype=np.int64), "episode_sums": f(N, num_reward_slots),
            "obs_history": f(N, P.history_len, P.num_proprio), "last_contacts": np.zeros((N, P.num_feet), np.uint8),
            "last_contact_heights": f(N, P.num_feet), "feet_air_time": f(N, P.num_feet),
            "obs": f(N, P.num_obs), "priv": f(N, max(P.num_priv, 1)), "critic": f(N, P.num_critic),
            "est": f(N, max(P.num_est, 1)), "scan": f(N, max(P.num_scan, 1)), "rew": f(N),
            "reset": np.zeros(N, np.uint8), "time_out": np.zeros(N, np.uint8),
            "base_lin_vel": f(N, 3), "base_ang_vel": f(N, 3), "projected_gravity": f(N, 3), "rpy_phase": f(N, 8),
            "measured_heights": f(N, P.num_height_points),
            "friction": f(N), "mass_params": f(N, 4), "kp_kd": f(2, N, D), "env_origins": f(N, 3),
            "terrain_levels": None, "terrain_types": None, "terrain_origins": None, "height_samples": None,
            "terrain_mesh": None,
            "sea_hidden": f(2, N * D, 8) if P.actuator_net else None,
            "sea_cell": f(2, N * D, 8) if P.actuator_net else None,
            "episode_stats": f(num_reward_slots + 1),
        }
        self.a["kp_kd"][:] = 1.0
        self.B = _abi.Buffers()
        self.rebind()

    def rebind(self):
        for k, v in self.a.items():
            setattr(self.B, k, _ptr(v))

    def post_physics(self, seed, step):
        lib().oracle_post_physics(C.byref(self.P), C.byref(self.B), seed, step)

    def set_terrain(self, height_samples, mesh_words, levels=None, types=None, origins=None):
        """Bind a terrain: int16 samples + packed uint32 mesh words [rows, cols]; the
        curriculum tables when given (int64 levels/types [N], float32 origins [R, C, 3])."""
        self.a["height_samples"] = np.ascontiguousarray(height_samples, dtype=np.int16)
        self.a["terrain_mesh"] = np.ascontiguousarray(mesh_words, dtype=np.uint32)
        if levels is not None:
            self.a["terrain_levels"] = np.ascontiguousarray(levels, dtype=np.int64)
            self.a["terrain_types"] = np.ascontiguousarray(types, dtype=np.int64)
            self.a["terrain_origins"] = np.ascontiguousarray(origins, dtype=np.float32)
        self.rebind()

    def reset_envs(self, mask, seed, call, after_init=1):
        m = np.ascontiguousarray(mask.astype(np.uint8))
        lib().oracle_reset_envs(C.byref(self.P), C.byref(self.B), _ptr(m), seed, call, after_init)

    def clip_actions(self):
        lib().oracle_clip_actions(C.byref(self.P), C.byref(self.B))

    def compute_torques(self):
        for e in range(self.P.num_envs):
            lib().oracle_compute_torques(C.byref(self.P), C.byref(self.B), e)

    def physics_substep(self):
        for e in range(self.P.num_envs):
            lib().oracle_physics_substep(C.byref(self.M), C.byref(self.P), C.byref(self.B), e)

    def step(self, seed, step):
        lib().oracle_step(C.byref(self.M), C.byref(self.P), C.byref(self.B), seed, step)

    def energy(self, e):
        return lib().oracle_energy(C.byref(self.M), C.byref(self.P), C.byref(self.B), e)


def last_rows(n):
    """Constraint rows of each env's latest physics substep (numpy int array)."""
    L = lib()
    return np.array([L.oracle_debug_rows(e) for e in range(n)])
