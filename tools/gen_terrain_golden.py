#!/usr/bin/env python3
"""Terrain golden vectors: runs the REFERENCE's own terrain code (legged_gym/utils/
terrain.py, terrain_utils.py; read-only at /root/reference) in this container and
records outputs as data under tests/golden/terrain.npz. Test infrastructure only.

scipy 1.15 no longer has `interpolate.interp2d` (terrain_utils.py:42 uses it). The
harness supplies the call the reference makes, interp2d(x, y, z, kind='linear') on a
rectilinear grid, through scipy's RegularGridInterpolator (an implementation
independent of the product's `_bilinear_upsample`).

Records:
  * gen.<case>        every generator on a small tile with a fixed np.random seed;
  * mesh.*            convert_heightfield_to_trimesh of a stepped tile (slope threshold);
  * configs.json      class_to_dict of each task's env/train config;
  * field.<task>.*    whole-field Terrain for the task configs (sha1 of height_field_raw,
                      shape, env_origins; for go2_parkour also the trimesh sha1s).

Usage:  python tools/gen_terrain_golden.py
"""
import hashlib
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path[:0] = [os.path.join(HERE, "refharness"), REF, os.path.join(REF, "rsl_rl")]

import numpy as np  # noqa: E402
import scipy.interpolate as _si  # noqa: E402


class _Interp2dLinear:
    """interp2d(x, y, z, kind='linear') on a rectilinear grid: z[len(y), len(x)];
    __call__(xn, yn) -> [len(yn), len(xn)]."""

    def __init__(self, x, y, z, kind="linear"):
        assert kind == "linear"
        self._f = _si.RegularGridInterpolator((np.asarray(y, float), np.asarray(x, float)), np.asarray(z, float),
                                              method="linear")

    def __call__(self, xn, yn):
        yy, xx = np.meshgrid(np.asarray(yn, float), np.asarray(xn, float), indexing="ij")
        return self._f(np.stack([yy.ravel(), xx.ravel()], -1)).reshape(yy.shape)


_si.interp2d = _Interp2dLinear

_tb = types.ModuleType("torch.utils.tensorboard")
_tb.SummaryWriter = object
sys.modules["torch.utils.tensorboard"] = _tb

import isaacgym  # noqa: E402,F401  (the stub)
import legged_gym.envs  # noqa: E402,F401  (import order: envs before utils)
from legged_gym.utils import terrain_utils as ref_tu  # noqa: E402
from legged_gym.utils import terrain as ref_terrain  # noqa: E402
from legged_gym.utils.task_registry import task_registry  # noqa: E402

ref_tu.interpolate.interp2d = _Interp2dLinear


def sha1(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()


# (name, fn name, kwargs, seed); tile 64 x 48 cells, hs 0.1, vs 0.005
GEN_CASES = [
    ("random_uniform", "random_uniform_terrain", dict(min_height=-0.06, max_height=0.06, step=0.005,
                                                      downsampled_scale=0.2), 3),
    ("random_uniform_coarse", "random_uniform_terrain", dict(min_height=-0.01, max_height=0.01, step=0.005,
                                                             downsampled_scale=0.3), 4),
    ("sloped", "sloped_terrain", dict(slope=0.3), 0),
    ("pyramid_sloped_up", "pyramid_sloped_terrain", dict(slope=0.35, platform_size=3.0), 0),
    ("pyramid_sloped_down", "pyramid_sloped_terrain", dict(slope=-0.25, platform_size=3.0), 0),
    ("discrete_obstacles", "discrete_obstacles_terrain", dict(max_height=0.17, min_size=1.0, max_size=2.0,
                                                              num_rects=20, platform_size=3.0), 5),
    ("wave", "wave_terrain", dict(num_waves=2, amplitude=0.7), 0),
    ("stairs", "stairs_terrain", dict(step_width=0.3, step_height=0.08), 0),
    ("pyramid_stairs_up", "pyramid_stairs_terrain", dict(step_width=0.25, step_height=0.1, platform_size=2.0), 0),
    ("pyramid_stairs_down", "pyramid_stairs_terrain", dict(step_width=0.25, step_height=-0.1, platform_size=2.0), 0),
    ("stepping_stones", "stepping_stones_terrain", dict(stone_size=0.9, stone_distance=0.1, max_height=0.0,
                                                        platform_size=2.0), 6),
    ("stepping_stones_h", "stepping_stones_terrain", dict(stone_size=0.6, stone_distance=0.4, max_height=0.4,
                                                          platform_size=3.0, depth=-5.0), 7),
    ("parkour", "parkour_terrain", dict(start_platform_length=1.0, start_platform_height=0.1,
                                        x_positions=[2.0, 3.5, 5.0], y_positions=[0.0, 0.5, -0.7],
                                        obstacle_lengths=[0.3, 0.35, 0.5], obstacle_heights=[0.2, -2.0, 0.35],
                                        half_valid_width=1.5, border_width=0.2, border_height=0.5), 0),
    ("parkour_hurdle_randomized", "parkour_hurdle_terrain_randomized",
     dict(platform_len=1.0, platform_height=0.1, x_range=(1.0, 1.6), y_range=(-0.5, 0.5), num_hurdles=3,
          hurdle_thickness=0.3, hurdle_height_range=(0.2, 0.3), half_valid_width=(1.0, 1.4), border_width=0.1,
          border_height=0.5), 8),
    ("gap", "gap_terrain", dict(gap_size=0.6, platform_size=2.0), 0),
    ("pit", "pit_terrain", dict(depth=0.4, platform_size=2.0), 0),
]


def gen_cases(out):
    for name, fn, kw, seed in GEN_CASES:
        np.random.seed(seed)
        t = ref_tu.SubTerrain("terrain", width=48, length=64, vertical_scale=0.005, horizontal_scale=0.1)
        f = getattr(ref_tu, fn, None) or getattr(ref_terrain, fn)
        import contextlib
        import io
        with contextlib.redirect_stdout(io.StringIO()):
            f(t, **kw)
        out[f"gen.{name}"] = t.height_field_raw.copy()
        out[f"gen.{name}.rng_after"] = np.array([np.random.randint(0, 2**31 - 1)])
        for attr in ("hurdle_positions", "hurdles"):
            if hasattr(t, attr):
                out[f"gen.{name}.{attr}"] = np.array(getattr(t, attr), dtype=np.float64)


def gen_mesh(out):
    np.random.seed(11)
    t = ref_tu.SubTerrain("terrain", width=40, length=36, vertical_scale=0.005, horizontal_scale=0.1)
    ref_tu.pyramid_stairs_terrain(t, step_width=0.3, step_height=0.12, platform_size=1.0)
    ref_tu.random_uniform_terrain(t, min_height=-0.03, max_height=0.03, step=0.005, downsampled_scale=0.2)
    hf = t.height_field_raw.copy()
    v, tri = ref_tu.convert_heightfield_to_trimesh(hf, 0.1, 0.005, 0.75)
    out["mesh.hf"] = hf
    out["mesh.vertices"] = v
    out["mesh.triangles"] = tri
    v0, tri0 = ref_tu.convert_heightfield_to_trimesh(hf, 0.1, 0.005, None)
    out["mesh.vertices_noslope"] = v0


def _terrain_cfg(task, edit=None):
    env_cfg, _ = task_registry.get_cfgs(task)
    if edit:
        edit(env_cfg.terrain)
    return env_cfg.terrain


def gen_fields(out):
    cases = [
        ("go2_parkour", "go2_parkour", None, 1, True),
        ("go2_parkour_finetune", "go2_parkour_finetune", None, 1, False),
        ("anymal_c_rough", "anymal_c_rough", None, 1, False),
        ("randomized_small", "anymal_c_rough",
         lambda t: (setattr(t, "curriculum", False), setattr(t, "num_rows", 3), setattr(t, "num_cols", 4),
                    setattr(t, "mesh_type", "heightfield")), 5, False),
        ("selected_small", "anymal_c_rough",
         lambda t: (setattr(t, "curriculum", False), setattr(t, "selected", True), setattr(t, "num_rows", 2),
                    setattr(t, "num_cols", 3), setattr(t, "mesh_type", "heightfield"),
                    setattr(t, "terrain_kwargs", {"type": "terrain_utils.discrete_obstacles_terrain",
                                                  "max_height": 0.2, "min_size": 1.0, "max_size": 2.0,
                                                  "num_rects": 10, "platform_size": 2.0})), 9, False),
        ("roughness_small", "go2_parkour",
         lambda t: (setattr(t, "add_roughness_to_selected_terrain", True), setattr(t, "num_rows", 2),
                    setattr(t, "num_cols", 3), setattr(t, "mesh_type", "heightfield")), 2, False),
    ]
    for name, task, edit, seed, mesh in cases:
        cfg = _terrain_cfg(task, edit)
        np.random.seed(seed)
        ter = ref_terrain.Terrain(cfg, 64)
        hf = ter.height_field_raw
        out[f"field.{name}.sha1"] = np.array(sha1(hf))
        out[f"field.{name}.shape"] = np.array(hf.shape)
        out[f"field.{name}.minmax"] = np.array([hf.min(), hf.max()])
        out[f"field.{name}.env_origins"] = ter.env_origins.copy()
        out[f"field.{name}.seed"] = np.array(seed)
        out[f"field.{name}.rng_after"] = np.array([np.random.randint(0, 2**31 - 1)])
        if hf.size <= 600_000:
            out[f"field.{name}.hf"] = hf.copy()
        if mesh and cfg.mesh_type == "trimesh":
            out[f"field.{name}.vertices_sha1"] = np.array(sha1(ter.vertices))
            out[f"field.{name}.triangles_sha1"] = np.array(sha1(ter.triangles))
        print(name, hf.shape, sha1(hf)[:12], hf.min(), hf.max())


def _jsonable(x):
    if isinstance(x, dict):
        return {k: _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    if isinstance(x, np.generic):
        return x.item()
    return x


def gen_configs():
    """class_to_dict of every registered task's (env_cfg, train_cfg) — the drop-in
    config surface (base_config.py:33-55, helpers.py class_to_dict)."""
    import json
    from legged_gym.utils.helpers import class_to_dict
    out = {}
    for task in ("go2", "go2_parkour", "go2_parkour_finetune", "anymal_c_rough", "anymal_c_flat"):
        env_cfg, train_cfg = task_registry.get_cfgs(task)
        out[task] = {"env": _jsonable(class_to_dict(env_cfg)), "train": _jsonable(class_to_dict(train_cfg))}
    path = os.path.join(REPO, "tests", "golden", "configs.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    gen_configs()
    out = {}
    gen_cases(out)
    gen_mesh(out)
    gen_fields(out)
    path = os.path.join(REPO, "tests", "golden", "terrain.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")
