"""Terrain generation: legged_gym_custom_amd.utils.terrain /
terrain_utils against the reference's own outputs (tests/golden/terrain.npz, written by
tools/gen_terrain_golden.py from legged_gym/utils/terrain.py + terrain_utils.py).

Bit-exact: int16 height fields, env origins, trimesh vertices/triangles, and the numpy
RNG state after each generator (same draws in the same order). Whole fields are pinned
by sha1 (go2_parkour: 240080b3f8ed..., the value SURVEY.md a17 measured)."""
import hashlib

import numpy as np
import pytest

import golden_util as G
from legged_gym_custom_amd.envs import task_registry_configs
from legged_gym_custom_amd.utils import terrain as T
from legged_gym_custom_amd.utils import terrain_utils as TU


@pytest.fixture(scope="module")
def gold():
    return G.load("terrain.npz")


def _sha1(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()


# must mirror tools/gen_terrain_golden.py GEN_CASES
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


@pytest.mark.parametrize("case", GEN_CASES, ids=[c[0] for c in GEN_CASES])
def test_generator_matches_reference(gold, case):
    name, fn, kw, seed = case
    np.random.seed(seed)
    t = TU.SubTerrain("terrain", width=48, length=64, vertical_scale=0.005, horizontal_scale=0.1)
    (getattr(TU, fn, None) or getattr(T, fn))(t, **kw)
    assert t.height_field_raw.dtype == np.int16
    np.testing.assert_array_equal(t.height_field_raw, gold[f"gen.{name}"])
    assert np.random.randint(0, 2**31 - 1) == int(gold[f"gen.{name}.rng_after"][0]), "RNG draw order differs"
    for attr in ("hurdle_positions", "hurdles"):
        if f"gen.{name}.{attr}" in gold:
            np.testing.assert_array_equal(np.array(getattr(t, attr), np.float64), gold[f"gen.{name}.{attr}"])


def test_trimesh_conversion_matches_reference(gold):
    hf = gold["mesh.hf"]
    v, tri = TU.convert_heightfield_to_trimesh(hf, 0.1, 0.005, 0.75)
    assert v.dtype == np.float32 and tri.dtype == np.uint32
    np.testing.assert_array_equal(v, gold["mesh.vertices"])
    np.testing.assert_array_equal(tri, gold["mesh.triangles"])
    v0, _ = TU.convert_heightfield_to_trimesh(hf, 0.1, 0.005, None)
    np.testing.assert_array_equal(v0, gold["mesh.vertices_noslope"])
    # the slope correction really produced vertical walls on this stepped tile
    assert not np.array_equal(v, v0)


def _field_cfg(name):
    task = {"go2_parkour": "go2_parkour", "go2_parkour_finetune": "go2_parkour_finetune",
            "anymal_c_rough": "anymal_c_rough", "randomized_small": "anymal_c_rough",
            "selected_small": "anymal_c_rough", "roughness_small": "go2_parkour"}[name]
    t = task_registry_configs(task)[0].terrain
    if name == "randomized_small":
        t.curriculum, t.num_rows, t.num_cols, t.mesh_type = False, 3, 4, "heightfield"
    elif name == "selected_small":
        t.curriculum, t.selected, t.num_rows, t.num_cols, t.mesh_type = False, True, 2, 3, "heightfield"
        t.terrain_kwargs = {"type": "terrain_utils.discrete_obstacles_terrain", "max_height": 0.2,
                            "min_size": 1.0, "max_size": 2.0, "num_rects": 10, "platform_size": 2.0}
    elif name == "roughness_small":
        t.add_roughness_to_selected_terrain, t.num_rows, t.num_cols, t.mesh_type = True, 2, 3, "heightfield"
    return t


FIELDS = ["go2_parkour", "go2_parkour_finetune", "anymal_c_rough", "randomized_small", "selected_small",
          "roughness_small"]


@pytest.mark.parametrize("name", FIELDS)
def test_whole_field_matches_reference(gold, name):
    cfg = _field_cfg(name)
    np.random.seed(int(gold[f"field.{name}.seed"]))
    ter = T.Terrain(cfg, 64)
    hf = ter.height_field_raw
    assert tuple(hf.shape) == tuple(gold[f"field.{name}.shape"])
    if f"field.{name}.hf" in gold:
        np.testing.assert_array_equal(hf, gold[f"field.{name}.hf"])
    assert _sha1(hf) == str(gold[f"field.{name}.sha1"])
    np.testing.assert_array_equal(ter.env_origins, gold[f"field.{name}.env_origins"])
    assert np.random.randint(0, 2**31 - 1) == int(gold[f"field.{name}.rng_after"][0])
    if f"field.{name}.vertices_sha1" in gold:
        assert _sha1(ter.vertices) == str(gold[f"field.{name}.vertices_sha1"])
        assert _sha1(ter.triangles) == str(gold[f"field.{name}.triangles_sha1"])


def test_parkour_field_is_the_surveyed_one(gold):
    assert str(gold["field.go2_parkour.sha1"]).startswith("240080b3f8ed")
    assert tuple(gold["field.go2_parkour.shape"]) == (3860, 2500)


def test_selected_terrain_leaves_cfg_intact():
    cfg = _field_cfg("selected_small")
    np.random.seed(0)
    T.Terrain(cfg, 8)
    assert cfg.terrain_kwargs["type"] == "terrain_utils.discrete_obstacles_terrain"


def test_plane_builds_nothing():
    cfg = task_registry_configs("go2")[0].terrain
    ter = T.Terrain(cfg, 8)
    assert not hasattr(ter, "height_field_raw")


def test_packed_mesh_rebuilds_the_reference_trimesh(gold):
    """lgx_buffers.terrain_mesh words decode to the reference trimesh's vertices
    (positions to fp32 rounding; heights exact), with and without the slope walls."""
    hf = gold["mesh.hf"]
    for thr, key in ((0.75, "mesh.vertices"), (None, "mesh.vertices_noslope")):
        w = TU.pack_mesh(hf, 0.1, 0.005, thr)
        assert w.dtype == np.uint32 and w.shape == hf.shape
        h = (w & 0xFFFF).astype(np.uint16).view(np.int16)
        dx = ((w >> 16) & 3).astype(np.int64) - 1
        dy = ((w >> 18) & 3).astype(np.int64) - 1
        ii, jj = np.meshgrid(np.arange(hf.shape[0]), np.arange(hf.shape[1]), indexing="ij")
        v = np.stack([(ii + dx) * 0.1, (jj + dy) * 0.1, h * 0.005], -1).reshape(-1, 3)
        np.testing.assert_array_equal(h, hf)
        np.testing.assert_allclose(v, gold[key], atol=2e-6, rtol=0)
        assert (np.abs(dx) <= 1).all() and (np.abs(dy) <= 1).all()


def test_torchscript_reader_round_trip(tmp_path):
    """actuator.read_torchscript_tensors (no deserialisation) returns exactly the
    tensors torch.jit.save wrote, for the SEA net architecture (anymal.py:24)."""
    from legged_gym_custom_amd import actuator as act
    w = act.random_sea_weights(7)
    p = str(tmp_path / "net.pt")
    act.save_sea_archive(w, p)
    r = act.load_sea_lstm(p)
    for k in act.SEA_KEYS:
        np.testing.assert_array_equal(r[k], w[k])


def test_sea_lstm_restatement_matches_torch_lstm_cell():
    """SeaLSTM == x*in_scale -> 2-layer nn.LSTM step -> Linear -> *out_scale, checked
    against an explicit gate-by-gate fp64 evaluation (gate order i f g o)."""
    import torch
    from legged_gym_custom_amd import actuator as act
    w = act.random_sea_weights(4)
    net = act.SeaLSTM(w).double()
    g = torch.Generator().manual_seed(0)
    x = torch.randn(50, 1, 2, generator=g, dtype=torch.float64)
    h = torch.randn(2, 50, 8, generator=g, dtype=torch.float64)
    c = torch.randn(2, 50, 8, generator=g, dtype=torch.float64)
    with torch.no_grad():
        tau, (h1, c1) = net(x, (h, c))
    W = {k: torch.from_numpy(v).double() for k, v in w.items()}
    inp = x[:, 0, :] * W["in_scale"].reshape(2)
    hs, cs = [], []
    for layer in range(2):
        gates = inp @ W[f"lstm.weight_ih_l{layer}"].T + W[f"lstm.bias_ih_l{layer}"] + \
            h[layer] @ W[f"lstm.weight_hh_l{layer}"].T + W[f"lstm.bias_hh_l{layer}"]
        i, f, gg, o = gates.split(8, dim=1)
        cn = torch.sigmoid(f) * c[layer] + torch.sigmoid(i) * torch.tanh(gg)
        hn = torch.sigmoid(o) * torch.tanh(cn)
        hs.append(hn); cs.append(cn)
        inp = hn
    want = W["out_scale"] * (inp @ W["linear.weight"].T + W["linear.bias"])[:, 0]
    torch.testing.assert_close(tau, want)
    torch.testing.assert_close(h1, torch.stack(hs))
    torch.testing.assert_close(c1, torch.stack(cs))
