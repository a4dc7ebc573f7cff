"""Drop-in config surface: class_to_dict of every task's (env_cfg, train_cfg) equals the
reference's (tests/golden/configs.json, written by tools/gen_terrain_golden.py from the
reference's own config classes; base_config.py:33-55, helpers.py class_to_dict)."""
import json
import os

import pytest

from legged_gym_custom_amd.envs import task_registry_configs
from legged_gym_custom_amd.utils.helpers import class_to_dict

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "configs.json")


def _norm(x):
    if isinstance(x, dict):
        return {k: _norm(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_norm(v) for v in x]
    if hasattr(x, "item"):
        return x.item()
    return x


def _diff(a, b, path=""):
    if isinstance(a, dict) and isinstance(b, dict):
        out = []
        for k in sorted(set(a) | set(b)):
            if k not in a or k not in b:
                out.append(f"{path}.{k}: {'missing here' if k not in a else 'extra here'}")
            else:
                out.extend(_diff(a[k], b[k], f"{path}.{k}"))
        return out
    return [] if a == b else [f"{path}: {a!r} != {b!r}"]


@pytest.mark.parametrize("task", ["go2", "go2_parkour", "go2_parkour_finetune", "anymal_c_rough", "anymal_c_flat"])
def test_config_matches_reference(task):
    with open(GOLDEN) as f:
        want = json.load(f)[task]
    env_cfg, train_cfg = task_registry_configs(task)
    env_cfg.seed = train_cfg.seed  # what task_registry.get_cfgs adds (task_registry.py:52-58)
    got = {"env": _norm(class_to_dict(env_cfg)), "train": _norm(class_to_dict(train_cfg))}
    problems = _diff(json.loads(json.dumps(got)), want)
    assert not problems, "\n".join(problems[:40])


def test_command_curriculum_needs_the_tracking_term():
    """commands.curriculum (go2.py:80-107) reads episode_sums['tracking_lin_vel']; without
    that reward term the reference raises KeyError at the first curriculum step — here at
    build time, before anything is launched."""
    import pytest
    from legged_gym_custom_amd import model as mdl, params as prm
    from legged_gym_custom_amd.envs import task_registry_configs
    env_cfg, _ = task_registry_configs("go2")
    env_cfg.commands.curriculum = True
    env_cfg.rewards.scales.tracking_lin_vel = 0.0
    m = mdl.load_model(env_cfg.asset.file, env_cfg.asset.foot_name)
    with pytest.raises(KeyError, match="tracking_lin_vel"):
        prm.build_task_params(env_cfg, m, 4)


def test_device_command_ranges_write_through():
    """command_ranges under the command curriculum lives in a device buffer: the reference's
    per-end idiom `command_ranges["lin_vel_x"][1] = v` (go2.py:96-107) must reach it."""
    import torch
    from legged_gym_custom_amd.envs.base.legged_robot import _DeviceCommandRanges
    buf = torch.tensor([-1.0, 1.0, -0.5, 0.5, -1.0, 1.0, -3.14, 3.14], dtype=torch.float64)
    r = _DeviceCommandRanges(buf)
    r["lin_vel_x"][1] = 2.5
    r["lin_vel_y"][0] = -0.75
    assert r["lin_vel_x"] == [-1.0, 2.5] and r["lin_vel_y"] == [-0.75, 0.5]
    r["heading"] = [0.0, 1.0]
    assert buf.tolist() == [-1.0, 2.5, -0.75, 0.5, -1.0, 1.0, 0.0, 1.0]
    assert dict(r.items())["ang_vel_yaw"] == [-1.0, 1.0]
