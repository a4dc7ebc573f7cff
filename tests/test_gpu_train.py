"""`train.py --task=go2` end to end on the MI355X (legged_gym/scripts/train.py flow):
registry -> env (liblgx.so) -> runner (HIP MLP GEMMs, graph-captured update) -> logs and
reference-format checkpoints."""
import glob
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_train_entry_point_runs_and_checkpoints(tmp_path, monkeypatch):
    import sys
    from legged_gym_custom_amd.scripts import train
    trm = sys.modules["legged_gym_custom_amd.utils.task_registry"]  # the module (the package re-exports the instance)
    monkeypatch.setattr(trm, "LEGGED_GYM_ROOT_DIR", str(tmp_path))
    train.main(["--task=go2", "--headless", "--num_envs=256", "--max_iterations=4", "--seed=3"])
    ck = sorted(glob.glob(os.path.join(tmp_path, "logs", "go2", "*", "model_*.pt")))
    assert any(c.endswith("model_4.pt") for c in ck), ck
    d = torch.load([c for c in ck if c.endswith("model_4.pt")][0], weights_only=True)
    assert d["iter"] == 4
    assert all(torch.isfinite(v).all() for v in d["model_state_dict"].values())
