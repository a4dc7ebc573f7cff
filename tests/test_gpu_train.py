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


def test_play_loads_latest_checkpoint_and_exports(tmp_path, monkeypatch):
    """play.py flow (legged_gym/scripts/play.py:12-105) after a short train: the latest
    model_*.pt of the experiment is loaded, the four TorchScript files are exported and
    reproduce the GPU inference policy on CPU, and the headless play loop runs."""
    import copy
    import sys
    from legged_gym_custom_amd.scripts import play, train
    from legged_gym_custom_amd.utils.helpers import get_args
    trm = sys.modules["legged_gym_custom_amd.utils.task_registry"]
    reg = trm.task_registry
    monkeypatch.setattr(trm, "LEGGED_GYM_ROOT_DIR", str(tmp_path))
    monkeypatch.setitem(reg.env_cfgs, "go2", copy.deepcopy(reg.env_cfgs["go2"]))
    monkeypatch.setitem(reg.train_cfgs, "go2", copy.deepcopy(reg.train_cfgs["go2"]))
    train.main(["--task=go2", "--headless", "--num_envs=128", "--max_iterations=2", "--seed=5"])
    env, runner, logger, path = play.play(get_args(["--task=go2", "--headless"]), num_steps=120, root=str(tmp_path))
    assert runner.current_learning_iteration == 2
    assert sorted(os.listdir(path)) == ["adaptation_module.pt", "estimator.pt", "policy.pt", "scan_encoder.pt"]
    assert len(logger.state_log["dof_pos"]) == 100
    # deploy pipeline on CPU == the live GPU policy
    ac, est = runner.alg.actor_critic, runner.alg.estimator
    obs, scan = env.obs_buf.clone(), env.scan_obs_buf.clone()
    with torch.no_grad():
        want = ac.act_inference(obs, env.privileged_obs_buf, est(obs), scan, adaptation_mode=True).cpu()
        jl = lambda f: torch.jit.load(os.path.join(path, f))  # noqa: E731
        o, s = obs.cpu(), scan.cpu()
        hist = o[:, :-env.num_proprio].reshape(o.shape[0], env.cfg.env.history_buffer_length, env.num_proprio)
        got = jl("policy.pt")(torch.cat((o, jl("adaptation_module.pt")(hist), jl("scan_encoder.pt")(s),
                                         jl("estimator.pt")(o)), dim=-1))
    torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-4)  # GPU bf16x3 GEMMs vs CPU fp32
