"""TorchScript export (helpers.py:180-214), CPU. (The checkpoint
format, on_policy_runner.py:283-297, is covered by test_runner_cpu.py.)

The four exported files are what deploy/base/deploy_base.py:32-35 loads and
deploy_base.py:249-264 calls: policy(cat(obs, adaptation(hist), scan_encoder(scan),
estimator(obs))). The exports must compute exactly the live modules' forward (fp32, same
device) and keep the reference's state_dict keys, although the live MLPs are HipMLP and
the adaptation encoder has a HIP forward."""
import os

import torch

from test_ppo_update import A, EST, H, P, PRIV, SCAN, _make
from legged_gym_custom_amd.utils.helpers import export_policy_as_jit


def test_exported_modules_match_live_modules(tmp_path):
    alg = _make("fixed", seed=3)
    ac, est = alg.actor_critic, alg.estimator
    export_policy_as_jit(ac, est, str(tmp_path))
    files = sorted(os.listdir(tmp_path))
    assert files == ["adaptation_module.pt", "estimator.pt", "policy.pt", "scan_encoder.pt"]
    policy = torch.jit.load(str(tmp_path / "policy.pt"))
    adapt = torch.jit.load(str(tmp_path / "adaptation_module.pt"))
    estim = torch.jit.load(str(tmp_path / "estimator.pt"))
    scan_enc = torch.jit.load(str(tmp_path / "scan_encoder.pt"))
    # same parameter names as the live modules (= the reference's, e.g. actor '0.weight')
    assert list(policy.state_dict()) == list(ac.actor.state_dict())
    assert list(adapt.state_dict()) == list(ac.adaptation_encoder_.state_dict())
    assert list(estim.state_dict()) == list(est.state_dict())
    assert list(scan_enc.state_dict()) == list(ac.scan_encoder.state_dict())
    g = torch.Generator().manual_seed(0)
    B = 7
    obs = torch.randn(B, P * (1 + H), generator=g)
    priv = torch.randn(B, PRIV, generator=g)
    scan = torch.randn(B, SCAN, generator=g)
    with torch.no_grad():
        hist = obs[:, :H * P].reshape(B, H, P)
        z, s, e = adapt(hist), scan_enc(scan), estim(obs)
        torch.testing.assert_close(z, ac.adaptation_encoder_(hist), rtol=0, atol=0)
        torch.testing.assert_close(s, ac.scan_encoder(scan), rtol=0, atol=0)
        torch.testing.assert_close(e, est(obs), rtol=0, atol=0)
        # the deploy pipeline (deploy_base.py:249-264) == act_inference in adaptation mode
        a = policy(torch.cat((obs, z, s, e), dim=-1))
        want = ac.act_inference(obs, priv, est(obs), scan, adaptation_mode=True)
        torch.testing.assert_close(a, want, rtol=0, atol=0)
        assert a.shape == (B, A)


def test_exported_files_load_without_this_package(tmp_path):
    """The export is self-contained TorchScript: no legged_gym_custom_amd class is needed
    to load and run it (a deploy box has only torch)."""
    import subprocess
    import sys
    alg = _make("fixed", seed=1)
    export_policy_as_jit(alg.actor_critic, alg.estimator, str(tmp_path))
    code = ("import torch,sys; m=torch.jit.load(sys.argv[1]); "
            "print(tuple(m(torch.zeros(2, %d)).shape))" % SCAN)
    env = dict(os.environ, PYTHONPATH="")
    out = subprocess.run([sys.executable, "-c", code, str(tmp_path / "scan_encoder.pt")], capture_output=True,
                         text=True, cwd=str(tmp_path), env=env, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().endswith("(2, 4)")
