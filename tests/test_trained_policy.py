"""Physics plausibility with the reference's trained deploy networks (SURVEY.md
§4/§7 step 5). The policy trained in Isaac Gym / PhysX (deploy/networks/go2/parkour_v12_ft_iii,
read in place by the parse-only TorchScript reader, nothing stored here) drives this build's
physics (the CPU oracle: the same model as the HIP kernel, pinned to it by
tests/test_gpu_trajectory.py) on flat ground for 600 steps. It must walk: >= 95 % of the robots
survive, the mean base height is within 3.5 cm of the 0.296 m the reference's recorded deploy
scan implies (deploy/base/SCAN_v12_ft_iii.txt), the robot moves forward at >= half the command,
and foot contacts follow the gait clock more often than not. Runs only where /root/reference
exists (this container). Measured numbers: profiles/r02_trained_policy.txt."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NETS = "/root/reference/deploy/networks/go2/parkour_v12_ft_iii"
pytestmark = pytest.mark.skipif(not os.path.isdir(NETS), reason="reference deploy networks not present")


def test_reader_matches_torch_serializer():
    import torch
    import tempfile
    from legged_gym_custom_amd.utils import ts_archive as ts
    from legged_gym_custom_amd.rsl_rl.modules.support_networks import AdaptationEncoderTS

    class Nested(torch.nn.Module):  # the exported ScanEncoder / MlpEstimator layout
        def __init__(self):
            super().__init__()
            self.scan_encoder = torch.nn.Sequential(torch.nn.Linear(132, 128), torch.nn.ELU(), torch.nn.Linear(128, 32))

        def forward(self, x):
            return self.scan_encoder(x)

    for m in (AdaptationEncoderTS(52, 10, 20), Nested()):
        p = os.path.join(tempfile.mkdtemp(), "m.pt")
        torch.jit.script(m).save(p)
        st, sd = ts.read_state(p), m.state_dict()
        assert list(st) == list(sd)
        for k in sd:
            assert torch.equal(torch.from_numpy(st[k]), sd[k]), k


@pytest.mark.parametrize("vx", [0.5, 1.0])
def test_trained_parkour_policy_walks_in_build_physics(vx):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import trained_policy_rollout as tp
    r = tp.rollout("parkour_v12_ft_iii", n=64, steps=600, vx=vx)
    print(r)
    assert r["survival"] >= 0.95
    assert abs(r["base_height_mean"] - r["scan_trace_height"]) < 0.035
    assert r["vx_mean"] >= 0.5 * vx
    assert r["contact_matches_gait_clock"] > 0.55
    assert min(r["duty_cycle"]) > 0.25 and max(r["duty_cycle"]) < 0.75


def test_shipped_estimators_are_untrained():
    """The velocity estimator shipped beside each trained policy reads ~0 m/s on this physics
     because it was never trained: the runner's checkpoint does not save the
    estimator (on_policy_runner.py:283-289, Appendix B Q13), so play.py's export writes a freshly
    initialised one (helpers.py:180-214). Its weights have nn.Linear's default-init statistics
    (U(+-1/sqrt(fan_in)): mean |w| = bound / 2 for every layer), and the two parkour runs' (and
    the two cheetah runs') estimators are bit-identical — the same seeded initialisation."""
    import numpy as np
    from legged_gym_custom_amd.utils import ts_archive as ts
    base = os.path.dirname(NETS)
    st = {r: ts.read_state(os.path.join(base, r, "estimator.pt"))
          for r in ("parkour_v12_ft_iii", "parkour_v12_ft_i", "cheetah_v8", "cheetah_v8_rough")}
    for a, b in (("parkour_v12_ft_iii", "parkour_v12_ft_i"), ("cheetah_v8", "cheetah_v8_rough")):
        assert all(np.array_equal(st[a][k], st[b][k]) for k in st[a])
    for r, s in st.items():
        for k, w in s.items():
            if k.endswith(".weight"):
                bound = 1.0 / np.sqrt(w.shape[1])
                assert np.abs(w).max() <= bound, (r, k)  # never left the init interval
                if w.size >= 1000:
                    assert abs(np.abs(w).mean() / (bound / 2) - 1.0) < 0.02, (r, k)
    # the policies and adaptation modules beside them are trained: weights far outside that interval
    for r in ("parkour_v12_ft_iii", "cheetah_v8"):
        for f in ("policy.pt", "adaptation_module.pt"):
            s = ts.read_state(os.path.join(base, r, f))
            w = next(v for k, v in s.items() if k.endswith("weight") and v.ndim == 2)
            assert np.abs(w).max() > 1.3 / np.sqrt(w.shape[1]), (r, f)


def test_trained_policy_with_deploy_gait_clock_and_true_velocity():
    """The settings the reference deployed this policy with (deploy/configs/go2.yaml: gait
    period 0.35 s) and the velocity a trained estimator would supply (the env's true estimated
    observation, which PPO.update trains the estimator toward, ppo.py:224-231): the stance
    height matches the recorded deploy scan's 0.296 m to 1 cm and the feet follow the gait clock
    in >= 70 % of the steps (profiles/r03_trained_policy.txt)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import trained_policy_rollout as tp
    r = tp.rollout("parkour_v12_ft_iii", n=64, steps=600, vx=1.0, est_source="true", period=0.35)
    print(r)
    assert r["survival"] >= 0.95
    assert abs(r["base_height_mean"] - r["scan_trace_height"]) < 0.01
    assert r["contact_matches_gait_clock"] >= 0.7
