"""GPU diagnostic: kernel vs oracle physics on random contact-heavy states, with the
solver knobs varied to localise a discrepancy (dev tool, not a test)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import golden_util as G  # noqa: E402
from native_util import Twin  # noqa: E402
from test_gpu_parity import _random_state  # noqa: E402
from legged_gym_custom_amd import model as mdl, _native  # noqa: E402


def run(decim, iters, margin=None, seed=7, n=64):
    cfg, m, P = G.go2_setup(n)
    P.push_robots = 0
    P.decimation = decim
    P.solver_iterations = iters
    if margin is not None:
        P.contact_margin = margin
    tw = Twin(P, mdl.to_struct(m), P.num_reward_terms + P.has_termination_reward)
    rng = np.random.default_rng(seed)
    _random_state(tw, P, rng, n)
    tw.push()
    tw.o.step(3, 11)
    tw.native.step(3, 11, tw.stream())
    tw.sync()
    a = tw.a
    d_dof = np.abs(tw.gpu("dof_state") - a["dof_state"]).reshape(n, -1).max(1)
    d_root = np.abs(tw.gpu("root_states") - a["root_states"]).max(1)
    d_cf = np.abs(tw.gpu("contact_forces") - a["contact_forces"]).reshape(n, -1).max(1)
    ncon_o = (np.abs(a["contact_forces"][:, :, 2]) > 0).sum(1)
    ncon_g = (np.abs(tw.gpu("contact_forces")[:, :, 2]) > 0).sum(1)
    bad = np.argsort(-d_dof)[:6]
    print(f"decim={decim} iters={iters} margin={margin}: max dof {d_dof.max():.3e} root {d_root.max():.3e} "
          f"cf {d_cf.max():.3e}")
    for e in bad:
        dd = np.abs(tw.gpu("dof_state")[e] - a["dof_state"][e])
        print(f"   env {e}: dof {d_dof[e]:.3e} root {d_root[e]:.3e} cf {d_cf[e]:.3e} bodies_w_force oracle {ncon_o[e]} "
              f"gpu {ncon_g[e]} worst joint {np.unravel_index(dd.argmax(), dd.shape)} reset o/g {a['reset'][e]}/{tw.gpu('reset')[e]}")


for decim, iters in [(1, 0), (1, 1), (1, 8), (4, 8)]:
    run(decim, iters)
run(1, 8, margin=0.0)
