"""Adam moments after the C2 golden update: S8 minibatch path vs the autograd path, each vs the
reference fixture (tests/golden/learner_go2_c2.npz) — how much of the difference is the path
and how much is the update's sensitivity to rounding (dev tool)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402

import learner_case as LC  # noqa: E402
import learner_replay as R  # noqa: E402
from legged_gym_custom_amd.rsl_rl.algorithms import ppo as P  # noqa: E402


def worst(case, res, d):
    out = {}
    for n, m in res["exp_avg"].items():
        for key in ("exp_avg", "exp_avg_sq"):
            ref = d[f"{key}.{n}.v"]
            got = (m if key == "exp_avg" else res["exp_avg_sq"][n]).reshape(-1)[LC.sample_index(n, m.size)]
            out[(key, n)] = float(np.abs(got - ref).max()) / (float(np.abs(ref).max()) + 1e-30)
    return out


case = sys.argv[1] if len(sys.argv) > 1 else "go2_c2"
d = R.load(case)
runs = {}
for s8 in (False, True):
    P.USE_S8 = s8
    res, alg = R.run(case, "cuda:0")
    assert (alg._s8 is not None) == s8
    runs[s8] = res
    w = worst(case, res, d)
    top = sorted(w.items(), key=lambda kv: -kv[1])[:6]
    print(f"s8={s8}: worst moments vs reference", [(k[0], k[1], round(v, 5)) for k, v in top])
# S8 vs autograd path directly
diff = []
for n, m in runs[True]["exp_avg"].items():
    r = runs[False]["exp_avg"][n]
    diff.append((n, float(np.abs(m - r).max()) / (float(np.abs(r).max()) + 1e-30)))
print("S8 vs autograd path, exp_avg", sorted(diff, key=lambda x: -x[1])[:6])
g0 = [(n, float(np.abs(runs[True]["grad0"][n] - g).max() / (np.abs(g).max() + 1e-30))) for n, g in runs[False]["grad0"].items()]
print("minibatch-0 gradients, S8 vs autograd", sorted(g0, key=lambda x: -x[1])[:4])
pa = [(n, float(np.abs(runs[True]["after"][n] - p).max())) for n, p in runs[False]["after"].items()]
print("params after the update, max |S8 - autograd|", sorted(pa, key=lambda x: -x[1])[:4])
