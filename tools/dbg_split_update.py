"""Dev debug (GPU): record every minibatch's gradients of the go2_c2 golden update (tests/
learner_replay.py flow) under this process's knobs; with --compare A B print per-minibatch max
relative differences between two recordings."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    keys = sorted(a.files)
    mbs = sorted({int(k.split(".")[0][2:]) for k in keys})
    for mb in mbs:
        worst = []
        for k in keys:
            if k.startswith(f"mb{mb}."):
                x, y = a[k], b[k]
                d = float(np.abs(x - y).max() / (np.abs(x).max() + 1e-30))
                worst.append((d, k))
        worst.sort(reverse=True)
        print(mb, [(k, f"{d:.2e}") for d, k in worst[:3]])
    sys.exit(0)

import torch  # noqa: E402
import learner_replay as LR  # noqa: E402

out = sys.argv[1]
rec = {}
orig_build = LR.build


def build(case, device, use_graphs=None):
    alg = orig_build(case, device, use_graphs=False)
    f = alg._minibatch_grads
    cnt = [0]

    def grads(mb):
        r = f(mb)
        for n, p in LR.named_params(alg):
            if p.grad is not None:
                rec[f"mb{cnt[0]}.{n}"] = p.grad.detach().cpu().numpy().copy()
        cnt[0] += 1
        return r
    alg._minibatch_grads = grads
    return alg


LR.build = build
LR.run("go2_c2", "cuda")
np.savez(out, **rec)
print("recorded", len(rec))
