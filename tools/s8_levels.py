"""Launch-schedule experiment for the S8 minibatch (dev tool): µs per minibatch (HIP events over
eager minibatches, median of rounds) for level shifts of the critic / estimator chains.
Usage: PYTHONPATH=.:tests python tools/s8_levels.py [case]"""
import itertools
import json
import statistics
import sys

import torch

import learner_case as LC
import learner_replay as R

dev = "cuda:0"


def main():
    case = sys.argv[1] if len(sys.argv) > 1 else "go2_c2"
    alg = R.build(case, dev, use_graphs=False)
    R.rollout(alg, case, 1, {}, False, dev)
    alg.total_updates = LC.TOTAL_UPDATES
    alg._reg_coef.fill_(alg.reg_coef())
    alg._perm.copy_(torch.from_numpy(LC.permutation(case, 1)).to(dev))
    alg._precompute()
    s8 = alg._s8
    assert s8 is not None
    mbs = list(alg._minibatches())
    configs = [(3, 3, 0, 2, sl) for sl in (1, 2, 3, 4)] + [(3, 3, 0, 0, 4), (3, 3, 1, 2, 4)]
    res = {c: [] for c in configs}

    def run():
        for idx in mbs:
            alg._minibatch_grads(idx)
    for rnd in range(5):
        for c in configs:
            s8.fwd_shift = {"critic": c[0], "est": c[1]}
            s8.dx_shift = {"critic": c[2], "est": c[3]}
            s8.l0_slices = {"critic": c[4]}
            run()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(3):
                run()
            b.record()
            b.synchronize()
            res[c].append(a.elapsed_time(b) * 1000 / (3 * len(mbs)))
    out = sorted(((round(statistics.median(v), 1), c) for c, v in res.items()))
    for t, c in out:
        print(f"{t:8.1f} us/minibatch  fwd shift critic {c[0]} est {c[1]}  dx shift critic {c[2]} est {c[3]}"
              f"  critic L0 slices {c[4]}")
    print(json.dumps({str(c): t for t, c in out}))


if __name__ == "__main__":
    main()
