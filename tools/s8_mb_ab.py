"""Per-minibatch time of the S8 update (dev tool): the go2_c2 learner case (24,576-row minibatches),
eager minibatches (weight split, forward levels, heads, input-gradient levels, weight gradients,
reduce, optimizer tail) timed with HIP events, median of rounds. The library is the product one
or LGX_S8_LIB (a build variant). Usage: PYTHONPATH=.:tests python tools/s8_mb_ab.py [case]"""
import json
import os
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
    assert alg._s8 is not None
    mbs = list(alg._minibatches())
    ts = []
    for rnd in range(7):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(2):
            for idx in mbs:
                alg._minibatch_grads(idx)
        b.record()
        b.synchronize()
        if rnd >= 2:
            ts.append(a.elapsed_time(b) * 1000 / (2 * len(mbs)))
    print(json.dumps({"lib": os.environ.get("LGX_S8_LIB", "product"), "us_per_minibatch": round(statistics.median(ts), 1),
                      "all": [round(t, 1) for t in ts]}))


if __name__ == "__main__":
    main()
