"""The PPO minibatch's optimizer tail alone (dev tool): the go2_c2 learner case after one eager
update, lgx_ppo_tail timed with HIP events over 200 calls, with the S8 copies (the product) and
without (the table withheld: the kernel then writes no S8, as with LGX_TAIL_S8=0), interleaved.
The library is the product one or LGX_MLP_LIB (a build variant).
Usage: PYTHONPATH=.:tests python tools/tail_ab.py"""
import json
import os
import statistics

import torch

import learner_case as LC
import learner_replay as R

dev = "cuda:0"


def main():
    case = "go2_c2"
    alg = R.build(case, dev, use_graphs=False)
    R.rollout(alg, case, 1, {}, False, dev)
    alg.total_updates = LC.TOTAL_UPDATES
    alg._reg_coef.fill_(alg.reg_coef())
    alg._perm.copy_(torch.from_numpy(LC.permutation(case, 1)).to(dev))
    alg._precompute()
    s8 = alg._s8
    assert s8 is not None and s8.tail_table() is not None
    table = s8.tail_table
    res = {"with_s8": [], "without": []}
    for rnd in range(6):
        for mode in ("with_s8", "without"):
            s8.tail_table = table if mode == "with_s8" else (lambda: None)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(5):
                alg._minibatch_step()
            a.record()
            for _ in range(200):
                alg._minibatch_step()
            b.record()
            b.synchronize()
            if rnd:
                res[mode].append(a.elapsed_time(b) * 1000 / 200)
    s8.tail_table = table
    print(json.dumps({"lib": os.environ.get("LGX_MLP_LIB", "product"),
                      **{k: round(statistics.median(v), 2) for k, v in res.items()}}))


if __name__ == "__main__":
    main()
