"""The one-launch act kernel (lgx_s8_act) on a go2 C2 batch (4096 envs): HIP-event time per
launch, the product library and build variants interleaved (dev tool).
Usage: PYTHONPATH=.:tests:tools python tools/act_bench.py [variant.so ...]"""
import json
import sys

import torch

import learner_case as LC
import learner_replay as R
from legged_gym_custom_amd.rsl_rl.modules import hip_s8 as S
from s8_bench import timeit_many

dev = "cuda:0"


def main():
    case = "go2_c2"
    alg = R.build(case, dev, use_graphs=False)
    R.rollout(alg, case, 1, {}, False, dev)
    fa = alg._s8act
    assert fa is not None
    N = LC.n_envs(case)
    c = LC.CASES[case]
    g = torch.Generator(device="cpu").manual_seed(0)
    mk = lambda w: torch.randn(N, w, generator=g).to(dev)  # noqa: E731
    obs, priv, critic, scan = mk(c["P"] * (c["H"] + 1)), mk(c["priv"]), mk(c["critic"]), mk(c["scan"])
    fa.run(obs, priv, critic, scan)
    libs = {"product": S.lib()}
    for v in sys.argv[1:]:
        libs[v.split("/")[-1]] = S.load(v)
    res = timeit_many({k: (lambda L=L: S.act(fa.args, L)) for k, L in libs.items()}, n=20, rounds=5)
    print(json.dumps(res))
    # fewer blocks per XCD (the first rows only): per-CU vs per-XCD bound
    for b in (2048, 1024, 256, 32):
        fa.args.B = b
        print(b, json.dumps(timeit_many({"product": lambda: S.act(fa.args)}, n=20, rounds=3)))
    fa.args.B = N


if __name__ == "__main__":
    main()
