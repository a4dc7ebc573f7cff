"""Per-layer wall-clock stamps of the act kernel (a dev build, exp/libact_clock.so, that writes
wall_clock64() per layer of row blocks 0 and last into the est storage-row pointer): warm (back
to back) and cold (a 256 MB write between launches, as the env step evicts L2), with and
without the storage-row copies."""
import sys

import torch

import learner_case as LC
import learner_replay as R
from legged_gym_custom_amd.rsl_rl.modules import hip_s8 as S

dev = "cuda:0"
case = "go2_c2"
alg = R.build(case, dev, use_graphs=False)
R.rollout(alg, case, 1, {}, False, dev)
fa = alg._s8act
L = S.load(sys.argv[1])
dbg = torch.zeros(128, dtype=torch.int64, device=dev)
a = fa.args
junk = torch.empty(64 * 1024 * 1024, device=dev)
N = LC.n_envs(case)
st = [torch.empty(N, w, device=dev) for w in (a.n_obs, a.n_priv_in, a.n_critic_in, 3, a.n_scan_in)]


def stamps(cold, rows):
    for _ in range(5):
        if cold:
            junk.zero_()
        if rows:
            a.obs_st, a.priv_st, a.critic_st, a.scan_st = st[0].data_ptr(), st[1].data_ptr(), st[2].data_ptr(), \
                st[4].data_ptr()
        else:
            a.obs_st = a.priv_st = a.critic_st = a.scan_st = None
        a.est_st = dbg.data_ptr()
        S.act(a, L)
    torch.cuda.synchronize()
    d = dbg.cpu().numpy()
    names_a = [f"est{i}" for i in range(a.n_est)] + [f"scan{i}" for i in range(a.n_scan)] + \
        [f"priv{i}" for i in range(a.n_priv)] + [f"actor{i}" for i in range(a.n_actor)]
    names_c = [f"critic{i}" for i in range(a.n_critic)]
    for base, names, tag in ((0, names_a, "actor rb0"), (32, names_c, "critic rb0")):
        t = d[base:base + len(names) + 2]
        us = (t - t[0]) / 100.0  # 100 MHz
        print(f"cold={cold} rows={rows} {tag}", "prologue %.1f" % us[1],
              " ".join(f"{n}:{us[i + 2] - us[i + 1]:.1f}" for i, n in enumerate(names)), "total %.1f us" % us[-1])


for cold in (False, True):
    for rows in (False, True):
        stamps(cold, rows)
