"""Kernels of one runner iteration outside the rollout steps and the PPO minibatches (dev
tool): python tools/trace_outside.py <trace.csv>. Prints, for the last complete iteration
(between two first-env-step-of-iteration markers), the kernels that run between the last env
step and the first minibatch gather, and after the last minibatch."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
env = [i for i, k in enumerate(ks) if "env_step" in k[2]]
# iterations: 24 env steps each; the last full iteration ends before the trace's last env block
blocks = [env[0]]
for a, b in zip(env, env[1:]):
    if b - a > 200:
        blocks.append(b)
if len(blocks) < 3:
    sys.exit("not enough iterations in the trace")
start, end = blocks[-2], blocks[-1]
last_env = max(i for i in env if i < end)
t0 = ks[start][0]
print(f"iteration: {(ks[end][0] - t0) / 1e3:.1f} us; after the last env step:")
tot = 0
for s, e, n in ks[last_env + 1:end]:
    nm = n.split("(")[0]
    if "gemm" in nm or "loss_heads" in nm or "tail_" in nm or "splitk" in nm or "transpose" in nm:
        continue
    tot += e - s
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  {nm[:90]}")
print(f"non-GEMM/non-head kernels after the rollout: {tot / 1e3:.1f} us")
