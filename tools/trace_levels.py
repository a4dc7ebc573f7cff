"""Per-launch medians of the update's minibatch sequence from a rocprofv3 kernel trace (dev tool):
the launches between consecutive minibatch-start dispatches (the encoder chain launch, lgxc::chain_kernel,
since round 6 the first launch of a minibatch: the weight split runs once per update),
position by position, and the median span of a minibatch.
Usage: python tools/trace_levels.py <run_kernel_trace.csv> [...]"""
import collections
import csv
import statistics
import sys


def levels(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    seqs, cur = [], None
    for r in rows:
        short = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "lgxc::chain_kernel" in short:
            if cur:
                seqs.append(cur)
            cur = []
        if cur is not None:
            cur.append((short[:44], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000,
                        int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    if cur:
        seqs.append(cur)
    n = collections.Counter(len(s) for s in seqs).most_common(1)[0][0]
    good = [s for s in seqs if len(s) == n][-40:]
    out = [(good[0][k][0], statistics.median(s[k][1] for s in good)) for k in range(n)]
    span = statistics.median((s[-1][3] - s[0][2]) / 1000 for s in good)
    return out, span


if __name__ == "__main__":
    res = [levels(p) for p in sys.argv[1:]]
    for k in range(len(res[0][0])):
        print(f"{k:2d} {res[0][0][k][0]:46s}" + "".join(f"{r[0][k][1]:9.1f}" for r in res if k < len(r[0])))
    print("span" + " " * 45 + "".join(f"{r[1]:9.1f}" for r in res))
