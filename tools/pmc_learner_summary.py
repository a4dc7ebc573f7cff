"""Per-launch PMC means of the learner's grouped GEMM launches and the env kernel, keyed by
kernel and grid size (one grid = one launch shape of the runner iteration), from the passes
of tools/gpu/pmc_learner.sh: python tools/pmc_learner_summary.py gpurun_out/pmc_learner"""
import collections
import csv
import glob
import sys


def main(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + "/p*/*/*_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"].split("(")[0]
            if "gemm_group_kernel" not in n and "env_step" not in n:
                continue
            agg[(n.split("::")[-1], int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"{'kernel':30s} {'grid':>7s} {'L2 hit':>6s} {'L2 req MB':>9s} {'FETCH MB':>8s} {'wait':>5s} "
          f"{'MFMA busy':>9s} {'VALU/MFMA':>9s}")
    rows = []
    for (k, grid), c in agg.items():
        m = {n: sum(v) / len(v) for n, v in c.items()}
        hit, miss = m.get("TCC_HIT_sum", 0.0), m.get("TCC_MISS_sum", 0.0)
        gui = m.get("GRBM_GUI_ACTIVE", 0.0) / 8  # summed over the 8 XCDs
        busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (1024 * gui) if gui else 0.0  # per SIMD
        rows.append((m.get("SQ_WAVE_CYCLES", 0.0), f"{k:30s} {grid:7d} {hit / max(hit + miss, 1):6.3f} "
                     f"{(hit + miss) * 128 / 1e6:9.1f} {m.get('FETCH_SIZE', 0.0) / 1024:8.1f} "
                     f"{m.get('SQ_WAIT_ANY', 0.0) / max(m.get('SQ_WAVE_CYCLES', 1.0), 1.0):5.2f} {busy:9.3f} "
                     f"{m.get('SQ_INSTS_VALU', 0.0) / max(m.get('SQ_INSTS_MFMA', 1.0), 1.0):9.2f}"))
    for _w, line in sorted(rows, key=lambda r: -r[0]):
        print(line)


if __name__ == "__main__":
    main(sys.argv[1])
