# DW group alone: kernel stats and FETCH_SIZE with the XCD-unit deal on / off
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dw_probe
rm -rf $O && mkdir -p $O
for v in 1 0; do
  LGX_S8_DW_XCD=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$v -o run -- python3 $R/tools/dw_probe.py > $O/t$v.log 2>&1 || { tail -5 $O/t$v.log; exit 1; }
  LGX_S8_DW_XCD=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --output-format csv -d $O/p$v -o run -- python3 $R/tools/dw_probe.py > $O/p$v.log 2>&1 || { tail -5 $O/p$v.log; exit 1; }
  echo "== XCD units $v"; grep achieved $O/t$v.log | cut -c1-300
  grep -h "s8_gemm\|s8_reduce" $(find $O/t$v -name "*kernel_stats.csv") | cut -d, -f1-8
  python3 - $O/p$v <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "s8_gemm" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(k, "mean", sum(v) / len(v), "n", len(v))
PY
done
