set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tail_prof; rm -rf $O; mkdir -p $O
cd $R && timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_s8.py -k "tail or heads" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log; cd /tmp
for v in 1 0; do
LGX_HEADS_TAIL=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$v -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no_cpu_baseline > $O/b$v.log 2>&1 || { tail -5 $O/b$v.log; exit 1; }
f=$(find $O/t$v -name "*kernel_stats.csv" | head -1)
echo "== LGX_HEADS_TAIL=$v $(tail -1 $O/b$v.log | cut -c1-60)"
python3 - "$f" <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if any(k in r["Name"] for k in ("loss_heads", "s8_gemm", "s8_reduce")): print(r["Name"][:44], r["Calls"], r["AverageNs"], r["TotalDurationNs"])
PY
done
