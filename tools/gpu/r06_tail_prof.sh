# round 6: kernel times of the optimizer tail with / without the S8 copies (LGX_TAIL_S8), one box.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r06_tailp}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in 1 0; do
  LGX_TAIL_S8=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$v -o run -- python3 $R/bench.py --no_cpu_baseline --steps 3 --warmup 1 > $O/b$v.json 2> $O/b$v.err || { tail -5 $O/b$v.err; exit 1; }
  f=$(find $O/p$v -name "*kernel_stats.csv" | head -1)
  python3 - $f $v <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if any(k in n for k in ('tail_','s8_split','s8f_kernel','s8_gemm_kernel<2>')):
        print(sys.argv[2], f"{int(r['Calls']):6d} x {float(r['AverageNs'])/1e3:8.1f} us  {n[:70]}")
PY
done
