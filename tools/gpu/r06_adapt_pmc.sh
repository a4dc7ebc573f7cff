# round 6: PMC of the two adaptation-forward kernels (tools/adapt_fwd_timing.py; separate --pmc passes)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${TAG:-r06_adapt_pmc}; rm -rf $O; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
K=$R/legged_gym_custom_amd/lib/dev/liblgx_mlp_knobs.so
i=0
for c in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for v in 1 0; do
    LGX_MLP_LIB=$K LGX_ADAPT_FWD2=$v timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $O/p${i}_$v -- python3 $R/tools/adapt_fwd_timing.py > $O/p${i}_$v.log 2>&1 || { echo "pass $i $v failed"; tail -5 $O/p${i}_$v.log; exit 1; }
  done
done
cd $R && python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
for v in ("1", "0"):
    acc = collections.defaultdict(list)
    for f in glob.glob(f"{O}/p*_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "adapt_fwd" not in r["Kernel_Name"] or int(r.get("Grid_Size", 0) or 0) < 256 * 1000:
                continue
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("fwd2" if v == "1" else "old ", {k: round(sum(x) / len(x)) for k, x in sorted(acc.items())})
PY
