# go2_parkour (C4, 8192 envs) bench line with one and two envs per wavefront (A/B, one box)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/c4_epw; mkdir -p $O
cd $R
for e in 1 2 1 2; do
  LGX_ENVS_PER_WAVE=$e timeout -k 10 400 python bench.py --task go2_parkour --num_envs 8192 --no_cpu_baseline > $O/epw$e.log 2>&1 || exit $?
  python -c "import json; b=json.loads(open('$O/epw$e.log').read().strip().splitlines()[-1]); print('epw=$e', b['value'], b['env_kernel'])"
done
