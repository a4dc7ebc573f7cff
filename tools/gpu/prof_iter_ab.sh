# prof_iter.sh for the S8 update and for the autograd update (LGX_S8_UPDATE=0), side by side
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu/prof_iter.sh && mv $R/gpurun_out/prof_iter $R/gpurun_out/prof_iter_s8 && \
LGX_S8_UPDATE=0 bash $R/tools/gpu/prof_iter.sh && mv $R/gpurun_out/prof_iter $R/gpurun_out/prof_iter_ag
