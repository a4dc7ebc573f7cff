cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 300 python tools/diag_physics.py > gpurun_out/diag.log 2>&1; cat gpurun_out/diag.log | grep -v amdgpu.ids
