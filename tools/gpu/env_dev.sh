# Env-kernel dev loop on the GPU box: physics/post-physics parity tests, then the
# per-phase cycle profile (tools/phase_clock.py, liblgx_prof.so) at 4096 envs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_terrain.py} > gpurun_out/env_tests.log 2>&1
rc=$?; tail -15 gpurun_out/env_tests.log; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/phase_clock.py > gpurun_out/phase.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/phase.log | tail -19; exit $rc
