# isolate the round-4 S8 run's failures: the legacy learner tests alone, then the c2 golden moments (dev)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/dbg_learner.log 2>&1
rc=$?
grep -v "^  File\|^frame" gpurun_out/dbg_learner.log | tail -60
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner_golden.py -x -v --timeout 250 --timeout-method thread -p no:cacheprovider -k "go2_c2" > gpurun_out/dbg_c2.log 2>&1
rc=$?
grep -v "^  File\|^frame" gpurun_out/dbg_c2.log | tail -40
exit $rc
