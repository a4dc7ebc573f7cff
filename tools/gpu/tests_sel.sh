# GPU box: a selection of -m gpu tests (TESTS="file::test ..."), verbose, per-test timeout, -s.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 ${TMO:-600} python -u -m pytest ${TESTS} -m gpu -v -s -p no:cacheprovider -rf --timeout ${PT:-300} --timeout-method thread > gpurun_out/pytest_sel.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -${TAILN:-40} gpurun_out/pytest_sel.log
exit $rc
