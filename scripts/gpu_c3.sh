cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_conv3x3_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c3_test.log 2>&1; rc=$?; tail -3 gpurun_out/c3_test.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/c3_time.py $C3_ARGS > gpurun_out/c3_time.log 2>&1; rc=$?; cat gpurun_out/c3_time.log; exit $rc
