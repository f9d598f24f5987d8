cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest _bisect/old/tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread -k graphed > gpurun_out/bis_old.log 2>&1; echo "old rc=$?"
timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread -k graphed > gpurun_out/bis_new.log 2>&1; echo "new rc=$?"
timeout -k 10 300 python -u -m pytest _bisect/old/tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread -k graphed > gpurun_out/bis_old2.log 2>&1; echo "old2 rc=$?"
grep -h "AssertionError\|passed\|failed" gpurun_out/bis_*.log
