#!/bin/bash
# conv1x1 GEMM tests (incl. the BN-reduce epilogue hand-off) + A/B bench of XDDP_CONV_EPI.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest tests/test_conv_gemm_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/epi_tests.log 2>&1 || { tail -40 gpurun_out/epi_tests.log; exit 1; }
tail -3 gpurun_out/epi_tests.log
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/epi_on.log 2>&1 || { tail -20 gpurun_out/epi_on.log; exit 1; }
tail -1 gpurun_out/epi_on.log
XDDP_CONV_EPI=0 timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/epi_off.log 2>&1 || { tail -20 gpurun_out/epi_off.log; exit 1; }
tail -1 gpurun_out/epi_off.log
