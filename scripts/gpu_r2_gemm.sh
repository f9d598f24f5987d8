#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
timeout -k 10 300 python scripts/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1; rc=$?; cat gpurun_out/gemm_bench.log; exit $rc
