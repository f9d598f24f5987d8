#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
GEMM_SET=resnet timeout -k 10 300 python scripts/gemm_bench.py > gpurun_out/gemm_bench_r50.log 2>&1; rc=$?; cat gpurun_out/gemm_bench_r50.log; exit $rc
