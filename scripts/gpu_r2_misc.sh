#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -6 "gpurun_out/$name.log" | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi; }
step epilink 300 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread tests/test_sync_bn_gpu.py tests/test_epilink_gpu.py tests/test_headline_gpu.py
GEMM_SET=resnet step gemm_r50 300 python scripts/gemm_bench.py
