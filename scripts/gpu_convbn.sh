#!/bin/bash
# Fused 1x1-conv + BN: kernel tests, model tests, then the headline bench with the fusion on/off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -12 "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_convgemm 400 python -u -m pytest tests/test_conv_gemm_gpu.py tests/test_ddp_gpu.py -x -v --timeout 120 --timeout-method thread
step bench_fused 400 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/bench_fused.json
XDDP_CONV_BN_FUSION=0 step bench_unfused 400 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/bench_unfused.json
