#!/bin/bash
# Deep-K 1x1 forward on hipBLASLt + stats pass (XDDP_C1_BLAS_MIN_K) vs the fused-stats GEMM.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -3 | cut -c1-200; grep -o '"value": [0-9.]*' "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step t_head 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_headline_gpu.py tests/test_conv_gemm_gpu.py -k "resnet or bottleneck or handoff or headline"
step c_1024 300 python bench.py --steps 30 --warmup 10
step c_off 300 env XDDP_C1_BLAS_MIN_K=0 python bench.py --steps 30 --warmup 10
step c_512 300 env XDDP_C1_BLAS_MIN_K=512 python bench.py --steps 30 --warmup 10
step c_1024b 300 python bench.py --steps 30 --warmup 10
