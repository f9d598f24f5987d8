#!/bin/bash
# Downsample BN apply folded into the final apply pass: tests + A/B bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value": [0-9.]*' "gpurun_out/$name.log"; grep -v amdgpu "gpurun_out/$name.log" | tail -2 | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
step t_def 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gemm_gpu.py tests/test_headline_gpu.py tests/test_epilink_gpu.py tests/test_norm_gpu.py
step t_def2 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_conv_gemm_gpu.py -k "deferred or downsample or handoff"
step d_on 300 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/d_on.json
step d_off 300 env XDDP_DS_DEFER=0 python bench.py --steps 30 --warmup 10
step d_on2 300 python bench.py --steps 30 --warmup 10
