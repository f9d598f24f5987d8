#!/bin/bash
# BN2 backward reduce folded into conv3's input-gradient epilogue (XDDP_CONV_EPI2) A/B, now that the
# EPI variants run at occupancy 2 without spills.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value": [0-9.]*' "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then tail -3 "gpurun_out/$name.log"; exit $rc; fi; }
step e2_test 300 env XDDP_CONV_EPI2=1 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gemm_gpu.py -k "epilogue or handoff or resnet"
step e0 300 python bench.py --steps 30 --warmup 10
step e2 300 env XDDP_CONV_EPI2=1 python bench.py --steps 30 --warmup 10
step e0b 300 python bench.py --steps 30 --warmup 10
step e2b 300 env XDDP_CONV_EPI2=1 python bench.py --steps 30 --warmup 10
