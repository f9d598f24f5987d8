#!/bin/bash
# 64x128 tiles for the forward-with-statistics and BN-backward-prologue GEMMs (XDDP_GEMM_BM64): tests + A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -2 | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
step t_bm64 300 env XDDP_GEMM_BM64=fwd,pro python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gemm_gpu.py tests/test_headline_gpu.py
bash scripts/gpu_ab.sh "" "XDDP_GEMM_BM64=fwd" "XDDP_GEMM_BM64=pro" "XDDP_GEMM_BM64=fwd,pro" ""
