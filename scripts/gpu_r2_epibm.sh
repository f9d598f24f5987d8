#!/bin/bash
# EPI GEMM on 64x128 tiles (XDDP_GEMM_EPI_BM=64): tests, per-shape timing, bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -5 | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
step t_bm 300 env XDDP_GEMM_EPI_BM=64 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gemm_gpu.py tests/test_headline_gpu.py tests/test_epilink_gpu.py
step epi_bm64 120 env XDDP_GEMM_EPI_BM=64 python scripts/pmc_epi.py
step epi_bm128 120 python scripts/pmc_epi.py
bash scripts/gpu_ab.sh "" "XDDP_GEMM_EPI_BM=64" "" "XDDP_GEMM_EPI_BM=64"
