#!/bin/bash
# EPI dgrad GEMM with the epilogue loads hoisted to the tile start: per-shape timing and bench, at
# occupancy 4 (spills) and 2 (XDDP_GEMM_EPI_OCC=2, no spills).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -4 | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
step t_epi 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gemm_gpu.py -k "epilogue or handoff"
step epi_o4 120 python scripts/pmc_epi.py
step epi_o2 120 env XDDP_GEMM_EPI_OCC=2 python scripts/pmc_epi.py
step b_o4 300 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_o4.json
step b_o2 300 env XDDP_GEMM_EPI_OCC=2 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_o2.json
