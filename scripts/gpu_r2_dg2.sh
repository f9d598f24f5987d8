#!/bin/bash
# DG2 (stride-2 3x3 input gradient) tile A/B: micro-bench per shape vs MIOpen, then the headline bench per tile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -4 | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi; }
step dg2_bench 300 python scripts/dg2_bench.py
for t in 4 0 1; do step b_t$t 300 env XDDP_DG2_TILE=$t python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_t$t.json; done
step b_epiocc2 300 env XDDP_GEMM_EPI_OCC=2 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_epiocc2.json
step b_bpc3 300 env XDDP_GEMM_BLOCKS_PER_CU=3 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_bpc3.json
