#!/bin/bash
# Headline bench under GEMM knob variants (A/B on one box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value": [0-9.]*' "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step k_base 300 python bench.py --steps 30 --warmup 10
step k_occ2 300 env XDDP_GEMM_OCC=2 python bench.py --steps 30 --warmup 10
step k_base2 300 python bench.py --steps 30 --warmup 10
