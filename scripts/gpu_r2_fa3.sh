#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -4 | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi; }
step fa_test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_flash_attn_gpu.py
step fa_bench 300 python scripts/attn_bench.py
XDDP_FA_DKDV_KW=4 step fa_bench_kw4 300 python scripts/attn_bench.py
step loss_curve 400 python scripts/loss_curve.py
