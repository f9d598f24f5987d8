#!/bin/bash
# Flash attention: numerics tests, xddp-vs-SDPA timing, per-kernel profile of the attention bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi; }
step fa_test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_flash_attn_gpu.py
step fa_bench 300 python scripts/attn_bench.py
XDDP_FA_WAVES=4 step fa_bench4 300 python scripts/attn_bench.py
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_fa" -o prof --output-format csv -- python3 "$R/scripts/attn_bench.py" > "$R/gpurun_out/prof_fa.log" 2>&1; echo "prof fa rc=$?"
