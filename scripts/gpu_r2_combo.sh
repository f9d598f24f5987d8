#!/bin/bash
# FA (tests, bench, profile) + stem (tests, fused-wgrad A/B bench, profile) + bench-config loss curves.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi; }
step fa_test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_flash_attn_gpu.py
step stem_test 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_stem_gpu.py
step fa_bench 300 python scripts/attn_bench.py
step r50 300 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/r50.json
XDDP_STEM_WGRAD_FUSED=0 step r50_unfused 300 python bench.py --steps 30 --warmup 10 --diag-steps 0
step loss_curve 400 python scripts/loss_curve.py
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_fa" -o prof --output-format csv -- python3 "$R/scripts/attn_bench.py" > "$R/gpurun_out/prof_fa.log" 2>&1; echo "prof fa rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r50" -o prof --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 5 --diag-steps 0 > "$R/gpurun_out/prof_r50.log" 2>&1; echo "prof r50 rc=$?"
