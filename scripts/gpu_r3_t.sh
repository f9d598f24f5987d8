#!/bin/bash
# r3 call T: stem pool-BN backward with software-pipelined loads: stem tests, bench x2, trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ge 124 ]; then exit $rc; fi; }
step pytest_s 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_stem_gpu.py
step r50_a 300 python -u bench.py --json-out gpurun_out/r3t_a.json
step r50_b 300 python -u bench.py --json-out gpurun_out/r3t_b.json
cd /tmp && export TMPDIR=/tmp
step prof_r50 300 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/prof_r50t" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 5 --diag-steps 0
python3 "$ROOT/scripts/trace_groups.py" "$ROOT/gpurun_out/prof_r50t/run_kernel_trace.csv" 15 120 > "$ROOT/gpurun_out/r3_resnet50_bs256_kernel_groups_t.txt"
grep -n "total\|stem_pool" "$ROOT/gpurun_out/r3_resnet50_bs256_kernel_groups_t.txt" | cut -c1-150
