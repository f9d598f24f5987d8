#!/bin/bash
# full GPU tests + default bench + kernel profile (no risky probes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1 XDDP_NATIVE_BACKTRACE=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E "passed|failed|value|^FAILED|^ERROR" "gpurun_out/$name.log" | cut -c1-240 | tail -8; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step pytest_gpu 900 python -m pytest tests -m gpu -q
step b_default 900 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_default.json
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o prof --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 5 > "$R/gpurun_out/prof.log" 2>&1; echo "prof rc=$?"
