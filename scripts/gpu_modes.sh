#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E "warmup step 1/|value" "gpurun_out/$name.log" | cut -c1-160; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
for m in 5 3 2 1; do MIOPEN_FIND_MODE=$m step mode$m 900 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/b_mode$m.json; done
