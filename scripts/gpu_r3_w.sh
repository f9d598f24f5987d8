#!/bin/bash
# r3 call W: own global-avg-pool backward + PMC roofline passes of every kernel (incl. r3 ones) + bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ge 124 ]; then exit $rc; fi; }
step pytest_n 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_norm_gpu.py tests/test_headline_gpu.py
step r50_a 300 python -u bench.py --json-out gpurun_out/r3w_a.json
step r50_b 300 python -u bench.py --json-out gpurun_out/r3w_b.json
bash scripts/gpu_r3_pmc2.sh
