#!/bin/bash
# r3 call K: pending-apply tests (yardstick cosine), 3x3 conv vs explicit-GEMM ceiling.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ge 124 ]; then exit $rc; fi; }
PYT="python -u -m pytest -v --timeout 240 --timeout-method thread"
step pytest_pend 300 $PYT -s tests/test_pending_apply_gpu.py
step ceiling 300 python -u scripts/conv3x3_ceiling.py --out gpurun_out/r3_conv3x3_ceiling.txt
cat gpurun_out/r3_conv3x3_ceiling.txt
