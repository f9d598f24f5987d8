#!/bin/bash
# r3 call P2: the own deep-K statistics GEMM arm of call P (fixed binding), interleaved with base.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ge 124 ]; then exit $rc; fi; }
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
step pytest_g 300 $PYT tests/test_gemm_gpu.py
step pytest_h 300 env XDDP_DEEP_K_OWN=1 $PYT tests/test_headline_gpu.py
for r in 1 2; do
step base$r 300 python -u bench.py --json-out gpurun_out/r3p_base$r.json
step own$r 300 env XDDP_DEEP_K_OWN=1 python -u bench.py --json-out gpurun_out/r3p_own$r.json
done
