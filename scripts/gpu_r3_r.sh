#!/bin/bash
# r3 call R: plain 1x1 forwards (downsamples) on the LDS-DMA GEMM: test + bench arms interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ge 124 ]; then exit $rc; fi; }
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
step pytest_c 300 $PYT tests/test_conv_gemm_gpu.py -k "gemm_nt or conv1x1_gemm_matches"
step pytest_h 300 env XDDP_C1_NT=1 $PYT tests/test_headline_gpu.py
for r in 1 2; do
step base$r 300 python -u bench.py --json-out gpurun_out/r3r_base$r.json
step s2_$r 300 env XDDP_C1_NT=s2 python -u bench.py --json-out gpurun_out/r3r_s2_$r.json
step all$r 300 env XDDP_C1_NT=1 python -u bench.py --json-out gpurun_out/r3r_all$r.json
done
