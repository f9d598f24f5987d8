#!/bin/bash
# r3 call X: persistent weights-resident halo kernel for 64->64 (XDDP_C3_HALO64 on/off).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ge 124 ]; then exit $rc; fi; }
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
step pytest_c3 300 $PYT tests/test_conv3x3_gpu.py
step ceil_on 300 python -u scripts/conv3x3_ceiling.py --out gpurun_out/r3_conv3x3_ceiling_halo64.txt
step ceil_off 300 env XDDP_C3_HALO64=0 python -u scripts/conv3x3_ceiling.py --out gpurun_out/r3_conv3x3_ceiling_halo64_off.txt
cat gpurun_out/r3_conv3x3_ceiling_halo64.txt gpurun_out/r3_conv3x3_ceiling_halo64_off.txt
step pytest_conv 400 $PYT tests/test_conv_gemm_gpu.py tests/test_headline_gpu.py tests/test_pending_apply_gpu.py
for r in 1 2; do
step r50_on$r 300 python -u bench.py --json-out gpurun_out/r3x_on$r.json
step r50_off$r 300 env XDDP_C3_HALO64=0 python -u bench.py --json-out gpurun_out/r3x_off$r.json
done
