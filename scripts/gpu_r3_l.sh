#!/bin/bash
# r3 call L: wide 3x3 convs (N >= 256) on the dense GEMM pipeline: tests, per-shape ceiling on/off,
# ResNet-50 bench interleaved on/off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ge 124 ]; then exit $rc; fi; }
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
step pytest_c3 300 $PYT tests/test_conv3x3_gpu.py
step pytest_conv 400 $PYT tests/test_conv_gemm_gpu.py tests/test_headline_gpu.py tests/test_pending_apply_gpu.py
step ceil_on 300 python -u scripts/conv3x3_ceiling.py --out gpurun_out/r3_conv3x3_ceiling_gemm.txt
step ceil_off 300 env XDDP_C3_GEMM_MIN_N=0 python -u scripts/conv3x3_ceiling.py --out gpurun_out/r3_conv3x3_ceiling_old.txt
cat gpurun_out/r3_conv3x3_ceiling_gemm.txt gpurun_out/r3_conv3x3_ceiling_old.txt
step r50_on1 300 python -u bench.py --json-out gpurun_out/r3l_on1.json
step r50_off1 300 env XDDP_C3_GEMM_MIN_N=0 python -u bench.py --json-out gpurun_out/r3l_off1.json
step r50_on2 300 python -u bench.py --json-out gpurun_out/r3l_on2.json
step r50_off2 300 env XDDP_C3_GEMM_MIN_N=0 python -u bench.py --json-out gpurun_out/r3l_off2.json
