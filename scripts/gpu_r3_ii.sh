#!/bin/bash
# r3 call II: split MFMA chains in the flash dK/dV backward: tests, standalone timing, ViT bench x2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_fa 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_flash_attn_gpu.py tests/test_transformer_gpu.py
step fa_a 120 python -u scripts/fa_vit_time.py
step fa_b 120 python -u scripts/fa_vit_time.py
step v1 400 python -u bench.py --model vit_l_16 --steps 10 --warmup 3 --json-out gpurun_out/r3ii_v1.json
step v2 400 python -u bench.py --model vit_l_16 --steps 10 --warmup 3 --json-out gpurun_out/r3ii_v2.json
