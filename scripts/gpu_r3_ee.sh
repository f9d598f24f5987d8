#!/bin/bash
# r3 call EE/FF: whole-K/V flash attention forward and whole-item dK/dV backward for short non-causal heads: tests, standalone A/B, ViT bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_fa 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_flash_attn_gpu.py
step fa1 120 python -u scripts/fa_vit_time.py
XDDP_FA_WHOLE=0 step fa0 120 python -u scripts/fa_vit_time.py
step fa1b 120 python -u scripts/fa_vit_time.py
step v_on1 400 python -u bench.py --model vit_l_16 --steps 10 --warmup 3 --json-out gpurun_out/r3ff_on1.json
XDDP_FA_WHOLE=0 step v_off1 400 python -u bench.py --model vit_l_16 --steps 10 --warmup 3 --json-out gpurun_out/r3ff_off1.json
step v_on2 400 python -u bench.py --model vit_l_16 --steps 10 --warmup 3 --json-out gpurun_out/r3ff_on2.json
XDDP_FA_WHOLE=0 step v_off2 400 python -u bench.py --model vit_l_16 --steps 10 --warmup 3 --json-out gpurun_out/r3ff_off2.json
