#!/bin/bash
# r3 call JJ: LayerNorm backward with the residual gradient prefetched with the next row: tests,
# standalone A/B, ViT bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_ln 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_norm_gpu.py tests/test_encoder_block_gpu.py tests/test_transformer_gpu.py
step ln1 120 python -u scripts/ln_bwd_time.py
XDDP_LN_RESPF=0 step ln0 120 python -u scripts/ln_bwd_time.py
step ln1b 120 python -u scripts/ln_bwd_time.py
XDDP_LN_BWD_GRID=512 step ln1_g512 120 python -u scripts/ln_bwd_time.py
XDDP_LN_RESPF=0 XDDP_LN_BWD_GRID=512 step ln0_g512 120 python -u scripts/ln_bwd_time.py
step v_on1 400 python -u bench.py --model vit_l_16 --steps 10 --warmup 3 --json-out gpurun_out/r3jj_on1.json
XDDP_LN_RESPF=0 step v_off1 400 python -u bench.py --model vit_l_16 --steps 10 --warmup 3 --json-out gpurun_out/r3jj_off1.json
step v_on2 400 python -u bench.py --model vit_l_16 --steps 10 --warmup 3 --json-out gpurun_out/r3jj_on2.json
XDDP_LN_RESPF=0 step v_off2 400 python -u bench.py --model vit_l_16 --steps 10 --warmup 3 --json-out gpurun_out/r3jj_off2.json
