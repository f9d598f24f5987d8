#!/bin/bash
# r3 call KK: LN backward defaults (residual prefetch, 2 blocks per CU): tests, timing, ViT / Llama benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_ln 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_norm_gpu.py tests/test_encoder_block_gpu.py tests/test_transformer_gpu.py
step ln 120 python -u scripts/ln_bwd_time.py
step vit1 400 python -u bench.py --model vit_l_16 --steps 10 --warmup 3 --json-out gpurun_out/r3kk_vit1.json
step vit2 400 python -u bench.py --model vit_l_16 --steps 10 --warmup 3 --json-out gpurun_out/r3kk_vit2.json
step llama 400 python -u bench.py --model llama3_8b --steps 10 --warmup 3 --json-out gpurun_out/r3kk_llama.json
