#!/bin/bash
# Flash-attention tests + ViT-L/16 bench: one-block dK/dV (KW = 8) vs two 128-key blocks.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value": [0-9.]*' "gpurun_out/$name.log"; grep -v amdgpu "gpurun_out/$name.log" | tail -2 | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
step t_fa 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_flash_attn_gpu.py tests/test_encoder_block_gpu.py
step attn 200 python scripts/attn_bench.py
step v_kw8 400 python bench.py --model vit_l_16 --steps 10 --warmup 4 --diag-steps 0 --json-out gpurun_out/v_kw8.json
step v_kw4 400 env XDDP_FA_DKDV_KW=4 python bench.py --model vit_l_16 --steps 10 --warmup 4 --diag-steps 0
