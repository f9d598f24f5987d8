#!/bin/bash
# ViT-L/16 bs256: bias_grad+GELU-backward thread count A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value": [0-9.]*' "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then tail -3 "gpurun_out/$name.log"; exit $rc; fi; }
step t_tx 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_transformer_gpu.py tests/test_encoder_block_gpu.py
step v512k 400 python bench.py --model vit_l_16 --steps 10 --warmup 4 --diag-steps 0
step v128k 400 env XDDP_BIAS_GRAD_THREADS=131072 python bench.py --model vit_l_16 --steps 10 --warmup 4 --diag-steps 0
step v1m 400 env XDDP_BIAS_GRAD_THREADS=1048576 python bench.py --model vit_l_16 --steps 10 --warmup 4 --diag-steps 0
