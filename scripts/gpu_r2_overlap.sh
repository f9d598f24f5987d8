#!/bin/bash
# Overlapped optimizer (per-bucket AdamW on a side stream during backward): GPU test + Llama/ViT A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value": [0-9.]*' "gpurun_out/$name.log"; grep -v amdgpu "gpurun_out/$name.log" | tail -2 | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
step t_ov 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ddp_gpu.py
step llama_ov 500 python bench.py --model llama3_8b --batch-size 1 --steps 8 --warmup 3 --diag-steps 0 --json-out gpurun_out/llama_ov.json
step llama_base 500 python bench.py --model llama3_8b --batch-size 1 --steps 8 --warmup 3 --diag-steps 0 --overlap-optim 0
step vit_ov 400 python bench.py --model vit_l_16 --steps 10 --warmup 4 --diag-steps 0 --json-out gpurun_out/vit_ov.json
step vit_base 400 python bench.py --model vit_l_16 --steps 10 --warmup 4 --diag-steps 0 --overlap-optim 0
