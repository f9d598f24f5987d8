#!/bin/bash
# LN param-grad fix + patch-embed GEMM: norm tests, TunableOp GEMM tuning for the transformer
# configs, then benches with the tuned solutions.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_norm 300 python -u -m pytest tests/test_norm_gpu.py -x -q --timeout 120 --timeout-method thread
step vit_notune 300 python bench.py --model vit_l_16 --batch-size 64 --steps 10 --warmup 5 --tunableop off --json-out gpurun_out/vit_notune.json
step vit_tune 600 python bench.py --model vit_l_16 --batch-size 64 --steps 3 --warmup 3 --tunableop tune --diag-steps 0
step llama_tune 900 python bench.py --model llama3_8b --batch-size 1 --seq-len 4096 --steps 2 --warmup 2 --tunableop tune --diag-steps 0
mkdir -p tuning/tunableop && cp gpurun_out/tunableop_*.csv tuning/tunableop/
step vit 300 python bench.py --model vit_l_16 --batch-size 64 --steps 10 --warmup 5 --json-out gpurun_out/vit.json
step llama 600 python bench.py --model llama3_8b --batch-size 1 --seq-len 4096 --steps 4 --warmup 2 --json-out gpurun_out/llama.json
