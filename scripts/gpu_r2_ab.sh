#!/bin/bash
# GPU tests touched this round, ResNet-50 A/B (BN2-backward fold, GEMM occupancy), transformer
# TunableOp tuning + benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_k 600 python -u -m pytest tests/test_conv_gemm_gpu.py tests/test_norm_gpu.py tests/test_conv3x3_gpu.py -x -q --timeout 120 --timeout-method thread
step r50_epi2 300 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/r50_epi2.json
XDDP_CONV_EPI2=0 step r50_noepi2 300 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/r50_noepi2.json
XDDP_GEMM_OCC=2 step r50_occ2 300 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/r50_occ2.json
step r50_epi2b 300 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/r50_epi2b.json
step vit_tune 600 python bench.py --model vit_l_16 --batch-size 64 --steps 3 --warmup 3 --tunableop tune --diag-steps 0
step vit_notune 300 python bench.py --model vit_l_16 --batch-size 64 --steps 10 --warmup 5 --tunableop off --json-out gpurun_out/vit_notune.json
mkdir -p tuning/tunableop && cp gpurun_out/tunableop_vit_l_16.csv tuning/tunableop/
step vit 300 python bench.py --model vit_l_16 --batch-size 64 --steps 10 --warmup 5 --json-out gpurun_out/vit.json
step llama_tune 900 python bench.py --model llama3_8b --batch-size 1 --seq-len 4096 --steps 2 --warmup 2 --tunableop tune --diag-steps 0
cp gpurun_out/tunableop_llama3_8b.csv tuning/tunableop/
step llama 600 python bench.py --model llama3_8b --batch-size 1 --seq-len 4096 --steps 4 --warmup 2 --json-out gpurun_out/llama.json
