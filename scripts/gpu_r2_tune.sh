#!/bin/bash
# Transformer configs: TunableOp GEMM tuning (results under gpurun_out, copied into tuning/ by
# hand), ViT profile, 3x3 wgrad split sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi; }
step wgrad3 300 python scripts/wgrad3_bench.py
step vit_tune 600 python bench.py --model vit_l_16 --batch-size 64 --steps 2 --warmup 2 --tunableop tune --diag-steps 0
mkdir -p tuning/tunableop && cp gpurun_out/tunableop_vit_l_16.csv tuning/tunableop/
step vit 300 python bench.py --model vit_l_16 --batch-size 64 --steps 10 --warmup 5 --json-out gpurun_out/vit.json
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_vit" -o prof --output-format csv -- python3 "$R/bench.py" --model vit_l_16 --batch-size 64 --steps 5 --warmup 3 --diag-steps 0 > "$R/gpurun_out/prof_vit.log" 2>&1; echo "prof vit rc=$?"
cd "$R"
step llama_tune 900 python bench.py --model llama3_8b --batch-size 1 --seq-len 4096 --steps 1 --warmup 1 --tunableop tune --diag-steps 0
cp gpurun_out/tunableop_llama3_8b.csv tuning/tunableop/
step llama 600 python bench.py --model llama3_8b --batch-size 1 --seq-len 4096 --steps 4 --warmup 2 --json-out gpurun_out/llama.json
