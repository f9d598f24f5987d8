#!/bin/bash
# Transformer configs (BASELINE.json 4-5): benches (own flash attention vs SDPA) + rocprofv3 kernel traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
step vit 300 python bench.py --model vit_l_16 --batch-size 64 --steps 10 --warmup 5 --json-out gpurun_out/vit.json
XDDP_FLASH_ATTN=0 step vit_sdpa 300 python bench.py --model vit_l_16 --batch-size 64 --steps 10 --warmup 5 --diag-steps 0
step llama 600 python bench.py --model llama3_8b --batch-size 1 --seq-len 4096 --steps 4 --warmup 2 --json-out gpurun_out/llama.json
XDDP_FLASH_ATTN=0 step llama_sdpa 600 python bench.py --model llama3_8b --batch-size 1 --seq-len 4096 --steps 4 --warmup 2 --diag-steps 0
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_vit" -o prof --output-format csv -- python3 "$R/bench.py" --model vit_l_16 --batch-size 64 --steps 3 --warmup 2 --diag-steps 0 > "$R/gpurun_out/prof_vit.log" 2>&1; echo "prof vit rc=$?"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_llama" -o prof --output-format csv -- python3 "$R/bench.py" --model llama3_8b --batch-size 1 --seq-len 4096 --steps 2 --warmup 1 --diag-steps 0 > "$R/gpurun_out/prof_llama.log" 2>&1; echo "prof llama rc=$?"
