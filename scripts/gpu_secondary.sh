#!/bin/bash
# Secondary configs (ViT-L/16, Llama-3-8B fused vs reference ops, reference SimpleCNN eager/graphs),
# rocprofv3 kernel stats of the headline config, and the PMC counter list.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
step b_vit 400 python bench.py --model vit_l_16 --batch-size 64 --steps 10 --warmup 5 --json-out gpurun_out/b_vit.json
step b_llama 500 python bench.py --model llama3_8b --batch-size 1 --seq-len 4096 --steps 5 --warmup 3 --json-out gpurun_out/b_llama.json
XDDP_FUSED_TRANSFORMER=0 step b_llama_ref 500 python bench.py --model llama3_8b --batch-size 1 --seq-len 4096 --steps 5 --warmup 3 --json-out gpurun_out/b_llama_ref.json
step b_cnn 300 python bench.py --model simplecnn --batch-size 32 --image-size 32 --steps 200 --warmup 20 --json-out gpurun_out/b_cnn.json
step b_cnn_graph 300 python bench.py --model simplecnn --batch-size 32 --image-size 32 --steps 200 --warmup 20 --graphs 1 --json-out gpurun_out/b_cnn_graph.json
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/pmc_list.txt" 2>&1; echo "list rc=$?"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o prof --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 5 > "$R/gpurun_out/prof.log" 2>&1; echo "prof rc=$?"
