#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -1 | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
step vit 300 python bench.py --model vit_l_16 --batch-size 64 --steps 10 --warmup 5 --json-out gpurun_out/vit.json
step llama 600 python bench.py --model llama3_8b --batch-size 1 --seq-len 4096 --steps 4 --warmup 2 --json-out gpurun_out/llama.json
