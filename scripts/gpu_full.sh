#!/bin/bash
# GPU tests + headline bench + rocprof profile + secondary configs (ViT-L/16, Llama-3-8B).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step pytest_gpu 900 python -m pytest tests -m gpu -q
step b_default 900 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_default.json
if [ "${PROFILE:-1}" = "1" ]; then
  R=$PWD; cd /tmp && export TMPDIR=/tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o prof --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 5 > "$R/gpurun_out/prof.log" 2>&1; echo "prof rc=$?"
  cd "$R"
fi
if [ "${EXTRA:-1}" = "1" ]; then
  step b_vit 900 python bench.py --model vit_l_16 --batch-size 64 --steps 10 --warmup 5 --json-out gpurun_out/b_vit.json
  step b_llama 900 python bench.py --model llama3_8b --batch-size 1 --seq-len 4096 --steps 5 --warmup 3 --json-out gpurun_out/b_llama.json
fi
cat gpurun_out/b_*.json
