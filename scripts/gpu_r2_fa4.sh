#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -4 | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi; }
step fa_test 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_flash_attn_gpu.py
step fa_bench 300 python scripts/attn_bench.py
XDDP_FA_DKDV_SPLIT=1 step fa_bench_nosplit 300 python scripts/attn_bench.py
step llama 600 python bench.py --model llama3_8b --batch-size 1 --seq-len 4096 --steps 4 --warmup 2 --json-out gpurun_out/llama.json
