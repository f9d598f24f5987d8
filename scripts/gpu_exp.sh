#!/bin/bash
# GPU experiment: full GPU tests, then bench variants (MIOpen find modes), each time-limited.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step pytest_gpu 900 python -m pytest tests -m gpu -q
step b_default 600 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/b_default.json
XDDP_CUDNN_BENCHMARK=1 step b_benchmark 900 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/b_benchmark.json
MIOPEN_FIND_MODE=1 step b_findnormal 900 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/b_findnormal.json
step b_bs512 600 python bench.py --steps 20 --warmup 10 --batch-size 512 --json-out gpurun_out/b_bs512.json
step b_bs128 600 python bench.py --steps 20 --warmup 10 --batch-size 128 --json-out gpurun_out/b_bs128.json
grep -h '"value"' gpurun_out/b_*.json | python3 -c "import sys,json; [print(json.loads(l)['value'], json.loads(l)['ms_per_step'], json.loads(l)['config']['per_gpu_batch']) for l in sys.stdin]"
