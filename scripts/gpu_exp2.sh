#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step pytest_gpu 900 python -m pytest tests -m gpu -q
step b_find1 900 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_find1.json
MIOPEN_FIND_MODE=5 step b_find5 900 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_find5.json
MIOPEN_FIND_MODE=5 XDDP_CUDNN_BENCHMARK=1 step b_bench 900 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_bench.json
step b_find1_again 900 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_find1_again.json
R=$PWD; cd /tmp && export TMPDIR=/tmp
MIOPEN_FIND_MODE=5 timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o prof --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 5 > "$R/gpurun_out/prof.log" 2>&1; echo "prof rc=$?"
cd "$R"
for f in gpurun_out/b_*.json; do echo "$f $(python3 -c "import json;d=json.load(open('$f'));print(d['value'], d['ms_per_step'])")"; done
