#!/bin/bash
# graph-capture probe (DDP cases) then the graphed DDP test and graphed benches.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1 XDDP_NATIVE_BACKTRACE=1
PROBE_CASES="ddp_linear our_bn llama simplecnn" bash scripts/gpu_graph_probe.sh || exit $?
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E "passed|failed|Error|value" "gpurun_out/$name.log" | cut -c1-220 | tail -4; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step pytest_graph 600 python -m pytest tests/test_ddp_gpu.py -q -k "graphed"
REF="--model simplecnn --image-size 32 --batch-size 32 --steps 200 --warmup 20"
step ref_xddp_eager 600 python bench.py $REF --json-out gpurun_out/ref_xddp_eager.json
step ref_xddp_graphs 600 python bench.py $REF --graphs 1 --json-out gpurun_out/ref_xddp_graphs.json
step r50_graphs 900 python bench.py --steps 30 --warmup 10 --graphs 1 --json-out gpurun_out/r50_graphs.json
for f in gpurun_out/*.json; do echo "$f $(python3 -c "import json;d=json.load(open('$f'));print(d['value'], d['ms_per_step'])")"; done
