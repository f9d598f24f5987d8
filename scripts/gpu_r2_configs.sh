#!/bin/bash
# BASELINE.json configs 2 and 3 on one MI355X (configs 4/5: gpu_r2_transformers.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
step cfg2 300 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/cfg2.json
step cfg3_m2 300 python bench.py --steps 20 --warmup 5 --batch-size 128 --no-sync-accum 2 --json-out gpurun_out/cfg3_m2.json
step cfg3_m4 300 python bench.py --steps 20 --warmup 5 --batch-size 64 --no-sync-accum 4 --json-out gpurun_out/cfg3_m4.json
step cfg3_m2_256 300 python bench.py --steps 15 --warmup 5 --batch-size 256 --no-sync-accum 2 --json-out gpurun_out/cfg3_m2_256.json
