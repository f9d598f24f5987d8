#!/bin/bash
# Generate MIOpen tuning (find-db, perf-db, kernel cache) for the headline config with an
# exhaustive search, then verify that a fresh process given copies of them skips the search.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=gpurun_out/tuning/miopen
rm -rf $T; mkdir -p $T/db $T/cache
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -E "warmup step 1/|value" "gpurun_out/$name.log" | cut -c1-200; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
MIOPEN_USER_DB_PATH=$PWD/$T/db MIOPEN_CUSTOM_CACHE_DIR=$PWD/$T/cache XDDP_CUDNN_BENCHMARK=1 \
  step tune 900 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/b_tune.json
find $T -type f | xargs ls -la; du -sh $T
mkdir -p tuning && rm -rf tuning/miopen && cp -r $T tuning/miopen
step fresh 900 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/b_fresh.json
step fresh2 900 python bench.py --steps 20 --warmup 5 --json-out gpurun_out/b_fresh2.json
