#!/bin/bash
# Round-2 baseline call: GPU tests, headline bench, forced-RCCL bench (real RCCL kernels at W=1),
# config-3 (no_sync accumulation) benches, and a kernel trace of the forced-RCCL step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step bench 300 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/bench.json
XDDP_RCCL_FORCE_LAUNCH=1 step bench_forced 300 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/bench_forced.json
step bench_nosync2 300 python bench.py --steps 20 --warmup 10 --no-sync-accum 2 --json-out gpurun_out/bench_nosync2.json
step bench_nosync4 300 python bench.py --steps 20 --warmup 10 --no-sync-accum 4 --json-out gpurun_out/bench_nosync4.json
R=$PWD; cd /tmp && export TMPDIR=/tmp
export XDDP_RCCL_FORCE_LAUNCH=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_forced" -o prof --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 5 > "$R/gpurun_out/prof_forced.log" 2>&1; echo "prof rc=$?"
