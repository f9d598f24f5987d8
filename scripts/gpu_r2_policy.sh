#!/bin/bash
# xGMI bucket policy + grouped launches: GPU tests, headline bench, forced-RCCL A/B (reference vs
# xgmi policy), kernel trace of the forced-RCCL step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench 300 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/bench.json
XDDP_RCCL_FORCE_LAUNCH=1 step forced_xgmi 300 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/forced_xgmi.json
XDDP_RCCL_FORCE_LAUNCH=1 step forced_ref 300 python bench.py --steps 20 --warmup 10 --bucket-policy reference --json-out gpurun_out/forced_ref.json
step bench2 300 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/bench2.json
R=$PWD; cd /tmp && export TMPDIR=/tmp
export XDDP_RCCL_FORCE_LAUNCH=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_forced" -o prof --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 5 > "$R/gpurun_out/prof_forced.log" 2>&1; echo "prof rc=$?"
