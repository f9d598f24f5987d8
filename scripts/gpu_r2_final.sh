#!/bin/bash
# Final validation: GPU suite, smoke, headline bench, 2 ranks on one GPU over the peer backend.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -2 | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/bench.json
step bench_peer2 600 python bench.py --gpus 2 --backend peer --steps 10 --warmup 5 --json-out gpurun_out/bench_peer2.json
