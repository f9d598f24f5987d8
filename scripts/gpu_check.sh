#!/bin/bash
# GPU sanity call: full GPU test suite, smoke(), headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -6 "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/bench.json
