#!/bin/bash
# r3 call LL: final HEAD validation — full GPU suite, smoke, ResNet-50 bench x2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ge 124 ]; then exit $rc; fi; }
step pytest_all 900 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step r50_a 300 python -u bench.py --json-out gpurun_out/r3ll_r50_a.json
step r50_b 300 python -u bench.py --json-out gpurun_out/r3ll_r50_b.json
