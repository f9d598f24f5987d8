#!/bin/bash
# Short GPU call: parity probe + norm tests + one bench (fused BN) + profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -8 "gpurun_out/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step parity 300 python scripts/debug_parity.py
DET=1 step parity_det 300 python scripts/debug_parity.py
step pytest_norm 600 python -m pytest tests/test_norm_gpu.py tests/test_kernels_gpu.py -x -q
step bench_xddp 600 python bench.py --norm xddp --steps 20 --warmup 10 --json-out gpurun_out/bench_xddp.json
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o prof --output-format csv -- python3 "$R/bench.py" --norm xddp --steps 5 --warmup 5 > "$R/gpurun_out/prof.log" 2>&1; echo "prof rc=$?"
