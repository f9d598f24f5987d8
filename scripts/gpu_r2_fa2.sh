#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi; }
bash scripts/gpu_r2_fa.sh || exit $?
step loss_curve 400 python scripts/loss_curve.py
