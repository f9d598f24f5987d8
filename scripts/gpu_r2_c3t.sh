#!/bin/bash
# 3x3 tile choice for the 64-channel (ResNet-50 layer1) convs: XDDP_C3_TILE64 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value": [0-9.]*' "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then tail -3 "gpurun_out/$name.log"; exit $rc; fi; }
step t4 300 python bench.py --steps 30 --warmup 10
for t in 2 3 5; do step t$t 300 env XDDP_C3_TILE64=$t python bench.py --steps 30 --warmup 10; done
step t4b 300 python bench.py --steps 30 --warmup 10
