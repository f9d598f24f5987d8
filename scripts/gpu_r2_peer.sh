#!/bin/bash
# Peer-memory one-shot all-reduce (2 processes on cuda:0), then the headline bench (DG2 default off).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1 XDDP_PEER_TIMEOUT_MS=5000
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -8 | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi; }
step t_peer 240 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_peer_allreduce_gpu.py
step b_default 300 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_default.json
step b_dg2on 300 env XDDP_CONV3X3_DGRAD_S2=1 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_dg2on.json
