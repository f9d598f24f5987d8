#!/bin/bash
# Multi-rank GPU paths on a 1-GPU box: 2 ranks on cuda:0 (staged CPU backend) + forced RCCL launches,
# then the headline bench with real RCCL all-reduce kernels on the comm stream.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -15 "gpurun_out/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_multirank 600 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 240 --timeout-method thread
step pytest_multirank2 600 python -u -m pytest tests/test_multirank_gpu.py -x -v --timeout 240 --timeout-method thread -k parity
XDDP_RCCL_FORCE_LAUNCH=1 step bench_forced 600 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/bench_forced.json
