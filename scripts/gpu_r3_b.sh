#!/bin/bash
# r3 call B: GEMM pipelines (test + bench), peer-backend DDP (tests + 2-rank bench diagnosis with a
# short peer timeout and flight dumps), config-3, PMC roofline passes, forced-RCCL kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -6 "$ROOT/gpurun_out/$name.log"; if [ $rc -ge 124 ]; then exit $rc; fi; }
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
step pytest_gemm 300 $PYT tests/test_gemm_gpu.py
step gemm_bench 400 python -u scripts/gemm_nt_bench.py --out gpurun_out/r3_gemm_nt_vs_hipblaslt.txt
step pytest_multirank 500 $PYT tests/test_multirank_gpu.py
export XDDP_PEER_TIMEOUT_MS=30000 XDDP_FLIGHT_DUMP_PREFIX=$ROOT/gpurun_out/flight_peer2_rank_
XDDP_PEER_TWO_SHOT_MIN_BYTES=1000000000000 step bench_peer2_oneshot 150 python -u bench.py --gpus 2 --backend peer --steps 5 --warmup 3 --diag-steps 1 --json-out gpurun_out/r3_bench_peer2_oneshot.json
step bench_peer2 150 python -u bench.py --gpus 2 --backend peer --steps 5 --warmup 3 --diag-steps 1 --json-out gpurun_out/r3_bench_peer2.json
unset XDDP_PEER_TIMEOUT_MS XDDP_FLIGHT_DUMP_PREFIX
step pytest_cfg3 400 $PYT tests/test_headline_gpu.py -k config3 -s
bash scripts/gpu_r3_pmc.sh
cd /tmp && export TMPDIR=/tmp
XDDP_RCCL_FORCE_LAUNCH=1 step prof_forced 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_forced" -o run --output-format csv -- python "$ROOT/bench.py" --steps 5 --warmup 3 --diag-steps 3
