#!/bin/bash
# r3 call A: own transformer GEMM (test + vs hipBLASLt), comm/peer checks, config-3, smoke, bench
# (plain / forced RCCL / 2-rank peer backend), forced-RCCL kernel trace, PMC roofline passes.
# A step that fails with an ordinary test failure (rc 1/2) does not stop the script; a timeout,
# abort or crash (rc >= 124) does.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
FAILED=0
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -6 "$ROOT/gpurun_out/$name.log"; if [ $rc -ge 124 ]; then exit $rc; fi; if [ $rc -ne 0 ]; then FAILED=1; fi; }
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
step pytest_gemm 300 $PYT tests/test_gemm_gpu.py
step gemm_bench 400 python scripts/gemm_nt_bench.py --out gpurun_out/r3_gemm_nt_vs_hipblaslt.txt
step pytest_peer 600 $PYT tests/test_peer_allreduce_gpu.py
step pytest_syncbn 400 $PYT tests/test_sync_bn_gpu.py
step pytest_cfg3 400 $PYT tests/test_headline_gpu.py -k config3 -s
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/r3_bench.json
XDDP_RCCL_FORCE_LAUNCH=1 step bench_forced 600 python bench.py --steps 10 --warmup 5 --json-out gpurun_out/r3_bench_forced.json
step bench_peer2 600 python bench.py --gpus 2 --backend peer --steps 10 --warmup 5 --json-out gpurun_out/r3_bench_peer2.json
cd /tmp && export TMPDIR=/tmp
XDDP_RCCL_FORCE_LAUNCH=1 step prof_forced 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_forced" -o run --output-format csv -- python "$ROOT/bench.py" --steps 5 --warmup 3 --diag-steps 3
cd "$ROOT" && bash scripts/gpu_r3_pmc.sh
echo "FAILED=$FAILED"
