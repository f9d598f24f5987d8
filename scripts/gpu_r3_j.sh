#!/bin/bash
# r3 call J: pending applies, 128-row tiles on 64-wide N (bitwise-matching statistics), A/B bench, trace.
# kernel/model A/B tests, ResNet-50 bench interleaved on/off, kernel trace with them on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ge 124 ]; then exit $rc; fi; }
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
step pytest_pend 400 $PYT -s tests/test_pending_apply_gpu.py
step pytest_conv 400 $PYT tests/test_conv_gemm_gpu.py tests/test_headline_gpu.py tests/test_epilink_gpu.py tests/test_norm_gpu.py tests/test_ddp_gpu.py tests/test_stem_gpu.py
step r50_on1 300 python -u bench.py --json-out gpurun_out/r3j_on1.json
step r50_off1 300 env XDDP_PENDING_APPLY=0 python -u bench.py --json-out gpurun_out/r3j_off1.json
step r50_on2 300 python -u bench.py --json-out gpurun_out/r3j_on2.json
step r50_off2 300 env XDDP_PENDING_APPLY=0 python -u bench.py --json-out gpurun_out/r3j_off2.json
cd /tmp && export TMPDIR=/tmp
step prof_r50 300 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/prof_r50j" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 5 --diag-steps 0
python3 "$ROOT/scripts/trace_groups.py" "$ROOT/gpurun_out/prof_r50j/run_kernel_trace.csv" 15 90 > "$ROOT/gpurun_out/r3_resnet50_bs256_kernel_groups_j.txt"
head -30 "$ROOT/gpurun_out/r3_resnet50_bs256_kernel_groups_j.txt" | cut -c1-160
