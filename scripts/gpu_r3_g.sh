#!/bin/bash
# r3 call G: BN-backward coefficient copy folded into the finalize kernel: BN / headline tests,
# ResNet-50 bench x2, kernel trace (copyBuffer count per iteration).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ge 124 ]; then exit $rc; fi; }
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
step pytest_bn 400 $PYT tests/test_norm_gpu.py tests/test_conv_gemm_gpu.py tests/test_headline_gpu.py tests/test_epilink_gpu.py
step r50_a 300 python -u bench.py --json-out gpurun_out/r3g_r50_a.json
step r50_b 300 python -u bench.py --json-out gpurun_out/r3g_r50_b.json
cd /tmp && export TMPDIR=/tmp
step prof_r50 300 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/prof_r50g" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 5 --diag-steps 0
python3 "$ROOT/scripts/trace_groups.py" "$ROOT/gpurun_out/prof_r50g/run_kernel_trace.csv" 15 90 > "$ROOT/gpurun_out/r3_resnet50_bs256_kernel_groups_g.txt"
grep -n "copyBuffer\|fillBuffer\|total" "$ROOT/gpurun_out/r3_resnet50_bs256_kernel_groups_g.txt"
