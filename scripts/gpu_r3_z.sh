#!/bin/bash
# r3 call Z: deep-K BN-reduce-epilogue input gradient on LDS-DMA stages (epi_dgrad_dma_kernel):
# tests, bench interleaved (XDDP_EPI_DMA_MIN_K default 256 / 128 / off), trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ge 124 ]; then exit $rc; fi; }
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
step pytest_c 400 $PYT tests/test_conv_gemm_gpu.py tests/test_headline_gpu.py tests/test_epilink_gpu.py
for r in 1 2; do
step on$r 300 python -u bench.py --json-out gpurun_out/r3z_on$r.json
step k128_$r 300 env XDDP_EPI_DMA_MIN_K=128 python -u bench.py --json-out gpurun_out/r3z_k128_$r.json
step off$r 300 env XDDP_EPI_DMA_MIN_K=0 python -u bench.py --json-out gpurun_out/r3z_off$r.json
done
cd /tmp && export TMPDIR=/tmp
step prof_r50 300 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/prof_r50z" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 5 --diag-steps 0
python3 "$ROOT/scripts/trace_groups.py" "$ROOT/gpurun_out/prof_r50z/run_kernel_trace.csv" 15 200 --steady sgd_master > "$ROOT/gpurun_out/r3_resnet50_bs256_kernel_groups_z.txt"
grep -n "total\|epi_dgrad\|true, true, 4>" "$ROOT/gpurun_out/r3_resnet50_bs256_kernel_groups_z.txt" | cut -c1-150
