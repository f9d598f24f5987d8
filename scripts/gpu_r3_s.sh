#!/bin/bash
# r3 call S: (1) plain 1x1 forwards on the LDS-DMA GEMM (XDDP_C1_NT arms), (2) 3 LDS stages for the
# 128-wide gemm_nt tile (XDDP_GEMM_STAGES=2 vs default 3): GEMM / 3x3 microbenches + bench arms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ge 124 ]; then exit $rc; fi; }
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
step pytest_c 300 $PYT tests/test_conv_gemm_gpu.py tests/test_gemm_gpu.py tests/test_conv3x3_gpu.py
step pytest_h 300 env XDDP_C1_NT=1 $PYT tests/test_headline_gpu.py
step gemm3 300 env XDDP_GEMM_BN=128 python -u scripts/gemm_nt_bench.py --out gpurun_out/r3_gemm_nt_bn128_s3.txt
step gemm2 300 env XDDP_GEMM_BN=128 XDDP_GEMM_STAGES=2 python -u scripts/gemm_nt_bench.py --out gpurun_out/r3_gemm_nt_bn128_s2.txt
step gemm256 300 env XDDP_GEMM_BN=256 python -u scripts/gemm_nt_bench.py --out gpurun_out/r3_gemm_nt_bn256.txt
step ceil3 300 python -u scripts/conv3x3_ceiling.py --out gpurun_out/r3_conv3x3_ceiling_s3.txt
step ceil2 300 env XDDP_GEMM_STAGES=2 python -u scripts/conv3x3_ceiling.py --out gpurun_out/r3_conv3x3_ceiling_s2.txt
for r in 1 2; do
step base$r 300 env XDDP_GEMM_STAGES=2 python -u bench.py --json-out gpurun_out/r3s_base$r.json
step s3_$r 300 python -u bench.py --json-out gpurun_out/r3s_s3_$r.json
step s3nt_$r 300 env XDDP_C1_NT=s2 python -u bench.py --json-out gpurun_out/r3s_s3nts2_$r.json
step s3nt1_$r 300 env XDDP_C1_NT=1 python -u bench.py --json-out gpurun_out/r3s_s3nt1_$r.json
done
