#!/bin/bash
# Packed C-tile LDS stores (transposed MFMA) in the 1x1 GEMM and 3x3 implicit GEMM: tests, EPI timing, bench, profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -5 | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
step t_conv 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_conv_gemm_gpu.py tests/test_conv3x3_gpu.py tests/test_headline_gpu.py
step epi_time 120 python scripts/pmc_epi.py
step b_pack 300 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_pack.json
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_pack" -o prof --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 5 --diag-steps 0 > "$R/gpurun_out/prof_pack.log" 2>&1; echo "prof rc=$?"
