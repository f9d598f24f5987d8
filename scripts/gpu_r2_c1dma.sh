#!/bin/bash
# 1x1 forward on the LDS-DMA pipeline: tests, ResNet-50 A/B over the Cin threshold, kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -2 | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
step c1_test 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_conv_gemm_gpu.py tests/test_headline_gpu.py
for v in 0 1024 512 256 1; do XDDP_C1_DMA=$v step r50_c1dma_$v 300 python bench.py --steps 30 --warmup 10 --diag-steps 0; done
R=$PWD; cd /tmp && export TMPDIR=/tmp
XDDP_C1_DMA=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c1" -o prof --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 5 --diag-steps 0 > "$R/gpurun_out/prof_c1.log" 2>&1; echo "prof rc=$?"
