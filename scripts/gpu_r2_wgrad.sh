#!/bin/bash
# New 3x3 weight-gradient kernel + BN2-backward fold: kernel tests, model tests, ResNet-50 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-200; if [ $rc -ne 0 ]; then exit $rc; fi; }
step pytest_k 600 python -u -m pytest tests/test_conv3x3_gpu.py tests/test_conv_gemm_gpu.py tests/test_norm_gpu.py -x -q --timeout 120 --timeout-method thread
step pytest_head 600 python -u -m pytest tests/test_headline_gpu.py tests/test_ddp_gpu.py -x -q --timeout 240 --timeout-method thread
step r50 300 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/r50.json
XDDP_CONV3X3_WGRAD=0 step r50_miopen_wgrad 300 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/r50_mw.json
XDDP_CONV_EPI2=0 step r50_noepi2 300 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/r50_noepi2.json
XDDP_GEMM_OCC=2 step r50_occ2 300 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/r50_occ2.json
step r50b 300 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/r50b.json
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r50" -o prof --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 5 --diag-steps 0 > "$R/gpurun_out/prof_r50.log" 2>&1; echo "prof rc=$?"
