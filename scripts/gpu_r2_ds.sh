#!/bin/bash
# Stride-2 kernels (3x3 phase dgrad, 1x1 downsample gradient into conv1's epilogue): tests + A/B bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -4 | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
step t_s2 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv3x3_gpu.py tests/test_conv_gemm_gpu.py -k "s2 or stride2 or downsample or handoff or dgrad_bn"
step b_new 300 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_new.json
step b_old 300 env XDDP_CONV3X3_DGRAD_S2=0 XDDP_CONV_EPI_DS=0 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_old.json
step b_new2 300 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_new2.json
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_ds" -o prof --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 5 --diag-steps 0 > "$R/gpurun_out/prof_ds.log" 2>&1; echo "prof rc=$?"
cd "$R"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
