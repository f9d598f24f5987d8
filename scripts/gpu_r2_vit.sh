#!/bin/bash
# LayerNorm tests + ViT-L/16 bs256 bench + kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -3 | cut -c1-250; if [ $rc -ne 0 ]; then exit $rc; fi; }
step t_ln 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_norm_gpu.py tests/test_encoder_block_gpu.py tests/test_transformer_gpu.py
step vit 400 python bench.py --model vit_l_16 --steps 10 --warmup 4 --diag-steps 0 --json-out gpurun_out/vit.json
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_vit" -o prof --output-format csv -- python3 "$R/bench.py" --model vit_l_16 --steps 3 --warmup 2 --diag-steps 0 > "$R/gpurun_out/prof_vit.log" 2>&1; echo "prof vit rc=$?"
