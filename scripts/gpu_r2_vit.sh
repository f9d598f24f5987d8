#!/bin/bash
# fused encoder block: kernel/block tests, ViT-L/16 bs256 bench A/B (fused vs unfused), kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -3 | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
step vit_test 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_encoder_block_gpu.py tests/test_flash_attn_gpu.py tests/test_ddp_gpu.py -k "not resnet or vit"
step vit_fused 300 python -u bench.py --model vit_l_16 --steps 10 --warmup 5 --diag-steps 0 --tunableop off
XDDP_FUSED_BLOCK=0 step vit_unfused 300 python -u bench.py --model vit_l_16 --steps 10 --warmup 5 --diag-steps 0 --tunableop off
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_vit" -o prof --output-format csv -- python3 "$R/bench.py" --model vit_l_16 --steps 3 --warmup 2 --diag-steps 0 --tunableop off > "$R/gpurun_out/prof_vit.log" 2>&1; echo "prof vit rc=$?"
