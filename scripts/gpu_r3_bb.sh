#!/bin/bash
# r3 call BB: LDS-tiled transpose for the fused dGELU GEMM's Wᵀ: encoder tests, ViT bench x2, profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ge 124 ]; then exit $rc; fi; }
step pytest_e 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_encoder_block_gpu.py tests/test_transformer_gpu.py
step vit1 400 python -u bench.py --model vit_l_16 --steps 10 --warmup 3 --json-out gpurun_out/r3bb_vit1.json
step vit2 400 python -u bench.py --model vit_l_16 --steps 10 --warmup 3 --json-out gpurun_out/r3bb_vit2.json
cd /tmp && export TMPDIR=/tmp
step prof_vit 400 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/prof_vitbb" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_l_16 --steps 4 --warmup 2 --diag-steps 0
python3 "$ROOT/scripts/trace_groups.py" "$ROOT/gpurun_out/prof_vitbb/run_kernel_trace.csv" 6 60 --steady adam_kernel > "$ROOT/gpurun_out/r3_vit_l16_kernel_groups_bb.txt"
grep -n "total\|transpose\|elementwise" "$ROOT/gpurun_out/r3_vit_l16_kernel_groups_bb.txt" | cut -c1-150
