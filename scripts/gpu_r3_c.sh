#!/bin/bash
# r3 call C: GEMM odd-K path, two-shot peer stress (which factor makes 2 processes on one GPU stall),
# ViT / Llama step with the own GEMM on and off, PMC roofline passes (incl. gemm_nt vs hipBLASLt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "$ROOT/gpurun_out/$name.log"; if [ $rc -ge 124 ]; then exit $rc; fi; }
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
step pytest_gemm 300 $PYT tests/test_gemm_gpu.py
XDDP_GEMM_WAVES=4 step pytest_gemm_w4 300 $PYT tests/test_gemm_gpu.py
step gemm_bench 400 python -u scripts/gemm_nt_bench.py --out gpurun_out/r3_gemm_nt_vs_hipblaslt_v3.txt
step stress_nocompute 100 python -u scripts/peer_stress.py --compute 0 --iters 4
step stress_default 100 python -u scripts/peer_stress.py --iters 4
step stress_b64 100 python -u scripts/peer_stress.py --blocks 64 --iters 4
step stress_normalprio 100 python -u scripts/peer_stress.py --priority normal --iters 4
step vit_own1 300 python -u bench.py --model vit_l_16 --steps 5 --warmup 3 --json-out gpurun_out/r3_vit_own1.json
XDDP_OWN_GEMM=0 step vit_own0 300 python -u bench.py --model vit_l_16 --steps 5 --warmup 3 --json-out gpurun_out/r3_vit_own0.json
step llama_own1 400 python -u bench.py --model llama3_8b --steps 3 --warmup 2 --json-out gpurun_out/r3_llama_own1.json
XDDP_OWN_GEMM=0 step llama_own0 400 python -u bench.py --model llama3_8b --steps 3 --warmup 2 --json-out gpurun_out/r3_llama_own0.json
bash scripts/gpu_r3_pmc.sh
