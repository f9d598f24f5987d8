#!/bin/bash
# r3 call D: GEMM grouped order + dGELU epilogue, LDS-free peer barrier (stress + 2-rank peer
# bench), ViT / Llama own-GEMM A/B, PMC passes, then the whole GPU test suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "$ROOT/gpurun_out/$name.log"; if [ $rc -ge 124 ]; then exit $rc; fi; }
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
step pytest_gemm 300 $PYT tests/test_gemm_gpu.py tests/test_encoder_block_gpu.py
step gemm_bench 400 python -u scripts/gemm_nt_bench.py --out gpurun_out/r3_gemm_nt_vs_hipblaslt_v4.txt
step stress_b64 100 python -u scripts/peer_stress.py --iters 4
step stress_b256 100 python -u scripts/peer_stress.py --blocks 256 --iters 4
export XDDP_PEER_TIMEOUT_MS=30000 XDDP_FLIGHT_DUMP_PREFIX=$ROOT/gpurun_out/flight_peer2d_rank_
step bench_peer2 200 python -u bench.py --gpus 2 --backend peer --steps 5 --warmup 3 --diag-steps 2 --json-out gpurun_out/r3_bench_peer2.json
unset XDDP_PEER_TIMEOUT_MS XDDP_FLIGHT_DUMP_PREFIX
step vit_own1 300 python -u bench.py --model vit_l_16 --steps 5 --warmup 3 --json-out gpurun_out/r3_vit_own1.json
XDDP_OWN_GEMM=0 step vit_own0 300 python -u bench.py --model vit_l_16 --steps 5 --warmup 3 --json-out gpurun_out/r3_vit_own0.json
step llama_own1 400 python -u bench.py --model llama3_8b --steps 3 --warmup 2 --json-out gpurun_out/r3_llama_own1.json
XDDP_OWN_GEMM=0 step llama_own0 400 python -u bench.py --model llama3_8b --steps 3 --warmup 2 --json-out gpurun_out/r3_llama_own0.json
bash scripts/gpu_r3_pmc.sh || exit $?
cd /tmp && export TMPDIR=/tmp
XDDP_RCCL_FORCE_LAUNCH=1 step prof_llama_overlap 500 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/prof_llama_overlap" -o run --output-format csv -- python3 "$ROOT/bench.py" --model llama3_8b --steps 3 --warmup 2 --diag-steps 0 --overlap-optim 1
python3 "$ROOT/scripts/overlap_trace.py" "$ROOT/gpurun_out/prof_llama_overlap" --out "$ROOT/gpurun_out/r3_llama_overlap_tail.txt"
cd "$ROOT"
step pytest_all 1000 $PYT -m gpu tests
