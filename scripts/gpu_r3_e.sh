#!/bin/bash
# r3 call E: whole GPU suite after the knob cleanup, smoke, ResNet-50 bench, ViT own-GEMM modes A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "$ROOT/gpurun_out/$name.log" | cut -c1-400; if [ $rc -ge 124 ]; then exit $rc; fi; }
PYT="python -u -m pytest -x -v --timeout 240 --timeout-method thread"
step pytest_all 600 $PYT -m gpu tests
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
step r50_a 300 python -u bench.py --json-out gpurun_out/r3e_r50_a.json
for i in 1 2; do
  XDDP_OWN_GEMM=0 step vit_0_$i 300 python -u bench.py --model vit_l_16 --steps 8 --warmup 3 --diag-steps 0 --json-out gpurun_out/r3e_vit_0_$i.json
  XDDP_OWN_GEMM=bwd step vit_bwd_$i 300 python -u bench.py --model vit_l_16 --steps 8 --warmup 3 --diag-steps 0 --json-out gpurun_out/r3e_vit_bwd_$i.json
done
step r50_b 300 python -u bench.py --json-out gpurun_out/r3e_r50_b.json
cd /tmp && export TMPDIR=/tmp
R=$ROOT
gpass() { local name=$1; shift; echo "== $name"; timeout -s KILL 150 rocprofv3 "$@" -d "$R/gpurun_out/pmc3_$name" -o run --output-format csv -- python3 "$R/scripts/pmc_r3.py" --only-gemm > "$R/gpurun_out/pmc3_$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$R/gpurun_out/pmc3_$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
gpass gt --kernel-trace
gpass gs --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace
python3 "$R/scripts/pmc_summary.py" --plan "$R/gpurun_out/pmc_r3_gemm_plan.json" --trace "$R/gpurun_out/pmc3_gt" --pmc "$R/gpurun_out/pmc3_gs" --out "$R/gpurun_out/r3_pmc_gemm_stalls.txt"
