#!/bin/bash
# r3 call CC: stall counters (wait / busy per wave-cycle) over the ResNet-50 kernels that sit
# below their roofline: EPI input gradient per stage, halo 3x3, conv on gemm_nt, pending prologue.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
ONLY="EPI,conv3x3 fwd,conv3x3 dgrad,pending,deep-K"
spass() { local name=$1; shift; echo "== $name"; timeout -s KILL 150 rocprofv3 "$@" -d "$R/gpurun_out/pmc3c_$name" -o run --output-format csv -- python3 "$R/scripts/pmc_r3.py" --only "$ONLY" --plan-out "$R/gpurun_out/pmc_r3c_plan.json" > "$R/gpurun_out/pmc3c_$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$R/gpurun_out/pmc3c_$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
spass t --kernel-trace
spass s --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace
python3 "$R/scripts/pmc_summary.py" --plan "$R/gpurun_out/pmc_r3c_plan.json" --trace "$R/gpurun_out/pmc3c_t" --pmc "$R/gpurun_out/pmc3c_s" --out "$R/gpurun_out/r3_pmc_resnet_stalls.txt"
cat "$R/gpurun_out/r3_pmc_resnet_stalls.txt"
