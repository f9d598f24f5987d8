#!/bin/bash
# r3 call GG: stall counters over the flash attention kernels (ViT and Llama shapes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
ONLY="flash"
spass() { local name=$1; shift; echo "== $name"; timeout -s KILL 150 rocprofv3 "$@" -d "$R/gpurun_out/pmc3g_$name" -o run --output-format csv -- python3 "$R/scripts/pmc_r3.py" --only "$ONLY" --plan-out "$R/gpurun_out/pmc_r3g_plan.json" > "$R/gpurun_out/pmc3g_$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$R/gpurun_out/pmc3g_$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
spass t --kernel-trace
spass s --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace
python3 "$R/scripts/pmc_summary.py" --plan "$R/gpurun_out/pmc_r3g_plan.json" --trace "$R/gpurun_out/pmc3g_t" --pmc "$R/gpurun_out/pmc3g_s" --out "$R/gpurun_out/r3_pmc_flash_stalls.txt"
cat "$R/gpurun_out/r3_pmc_flash_stalls.txt"
