#!/bin/bash
# PMC roofline of HEAD (scripts/pmc_r3.py workload): one counter-free trace pass for time, then three
# counter passes (SQ MFMA / LDS / stall counters + GRBM, FETCH_SIZE, WRITE_SIZE), summarized by
# scripts/pmc_summary.py into gpurun_out/pmc_kernels.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
R=$PWD; cd /tmp && export TMPDIR=/tmp
pass() {  # name, rocprofv3 counter args...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 "$@" --kernel-trace -d "$R/gpurun_out/$name" -o pmc --output-format csv -- python3 "$R/scripts/pmc_r3.py" > "$R/gpurun_out/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
pass pmcT
pass pmcA --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
pass pmcB --pmc FETCH_SIZE
pass pmcC --pmc WRITE_SIZE
cd "$R" && python3 scripts/pmc_summary.py --plan gpurun_out/pmc_r3_plan.json --trace gpurun_out/pmcT --pmc gpurun_out/pmcA gpurun_out/pmcB gpurun_out/pmcC --out gpurun_out/pmc_kernels.txt && cat gpurun_out/pmc_kernels.txt
