#!/bin/bash
# PMC pass over the stride-1 3x3 kernels (scripts/c3_pmc.py): stall / MFMA / LDS counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d "$R/gpurun_out/c3pmc" -o pmc --output-format csv -- python3 "$R/scripts/c3_pmc.py" ${C3_ONLY:-} > "$R/gpurun_out/c3pmc.log" 2>&1; rc=$?; echo "pmc rc=$rc"; tail -2 "$R/gpurun_out/c3pmc.log"
cd "$R" && python3 scripts/pmc_group.py gpurun_out/c3pmc --filter conv3x3 > gpurun_out/c3pmc_table.txt; cat gpurun_out/c3pmc_table.txt | cut -c1-250
exit $rc
