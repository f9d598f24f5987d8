#!/bin/bash
# Flash-attention backward: per-call timing, then one SQ stall/MFMA/LDS counter pass (scripts/fa_bwd_time.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
timeout -k 10 300 python -u scripts/fa_bwd_time.py > gpurun_out/fa_time.log 2>&1 || exit $?
cat gpurun_out/fa_time.log
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d "$R/gpurun_out/fapmc" -o pmc --output-format csv -- python3 "$R/scripts/fa_bwd_time.py" --iters 3 > "$R/gpurun_out/fapmc.log" 2>&1; rc=$?; echo "pmc rc=$rc"
cd "$R" && python3 scripts/pmc_group.py gpurun_out/fapmc --filter fa_ | cut -c1-230
exit $rc
