#!/bin/bash
# Flash-attention backward: per-call timing, then one SQ stall/MFMA/LDS counter pass.
# FA_SCRIPT selects the workload (default scripts/fa_bwd_time.py, the Llama shape; the ViT shape:
# FA_SCRIPT=scripts/fa_vit_time.py FA_PMC_ARGS=""), FA_PMC_ARGS its arguments under the profiler.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
S=${FA_SCRIPT:-scripts/fa_bwd_time.py}
timeout -k 10 300 python -u "$S" > gpurun_out/fa_time.log 2>&1 || exit $?
cat gpurun_out/fa_time.log
R=$PWD; cd /tmp && export TMPDIR=/tmp
# shellcheck disable=SC2086
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d "$R/gpurun_out/fapmc" -o pmc --output-format csv -- python3 "$R/$S" ${FA_PMC_ARGS---iters 3} > "$R/gpurun_out/fapmc.log" 2>&1; rc=$?; echo "pmc rc=$rc"
cd "$R" && python3 scripts/pmc_group.py gpurun_out/fapmc --filter fa_ | cut -c1-230
exit $rc
