#!/bin/bash
# PMC counters behind the round-2 kernels (scripts/pmc_r3.py workload): a counter-free trace pass
# for time, one SQ pass (MFMA ops / busy, LDS bank conflicts) and one pass each for FETCH_SIZE and
# WRITE_SIZE; scripts/pmc_summary.py turns them into a roofline table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
pass() { local name=$1; shift; echo "== $name"; timeout -s KILL 150 rocprofv3 "$@" -d "$R/gpurun_out/pmc3_$name" -o run --output-format csv -- python3 "$R/scripts/pmc_r3.py" > "$R/gpurun_out/pmc3_$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$R/gpurun_out/pmc3_$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
pass t --kernel-trace
pass a --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace
pass f --pmc FETCH_SIZE --kernel-trace
pass w --pmc WRITE_SIZE --kernel-trace
python3 "$R/scripts/pmc_summary.py" --plan "$R/gpurun_out/pmc_r3_plan.json" --trace "$R/gpurun_out/pmc3_t" --pmc "$R/gpurun_out/pmc3_a" "$R/gpurun_out/pmc3_f" "$R/gpurun_out/pmc3_w" --out "$R/gpurun_out/r3_pmc_kernels.txt"
# stall counters over the transformer GEMMs (own gemm_nt vs hipBLASLt) in passes of their own
gpass() { local name=$1; shift; echo "== $name"; timeout -s KILL 150 rocprofv3 "$@" -d "$R/gpurun_out/pmc3_$name" -o run --output-format csv -- python3 "$R/scripts/pmc_r3.py" --only-gemm > "$R/gpurun_out/pmc3_$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$R/gpurun_out/pmc3_$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
gpass gt --kernel-trace
gpass gs --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace
python3 "$R/scripts/pmc_summary.py" --plan "$R/gpurun_out/pmc_r3_gemm_plan.json" --trace "$R/gpurun_out/pmc3_gt" --pmc "$R/gpurun_out/pmc3_gs" --out "$R/gpurun_out/r3_pmc_gemm_stalls.txt"
