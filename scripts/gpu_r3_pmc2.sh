#!/bin/bash
# r3 call V: PMC roofline of every hand-written kernel incl. the round-3 ones (halo 3x3, conv on gemm_nt,
# pending-apply prologues, deep-K statistics GEMM): trace pass, one SQ pass, FETCH_SIZE, WRITE_SIZE.
#
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp
pass() { local name=$1; shift; echo "== $name"; timeout -s KILL 150 rocprofv3 "$@" -d "$R/gpurun_out/pmc3b_$name" -o run --output-format csv -- python3 "$R/scripts/pmc_r3.py" > "$R/gpurun_out/pmc3b_$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$R/gpurun_out/pmc3b_$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
pass t --kernel-trace
pass a --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace
pass f --pmc FETCH_SIZE --kernel-trace
pass w --pmc WRITE_SIZE --kernel-trace
python3 "$R/scripts/pmc_summary.py" --plan "$R/gpurun_out/pmc_r3_plan.json" --trace "$R/gpurun_out/pmc3b_t" --pmc "$R/gpurun_out/pmc3b_a" "$R/gpurun_out/pmc3b_f" "$R/gpurun_out/pmc3b_w" --out "$R/gpurun_out/r3_pmc_kernels_v3.txt"
