#!/bin/bash
# Headline bench (channels_last global avg-pool backward) + EPI dgrad GEMM timing and PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -5 | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
step b_avgpool 300 python bench.py --steps 30 --warmup 10 --json-out gpurun_out/b_avgpool.json
step epi_time 120 python scripts/pmc_epi.py
R=$PWD; cd /tmp && export TMPDIR=/tmp
step2() { local name=$1; shift; timeout -s KILL 90 rocprofv3 "$@" --kernel-trace -d "$R/gpurun_out/$name" -o pmc --output-format csv -- python3 "$R/scripts/pmc_epi.py" > "$R/gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step2 pmc_a --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
step2 pmc_f --pmc FETCH_SIZE
step2 pmc_w --pmc WRITE_SIZE
step2 pmc_t --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
