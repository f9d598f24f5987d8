#!/bin/bash
# Graph-capture test + reference-workload graph bench, then PMC counter passes on the conv GEMM.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py -x -q --timeout 240 --timeout-method thread -k graphed > gpurun_out/graph_test.log 2>&1; echo "graph test rc=$?"; tail -1 gpurun_out/graph_test.log
timeout -k 10 300 python bench.py --model simplecnn --batch-size 32 --image-size 32 --steps 200 --warmup 20 --graphs 1 --json-out gpurun_out/b_cnn_graph.json > gpurun_out/b_cnn_graph.log 2>&1; echo "cnn graph rc=$?"; cat gpurun_out/b_cnn_graph.json
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/pmc1" -o pmc --output-format csv -- python3 "$R/scripts/pmc_gemm.py" > "$R/gpurun_out/pmc1.log" 2>&1; echo "pmc1 rc=$?"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmc2" -o pmc --output-format csv -- python3 "$R/scripts/pmc_gemm.py" > "$R/gpurun_out/pmc2.log" 2>&1; echo "pmc2 rc=$?"
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmc3" -o pmc --output-format csv -- python3 "$R/scripts/pmc_gemm.py" > "$R/gpurun_out/pmc3.log" 2>&1; echo "pmc3 rc=$?"
