cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export XDDP_NO_AUTOBUILD=1
for v in "XDDP_GRAPH_CUDNN_BENCHMARK=0" "XDDP_GRAPH_CUDNN_BENCHMARK=0 XDDP_MIOPEN_DB=none" "MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_V4R1=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_V4R1=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_V4R1=0"; do
  echo "== $v"; env $v timeout -k 10 120 python scripts/dbg/graph_dbg.py 2>&1 | grep -E "trial 0 step (1|2)|Error" | cut -c1-90
done
echo "== bench graphs benchmark0"
XDDP_GRAPH_CUDNN_BENCHMARK=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM=1 timeout -k 10 200 python bench.py --model simplecnn --batch-size 32 --image-size 32 --steps 200 --warmup 20 --graphs 1 2>&1 | tail -1 | cut -c1-200
