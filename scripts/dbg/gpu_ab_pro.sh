cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export XDDP_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_conv3x3_gpu.py tests/test_conv_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_conv.log 2>&1 || { tail -40 gpurun_out/t_conv.log; exit 1; }; tail -1 gpurun_out/t_conv.log
for v in "XDDP_GEMM_WT=1" "XDDP_GEMM_WT=0" "XDDP_GEMM_WT=1" "XDDP_GEMM_WT=0"; do
  env $v timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }; echo "$v $(tail -1 gpurun_out/ab.log | cut -c1-140)"
done
