cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread -k graphed > gpurun_out/g1.log 2>&1; echo "g1 rc=$?"
timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread -k graphed > gpurun_out/g2.log 2>&1; echo "g2 rc=$?"
timeout -k 10 300 python -u -m pytest tests/test_conv_gemm_gpu.py tests/test_ddp_gpu.py -x -q --timeout 120 --timeout-method thread -k "graphed or fusion" > gpurun_out/g3.log 2>&1; echo "g3 rc=$?"
timeout -k 10 400 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/bench_fused.json > gpurun_out/bench_fused.log 2>&1 && XDDP_CONV_BN_FUSION=0 timeout -k 10 400 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/bench_unfused.json > gpurun_out/bench_unfused.log 2>&1; echo "bench rc=$?"
cat gpurun_out/bench_fused.json gpurun_out/bench_unfused.json
