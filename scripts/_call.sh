bash scripts/gpu_steps.sh \
 "tailtest|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_tail_gpu.py tests/test_norm_gpu.py" \
 "tailtime|200|PYTHONPATH=. python -u scripts/bn_tail_time.py" \
 "r50_t1|200|python -u bench.py --steps 30 --warmup 10 --diag-steps 0 --json-out gpurun_out/r50_t1.json" \
 "r50_t0|200|XDDP_BN_TAIL=0 python -u bench.py --steps 30 --warmup 10 --diag-steps 0 --json-out gpurun_out/r50_t0.json" \
 "r50_t1b|200|python -u bench.py --steps 30 --warmup 10 --diag-steps 0 --json-out gpurun_out/r50_t1b.json" \
 "r50_t0b|200|XDDP_BN_TAIL=0 python -u bench.py --steps 30 --warmup 10 --diag-steps 0 --json-out gpurun_out/r50_t0b.json"
