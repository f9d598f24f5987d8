bash scripts/gpu_steps.sh \
 "g_new|200|python -u scripts/gemm1x1_time.py" \
 "g_old|200|cd ab_old && PYTHONPATH=. python -u ../scripts/gemm1x1_time.py" \
 "r_new|200|python -u bench.py --steps 30 --warmup 10 --diag-steps 0 --json-out gpurun_out/r_new.json" \
 "r_old|200|cd ab_old && python -u bench.py --steps 30 --warmup 10 --diag-steps 0 --json-out ../gpurun_out/r_old.json" \
 "r_new2|200|python -u bench.py --steps 30 --warmup 10 --diag-steps 0 --json-out gpurun_out/r_new2.json" \
 "r_old2|200|cd ab_old && python -u bench.py --steps 30 --warmup 10 --diag-steps 0 --json-out ../gpurun_out/r_old2.json"
