bash scripts/gpu_steps.sh \
 "ringtest|300|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_conv_gemm_gpu.py -k wgrad" \
 "wg_ring|200|python -u scripts/wgrad1x1_time.py" \
 "r50ring_a|240|python -u bench.py --steps 30 --warmup 10 --json-out gpurun_out/r50ring_a.json" \
 "r50old_a|240|XDDP_WGRAD_RING=0 python -u bench.py --steps 30 --warmup 10 --json-out gpurun_out/r50old_a.json" \
 "r50ring_b|240|python -u bench.py --steps 30 --warmup 10 --json-out gpurun_out/r50ring_b.json" \
 "r50old_b|240|XDDP_WGRAD_RING=0 python -u bench.py --steps 30 --warmup 10 --json-out gpurun_out/r50old_b.json" \
 "reftf_def|200|python -u tests/_ref_teacher_forced.py 8" \
 "reftf_det|200|XDDP_TEST_CUDNN_DETERMINISTIC=1 python -u tests/_ref_teacher_forced.py 8" \
 "reftf_nowino|200|MIOPEN_DEBUG_CONV_WINOGRAD=0 python -u tests/_ref_teacher_forced.py 8" \
 "reftf_noimpl|200|MIOPEN_DEBUG_CONV_IMPLICIT_GEMM=0 python -u tests/_ref_teacher_forced.py 8"
