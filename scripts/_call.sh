bash scripts/gpu_steps.sh \
 "commtests|600|python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_calibrate_gpu.py tests/test_peer_allreduce_gpu.py tests/test_replicas_gpu.py" \
 "bench_peer2|300|python -u bench.py --gpus 2 --backend peer --model resnet50 --batch-size 64 --steps 10 --warmup 3 --diag-steps 0 --json-out gpurun_out/bench_peer2.json"
