bash scripts/gpu_steps.sh \
 "r50|240|python -u bench.py --json-out gpurun_out/r50.json" \
 "ref_x1|200|python -u bench.py --model simplecnn --batch-size 32 --image-size 32 --recipe reference --steps 300 --warmup 30 --json-out gpurun_out/ref_x1.json" \
 "ref_t1|200|python -u bench.py --impl torch --norm torch --channels-last 0 --model simplecnn --batch-size 32 --image-size 32 --recipe reference --steps 300 --warmup 30 --json-out gpurun_out/ref_t1.json" \
 "ref_xf1|200|python -u bench.py --model simplecnn --batch-size 32 --image-size 32 --recipe reference --steps 300 --warmup 30 --fast-convs 1 --json-out gpurun_out/ref_xf1.json" \
 "ref_tf1|200|python -u bench.py --impl torch --norm torch --channels-last 0 --model simplecnn --batch-size 32 --image-size 32 --recipe reference --steps 300 --warmup 30 --fast-convs 1 --json-out gpurun_out/ref_tf1.json" \
 "ref_x2|200|python -u bench.py --model simplecnn --batch-size 32 --image-size 32 --recipe reference --steps 300 --warmup 30 --json-out gpurun_out/ref_x2.json" \
 "ref_t2|200|python -u bench.py --impl torch --norm torch --channels-last 0 --model simplecnn --batch-size 32 --image-size 32 --recipe reference --steps 300 --warmup 30 --json-out gpurun_out/ref_t2.json" \
 "ref_xf2|200|python -u bench.py --model simplecnn --batch-size 32 --image-size 32 --recipe reference --steps 300 --warmup 30 --fast-convs 1 --json-out gpurun_out/ref_xf2.json" \
 "ref_tf2|200|python -u bench.py --impl torch --norm torch --channels-last 0 --model simplecnn --batch-size 32 --image-size 32 --recipe reference --steps 300 --warmup 30 --fast-convs 1 --json-out gpurun_out/ref_tf2.json" \
 "reftest|400|python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_reference_workload_gpu.py"
