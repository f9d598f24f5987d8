bash scripts/gpu_steps.sh \
 "gputests|1000|python -u -m pytest -q --timeout 240 --timeout-method thread -m gpu tests" \
 "smoke|300|python -u -c \"import __graft_entry__ as g; g.smoke()\"" \
 "r50|240|python -u bench.py --gpus 1 --steps 20 --warmup 5 --json-out gpurun_out/r50.json"
