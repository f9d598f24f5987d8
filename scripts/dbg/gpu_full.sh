# full GPU suite + smoke + headline bench + graphed bench (resnet50 and the reference workload)
cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then tail -30 "gpurun_out/$name.log"; exit $rc; fi; }
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps 20 --warmup 10 --json-out gpurun_out/bench.json
step bench_graph 600 python bench.py --steps 20 --warmup 10 --graphs 1 --json-out gpurun_out/bench_graph.json
step b_cnn_graph 300 python bench.py --model simplecnn --batch-size 32 --image-size 32 --steps 200 --warmup 20 --graphs 1 --json-out gpurun_out/b_cnn_graph.json
