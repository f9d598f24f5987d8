cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
for i in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/b2_$i.log 2>&1 || exit 1; tail -1 gpurun_out/b2_$i.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])'; done
