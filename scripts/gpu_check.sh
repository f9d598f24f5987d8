#!/bin/bash
# One gpurun call: GPU tests, 1-GPU benches (xddp vs torch-DDP reference stack), rocprof stats.
# Every GPU step has its own time limit; a crash/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1 HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc in $name; stopping"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-20}
python -c "import torch; print(torch.cuda.get_device_name(0))"
run pytest_gpu 600 python -m pytest tests -m gpu -x -q
run bench_xddp 600 python bench.py --norm xddp --steps $STEPS --warmup 10 --json-out gpurun_out/bench_xddp.json
run bench_xddp_torchbn 600 python bench.py --norm torch --steps $STEPS --warmup 10 --json-out gpurun_out/bench_xddp_torchbn.json
run bench_torch 600 python bench.py --impl torch --norm torch --steps $STEPS --warmup 10 --json-out gpurun_out/bench_torch.json
if [ "${PROFILE:-1}" = "1" ]; then
  R=$PWD
  cd /tmp && export TMPDIR=/tmp
  run_prof() { timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o prof --output-format csv -- python3 "$R/bench.py" --norm xddp --steps 5 --warmup 5 > "$R/gpurun_out/prof.log" 2>&1; }
  run_prof; echo "prof rc=$?"
  cd "$R"
fi
cat gpurun_out/*.json 2>/dev/null
