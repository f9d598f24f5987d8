#!/bin/bash
# r3 call O: kernel-group profile of HEAD (pending applies, conv GEMM path, halo kernel) and the
# step's copy / fill attribution.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ge 124 ]; then exit $rc; fi; }
step step_ops 300 python -u scripts/step_ops.py --out gpurun_out/r3_resnet50_step_copies.txt
cd /tmp && export TMPDIR=/tmp
step prof_r50 300 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/prof_r50o" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 5 --diag-steps 0
python3 "$ROOT/scripts/trace_groups.py" "$ROOT/gpurun_out/prof_r50o/run_kernel_trace.csv" 15 120 > "$ROOT/gpurun_out/r3_resnet50_bs256_kernel_groups_o.txt"
head -3 "$ROOT/gpurun_out/r3_resnet50_bs256_kernel_groups_o.txt" | cut -c1-160
