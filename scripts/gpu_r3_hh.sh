#!/bin/bash
# r3 call HH: HEAD validation — full GPU suite, smoke, ResNet-50 bench x2, ViT-L/16 and Llama-3-8B
# benches, ViT steady-state profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ge 124 ]; then exit $rc; fi; }
step pytest_all 900 python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step r50_a 300 python -u bench.py --json-out gpurun_out/r3hh_r50_a.json
step r50_b 300 python -u bench.py --json-out gpurun_out/r3hh_r50_b.json
step vit 400 python -u bench.py --model vit_l_16 --steps 10 --warmup 3 --json-out gpurun_out/r3hh_vit.json
step llama 400 python -u bench.py --model llama3_8b --steps 10 --warmup 3 --json-out gpurun_out/r3hh_llama.json
cd /tmp && export TMPDIR=/tmp
step prof_vit 400 rocprofv3 --kernel-trace -d "$ROOT/gpurun_out/prof_vithh" -o run --output-format csv -- python3 "$ROOT/bench.py" --model vit_l_16 --steps 4 --warmup 2 --diag-steps 0
python3 "$ROOT/scripts/trace_groups.py" "$ROOT/gpurun_out/prof_vithh/run_kernel_trace.csv" 6 60 --steady adam_kernel > "$ROOT/gpurun_out/r3_vit_l16_kernel_groups_hh.txt"
head -2 "$ROOT/gpurun_out/r3_vit_l16_kernel_groups_hh.txt"
