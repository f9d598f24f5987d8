#!/bin/bash
# TunableOp search for a transformer bench config, then the bench with the tuned table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out tuning/tunableop
export XDDP_NO_AUTOBUILD=1 PYTORCH_TUNABLEOP_VERBOSE=1
M=${1:-vit_l_16}; shift
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -v amdgpu "gpurun_out/$name.log" | tail -2 | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
step tune_$M 900 python -u bench.py --model $M --steps 2 --warmup 1 --diag-steps 0 --tunableop tune "$@"
ls gpurun_out/ && cp "$(ls gpurun_out/tunableop_$M*.csv | head -1)" tuning/tunableop/tunableop_$M.csv && wc -l tuning/tunableop/*
step use_$M 300 python -u bench.py --model $M --steps 10 --warmup 5 --diag-steps 0 --tunableop use "$@"
step off_$M 300 python -u bench.py --model $M --steps 10 --warmup 5 --diag-steps 0 --tunableop off "$@"
