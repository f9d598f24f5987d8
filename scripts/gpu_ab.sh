#!/bin/bash
# Generic A/B of the headline bench (or any bench.py arguments) under environment variants, on one
# box, e.g.:
#   gpurun -- 'bash scripts/gpu_ab.sh "" "XDDP_DS_DEFER=0" "XDDP_PENDING_APPLY=0"'
#   BENCH_ARGS="--model vit_l_16 --steps 10 --warmup 4" gpurun -- 'bash scripts/gpu_ab.sh "" "XDDP_OWN_GEMM=0"'
# Each variant runs under its own time limit; the first failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
ARGS=${BENCH_ARGS:---steps 30 --warmup 10}
i=0
for variant in "$@"; do
  i=$((i + 1))
  echo "== variant $i: ${variant:-<default>}"
  # shellcheck disable=SC2086
  timeout -k 10 600 env $variant python bench.py $ARGS --diag-steps 0 > "gpurun_out/ab_$i.log" 2>&1
  rc=$?
  grep -o '"value": [0-9.]*' "gpurun_out/ab_$i.log"
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/ab_$i.log"; exit $rc; fi
done
