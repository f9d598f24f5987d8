#!/bin/bash
# HIP-graph capture bisect: smallest cases first; native backtrace on a crash.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export XDDP_NO_AUTOBUILD=1 XDDP_NATIVE_BACKTRACE=1
for c in ${PROBE_CASES:-mt_copy ln_fwd bn_fwd_only linear_only ddp_linear our_bn llama}; do
  timeout -k 10 200 python -X faulthandler scripts/graph_probe.py $c > gpurun_out/probe_$c.log 2>&1; rc=$?
  grep -E "^OK|^FAIL" gpurun_out/probe_$c.log; echo "$c rc=$rc"
  if [ $rc -ne 0 ]; then grep -B2 -A45 "native backtrace" gpurun_out/probe_$c.log | head -60; exit $rc; fi
done
