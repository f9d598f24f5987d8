#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export XDDP_NO_AUTOBUILD=1
for c in ddp_linear llama mt_copy ln_fwd bn_fwd_only our_bn; do
  timeout -k 10 200 python -X faulthandler scripts/graph_probe.py $c > gpurun_out/probe_$c.log 2>&1; rc=$?
  grep -E "^OK|^FAIL" gpurun_out/probe_$c.log; echo "$c rc=$rc"
  if [ $rc -ne 0 ]; then grep -A25 "Fatal Python error" gpurun_out/probe_$c.log | head -40; exit $rc; fi
done
