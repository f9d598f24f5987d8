#!/bin/bash
# rocprofv3 kernel-trace stats of the headline bench (5 warmup + 5 timed steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o prof --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 5 "$@" > "$R/gpurun_out/prof.log" 2>&1; echo "prof rc=$?"
tail -2 "$R/gpurun_out/prof.log"
