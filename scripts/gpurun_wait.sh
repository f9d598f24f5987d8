#!/bin/bash
# Submit one gpurun call, re-submitting ONLY while the pool reports no free box / backoff
# (gpurun exit 3 or a "transient" status: nothing ran, nothing charged). Any other outcome — the
# command ran, failed or was refused — ends the loop. Output: gpurun_out/_wait.log.
# usage: scripts/gpurun_wait.sh <timeout-seconds> '<command>'
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
t=$1
shift
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" > gpurun_out/_wait.log 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" gpurun_out/_wait.log; then
    echo "gpurun rc=$rc after $i attempt(s)" >> gpurun_out/_wait.log
    exit $rc
  fi
  sleep 45
done
echo "gave up after 40 attempts" >> gpurun_out/_wait.log
exit 3
