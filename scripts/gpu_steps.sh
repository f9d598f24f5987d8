#!/bin/bash
# One gpurun call = a list of named, individually time-limited steps, run in order; the first
# failing step ends the call (nothing more touches the GPU after a fault, abort or time limit).
# Each argument is "name|seconds|command"; the command's output goes to gpurun_out/<name>.log and
# its last lines are echoed. Examples:
#   gpurun -- 'bash scripts/gpu_steps.sh "tests|900|python -u -m pytest -v --timeout 240 --timeout-method thread -m gpu tests" \
#                                         "smoke|300|python -u -c \"import __graft_entry__ as g; g.smoke()\"" \
#                                         "r50|300|python -u bench.py --json-out gpurun_out/r50.json"'
# A command starting with "prof " runs under rocprofv3 --kernel-trace --stats (from /tmp, output
# in gpurun_out/<name>/; @R@ stands for the repo root): "r50prof|600|prof python3 @R@/bench.py --steps 5".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
for spec in "$@"; do
  name=${spec%%|*}
  rest=${spec#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  echo "== $name (limit ${secs}s): $cmd"
  if [ "${cmd#pmcpass }" != "$cmd" ]; then
    # "pmcpass <counters>": one rocprofv3 counter pass over $PMC_PROG (default scripts/pmc_wgrad.py)
    ctrs=${cmd#pmcpass }
    # shellcheck disable=SC2086
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL "$secs" rocprofv3 --pmc $ctrs --kernel-trace -d "$ROOT/gpurun_out/$name" \
      -o pmc --output-format csv -- python3 "$ROOT/${PMC_PROG:-scripts/pmc_wgrad.py}") > "$ROOT/gpurun_out/$name.log" 2>&1
  elif [ "${cmd#prof }" != "$cmd" ]; then
    prog=${cmd#prof }
    prog=${prog//@R@/$ROOT}
    # shellcheck disable=SC2086
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/$name" \
      -o prof --output-format csv -- $prog) > "$ROOT/gpurun_out/$name.log" 2>&1
  else
    timeout -k 10 "$secs" bash -c "$cmd" > "$ROOT/gpurun_out/$name.log" 2>&1
  fi
  rc=$?
  echo "== $name rc=$rc"
  tail -3 "$ROOT/gpurun_out/$name.log" | cut -c1-400
  if [ $rc -ne 0 ]; then exit $rc; fi
done
