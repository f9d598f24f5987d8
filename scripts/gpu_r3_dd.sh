#!/bin/bash
# r3 call DD: software-pipelined stem maxpool/ReLU/BN backward: stem tests, standalone A/B, bench A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "$ROOT/gpurun_out/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
# (stem tests passed on this tree in the first attempt of this call)
step t_pf1 120 python -u scripts/stem_bwd_time.py
XDDP_STEM_PF=0 step t_pf0 120 python -u scripts/stem_bwd_time.py
step t_pf1b 120 python -u scripts/stem_bwd_time.py
step b_on1 300 python -u bench.py --steps 20 --warmup 5 --json-out gpurun_out/r3dd_on1.json
XDDP_STEM_PF=0 step b_off1 300 python -u bench.py --steps 20 --warmup 5 --json-out gpurun_out/r3dd_off1.json
step b_on2 300 python -u bench.py --steps 20 --warmup 5 --json-out gpurun_out/r3dd_on2.json
XDDP_STEM_PF=0 step b_off2 300 python -u bench.py --steps 20 --warmup 5 --json-out gpurun_out/r3dd_off2.json
