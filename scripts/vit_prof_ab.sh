#!/bin/bash
# rocprofv3 kernel stats of a short ViT-L/16 bench for the working tree and ab_old/ (see ab_build_old.sh)
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/vprof_new" -o v -- python3 "$R/bench.py" --model vit_l_16 --steps 3 --warmup 2 > "$R/gpurun_out/vprof_new.log" 2>&1 || exit $?
cd "$R/ab_old" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/vprof_old" -o v -- python3 "$R/ab_old/bench.py" --model vit_l_16 --steps 3 --warmup 2 > "$R/gpurun_out/vprof_old.log" 2>&1
