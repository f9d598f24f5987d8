#!/bin/bash
# Interleaved A/B builds on one GPU box: build a git ref's version of the given source files into
# ab_old/ (a copy of the package with its own _C .so, plus bench.py and a tuning/ link), then
# rebuild the working tree. One gpurun call can then alternate the two builds minutes apart:
#   scripts/ab_build_old.sh distributeddataparallel_amd/csrc/kernels/conv_gemm.hip
#   gpurun -- 'bash scripts/gpu_steps.sh "n1|300|python -u bench.py --json-out gpurun_out/new1.json" \
#                 "o1|300|cd ab_old && python -u bench.py --json-out ../gpurun_out/old1.json" ...'
# (scripts run from ab_old import the repo package, not the old one: A/B benches, not scripts.)
# REF defaults to HEAD. Remove ab_old/ afterwards (it is not part of the tree).
set -e
cd "$(dirname "$0")/.."
REF=${REF:-HEAD}
keep=$(mktemp -d)
rm -rf ab_old
for f in "$@"; do mkdir -p "$keep/$(dirname "$f")"; cp "$f" "$keep/$f"; git show "$REF:$f" > "$f"; done
restore() { for f in "$@"; do cp "$keep/$f" "$f"; done; }
trap 'restore "$@"' EXIT
timeout 1800 python -c "import __graft_entry__ as g; g.build()" > /tmp/ab_build_old.log 2>&1
mkdir -p ab_old/distributeddataparallel_amd
(cd distributeddataparallel_amd && tar cf - --exclude=build --exclude="build_san_*" --exclude=__pycache__ --exclude=csrc .) | (cd ab_old/distributeddataparallel_amd && tar xf -)
cp bench.py ab_old/
ln -s ../tuning ab_old/tuning
restore "$@"
trap - EXIT
timeout 1800 python -c "import __graft_entry__ as g; g.build()" > /tmp/ab_build_new.log 2>&1
echo "ab_old/ = $REF of: $*"
