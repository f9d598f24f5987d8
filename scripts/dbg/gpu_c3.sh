cd "${GRAFT_REPO_ROOT}"; mkdir -p gpurun_out; export XDDP_NO_AUTOBUILD=1
for t in ${C3_TILES:-0 1 2 3}; do
  echo "== tile $t"; XDDP_C3_TILE=$t timeout -k 10 240 python scripts/conv3x3_bench.py > gpurun_out/c3_$t.log 2>&1 || { tail -20 gpurun_out/c3_$t.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/c3_$t.log | tail -8 | sed -e 's/.*||/||/' -e 's/^\(C[0-9]*->[0-9]* [0-9x]* s[12]\).*||/\1 ||/'
done
