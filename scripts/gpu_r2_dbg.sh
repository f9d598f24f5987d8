#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
timeout -k 10 300 python scripts/debug_bs.py > gpurun_out/dbg.log 2>&1; rc=$?; grep -v amdgpu gpurun_out/dbg.log | tail -8
[ $rc -ne 0 ] && exit $rc
XDDP_STEM_CONV=0 timeout -k 10 300 python scripts/debug_bs.py > gpurun_out/dbg2.log 2>&1; rc=$?; echo "-- XDDP_STEM_CONV=0"; grep -v amdgpu gpurun_out/dbg2.log | tail -8; [ $rc -ne 0 ] && exit $rc
XDDP_CONV_BN_FUSION=0 timeout -k 10 300 python scripts/debug_bs.py > gpurun_out/dbg3.log 2>&1; rc=$?; echo "-- XDDP_CONV_BN_FUSION=0"; grep -v amdgpu gpurun_out/dbg3.log | tail -8; exit $rc
