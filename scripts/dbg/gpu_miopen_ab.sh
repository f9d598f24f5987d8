cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export XDDP_NO_AUTOBUILD=1
b() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 10 > gpurun_out/ab_$tag.log 2>&1 || return 1; echo "$tag $(tail -1 gpurun_out/ab_$tag.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"; }
b base XDDP_X=1 && b nowrw MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 && b nobwd MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 && b noboth MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0
