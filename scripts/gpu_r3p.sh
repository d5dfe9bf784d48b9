#!/bin/bash
# call P: persistent GEMM 256 x 192 walk with B staged through VGPRs (LDS-DMA only for A) -- GEMM tests, isolated
# timings at 64k tokens (default tile choice, 256 x 192 forced, HEAD build), whole Mamba-2 280M step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_pipe_gpu.py > gpurun_out/t_p.log 2>&1; rc=$?; tail -2 gpurun_out/t_p.log; [ $rc -eq 0 ] || exit $rc
MAMBA_AMD_PK_TILE=192 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_pipe_gpu.py -k pk > gpurun_out/t_p2.log 2>&1; rc=$?; tail -2 gpurun_out/t_p2.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in t192 dflt base; do
    e=""; [ $v = t192 ] && e="MAMBA_AMD_PK_TILE=192"; [ $v = base ] && e="MAMBA_AMD_SO=$PWD/ab/base_C.so"
    env $e timeout -k 10 200 python -u scripts/pk_bench.py --M 65536 --rounds 1 --only in_fwd_pad,in_dgrad_pad,out_fwd,out_dgrad --no-wgrad 2>&1 | grep case | sed "s/^/[$v r$r] /" | sed 's/"rel_err[^,]*, "rel_err_rowscale[^,]*, //; s/, "gp_mm_us.*}/}/' || exit 1
  done
done
