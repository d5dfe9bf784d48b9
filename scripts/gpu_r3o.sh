#!/bin/bash
# call O: persistent GEMM with three A slots (256 x 192 tiles) and the epilogue's LDS staging through asm DS ops
# (no vmcnt(0) drain of the next tile's DMAs) vs MAMBA_AMD_PK3=0 (two-buffer walk, same epilogue fix) vs HEAD
# (ab/base_C.so): GEMM tests, isolated timings at 64k tokens, whole Mamba-2 280M step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_pipe_gpu.py > gpurun_out/t_o.log 2>&1; rc=$?; tail -2 gpurun_out/t_o.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "proj or padded or mamba2 or lm_head or model" > gpurun_out/t_o2.log 2>&1; rc=$?; tail -2 gpurun_out/t_o2.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in pk3 pk2 base; do
    e=""; [ $v = pk2 ] && e="MAMBA_AMD_PK3=0"; [ $v = base ] && e="MAMBA_AMD_SO=$PWD/ab/base_C.so"
    env $e timeout -k 10 200 python -u scripts/pk_bench.py --M 65536 --rounds 1 --only in_fwd_pad,in_dgrad_pad,out_fwd,out_dgrad --no-wgrad 2>&1 | grep case | sed "s/^/[$v r$r] /" | sed 's/"rel_err[^,]*, "rel_err_rowscale[^,]*, //; s/, "gp_mm_us.*}/}/' || exit 1
  done
done
bash scripts/gpu_envab.sh 2 "-" "MAMBA_AMD_PK3=0" "MAMBA_AMD_SO=$PWD/ab/base_C.so" -- --steps 3 --warmup 1 || exit 1
