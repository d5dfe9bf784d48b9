#!/bin/bash
# call P: (1) persistent GEMM 256 x 192 walk with B staged through VGPRs (LDS-DMA only for A): GEMM tests,
# isolated timings at 64k tokens (default tile choice, 256 x 192 forced, HEAD build); (2) the padded in_proj
# gradient's pad columns zeroed inside the SSD chunk backward (no separate fill); (3) the dt cumsum kernel as one
# workgroup per (b, chunk) with coalesced dt staging (kbench vs ab/pre_cumsum_C.so); whole Mamba-2 step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_pipe_gpu.py > gpurun_out/t_p.log 2>&1; rc=$?; tail -2 gpurun_out/t_p.log; [ $rc -eq 0 ] || exit $rc
MAMBA_AMD_PK_TILE=192 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_pipe_gpu.py -k pk > gpurun_out/t_p2.log 2>&1; rc=$?; tail -2 gpurun_out/t_p2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_varlen_gpu.py -k "padded or mamba2 or ssd or varlen" > gpurun_out/t_p3.log 2>&1; rc=$?; tail -2 gpurun_out/t_p3.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in t192 dflt base; do
    e=""; [ $v = t192 ] && e="MAMBA_AMD_PK_TILE=192"; [ $v = base ] && e="MAMBA_AMD_SO=$PWD/ab/base_C.so"
    env $e timeout -k 10 200 python -u scripts/pk_bench.py --M 65536 --rounds 1 --only in_fwd_pad,in_dgrad_pad,out_fwd,out_dgrad --no-wgrad 2>&1 | grep case | sed "s/^/[$v r$r] /" | sed 's/"rel_err[^,]*, "rel_err_rowscale[^,]*, //; s/, "gp_mm_us.*}/}/' || exit 1
  done
done
for r in 1 2; do
  for v in pre new; do
    so=""; [ $v = pre ] && so="MAMBA_AMD_SO=$PWD/ab/pre_cumsum_C.so"
    env $so timeout -k 10 200 python -u scripts/kbench.py --only ssd --B 64 --reps 20 2>&1 | grep -i "ssd" | sed "s/^/[cumsum $v r$r] /" || exit 1
  done
done
bash scripts/gpu_envab.sh 2 "-" "MAMBA_AMD_PK_TILE=192" "MAMBA_AMD_SO=$PWD/ab/pre_cumsum_C.so" -- --steps 3 --warmup 1 || exit 1
