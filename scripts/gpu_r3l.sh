#!/bin/bash
# call L: persistent GEMM with per-XCD tile ranges / claim counters vs one global counter (MAMBA_AMD_PK_XCD=0):
# GEMM tests, isolated timings at 64k tokens against hipBLASLt, whole-step A/B (Mamba-2 280M)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/lmhead_bench.py > gpurun_out/lm_l.log 2>&1 || { tail -20 gpurun_out/lm_l.log; exit 1; }
grep -E "chunk|fused" gpurun_out/lm_l.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_pipe_gpu.py tests/test_kernels_gpu.py -k "pk or gemm or lm_head or proj or padded" > gpurun_out/t_l.log 2>&1; rc=$?; tail -2 gpurun_out/t_l.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in xcd glob; do
    e=""; [ $v = glob ] && e="MAMBA_AMD_PK_XCD=0"
    env $e timeout -k 10 200 python -u scripts/pk_bench.py --M 65536 --rounds 1 --only in_fwd_pad,in_dgrad_pad,out_fwd,out_dgrad,lm_fwd --no-wgrad 2>&1 | grep case | sed "s/^/[$v r$r] /" || exit 1
  done
done
bash scripts/gpu_envab.sh 2 "-" "MAMBA_AMD_PK_XCD=0" -- --steps 3 --warmup 1 || exit 1
