#!/bin/bash
# call V: SSD chunk backward stages its dX tile as 4-byte column pairs (acc_to_lds_pk) instead of 2-byte writes:
# SSD GPU tests, kernel A/B against the previous build (ab/base_C.so), whole-step A/B on Mamba-2 280M
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_varlen_gpu.py -m gpu -x -q -k "ssd or mamba2 or varlen or padded" --timeout 120 --timeout-method thread > gpurun_out/t_v.log 2>&1; rc=$?; tail -2 gpurun_out/t_v.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  MAMBA_AMD_SO=$PWD/ab/base_C.so timeout -k 10 200 python -u scripts/kbench.py --only ssd --B 64 > gpurun_out/kb_base_$r.log 2>&1 || { tail -5 gpurun_out/kb_base_$r.log; exit 1; }
  timeout -k 10 200 python -u scripts/kbench.py --only ssd --B 64 > gpurun_out/kb_new_$r.log 2>&1 || { tail -5 gpurun_out/kb_new_$r.log; exit 1; }
  grep -h "ssd" gpurun_out/kb_base_$r.log | sed "s/^/[base r$r] /"; grep -h "ssd" gpurun_out/kb_new_$r.log | sed "s/^/[new r$r] /"
done
bash scripts/gpu_envab.sh 2 "-" "MAMBA_AMD_SO=$PWD/ab/base_C.so" -- --steps 4 --warmup 2 || exit 1
