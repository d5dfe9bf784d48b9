#!/bin/bash
# call I: row-chunked native lm_head + CE (GPU tests, node timing native vs hipBLASLt, whole-step A/B) and the
# Mamba-1 forward walk at 4 waves/SIMD (3-deep ring) vs the saved baseline build (ab/base_C.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "cross_entropy or lm_head or selscan or mamba1" > gpurun_out/t_i.log 2>&1; rc=$?; tail -2 gpurun_out/t_i.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/lmhead_bench.py > gpurun_out/lm_i.log 2>&1 || { tail -20 gpurun_out/lm_i.log; exit 1; }
cat gpurun_out/lm_i.log
for r in 1 2; do
  for v in base new; do
    so=""; [ $v = base ] && so="MAMBA_AMD_SO=$PWD/ab/base_C.so"
    env $so timeout -k 10 200 python -u scripts/kbench.py --only selscan --B 64 --reps 20 2>&1 | grep -i "selscan" | sed "s/^/[$v r$r] /" || exit 1
  done
done
bash scripts/gpu_envab.sh 2 "-" "MAMBA_AMD_LMHEAD=lib" -- --steps 3 --warmup 1 || exit 1
bash scripts/gpu_envab.sh 2 "-" "MAMBA_AMD_SO=$PWD/ab/base_C.so" -- --model mamba1-280m --steps 3 --warmup 1 || exit 1
