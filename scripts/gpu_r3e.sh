#!/bin/bash
# call E: SSD forward with two chunks of operand lookahead vs the saved baseline build (ab/base_C.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "ssd or mamba2_inner or padded" > gpurun_out/t_e.log 2>&1; rc=$?; tail -2 gpurun_out/t_e.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in base new; do
    so=""; [ $v = base ] && so="MAMBA_AMD_SO=$PWD/ab/base_C.so"
    env $so timeout -k 10 200 python -u scripts/kbench.py --only ssd --B 64 --reps 20 2>&1 | grep -i "ssd" | sed "s/^/[$v r$r] /" || exit 1
  done
done
bash scripts/gpu_envab.sh 2 "-" "MAMBA_AMD_SO=$PWD/ab/base_C.so" -- --steps 3 --warmup 1 || exit 1
