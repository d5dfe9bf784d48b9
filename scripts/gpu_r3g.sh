#!/bin/bash
# call G: bandwidth-kernel tuning (conv time tiles 64, gated-norm fwd 2 rows/wave, add-norm bwd early loads)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "norm or conv or mamba2_inner or native_vs_reference or varlen" > gpurun_out/t_g.log 2>&1; rc=$?; tail -2 gpurun_out/t_g.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_varlen_gpu.py > gpurun_out/t_g2.log 2>&1; rc=$?; tail -1 gpurun_out/t_g2.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in base new; do
    so=""; [ $v = base ] && so="MAMBA_AMD_SO=$PWD/ab/base_C.so"
    env $so timeout -k 10 200 python -u scripts/kbench.py --only conv,gnorm,norm --B 64 --reps 20 2>&1 | grep -E "conv|gated|norm" | sed "s/^/[$v r$r] /" || exit 1
  done
done
bash scripts/gpu_envab.sh 2 "-" "MAMBA_AMD_SO=$PWD/ab/base_C.so" -- --steps 3 --warmup 1 || exit 1
