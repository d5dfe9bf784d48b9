#!/bin/bash
# call M: Mamba-1 forward walk with B / C staged in LDS (wave-uniform float4 reads instead of v_readlane + SALU
# unpacking) vs HEAD (ab/base_C.so): selective-scan GPU tests, kbench, whole Mamba-1 280M step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_properties.py -k "selscan or selective or mamba1 or Mamba1" > gpurun_out/t_m.log 2>&1; rc=$?; tail -2 gpurun_out/t_m.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in base new; do
    so=""; [ $v = base ] && so="MAMBA_AMD_SO=$PWD/ab/base_C.so"
    env $so timeout -k 10 200 python -u scripts/kbench.py --only selscan --B 64 --reps 20 2>&1 | grep -i "selscan" | sed "s/^/[$v r$r] /" || exit 1
  done
done
bash scripts/gpu_envab.sh 2 "-" "MAMBA_AMD_SO=$PWD/ab/base_C.so" -- --model mamba1-280m --steps 3 --warmup 1 || exit 1
