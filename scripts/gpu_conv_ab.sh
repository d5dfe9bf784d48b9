#!/bin/bash
# channel-last conv: current build vs ab/_C_conv1.so (kernel A/B), conv GPU tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_varlen_gpu.py -k "conv" > gpurun_out/conv_tests.log 2>&1 || { tail -30 gpurun_out/conv_tests.log; exit 1; }
tail -2 gpurun_out/conv_tests.log
for so in mamba_distributed_amd/_C.so ab/_C_conv1.so mamba_distributed_amd/_C.so ab/_C_conv1.so; do
  echo "== $so"; MAMBA_AMD_SO=$so timeout -k 10 120 python scripts/kbench.py --only conv --reps 30 2>&1 | grep conv_ || exit 1
done
