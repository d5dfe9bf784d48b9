#!/bin/bash
# SSD forward: 2-deep prefetch (current build) vs ab/_C_ssd1.so; SSD GPU tests first
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_varlen_gpu.py -k "ssd or mamba2 or split_conv1d or chunk_scan or packed" > gpurun_out/ssd_tests.log 2>&1 || { tail -30 gpurun_out/ssd_tests.log; exit 1; }
tail -1 gpurun_out/ssd_tests.log
for so in mamba_distributed_amd/_C.so ab/_C_ssd1.so mamba_distributed_amd/_C.so ab/_C_ssd1.so; do
  echo "== $so"; MAMBA_AMD_SO=$so timeout -k 10 120 python scripts/kbench.py --only ssd --reps 30 2>&1 | grep ssd_ || exit 1
done
