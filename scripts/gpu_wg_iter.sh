#!/bin/bash
# Weight-gradient engine iteration on one GPU: its GPU tests, then the engine A/B (scripts/wg_bench.py).
#   bash scripts/gpu_wg_iter.sh [wg_bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_pipe_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "wg or xc or fp32_modes or headline" > gpurun_out/wg_tests.log 2>&1 || { tail -30 gpurun_out/wg_tests.log; exit 1; }
tail -2 gpurun_out/wg_tests.log
timeout -k 10 400 python -u scripts/wg_bench.py "$@" > gpurun_out/wg_bench.log 2>&1 || { tail -20 gpurun_out/wg_bench.log; exit 1; }
cat gpurun_out/wg_bench.log
