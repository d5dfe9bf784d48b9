#!/bin/bash
# One GPU: the GEMM / kernel GPU tests, then the headline bench and the Mamba-1 bench (short).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gemm_pipe_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/qc_tests.log 2>&1 || { tail -30 gpurun_out/qc_tests.log; exit 1; }
tail -2 gpurun_out/qc_tests.log
timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/qc_bench.log 2>&1 || { tail -20 gpurun_out/qc_bench.log; exit 1; }
tail -1 gpurun_out/qc_bench.log
timeout -k 10 300 python bench.py --model mamba1-280m --steps 4 --warmup 2 > gpurun_out/qc_bench_m1.log 2>&1 || { tail -20 gpurun_out/qc_bench_m1.log; exit 1; }
tail -1 gpurun_out/qc_bench_m1.log
