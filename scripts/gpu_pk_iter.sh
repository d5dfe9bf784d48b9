#!/bin/bash
# Persistent / staged-ring GEMM iteration on one GPU: the gemm GPU tests, then the persistent-engine A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_pipe_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pk_tests.log 2>&1 || { tail -30 gpurun_out/pk_tests.log; exit 1; }
tail -2 gpurun_out/pk_tests.log
timeout -k 10 500 python -u scripts/pk_bench.py --M 65536 --no-wgrad --rounds 2 --reps 10 "$@" > gpurun_out/pk_bench.log 2>&1 || { tail -20 gpurun_out/pk_bench.log; exit 1; }
grep case gpurun_out/pk_bench.log
