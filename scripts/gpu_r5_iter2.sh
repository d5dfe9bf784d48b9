#!/bin/bash
# Round-5 iteration: gemm tests, Mamba-1 gp_mm layout A/B (staged ring vs gemm_pipe_k), headline + Mamba-1 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_pipe_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pk_tests.log 2>&1 || { tail -30 gpurun_out/pk_tests.log; exit 1; }
tail -1 gpurun_out/pk_tests.log
timeout -k 10 300 python -u scripts/wg_bench.py --m1 --rounds 2 --reps 10 > gpurun_out/wg_m1.log 2>&1 || { tail -20 gpurun_out/wg_m1.log; exit 1; }
grep case gpurun_out/wg_m1.log
timeout -k 10 300 python bench.py --steps 6 --warmup 2 > gpurun_out/qc_bench.log 2>&1 || { tail -20 gpurun_out/qc_bench.log; exit 1; }
tail -1 gpurun_out/qc_bench.log
timeout -k 10 300 python bench.py --model mamba1-280m --steps 4 --warmup 2 > gpurun_out/qc_bench_m1.log 2>&1 || { tail -20 gpurun_out/qc_bench_m1.log; exit 1; }
tail -1 gpurun_out/qc_bench_m1.log
