#!/bin/bash
# GPU box: persistent GEMM correctness + microbenchmark + whole-step A/B of the projection engine.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pipe_gpu.py \
  > gpurun_out/r3/gemm_tests.log 2>&1 || { tail -30 gpurun_out/r3/gemm_tests.log; exit 1; }
tail -3 gpurun_out/r3/gemm_tests.log
timeout -k 10 300 python scripts/pk_bench.py --reps 20 --rounds 3 > gpurun_out/r3/pk_bench.log 2>&1 || { tail -20 gpurun_out/r3/pk_bench.log; exit 1; }
cat gpurun_out/r3/pk_bench.log
for e in lib pk lib pk; do
  MAMBA_AMD_PROJ_GEMM=$e timeout -k 10 300 python bench.py --steps 4 --warmup 2 > gpurun_out/r3/bench_$e.log 2>&1 || { tail -20 gpurun_out/r3/bench_$e.log; exit 1; }
  echo "$e $(tail -1 gpurun_out/r3/bench_$e.log | cut -c1-160)"
done
