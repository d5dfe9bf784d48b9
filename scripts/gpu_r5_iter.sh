#!/bin/bash
# Round-5 iteration on one GPU: gemm GPU tests, persistent-engine ring A/B, SSD kernel A/B vs ab/h (HEAD build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_pipe_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pk_tests.log 2>&1 || { tail -30 gpurun_out/pk_tests.log; exit 1; }
tail -2 gpurun_out/pk_tests.log
timeout -k 10 400 python -u scripts/pk_bench.py --M 65536 --no-wgrad --rounds 2 --reps 10 \
  --only out_fwd,out_dgrad,in_fwd_pad,in_dgrad_pad,lm_fwd > gpurun_out/pk_bench.log 2>&1 || { tail -20 gpurun_out/pk_bench.log; exit 1; }
grep case gpurun_out/pk_bench.log
KFILTER=ssd bash scripts/gpu_kstats_ab.sh h 2 scripts/kbench.py --only ssd --B 64 --reps 5 > gpurun_out/ssd_ab.log 2>&1 || { tail -20 gpurun_out/ssd_ab.log; exit 1; }
cat gpurun_out/ssd_ab.log
