#!/bin/bash
# call Q: Mamba-2 2.8B at T=8192 (micro-batch 4) measured 46.7k tok/s at the round-2 end and 31.1k at HEAD: the same
# bench at round-2 end (1830063) and at 791dcad, 72ab514, df8c6a7 (worktrees under ab/) vs the working tree, plus the
# SSD forward / dstate packed accumulator staging (SSD tests, kbench)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_varlen_gpu.py -k "ssd or mamba2 or varlen or padded" > gpurun_out/t_q.log 2>&1; rc=$?; tail -2 gpurun_out/t_q.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/kbench.py --only ssd --B 64 --reps 20 2>&1 | grep -i "ssd" | sed "s/^/[pk-staging] /" || exit 1
for d in . ab/w_1830063 ab/w_791dcad ab/w_72ab514 ab/w_df8c6a7; do
  (cd $d && timeout -k 10 300 python -u bench.py --model mamba2-2.8b --T 8192 --B 4 --steps 2 --warmup 1) > gpurun_out/q_$(basename $d).log 2>&1 || { echo "FAILED $d"; tail -5 gpurun_out/q_$(basename $d).log; exit 1; }
  echo "[$d] $(grep -o '"value": [0-9.]*' gpurun_out/q_$(basename $d).log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/q_$(basename $d).log) $(grep -o '"peak_mem_gb": [0-9.]*' gpurun_out/q_$(basename $d).log)"
done
