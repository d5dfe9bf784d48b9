#!/bin/bash
# call K: GPU suite at HEAD; whole-step A/B of HEAD vs the commit before the row-chunked lm_head (ab/prev, 2d1b5c0);
# Mamba-2 1.4B at HEAD vs the round-1 final commit (ab/r1, 4370fa4)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_k.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_k.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_tree.sh prev 2 --steps 3 --warmup 1 | sed 's/"metric.*"value"/"value"/; s/, "unit.*"peak_mem_gb"/ peak_mem_gb/' || exit 1
bash scripts/gpu_ab_tree.sh r1 2 --model mamba2-1.4b --steps 3 --warmup 1 | cut -c1-120 || exit 1
