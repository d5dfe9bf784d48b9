#!/bin/bash
# call B: persistent GEMM 256x192 tiles -- tests, then isolated timings vs hipBLASLt at the 64 x 1024-token micro-batch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_pipe_gpu.py -k pk > gpurun_out/t_pk.log 2>&1; rc=$?; tail -2 gpurun_out/t_pk.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/pk_bench.py --M 65536 --reps 10 --rounds 3 2>&1 | grep -v amdgpu.ids
