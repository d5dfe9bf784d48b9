#!/bin/bash
# GPU box: GEMM engine tests + A/B microbench vs hipBLASLt (writes gpurun_out/gemm_*.log)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== gemm tests"; date
timeout -k 10 300 python -u -m pytest tests/test_gemm_pipe_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1; rc=$?
tail -15 gpurun_out/gemm_tests.log; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
echo "== gemm bench"; date
timeout -k 10 300 python -u scripts/gemm_bench.py ${GB_ARGS} > gpurun_out/gemm_bench.log 2>&1; rc=$?
cat gpurun_out/gemm_bench.log | grep -v Warning; echo "bench rc=$rc"
exit $rc
