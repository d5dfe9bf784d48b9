#!/bin/bash
# GPU box: gemm_pipe tests, projection GEMM microbench (native tiles vs hipBLASLt), then an interleaved
# whole-step A/B of the native narrow-output projections (MAMBA_AMD_NATIVE_NARROW).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/gp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_pipe_gpu.py -m gpu \
  > gpurun_out/gp/test.log 2>&1; rc=$?; tail -3 gpurun_out/gp/test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/proj_gemm_bench.py > gpurun_out/gp/bench.log 2>&1; rc=$?
grep -v Warn gpurun_out/gp/bench.log | tail -30; [ $rc -eq 0 ] || exit $rc
[ "${AB:-1}" = "1" ] || exit 0
i=0
for n in 1 0 1 0; do
  i=$((i + 1))
  log=gpurun_out/gp/ab_${i}_narrow${n}.log
  MAMBA_AMD_NATIVE_NARROW=$n timeout -k 10 400 python bench.py --model ${MODEL:-mamba2-280m} --steps 5 --warmup 2 > $log 2>&1
  rc=$?; echo "narrow=$n: $(grep -o '"value": [0-9.]*' $log) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
