#!/bin/bash
# Iteration loop on the GPU box: kernel tests -> bench -> rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
echo "== pytest -m gpu"; date
timeout -k 10 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
ok $rc || exit $rc
echo "== bench"; date
timeout -k 10 900 python bench.py --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$?
grep -v Warn gpurun_out/bench.log | tail -2; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
[ "${PROFILE:-1}" = "1" ] || exit 0
echo "== rocprofv3"; date
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- \
  python3 bench.py --steps 1 --warmup 1 ${BENCH_ARGS} > gpurun_out/prof_bench.log 2>&1; rc=$?
echo "prof rc=$rc"
exit $rc
