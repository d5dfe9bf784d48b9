#!/bin/bash
# GPU box: kernel tests -> op microbench -> 1-GPU bench (tuned GEMM table).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest -m gpu"; date
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
echo "== kbench"; date
timeout -k 10 600 python scripts/kbench.py ${KB_ARGS} > gpurun_out/kbench.log 2>&1; rc=$?
grep -v Warn gpurun_out/kbench.log | tail -20; [ $rc -eq 0 ] || exit $rc
[ "${BENCH:-1}" = "1" ] || exit 0
echo "== bench"; date
timeout -k 10 600 python bench.py --steps ${STEPS:-3} --warmup 1 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; rc=$?
grep metric gpurun_out/bench.log; exit $rc
