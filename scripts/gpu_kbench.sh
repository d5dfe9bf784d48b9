#!/bin/bash
# quick kernel iteration: selected GPU tests + op microbenchmarks
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python scripts/kbench.py ${KB_ARGS} 2>&1 | grep -v Warn | tee gpurun_out/kbench.log; exit ${PIPESTATUS[0]}
