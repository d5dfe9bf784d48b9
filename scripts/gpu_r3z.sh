#!/bin/bash
# call Z: full GPU suite, smoke and the default bench at HEAD
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/z
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/z/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/z/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/z/smoke.log 2>&1 || { tail -5 gpurun_out/z/smoke.log; exit 1; }
tail -1 gpurun_out/z/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/z/bench.log 2>&1 || { tail -20 gpurun_out/z/bench.log; exit 1; }
tail -1 gpurun_out/z/bench.log
