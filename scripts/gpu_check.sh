#!/bin/bash
# GPU validation pass for gpurun: kernel tests -> smoke -> short bench.  Stops at the first
# crash / timeout (exit codes other than 0 = pass, 1 = test failures).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-3}
WARM=${WARM:-1}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
echo "== pytest -m gpu"; date
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -40 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
ok $rc || exit $rc
echo "== smoke"; date
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
cat gpurun_out/smoke.log | tail -5; echo "smoke rc=$rc"
[ $rc -eq 0 ] || exit $rc
echo "== bench"; date
timeout -k 10 900 python bench.py --steps $STEPS --warmup $WARM > gpurun_out/bench.log 2>&1; rc=$?
tail -5 gpurun_out/bench.log; echo "bench rc=$rc"
exit $rc
