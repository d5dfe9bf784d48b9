#!/bin/bash
# GPU box: tests -> op microbench -> bench -> rocprofv3 kernel stats -> decode bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
echo "== pytest -m gpu"; date
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -6 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
echo "== kbench"; date
timeout -k 10 600 python scripts/kbench.py --only ${KB_ONLY:-ssd,conv,gnorm,norm} > gpurun_out/kbench.log 2>&1 || exit $?
grep -v Warn gpurun_out/kbench.log | tail -12
echo "== bench"; date
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1 || exit $?
grep metric gpurun_out/bench.log
echo "== rocprofv3"; date
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- \
  python3 bench.py --steps 1 --warmup 1 > gpurun_out/prof_bench.log 2>&1 || exit $?
echo "== decode"; date
timeout -k 10 600 python scripts/bench_decode.py > gpurun_out/decode.log 2>&1; rc=$?
cat gpurun_out/decode.log | grep '{'; exit $rc
