#!/bin/bash
# rocprofv3 kernel trace + stats of the headline bench (1 timed step).  Output: gpurun_out/prof/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
STEPS=${STEPS:-1}
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- \
  python3 bench.py --steps $STEPS --warmup 1 ${BENCH_ARGS} > gpurun_out/prof_bench.log 2>&1
rc=$?
tail -3 gpurun_out/prof_bench.log
find gpurun_out/prof -name "*stats*" | head
exit $rc
