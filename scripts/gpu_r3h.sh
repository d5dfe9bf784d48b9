#!/bin/bash
# call H (re-entry baseline at HEAD): GPU suite, smoke, default bench, serialized kernel tables of Mamba-2 / Mamba-1 280M
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_h.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_h.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
timeout -k 10 300 python -u bench.py --steps 4 --warmup 2 > gpurun_out/bench_h.log 2>&1 || { tail -20 gpurun_out/bench_h.log; exit 1; }
tail -1 gpurun_out/bench_h.log
cd /tmp
MAMBA_AMD_WGRAD_STREAM=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_h2" -o m2 --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 > "$R/gpurun_out/prof_h2.log" 2>&1 || { tail -5 "$R/gpurun_out/prof_h2.log"; exit 1; }
MAMBA_AMD_WGRAD_STREAM=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_h1" -o m1 --output-format csv -- python3 "$R/bench.py" --model mamba1-280m --steps 2 --warmup 1 > "$R/gpurun_out/prof_h1.log" 2>&1 || { tail -5 "$R/gpurun_out/prof_h1.log"; exit 1; }
echo done
