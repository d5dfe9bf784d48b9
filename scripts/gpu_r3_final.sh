#!/bin/bash
# round-3 final check at HEAD on one MI355X: GPU suite, smoke, every README config, serialized Mamba-2 280M kernel table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/final/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -5 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
run() {  # name, bench args
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/final/bench_$n.log 2>&1 || { echo "FAILED $n"; tail -20 gpurun_out/final/bench_$n.log; exit 1; }
  echo "[$n $*] $(grep -o '"value": [0-9.]*' gpurun_out/final/bench_$n.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/final/bench_$n.log) $(grep -o '"peak_mem_gb": [0-9.]*' gpurun_out/final/bench_$n.log)"
}
run mamba2-280m --steps 5 --warmup 2 || exit 1
run mamba2-280m-rank8 --global-batch-tokens 65536 --steps 8 --warmup 3 || exit 1
run mamba1-280m --model mamba1-280m --steps 4 --warmup 2 || exit 1
run mamba1-370m --model mamba1-370m --steps 3 --warmup 1 || exit 1
run mamba2-1.4b --model mamba2-1.4b --steps 3 --warmup 1 || exit 1
run mamba2-2.8b-8k --model mamba2-2.8b --T 8192 --B 4 --steps 2 --warmup 1 || exit 1
cd /tmp
MAMBA_AMD_WGRAD_STREAM=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/final/prof_m2" -o m2 --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 > "$R/gpurun_out/final/prof_m2.log" 2>&1 || { tail -5 "$R/gpurun_out/final/prof_m2.log"; exit 1; }
echo done
