#!/bin/bash
# Every BASELINE config on the current tree (micro-batch auto unless given), one after another; logs in gpurun_out/.
#   bash scripts/gpu_bench_all.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in mamba2-280m:auto:1024 mamba1-280m:auto:1024 mamba1-370m:auto:1024 mamba2-1.4b:auto:1024 mamba2-2.8b:4:8192; do
  IFS=: read -r m B T <<< "$c"
  echo "== $m B=$B T=$T"
  timeout -k 10 600 python bench.py --model $m --B $B --T $T --steps ${STEPS:-3} --warmup 1 > gpurun_out/bench_$m.log 2>&1; rc=$?
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"micro_batch": [0-9]*\|"peak_mem_gb": [0-9.]*\|"peak_reserved_gb": [0-9.]*' gpurun_out/bench_$m.log | tr '\n' ' '; echo
  [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$m.log; exit $rc; }
done
