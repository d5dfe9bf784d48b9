#!/bin/bash
# Micro-batch 128 against 64 (one GPU, 524,288-token steps): fewer, larger micro-batches; interleaved on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/mb128
for r in 1 2; do
  for c in "mamba1-280m 64" "mamba1-280m 128" "mamba2-280m 64" "mamba2-280m 128"; do
    set -- $c
    log=gpurun_out/mb128/$1_b$2_$r.log
    timeout -k 10 400 python bench.py --model $1 --B $2 --steps 2 --warmup 1 > $log 2>&1
    echo "$1 B=$2 round $r (rc $?): $(grep -o '"value": [0-9.]*\|"peak_mem_gb": [0-9.]*\|"peak_reserved_gb": [0-9.]*\|"alloc_retries": [0-9]*\|OutOfMemory' $log | tr '\n' ' ')"
  done
done
