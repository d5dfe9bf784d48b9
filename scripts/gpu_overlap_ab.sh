#!/bin/bash
# Two-stream micro-batch overlap at micro-batch 64 (off by default since round 3: allocator pressure under the
# record_stream lifetimes) against the default and micro-batch 32 with overlap, interleaved on one box.
#   [MODEL=mamba2-280m] [ROUNDS=2] bash scripts/gpu_overlap_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/overlap
M=${MODEL:-mamba2-280m}
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in "64 off" "64 on" "32 on"; do
    set -- $c
    log=gpurun_out/overlap/${M}_b$1_$2_$r.log
    timeout -k 10 300 python bench.py --model $M --B $1 --overlap $2 --steps 3 --warmup 1 > $log 2>&1 || { tail -5 $log; exit 1; }
    echo "B=$1 overlap=$2 round $r: $(grep -o '"value": [0-9.]*\|"peak_reserved_gb": [0-9.]*\|"alloc_retries": [0-9]*' $log | tr '\n' ' ')"
  done
done
