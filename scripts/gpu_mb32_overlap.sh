#!/bin/bash
# Micro-batch 32 with the two-stream micro-batch overlap (auto at 32k-token micro-batches) vs the default micro-batch
# 64 without it, re-measured on the round-5 tree, interleaved.  Output: gpurun_out/mb32/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/mb32
mkdir -p $O
run() {  # tag model B
  timeout -k 10 400 python bench.py --model $2 --B $3 --steps 3 --warmup 1 > $O/$1.log 2>&1 || { tail -20 $O/$1.log; return 1; }
  echo "$1 $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"microbatch_overlap": [a-z]*\|"peak_reserved_gb": [0-9.]*' $O/$1.log | tr '\n' ' ')"
}
run m1_b64 mamba1-280m 64 || exit 1
run m1_b32 mamba1-280m 32 || exit 1
run m2_b64 mamba2-280m 64 || exit 1
run m2_b32 mamba2-280m 32 || exit 1
run m1_b64b mamba1-280m 64 || exit 1
run m1_b32b mamba1-280m 32 || exit 1
