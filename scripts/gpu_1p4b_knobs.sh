#!/bin/bash
# Mamba-2 1.4B scheduling knobs re-measured on the round-5 tree: default (no micro-batch overlap, micro-batch 32),
# the two-stream overlap forced on, and micro-batch 16.  Output: gpurun_out/k14/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/k14
mkdir -p $O
run() {  # tag args...
  local tag=$1; shift
  timeout -k 10 400 python bench.py --model mamba2-1.4b --steps 2 --warmup 1 "$@" > $O/$tag.log 2>&1 \
    || { tail -20 $O/$tag.log; return 1; }
  echo "$tag $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_reserved_gb": [0-9.]*\|"alloc_retries": [0-9]*' $O/$tag.log | tr '\n' ' ')"
}
run default || exit 1
run overlap_on --overlap on || exit 1
run b16 --B 16 || exit 1
run default2 || exit 1
