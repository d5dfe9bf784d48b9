#!/bin/bash
# GPU box: interleaved whole-step A/B over environment variants.
#   bash scripts/gpu_envab.sh <rounds> "<VAR=val ...>" "<VAR=val ...>" ... -- <bench.py args>
# A variant "-" means the default environment.  One line per run: variant, round, tok/s, peak memory.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/envab
rounds=$1; shift
variants=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do variants+=("$1"); shift; done
[ "$1" = "--" ] && shift
for r in $(seq 1 "$rounds"); do
  i=0
  for v in "${variants[@]}"; do
    i=$((i + 1))
    spec=$v; [ "$spec" = "-" ] && spec=""
    log=gpurun_out/envab/v${i}_r$r.log
    env $spec timeout -k 10 400 python -u bench.py "$@" > "$log" 2>&1 || { echo "FAILED: $v"; tail -20 "$log"; exit 1; }
    echo "[$v] r$r $(grep -o '"value": [0-9.]*' "$log") $(grep -o '"peak_mem_gb": [0-9.]*' "$log") $(grep -o '"peak_reserved_gb": [0-9.]*' "$log") $(grep -o '"alloc_retries": [0-9]*' "$log")"
  done
done
