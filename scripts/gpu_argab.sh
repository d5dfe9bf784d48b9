#!/bin/bash
# GPU box: interleaved whole-step A/B over bench.py argument variants.
#   bash scripts/gpu_argab.sh <rounds> "<args variant 1>" "<args variant 2>" ...
# A variant may start with "@<dir>" to run bench.py from another built tree (e.g. @ab/r1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
root=$PWD
mkdir -p gpurun_out/argab
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    dir=$root; args=$v
    if [ "${v#@}" != "$v" ]; then dir=$root/${v%% *}; dir=${dir/@/}; args=${v#* }; fi
    log=$root/gpurun_out/argab/v${i}_r$r.log
    (cd "$dir" && timeout -k 10 600 python -u bench.py $args) > "$log" 2>&1 || { echo "FAILED: $v"; tail -20 "$log"; exit 1; }
    echo "[$v] r$r $(grep -o '"value": [0-9.]*' "$log") $(grep -o '"ms_per_step": [0-9.]*' "$log") $(grep -o '"peak_mem_gb": [0-9.]*' "$log")"
  done
done
