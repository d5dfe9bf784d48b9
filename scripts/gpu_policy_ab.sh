#!/bin/bash
# GPU box: policy A/Bs by model (env switch on/off, interleaved): CASES="model:VAR ..."
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/policy
i=0
for c in ${CASES:-mamba2-1.4b:MAMBA_AMD_WGRAD_STREAM mamba1-280m:MAMBA_AMD_WGRAD_STREAM}; do
  IFS=: read -r m var <<< "$c"
  for v in 1 0 1 0; do
    i=$((i + 1)); log=gpurun_out/policy/${i}_${m}_${var}_$v.log
    env $var=$v timeout -k 10 500 python bench.py --model $m --steps 3 --warmup 1 > $log 2>&1; rc=$?
    echo "$m $var=$v: $(grep -o '"value": [0-9.]*' $log) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
