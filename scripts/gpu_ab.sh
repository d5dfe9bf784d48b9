#!/bin/bash
# interleaved A/B of two builds of the extension on one box: scripts/gpu_ab.sh <bench args...>  (builds in ab/C_old.so, ab/C_new.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for v in old new; do
    cp ab/C_$v.so mamba_distributed_amd/_C.so
    timeout -k 10 300 python -u bench.py "$@" > gpurun_out/ab_${v}_$r.log 2>&1 || exit $?
    echo "$v $r $(grep -o '"value": [0-9.]*' gpurun_out/ab_${v}_$r.log)"
  done
done
cp ab/C_new.so mamba_distributed_amd/_C.so
