#!/bin/bash
# GPU box: norm-backward partial-row grid (MAMBA_AMD_NORM_BWD_GRID) on the whole step, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/grid
i=0
for m in ${MODELS:-mamba2-280m}; do
  for k in 1 2; do
    for g in ${GRIDS:-2048 1024 768 512}; do
      i=$((i + 1)); log=gpurun_out/grid/${i}_${m}_$g.log
      MAMBA_AMD_NORM_BWD_GRID=$g timeout -k 10 500 python bench.py --model $m --steps ${STEPS:-4} --warmup 2 > $log 2>&1; rc=$?
      echo "$m grid=$g: $(grep -o '"value": [0-9.]*' $log) rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
