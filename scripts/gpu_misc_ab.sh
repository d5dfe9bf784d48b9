#!/bin/bash
# GPU box: quick interleaved A/Bs -- Mamba-1 280M micro-batch overlap on/off; norm-backward partial-row grid.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/misc
i=0
run() {  # label, env assignment or -, bench args...
  local lab=$1 e=$2; shift 2
  i=$((i + 1)); local log=gpurun_out/misc/${i}_$lab.log
  if [ "$e" = - ]; then timeout -k 10 400 python bench.py "$@" > $log 2>&1; else env $e timeout -k 10 400 python bench.py "$@" > $log 2>&1; fi
  local rc=$?; echo "$lab: $(grep -o '"value": [0-9.]*' $log) rc=$rc"; return $rc
}
for k in 1 2; do
  run m1_overlap_on - --model mamba1-280m --overlap on --steps 3 --warmup 1 || exit 1
  run m1_overlap_off - --model mamba1-280m --overlap off --steps 3 --warmup 1 || exit 1
done
for k in 1 2; do
  run m2_grid_default - --steps 4 --warmup 2 || exit 1
  run m2_grid_1024 MAMBA_AMD_NORM_BWD_GRID=1024 --steps 4 --warmup 2 || exit 1
  run m2_grid_4096 MAMBA_AMD_NORM_BWD_GRID=4096 --steps 4 --warmup 2 || exit 1
done
