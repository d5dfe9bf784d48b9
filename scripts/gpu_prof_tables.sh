#!/bin/bash
# Serialized (side stream off) rocprofv3 kernel tables of the BASELINE configs on the current tree.
#   [CONFIGS="mamba2-280m:64:1024 ..."] bash scripts/gpu_prof_tables.sh
# Output: gpurun_out/tables/<model>.md (unit = one micro-batch: (steps + warmup) x accumulation micro-batches).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp MAMBA_AMD_WGRAD_STREAM=0
mkdir -p gpurun_out/tables
sha=$(cat .git_head 2>/dev/null || echo tree)
for c in ${CONFIGS:-mamba2-280m:64:1024 mamba1-280m:64:1024 mamba2-1.4b:32:1024 mamba2-2.8b:4:8192}; do
  IFS=: read -r m B T <<< "$c"
  out=$R/gpurun_out/tables/$m
  rm -rf $out
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o k -- \
    python3 bench.py --model $m --B $B --T $T --steps 2 --warmup 1 > $out.log 2>&1 || { tail -20 $out.log; exit 1; }
  acc=$(( 524288 / (B * T) ))
  csv=$(find $out -name "*kernel_stats.csv" | head -1)
  { echo "# $m, micro-batch $B, T=$T, serialized (MAMBA_AMD_WGRAD_STREAM=0), rocprofv3 --kernel-trace --stats, 3 steps x $acc micro-batches"
    python3 scripts/prof_summary.py $csv $(( 3 * acc )) 32; } > $out.md
  grep -o '"value": [0-9.]*' $out.log
  head -3 $out.md | tail -1
  rm -rf $out
done
