#!/bin/bash
# The 8-GPU per-rank regime on one GPU: accumulation 1 (65,536 tokens per optimizer step) vs the headline
# accumulation 8, then a serialized kernel table of the accumulation-1 step (per-step extras: AdamW, casts,
# transposes, column sums, reductions).  Output: gpurun_out/accum1/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/accum1
timeout -k 10 300 python bench.py --B 64 --steps 3 --warmup 1 > gpurun_out/accum1/acc8.log 2>&1 || { tail -5 gpurun_out/accum1/acc8.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/accum1/acc8.log | tr '\n' ' '; echo " <- accum 8"
timeout -k 10 300 python bench.py --B 64 --global-batch-tokens 65536 --steps 24 --warmup 3 > gpurun_out/accum1/acc1.log 2>&1 || { tail -5 gpurun_out/accum1/acc1.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/accum1/acc1.log | tr '\n' ' '; echo " <- accum 1"
out=$R/gpurun_out/accum1/prof
rm -rf $out
MAMBA_AMD_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o k -- \
  python3 bench.py --B 64 --global-batch-tokens 65536 --steps 8 --warmup 2 > $out.log 2>&1 || { tail -20 $out.log; exit 1; }
csv=$(find $out -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py $csv 10 45 > gpurun_out/accum1/table_acc1.md
rm -rf $out
grep -o '"value": [0-9.]*' $out.log
head -2 gpurun_out/accum1/table_acc1.md
