#!/bin/bash
# Serialized per-kernel table of the accumulation-1 step under the native reducer (one torchrun rank, 65,536 tokens per
# optimizer step), plus the full names of every non-framework (torch) kernel.  Output: gpurun_out/acc1t/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/acc1t
mkdir -p $O
out=$O/prof
rm -rf $out
MAMBA_AMD_WGRAD_STREAM=0 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29731 \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o k -- \
  python3 bench.py --gpus 1 --global-batch-tokens 65536 --B 64 --steps 8 --warmup 2 > $out.log 2>&1 || { tail -20 $out.log; exit 1; }
csv=$(find $out -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py $csv 10 40 > $O/table_acc1_reducer.md
python3 - "$csv" > $O/torch_kernels.txt <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "mamba_amd" not in r["Name"]:
        print(f'{int(r["Calls"]):6d} {float(r["TotalDurationNs"])/1e6:8.2f} ms  {float(r["AverageNs"])/1e3:7.1f} us  {r["Name"][:400]}')
PY
rm -rf $out
grep -o '"value": [0-9.]*' $out.log
head -3 $O/table_acc1_reducer.md
