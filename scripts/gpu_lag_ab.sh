#!/bin/bash
# Side-stream operand keep-alive A/B on the headline bench: MAMBA_AMD_SIDE_LAG = -1 (record_stream), 4, 16, 64.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lag
for r in 1 2 3; do
  for lag in -1 16; do
    MAMBA_AMD_SIDE_LAG=$lag timeout -k 10 300 python bench.py --steps 5 --warmup 2 "$@" > gpurun_out/lag/l${lag}_$r.log 2>&1 || { tail -20 gpurun_out/lag/l${lag}_$r.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('lag', sys.argv[2], d['value'], d['config']['peak_reserved_gb'], d['config']['peak_mem_gb'])" gpurun_out/lag/l${lag}_$r.log $lag
  done
done
