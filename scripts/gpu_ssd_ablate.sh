#!/bin/bash
# Per-kernel times of the SSD kernels under MAMBA_AMD_SSD_ABLATE bit masks (profiling only: the
# ablated runs compute wrong results).   ABL="0 1 2 4" bash scripts/gpu_ssd_ablate.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
for m in ${ABL:-0 1 2 4}; do
  MAMBA_AMD_SSD_ABLATE=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/abl/m$m -o run -- python3 scripts/kbench.py --only ssd --reps 10 > gpurun_out/abl/m$m.log 2>&1 || exit 1
  f=$(find gpurun_out/abl/m$m -name "*kernel_stats.csv" | head -1)
  echo "== ablate $m"; python scripts/prof_summary.py "$f" 1 8 | grep -E "ssd_chunk_bwd|ssd_dstate|ssd_fused"
done
