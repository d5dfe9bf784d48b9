#!/bin/bash
# SSD kernels: correctness (GPU tests), A/B of the walk decomposition vs the sequential kernels, and a
# per-kernel rocprofv3 breakdown of the default path.   bash scripts/gpu_ssd_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ssd
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_varlen_gpu.py -k "ssd or mamba2_inner or split or packed or model_native or context_parallel" \
  > gpurun_out/ssd/tests.log 2>&1 || { tail -30 gpurun_out/ssd/tests.log; exit 1; }
tail -1 gpurun_out/ssd/tests.log
for walk in 0 1 2 3 0 2; do
  echo "== MAMBA_AMD_SSD_WALK=$walk"
  MAMBA_AMD_SSD_WALK=$walk timeout -k 10 100 python scripts/kbench.py --only ssd --reps 30 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ssd/prof -o run -- python3 scripts/kbench.py --only ssd --reps 10 \
  > gpurun_out/ssd/prof.log 2>&1 || exit 1
f=$(find gpurun_out/ssd/prof -name "*kernel_stats.csv" | head -1); python scripts/prof_summary.py "$f" 1 12
