#!/bin/bash
# Weight-gradient GEMM study on one GPU: timings of the split-K XC . XC engine against hipBLASLt and the old
# native kernel at 64k tokens, then PMC passes (kernel-trace + pmc only) over the same products.
#   bash scripts/gpu_wgrad_study.sh [only-list]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ONLY=${1:-in_wgrad,out_wgrad,in_fwd}
timeout -k 10 300 python -u scripts/gemm_bench.py --T 65536 --only "$ONLY" --reps 10 --rounds 2 > gpurun_out/wg_time.log 2>&1 \
  || { tail -20 gpurun_out/wg_time.log; exit 1; }
cat gpurun_out/wg_time.log
PMC_CMD="scripts/gemm_bench.py --T 65536 --only $ONLY --reps 2 --rounds 1" bash scripts/gpu_pmc.sh > gpurun_out/wg_pmc.log 2>&1 \
  || { tail -20 gpurun_out/wg_pmc.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc mamba_amd > gpurun_out/wg_pmc_summary.txt
rm -rf gpurun_out/pmc/p*/   # raw csv: the summary is what is kept
cat gpurun_out/wg_pmc_summary.txt
