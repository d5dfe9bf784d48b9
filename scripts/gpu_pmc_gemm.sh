#!/bin/bash
# L2 / memory counters of the projection GEMM engines on one shape (kernel-trace + pmc only).
#   SHAPE="65536 2048 8512" bash scripts/gpu_pmc_gemm.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
SHAPE=${SHAPE:-65536 2048 8512}
mkdir -p gpurun_out/pmcg
for eng in lib pk; do
  for ps in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_MFMA"; do
    n=$(echo $ps | cut -d' ' -f1)
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ps --output-format csv -d "$R/gpurun_out/pmcg/${eng}_$n" -o run -- \
      python3 scripts/gemm_one.py $eng $SHAPE 4 > gpurun_out/pmcg/${eng}_$n.log 2>&1 || { echo "fail $eng $n"; exit 1; }
  done
done
python3 scripts/pmc_summary.py gpurun_out/pmcg > gpurun_out/pmcg/summary.txt
echo done
