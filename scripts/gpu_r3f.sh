#!/bin/bash
# call F: PMC counters of the SSD kernels at the micro-batch-64 shape (kbench --only ssd --B 64)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_ssd
cd /tmp
i=0
for cs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
          "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU" \
          "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $cs --output-format csv -d "$R/gpurun_out/pmc_ssd/p$i" -o run -- \
    python3 "$R/scripts/kbench.py" --only ssd --B 64 --reps 2 > "$R/gpurun_out/pmc_ssd/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$R/gpurun_out/pmc_ssd/p$i.log"; exit 1; }
  echo "pass $i ok"
done
