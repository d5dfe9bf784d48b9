#!/bin/bash
# PMC counter passes over the op microbenchmark (kernel-trace + pmc only; no sys/runtime traces).
#   KB_ARGS="--only ssd --reps 2" bash scripts/gpu_pmc.sh
#   PMC_CMD="scripts/gemm_bench.py --only in_fwd --reps 3 --rounds 1" bash scripts/gpu_pmc.sh   (any script)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || { echo "list failed"; exit 1; }
have() { grep -qw "$1" gpurun_out/pmc/counters.txt; }
pass() {  # name counters...
  local name=$1; shift; local cs=()
  for c in "$@"; do have "$c" && cs+=("$c") || echo "skip $c"; done
  [ ${#cs[@]} -gt 0 ] || return 0
  echo "== pass $name: ${cs[*]}"; date
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "${cs[@]}" --output-format csv -d "$R/gpurun_out/pmc/$name" -o run -- \
    python3 ${PMC_CMD:-scripts/kbench.py ${KB_ARGS}} > gpurun_out/pmc/$name.log 2>&1
}
pass p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit $?
pass p2 SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_IDX_ACTIVE || exit $?
pass p3 FETCH_SIZE || exit $?
pass p4 WRITE_SIZE TCC_HIT_sum TCC_MISS_sum || exit $?
pass p5 SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT GRBM_GUI_ACTIVE || exit $?
echo done
