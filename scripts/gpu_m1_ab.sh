#!/bin/bash
# Mamba-1 280M whole-step A/B: sequential vs time-parallel selective-scan backward; then PMC of the kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for sg in 1 0 1 0; do
  echo "== BWD_SG=$sg"
  MAMBA_AMD_SELSCAN_BWD_SG=$sg timeout -k 10 400 python bench.py --model mamba1-280m --steps 3 --warmup 1 > gpurun_out/m1ab_$sg.log 2>&1 || { tail -5 gpurun_out/m1ab_$sg.log; exit 1; }
  grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/m1ab_$sg.log | tr '\n' ' '; echo
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_ss" -o pmc -- python3 "$GRAFT_REPO_ROOT/scripts/kbench.py" --only selscan --reps 3 > "$GRAFT_REPO_ROOT/gpurun_out/pmc_ss.log" 2>&1
echo "pmc rc=$?"
