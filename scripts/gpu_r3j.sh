#!/bin/bash
# call J: lm_head per-product timings at a 16384-row chunk; PMC counters of the persistent GEMM vs hipBLASLt at the
# two long-K projection shapes still on the library (out_proj fwd K=1536, padded in_proj dgrad K=3392), 64k tokens
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/lmhead_bench.py > gpurun_out/lm_j.log 2>&1 || { tail -20 gpurun_out/lm_j.log; exit 1; }
cat gpurun_out/lm_j.log
PMC_CMD="scripts/pk_bench.py --only out_fwd,in_dgrad_pad --M 65536 --reps 3 --rounds 1" timeout -k 10 600 bash scripts/gpu_pmc.sh || exit 1
python3 scripts/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_j.txt 2>&1; head -100 gpurun_out/pmc_j.txt
