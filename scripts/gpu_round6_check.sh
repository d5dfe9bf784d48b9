#!/bin/bash
# Round-6 tree: GPU suite + smoke + headline bench (gpu_final_check.sh), every BASELINE config, serialized kernel
# tables of the four training configs.  Stops at the first failing step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_final_check.sh || exit 1
bash scripts/gpu_bench_all.sh > gpurun_out/bench_all.txt 2>&1 || { cat gpurun_out/bench_all.txt; exit 1; }
cat gpurun_out/bench_all.txt
bash scripts/gpu_prof_tables.sh > gpurun_out/tables.txt 2>&1 || { cat gpurun_out/tables.txt; exit 1; }
cat gpurun_out/tables.txt
