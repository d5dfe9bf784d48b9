#!/bin/bash
# call R: second bisect round of the Mamba-2 2.8B @ T=8192 regression (round-2 end 46.3k, 791dcad 39.1k, df8c6a7 38.2k,
# HEAD 34.2k on one box): the commits in between
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in ab/w_20e3c6f ab/w_f249fea ab/w_92c9f0a ab/w_89bfe90 ab/w_313b536 ab/w_5ebdde3 .; do
  (cd $d && timeout -k 10 300 python -u bench.py --model mamba2-2.8b --T 8192 --B 4 --steps 2 --warmup 1) > gpurun_out/r_$(basename $d).log 2>&1 || { echo "FAILED $d"; tail -5 gpurun_out/r_$(basename $d).log; exit 1; }
  echo "[$d] $(grep -o '"value": [0-9.]*' gpurun_out/r_$(basename $d).log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r_$(basename $d).log) $(grep -o '"peak_mem_gb": [0-9.]*' gpurun_out/r_$(basename $d).log)"
done
