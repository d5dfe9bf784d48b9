#!/bin/bash
# decode kernel traces at batch 1 and 16 (graph mode is the last mode bench_decode runs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp
for b in 1 16; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_dec_b$b" -o dec --output-format csv -- python3 "$R/scripts/bench_decode.py" --batch $b --tokens 64 > "$R/gpurun_out/prof_dec_b$b.log" 2>&1 || { tail -5 "$R/gpurun_out/prof_dec_b$b.log"; exit 1; }
done
cd "$R"
for b in 1 16; do python3 scripts/dec_trace_summary.py gpurun_out/prof_dec_b$b/dec_kernel_trace.csv 2000 | tee gpurun_out/dec_trace_b$b.txt; rm -rf gpurun_out/prof_dec_b$b; done
