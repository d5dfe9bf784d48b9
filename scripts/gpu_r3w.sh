#!/bin/bash
# call W: decode at batch 1 / 16 (scripts/bench_decode.py) and its kernel table at batch 16
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/bench_decode.py > gpurun_out/dec_w.jsonl 2> gpurun_out/dec_w.err || { tail -5 gpurun_out/dec_w.err; exit 1; }
cat gpurun_out/dec_w.jsonl
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_dec" -o dec --output-format csv -- python3 "$R/scripts/bench_decode.py" --batch 16 --tokens 64 > "$R/gpurun_out/prof_dec.log" 2>&1 || { tail -5 "$R/gpurun_out/prof_dec.log"; exit 1; }
head -25 "$R/gpurun_out/prof_dec/dec_kernel_stats.csv" | cut -d, -f1-5 | cut -c1-200
