#!/bin/bash
# call Y: decode out_proj GEMV time vs batch rows (event-timed loop and rocprofv3 kernel durations)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/dec_kbench.py || exit 1
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d "$R/gpurun_out/prof_deck" -o dk --output-format csv -- python3 "$R/scripts/dec_kbench.py" > "$R/gpurun_out/prof_deck.log" 2>&1 || { tail -5 "$R/gpurun_out/prof_deck.log"; exit 1; }
echo done
