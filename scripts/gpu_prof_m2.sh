#!/bin/bash
# Serialized kernel profile of the Mamba-1 280M training step (no overlap, no side stream: clean durations)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
MAMBA_AMD_WGRAD_STREAM=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_m2" -o m2 --output-format csv -- python3 "$R/bench.py" --model mamba2-280m --steps 2 --warmup 1 --no-overlap > "$R/gpurun_out/prof_m2.log" 2>&1
echo "rc=$?"; tail -2 "$R/gpurun_out/prof_m2.log"
