#!/bin/bash
# round 3 session 3, call A: projection routing A/B at the default micro-batch (64) + serialized kernel table
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_envab.sh 2 "-" "MAMBA_AMD_PROJ_GEMM=auto" -- --steps 3 --warmup 1 || exit 1
cd /tmp
MAMBA_AMD_WGRAD_STREAM=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_m2b64" -o m2 --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 > "$R/gpurun_out/prof_m2b64.log" 2>&1
echo "rc=$?"; tail -2 "$R/gpurun_out/prof_m2b64.log"
