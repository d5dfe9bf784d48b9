#!/bin/bash
# call U: the in-place side-stream weight gradient gated on the allocated peak (< 70% of the device) and on
# allocator retries: 1.4B auto vs forced slabs (two interleaved rounds), 2.8B @ 8192 auto
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_envab.sh 2 "-" "MAMBA_AMD_WGRAD_INPLACE=0" -- --model mamba2-1.4b --steps 3 --warmup 1 || exit 1
bash scripts/gpu_envab.sh 1 "-" -- --model mamba2-2.8b --T 8192 --B 4 --steps 2 --warmup 1 || exit 1
