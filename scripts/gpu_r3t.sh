#!/bin/bash
# call T: the in-place side-stream weight gradient gated on allocator headroom (auto): 2.8B @ 8192 auto vs forced
# in-place (allocator retries reported), 1.4B and 280M auto, and the GPU tests of the touched paths
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_pipe_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_t.log 2>&1; rc=$?; tail -2 gpurun_out/t_t.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_envab.sh 1 "-" "MAMBA_AMD_WGRAD_INPLACE=1" -- --model mamba2-2.8b --T 8192 --B 4 --steps 2 --warmup 1 || exit 1
bash scripts/gpu_envab.sh 1 "-" "MAMBA_AMD_WGRAD_INPLACE=0" -- --model mamba2-1.4b --steps 3 --warmup 1 || exit 1
bash scripts/gpu_envab.sh 1 "-" -- --steps 4 --warmup 2 || exit 1
