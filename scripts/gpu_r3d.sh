#!/bin/bash
# call D: padded in_proj + auto routing: GPU tests, then whole-step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "padded or headline_width or mamba2_inner or in_place or overlap_is_bitwise" > gpurun_out/t_d.log 2>&1; rc=$?; tail -2 gpurun_out/t_d.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_envab.sh 2 "-" "MAMBA_AMD_PAD_PROJ=0" "MAMBA_AMD_PROJ_GEMM=lib MAMBA_AMD_PAD_PROJ=0" -- --steps 3 --warmup 1 || exit 1
bash scripts/gpu_envab.sh 1 "-" "MAMBA_AMD_PROJ_GEMM=lib" -- --model mamba1-280m --steps 3 --warmup 1 || exit 1
