#!/bin/bash
# call S: the two Mamba-2 2.8B @ T=8192 regressions located by bisection (89bfe90..791dcad: -13%, df8c6a7..313b536:
# -13%): HEAD with the candidate switches -- the lm_head chunk products (native, bf16-output library dW + fp32 add)
# and the non-deferred weight gradient (transient slabs on the main stream, the round-2 form) -- and 1.4B for the latter
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_envab.sh 1 "-" "MAMBA_AMD_LM_DW_F32=0" "MAMBA_AMD_LMHEAD=native" "MAMBA_AMD_WGRAD_INPLACE=0" "MAMBA_AMD_WGRAD_INPLACE=0 MAMBA_AMD_LM_DW_F32=0" -- --model mamba2-2.8b --T 8192 --B 4 --steps 2 --warmup 1 || exit 1
bash scripts/gpu_envab.sh 1 "-" "MAMBA_AMD_WGRAD_INPLACE=0" "MAMBA_AMD_LM_DW_F32=0" -- --model mamba2-1.4b --steps 3 --warmup 1 || exit 1
