#!/bin/bash
# Interleaved whole-step A/B: Mamba-1 280M weight gradients through deferred gemm_pipe slabs (default)
# vs gemm_wgrad_cm reduced every micro-step (MAMBA_AMD_M1_DEFER_WGRAD=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in 1 0 1 0; do
  echo "== MAMBA_AMD_M1_DEFER_WGRAD=$v"
  MAMBA_AMD_M1_DEFER_WGRAD=$v timeout -k 10 400 python bench.py --model mamba1-280m --steps 3 --warmup 1 2>/dev/null | tail -1 | cut -c1-200 || exit 1
done
