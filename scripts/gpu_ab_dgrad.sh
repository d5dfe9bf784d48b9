#!/bin/bash
# Interleaved whole-step A/B of the native short-K dgrad (MAMBA_AMD_NATIVE_DGRAD) on the headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in 1 0 1 0; do  # 1 = native dgrad (opt-in)
  echo "== MAMBA_AMD_NATIVE_DGRAD=$v"
  MAMBA_AMD_NATIVE_DGRAD=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 2>/dev/null | tail -1 | cut -c1-200 || exit 1
done
