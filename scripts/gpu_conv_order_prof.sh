#!/bin/bash
# In-step kernel times of the Mamba-1 280M step (serialized tables) with the channel-first conv rows in b-major (0)
# and memory (1) order.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for co in 0 1; do
  MAMBA_AMD_CONV_CF_ORDER=$co CONFIGS="mamba1-280m:64:1024" bash scripts/gpu_prof_tables.sh || exit 1
  mv gpurun_out/tables/mamba1-280m.md gpurun_out/tables/m1_order$co.md
  echo "== order $co"; grep -E 'conv_cf|selscan|total' gpurun_out/tables/m1_order$co.md
done
