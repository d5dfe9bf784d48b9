#!/bin/bash
# Projection GEMM routing re-measured on the round-5 tree: all-native (MAMBA_AMD_PROJ_GEMM=pk, default) vs "auto"
# (hipBLASLt with the tuned solution table where it measured faster: K > 1024 products) vs auto + the lm_head on
# hipBLASLt.  Interleaved whole-step benches.  Output: gpurun_out/route/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/route
mkdir -p $O
run() {  # tag model env...
  local tag=$1 m=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --model $m --steps ${STEPS:-3} --warmup 1 > $O/$tag.log 2>&1 \
    || { tail -20 $O/$tag.log; return 1; }
  echo "$tag $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"gemm_table": "[^"]*"' $O/$tag.log | tr '\n' ' ')"
}
for r in 1 2; do
  run m2_pk_$r mamba2-280m MAMBA_AMD_PROJ_GEMM=pk || exit 1
  run m2_auto_$r mamba2-280m MAMBA_AMD_PROJ_GEMM=auto || exit 1
  run m2_autolm_$r mamba2-280m MAMBA_AMD_PROJ_GEMM=auto MAMBA_AMD_LMHEAD=lib || exit 1
done
run m1_pk mamba1-280m MAMBA_AMD_PROJ_GEMM=pk || exit 1
run m1_auto mamba1-280m MAMBA_AMD_PROJ_GEMM=auto || exit 1
STEPS=2 run b14_pk mamba2-1.4b MAMBA_AMD_PROJ_GEMM=pk || exit 1
STEPS=2 run b14_auto mamba2-1.4b MAMBA_AMD_PROJ_GEMM=auto || exit 1
