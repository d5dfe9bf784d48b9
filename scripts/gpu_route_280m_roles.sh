#!/bin/bash
# Mamba-2 280M: the long-K projection products one at a time on hipBLASLt (role lists of MAMBA_AMD_PROJ_GEMM) against
# all-native, interleaved.  Output: gpurun_out/route/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/route
mkdir -p $O
run() {  # tag value
  MAMBA_AMD_PROJ_GEMM=$2 timeout -k 10 400 python bench.py --steps 3 --warmup 1 > $O/$1.log 2>&1 || { tail -20 $O/$1.log; return 1; }
  echo "$1 ($2) $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/$1.log | tr '\n' ' ')"
}
for r in 1 2; do
  run r280_pk_$r pk || exit 1
  run r280_outfwdlib_$r fwd_short,dgrad || exit 1
  run r280_indgradlib_$r fwd,dgrad_short || exit 1
done
