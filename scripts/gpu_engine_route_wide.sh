#!/bin/bash
# Wide models (d_model >= 2048): all-native projections vs hipBLASLt for the long-K fwd / dgrad products
# (MAMBA_AMD_PROJ_GEMM=pk / auto), interleaved.  Output: gpurun_out/route/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/route
mkdir -p $O
run() {  # tag model B T env...
  local tag=$1 m=$2 B=$3 T=$4; shift 4
  env "$@" timeout -k 10 500 python bench.py --model $m --B $B --T $T --steps 2 --warmup 1 > $O/$tag.log 2>&1 \
    || { tail -20 $O/$tag.log; return 1; }
  echo "$tag $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_reserved_gb": [0-9.]*' $O/$tag.log | tr '\n' ' ')"
}
for r in 2 3; do
  run b14_auto_$r mamba2-1.4b 32 1024 MAMBA_AMD_PROJ_GEMM=auto || exit 1
  run b14_pk_$r mamba2-1.4b 32 1024 MAMBA_AMD_PROJ_GEMM=pk || exit 1
done
run b28_pk mamba2-2.8b 4 8192 MAMBA_AMD_PROJ_GEMM=pk || exit 1
run b28_auto mamba2-2.8b 4 8192 MAMBA_AMD_PROJ_GEMM=auto || exit 1
