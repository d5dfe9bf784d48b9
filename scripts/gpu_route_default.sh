#!/bin/bash
# The default projection routing ("route") on the GPU: routing / engine tests, then 1.4B default vs all-native and
# 280M default.  Output: gpurun_out/route/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/route
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_gemm_routing.py -x -q --timeout 150 \
  --timeout-method thread -k "headline_width or bench_path or routing or tuned" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # tag model env...
  local tag=$1 m=$2; shift 2
  env "$@" timeout -k 10 400 python bench.py --model $m --steps 2 --warmup 1 > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; return 1; }
  echo "$tag $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"gemm_table": "[^"]*"' $O/$tag.log | tr '\n' ' ')"
}
run d14_default mamba2-1.4b MAMBA_AMD_X=1 || exit 1
run d14_pk mamba2-1.4b MAMBA_AMD_PROJ_GEMM=pk || exit 1
run d14_lmlib mamba2-1.4b MAMBA_AMD_LMHEAD=lib || exit 1
run d280_default mamba2-280m MAMBA_AMD_X=1 || exit 1
