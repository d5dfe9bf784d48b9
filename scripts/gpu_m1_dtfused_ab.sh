#!/bin/bash
# A/B of the fused dt_proj scan walk vs the separate delta GEMM (MAMBA_AMD_M1_DT_FUSED=0/1): the fused-dt tests, the
# serialized per-kernel table of each form (scan fwd / bwd, delta GEMM), and interleaved Mamba-1 280M benches.
# Output: gpurun_out/dtf/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/dtf
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread \
  -k "fused_dt" > $O/tests2.log 2>&1 || { tail -40 $O/tests2.log; exit 1; }
tail -1 $O/tests2.log
for v in 1 0; do
  out=$PWD/$O/prof$v
  rm -rf $out
  MAMBA_AMD_M1_DT_FUSED=$v MAMBA_AMD_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $out -o k -- python3 bench.py --model mamba1-280m --steps 1 --warmup 1 > $out.log 2>&1 || { tail -20 $out.log; exit 1; }
  csv=$(find $out -name "*kernel_stats.csv" | head -1)
  python3 scripts/prof_summary.py $csv 16 14 > $O/table_fused$v.md
  rm -rf $out
  echo "fused=$v"; grep "total GPU\|selscan_fwd\|selscan_bwd\|skinny" $O/table_fused$v.md
done
run() {  # tag env
  env $2 timeout -k 10 400 python bench.py --model mamba1-280m --steps ${STEPS:-3} --warmup 1 > $O/$1.log 2>&1 \
    || { tail -20 $O/$1.log; return 1; }
  echo "$1 $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/$1.log | tr '\n' ' ')"
}
for r in 1 2; do
  run b_off_$r MAMBA_AMD_M1_DT_FUSED=0 || exit 1
  run b_on_$r MAMBA_AMD_M1_DT_FUSED=1 || exit 1
done
