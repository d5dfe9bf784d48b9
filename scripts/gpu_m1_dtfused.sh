#!/bin/bash
# Mamba-1 dt_proj fused into the selective-scan walks: the scan / Mamba-1 GPU tests, then interleaved 1-GPU benches
# (MAMBA_AMD_M1_DT_FUSED=0/1) of Mamba-1 280M and 370M, then the per-kernel table of the fused 280M step.
# Output: gpurun_out/dtf/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/dtf
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread \
  -k "fused_dt or selective_scan or (Mamba1 and (native_vs_reference or bench_path))" > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # model tag env
  env $3 timeout -k 10 400 python bench.py --model $1 --steps ${STEPS:-3} --warmup 1 > $O/$2.log 2>&1 \
    || { tail -20 $O/$2.log; return 1; }
  echo "$2 $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_reserved_gb": [0-9.]*' $O/$2.log | tr '\n' ' ')"
}
for r in 1 2; do
  run mamba1-280m m1_off_$r MAMBA_AMD_M1_DT_FUSED=0 || exit 1
  run mamba1-280m m1_on_$r MAMBA_AMD_M1_DT_FUSED=1 || exit 1
done
run mamba1-370m m370_off MAMBA_AMD_M1_DT_FUSED=0 || exit 1
run mamba1-370m m370_on MAMBA_AMD_M1_DT_FUSED=1 || exit 1
out=$PWD/$O/prof
rm -rf $out
MAMBA_AMD_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o k -- \
  python3 bench.py --model mamba1-280m --steps 1 --warmup 1 > $out.log 2>&1 || { tail -20 $out.log; exit 1; }
csv=$(find $out -name "*kernel_stats.csv" | head -1)
python3 scripts/prof_summary.py $csv 16 30 > $O/table_m1_fused.md
rm -rf $out
head -24 $O/table_m1_fused.md
