#!/bin/bash
# bf16 dB / dC partials of the sequential selective-scan backward (MAMBA_AMD_SELSCAN_BC16=0/1): scan and Mamba-1 tests,
# serialized kernel times of the backward + reduction, interleaved Mamba-1 280M benches.  Output: gpurun_out/bc16/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/bc16
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread \
  -k "selective_scan or fused_dt or (Mamba1 and (native_vs_reference or bench_path or reducer))" > $O/tests.log 2>&1 \
  || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in 1 0; do
  out=$PWD/$O/prof$v
  rm -rf $out
  MAMBA_AMD_SELSCAN_BC16=$v MAMBA_AMD_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $out -o k -- python3 bench.py --model mamba1-280m --steps 1 --warmup 1 > $out.log 2>&1 || { tail -20 $out.log; exit 1; }
  csv=$(find $out -name "*kernel_stats.csv" | head -1)
  python3 scripts/prof_summary.py $csv 16 40 > $O/table$v.md
  rm -rf $out
  echo "bc16=$v"; grep "total GPU\|selscan" $O/table$v.md
done
run() {  # tag env
  env $2 timeout -k 10 400 python bench.py --model mamba1-280m --steps 3 --warmup 1 > $O/$1.log 2>&1 || { tail -20 $O/$1.log; return 1; }
  echo "$1 $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/$1.log | tr '\n' ' ')"
}
for r in 1 2; do
  run off_$r MAMBA_AMD_SELSCAN_BC16=0 || exit 1
  run on_$r MAMBA_AMD_SELSCAN_BC16=1 || exit 1
done
