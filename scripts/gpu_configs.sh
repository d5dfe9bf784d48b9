#!/bin/bash
# GPU box: extend the GEMM table with the shapes of the given configs, then bench each config.
#   CONFIGS="mamba1-280m:32:1024 mamba1-370m:32:1024" bash scripts/gpu_configs.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp mamba_distributed_amd/tuned/tunableop_gfx950.csv gpurun_out/tunableop_gfx950.csv
for c in ${CONFIGS}; do
  IFS=: read -r m B T <<< "$c"
  echo "== tune $m B=$B T=$T"; date
  timeout -k 10 900 python scripts/tune_gemms.py --models $m --B $B --T $T --max-ms ${MAXMS:-25} \
    --out gpurun_out/tunableop_gfx950.csv > gpurun_out/tune_$m.log 2>&1; rc=$?
  tail -2 gpurun_out/tune_$m.log; [ $rc -eq 0 ] || exit $rc
done
cp gpurun_out/tunableop_gfx950.csv mamba_distributed_amd/tuned/tunableop_gfx950.csv
for c in ${CONFIGS}; do
  IFS=: read -r m B T <<< "$c"
  echo "== bench $m"; date
  timeout -k 10 900 python bench.py --model $m --B $B --T $T --steps ${STEPS:-2} --warmup 1 > gpurun_out/bench_$m.log 2>&1; rc=$?
  grep metric gpurun_out/bench_$m.log; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$m.log; exit $rc; }
done
