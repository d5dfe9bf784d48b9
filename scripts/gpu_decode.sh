#!/bin/bash
# GPU box: tests -> SSD microbench -> bench -> decode GEMV tuning -> decode bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
cp mamba_distributed_amd/tuned/tunableop_gfx950.csv gpurun_out/tunableop_gfx950.csv
echo "== pytest -m gpu"; date
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/kbench.py --only ssd > gpurun_out/kbench.log 2>&1 || exit $?
grep -v Warn gpurun_out/kbench.log | tail -3
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench.log 2>&1 || exit $?
grep metric gpurun_out/bench.log
echo "== tune decode"; date
for m in ${MODELS:-mamba2-280m mamba1-280m}; do
  timeout -k 10 600 python scripts/tune_gemms.py --models $m --B 1 --T 64 --decode-batch 1 16 --max-ms 20 \
    --out gpurun_out/tunableop_gfx950.csv > gpurun_out/tune_decode_$m.log 2>&1 || { tail -5 gpurun_out/tune_decode_$m.log; exit 1; }
  tail -1 gpurun_out/tune_decode_$m.log
done
cp gpurun_out/tunableop_gfx950.csv mamba_distributed_amd/tuned/tunableop_gfx950.csv
echo "== decode bench"; date
for m in ${MODELS:-mamba2-280m mamba1-280m}; do
  timeout -k 10 600 python scripts/bench_decode.py --model $m > gpurun_out/decode_$m.log 2>&1 || { tail -5 gpurun_out/decode_$m.log; exit 1; }
  grep '{' gpurun_out/decode_$m.log
done
