#!/bin/bash
# GPU box: kernel tests -> GEMM solution search -> bench default vs tuned table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== pytest -m gpu"; date
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
echo "== tune"; date
timeout -k 10 1200 python scripts/tune_gemms.py --models ${MODELS:-mamba2-280m} --out gpurun_out/tunableop_gfx950.csv > gpurun_out/tune.log 2>&1; rc=$?
tail -30 gpurun_out/tune.log; echo "tune rc=$rc"
[ $rc -eq 0 ] || exit $rc
mkdir -p mamba_distributed_amd/tuned && cp gpurun_out/tunableop_gfx950.csv mamba_distributed_amd/tuned/
echo "== bench default"; date
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-tuned-gemms > gpurun_out/bench_default.log 2>&1; rc=$?
grep metric gpurun_out/bench_default.log; [ $rc -eq 0 ] || exit $rc
echo "== bench tuned"; date
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_tuned.log 2>&1; rc=$?
grep metric gpurun_out/bench_tuned.log; exit $rc
