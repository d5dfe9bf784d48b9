#!/bin/bash
# Row / workgroup order of the Mamba-1 channel-first kernels (conv_cf, selective-scan walks): GPU tests, then the
# Mamba-1 280M step interleaved over MAMBA_AMD_CONV_CF_ORDER / MAMBA_AMD_SELSCAN_ORDER (0 = b-major, 1 = memory order).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "conv1d or selective_scan" -x -q --timeout 120 --timeout-method thread > gpurun_out/order_tests.log 2>&1 || { tail -30 gpurun_out/order_tests.log; exit 1; }
tail -1 gpurun_out/order_tests.log
timeout -k 10 200 python -u scripts/conv_cf_bench.py --reps 30 --orders 0,1 > gpurun_out/order_conv.log 2>&1 || { tail -5 gpurun_out/order_conv.log; exit 1; }
cat gpurun_out/order_conv.log
for rep in 1 2; do
  for m in 0:0 1:0 1:1; do
    IFS=: read -r co so <<< "$m"
    MAMBA_AMD_CONV_CF_ORDER=$co MAMBA_AMD_SELSCAN_ORDER=$so timeout -k 10 300 python bench.py --model ${MODEL:-mamba1-280m} --steps 3 --warmup 1 > gpurun_out/order_b.log 2>&1 || { tail -5 gpurun_out/order_b.log; exit 1; }
    echo "conv=$co selscan=$so $(grep -o '"value": [0-9.]*' gpurun_out/order_b.log)"
  done
done
