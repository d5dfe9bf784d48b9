#!/bin/bash
# Sync micro-step weight gradients in place on the side stream (ops/grad_accum.py::sync_inplace) under the native
# reducer: the two-rank reducer tests, then the 8-GPU per-rank regime on one GPU -- one rank under torchrun (so the
# reducer's flat-buffer gradient views are live), 65,536 tokens per optimizer step (accumulation 1) -- A/B
# interleaved.  Output: gpurun_out/sync_inplace/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/sync_inplace
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 150 --timeout-method thread \
  -k "reducer_two_ranks or microbatch_overlap" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # model tag env
  local port=$((29600 + RANDOM % 300))
  env $3 timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 1 --model $1 --global-batch-tokens 65536 --B 64 --steps ${STEPS:-20} \
    --warmup 3 > $O/$2.log 2>&1 || { tail -20 $O/$2.log; return 1; }
  echo "$2 $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_reserved_gb": [0-9.]*' $O/$2.log | tr '\n' ' ')"
}
for r in 1 2; do
  run mamba2-280m m2_off_$r MAMBA_AMD_SYNC_INPLACE=0 || exit 1
  run mamba2-280m m2_on_$r MAMBA_AMD_SYNC_INPLACE=1 || exit 1
done
for r in 1 2; do
  run mamba1-280m m1_off_$r MAMBA_AMD_SYNC_INPLACE=0 || exit 1
  run mamba1-280m m1_on_$r MAMBA_AMD_SYNC_INPLACE=1 || exit 1
done
