#!/bin/bash
# In-place sync-step weight-gradient accumulation on the main stream (ops/grad_accum.py::sync_accumulable): the GPU
# tests that cover it, then the accumulation-1 regime (one torchrun rank, reducer live) and the headline bench,
# MAMBA_AMD_SYNC_INPLACE=0/1 interleaved.  Output: gpurun_out/sip/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/sip
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_optim_gpu.py -x -q --timeout 150 \
  --timeout-method thread -k "late_colsum or reducer_two_ranks or mamba1_fused or microbatch or bench_path or accum or optim or native_vs_reference" \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
acc1() {  # tag env model
  local port=$((29600 + RANDOM % 300))
  env $2 timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 1 --model $3 --global-batch-tokens 65536 --B 64 --steps 20 --warmup 3 \
    > $O/$1.log 2>&1 || { tail -20 $O/$1.log; return 1; }
  echo "$1 $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/$1.log | tr '\n' ' ')"
}
for r in 1 2; do
  acc1 a1_off_$r MAMBA_AMD_SYNC_INPLACE=0 mamba2-280m || exit 1
  acc1 a1_on_$r MAMBA_AMD_SYNC_INPLACE=1 mamba2-280m || exit 1
done
acc1 m1_off MAMBA_AMD_SYNC_INPLACE=0 mamba1-280m || exit 1
acc1 m1_on MAMBA_AMD_SYNC_INPLACE=1 mamba1-280m || exit 1
for v in 0 1; do
  MAMBA_AMD_SYNC_INPLACE=$v timeout -k 10 400 python bench.py --steps 3 --warmup 1 > $O/h$v.log 2>&1 || { tail -20 $O/h$v.log; exit 1; }
  echo "headline late=$v $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/h$v.log | tr '\n' ' ')"
done
