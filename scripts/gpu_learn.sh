#!/bin/bash
# Learning-curve evidence on a learnable synthetic stream (data/loader.py::markov_tokens): train the 280M
# model through train.py (native TokenLoader, accum 16) and keep the per-step logs under gpurun_out/learn/.
#   RUNS="m2_native m2_alt" STEPS=150 bash scripts/gpu_learn.sh
#   m2_native : Mamba-2, default fast path (micro-batch overlap, side-stream wgrad, deferred reductions)
#   m2_alt    : Mamba-2, every one of those switched off (sequential micro-batches, per-step reductions)
#   m1_native : Mamba-1 (the reference's default MambaConfig), default fast path
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/learn
STEPS=${STEPS:-150}
timeout -k 10 300 python -c "
from mamba_distributed_amd.data.loader import write_synthetic_shards as w
w('/tmp/markov', n_train=4, n_val=1, tokens_per_shard=25_000_000, kind='markov', seed=7)" || exit $?
for r in ${RUNS:-m2_native m2_alt}; do
  echo "== $r"; date
  common="--data-root /tmp/markov --steps $STEPS --max-steps $STEPS --warmup-steps 30 --val-every 50 --val-steps 5 \
          --ckpt-every 1000000 --sample-every 1000000 --log-dir /tmp/learn/$r --metrics-jsonl gpurun_out/learn/$r.jsonl"
  case $r in
    m2_native) timeout -k 10 1000 python -u train.py --layer Mamba2 $common ;;
    m2_alt) MAMBA_AMD_WGRAD_STREAM=0 MAMBA_AMD_DEFER_REDUCE=0 timeout -k 10 1000 python -u train.py --layer Mamba2 \
              --overlap-microbatches off $common ;;
    m1_native) timeout -k 10 1100 python -u train.py $common ;;
  esac > gpurun_out/learn/$r.log 2>&1
  rc=$?; cp /tmp/learn/$r/log.txt gpurun_out/learn/$r.txt 2>/dev/null; tail -3 gpurun_out/learn/$r.log
  [ $rc -eq 0 ] || exit $rc
done
