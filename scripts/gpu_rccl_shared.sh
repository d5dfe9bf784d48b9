#!/bin/bash
# GPU box (one MI355X): rehearse the multi-rank RCCL path with 2 ranks sharing the card
# (MAMBA_AMD_SHARE_GPU=1 wraps LOCAL_RANK onto the visible devices).  The bandwidths are NOT xGMI
# numbers (both ranks sit on one GPU); what this shows is that RCCL initialises, the bucketed reducer
# and torch DDP all-reduce over it, and bench.py's multi-rank JSON line comes out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp MAMBA_AMD_SHARE_GPU=1
mkdir -p gpurun_out/rccl
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name"; date
  timeout -k 10 "$secs" "$@" > "gpurun_out/rccl/$name.log" 2>&1; local rc=$?
  grep -E '^\{|busbw|Error|error' "gpurun_out/rccl/$name.log" | tail -12
  echo "$name rc=$rc"
  return $rc
}
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611"
run comm_bench 180 $TR scripts/comm_bench.py --ops all_reduce,reduce_scatter,all_gather --min-mb 1 --max-mb 256 --iters 10 || exit $?
run bench_native 300 python bench.py --gpus 2 --model mamba2-280m --B 16 --global-batch-tokens 131072 --steps 3 --warmup 1 || exit $?
run bench_ddp 300 python bench.py --gpus 2 --model mamba2-280m --B 16 --global-batch-tokens 131072 --steps 3 --warmup 1 --dp-impl ddp || exit $?
