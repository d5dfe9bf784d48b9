#!/bin/bash
# call N: persistent GEMM latency sensitivity -- the same products at 16384 rows (A operand MALL-resident across
# repeats) vs 65536 rows, TFLOP/s of pk and hipBLASLt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for M in 16384 65536; do
  timeout -k 10 200 python -u scripts/pk_bench.py --M $M --rounds 2 --only in_fwd_pad,in_dgrad_pad,out_fwd,out_dgrad --no-wgrad 2>&1 | grep case | sed "s/^/[M=$M] /" | sed 's/"rel_err[^,]*, "rel_err_rowscale[^,]*, //' || exit 1
done
