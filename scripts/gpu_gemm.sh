#!/bin/bash
# GEMM engine microbench on one GPU: persistent engine (8- and 4-wave forms) vs hipBLASLt, projection shapes.
#   PK_ARGS="--M 65536 --only in_fwd_pad,out_fwd" bash scripts/gpu_gemm.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/pk_bench.py ${PK_ARGS:---M 65536 --no-wgrad} > gpurun_out/pk_bench.log 2>&1; rc=$?
cat gpurun_out/pk_bench.log | grep -v Warn; exit $rc
