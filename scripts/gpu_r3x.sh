#!/bin/bash
# call X: decode GEMVs with fewer output rows per wave at 16 batch rows (no scratch accumulators, 2x the grid):
# decode GPU tests (batch 1/3/9/16), decode bench against the previous build (ab/pre_dec_C.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "decode" --timeout 120 --timeout-method thread > gpurun_out/t_x.log 2>&1; rc=$?; tail -2 gpurun_out/t_x.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  MAMBA_AMD_SO=$PWD/ab/pre_dec_C.so timeout -k 10 300 python -u scripts/bench_decode.py --batch 1 4 16 > gpurun_out/dec_base_$r.jsonl 2> gpurun_out/dec_base_$r.err || { tail -5 gpurun_out/dec_base_$r.err; exit 1; }
  timeout -k 10 300 python -u scripts/bench_decode.py --batch 1 4 16 > gpurun_out/dec_new_$r.jsonl 2> gpurun_out/dec_new_$r.err || { tail -5 gpurun_out/dec_new_$r.err; exit 1; }
  grep '"graph"' gpurun_out/dec_base_$r.jsonl | sed "s/^/[base r$r] /"; grep '"graph"' gpurun_out/dec_new_$r.jsonl | sed "s/^/[new r$r] /"
done
