cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x --timeout 120 --timeout-method thread -k "conv1d or mamba1_fused or (Mamba1 and native_vs_reference)" 2>&1 | tail -1
for r in 1 2; do
  echo "cur"; timeout -k 10 120 python scripts/conv_cf_bench.py || exit 1
  echo "old"; (cd ab/h && timeout -k 10 120 python scripts/conv_cf_bench.py) || exit 1
done
