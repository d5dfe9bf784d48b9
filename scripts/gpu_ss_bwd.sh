set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "sequential_backward or channel_walk or test_selective_scan" > gpurun_out/ss_tests.log 2>&1; rc=$?
tail -25 gpurun_out/ss_tests.log
[ $rc -eq 0 ] || exit $rc
for so in mamba_distributed_amd/_C.so ab/_C_pl1.so; do
  for sg in 1; do
    echo "== $so BWD_SG=$sg"
    MAMBA_AMD_SO=$so MAMBA_AMD_SELSCAN_BWD_SG=$sg timeout -k 10 120 python scripts/kbench.py --only selscan --reps 20 2>&1 | grep selscan || exit 1
  done
done
