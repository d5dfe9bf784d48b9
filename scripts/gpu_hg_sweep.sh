#!/bin/bash
# GPU box: SSD kernel tests, then the chunk-bwd head-group size sweep (MAMBA_AMD_SSD_HG override).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x > gpurun_out/pt.log 2>&1; rc=$?
tail -1 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
for hg in ${HGS:-8 12 24}; do
  echo "HG=$hg"; MAMBA_AMD_SSD_HG=$hg timeout -k 10 300 python scripts/kbench.py --only ssd 2>&1 | grep ssd_ || exit 1
done
