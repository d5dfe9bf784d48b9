#!/bin/bash
# GPU box: selective-scan GPU tests on the in-tree build, then kbench (selscan) and the Mamba-1 280M step,
# interleaved between the in-tree _C.so ("new") and saved builds ab/_C_<name>.so (MAMBA_AMD_SO).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ssab
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "selective or selscan" > gpurun_out/ssab/test.log 2>&1; rc=$?; tail -3 gpurun_out/ssab/test.log; [ $rc -eq 0 ] || exit $rc
pick() { if [ $1 = new ]; then unset MAMBA_AMD_SO; else export MAMBA_AMD_SO=$PWD/ab/_C_$1.so; fi; }
i=0
for so in ${KB_SOS:-base new base new}; do
  i=$((i + 1)); pick $so; log=gpurun_out/ssab/kb_${i}_$so.log
  timeout -k 10 300 python scripts/kbench.py --only selscan --reps 20 > $log 2>&1; rc=$?
  echo "$so: $(grep -E 'selscan_(fwd|bwd)' $log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
[ "${STEP:-1}" = "1" ] || exit 0
for so in ${STEP_SOS:-base new base new}; do
  i=$((i + 1)); pick $so; log=gpurun_out/ssab/bench_${i}_$so.log
  timeout -k 10 400 python bench.py --model mamba1-280m --steps 4 --warmup 2 > $log 2>&1; rc=$?
  echo "$so step: $(grep -o '"value": [0-9.]*' $log) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
