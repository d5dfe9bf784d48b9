#!/bin/bash
# GPU box: CU-partitioned stream A/B (utils/cu_mask.py) on the headline bench, interleaved.
#   CONFIGS="base side6 side4 ..."  (sideK: MAMBA_AMD_SIDE_CUS=K, otherK: MAMBA_AMD_OTHER_CUS=K)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/cumask
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cu_mask.py -m gpu \
  > gpurun_out/cumask/test.log 2>&1 || { tail -20 gpurun_out/cumask/test.log; exit 1; }
tail -1 gpurun_out/cumask/test.log
i=0
for c in ${CONFIGS:-base side6 side4 base side5 side3}; do
  i=$((i + 1))
  envs=""
  case $c in
    side*) envs="MAMBA_AMD_SIDE_CUS=${c#side}" ;;
    other*) envs="MAMBA_AMD_OTHER_CUS=${c#other}" ;;
  esac
  log=gpurun_out/cumask/${i}_${c}.log
  env $envs timeout -k 10 400 python bench.py --model ${MODEL:-mamba2-280m} --steps ${STEPS:-5} --warmup 2 > $log 2>&1
  rc=$?
  echo "$c: $(grep -o '"value": [0-9.]*' $log) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
