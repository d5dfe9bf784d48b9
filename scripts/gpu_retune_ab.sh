#!/bin/bash
# GPU box: fresh TunableOp search for the Mamba-2 280M step into a NEW table (the shipped one is not read),
# then an interleaved whole-step A/B: shipped table vs the fresh one (MAMBA_AMD_GEMM_TABLE).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/retune
NEW=$PWD/gpurun_out/retune/fresh.csv
rm -f $NEW
timeout -k 10 900 python scripts/tune_gemms.py --models ${MODELS:-mamba2-280m} --out $NEW --max-ms ${MAXMS:-40} \
  > gpurun_out/retune/tune.log 2>&1 &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 30; echo "tuning... $(date +%T)"; done  # heartbeat (silent search)
wait $pid; rc=$?; tail -3 gpurun_out/retune/tune.log; [ $rc -eq 0 ] || exit $rc
i=0
for t in shipped fresh shipped fresh; do
  i=$((i + 1)); log=gpurun_out/retune/${i}_$t.log
  if [ $t = fresh ]; then export MAMBA_AMD_GEMM_TABLE=$NEW; else unset MAMBA_AMD_GEMM_TABLE; fi
  timeout -k 10 400 python bench.py --model ${MODELS:-mamba2-280m} --steps 4 --warmup 2 > $log 2>&1; rc=$?
  echo "$t: $(grep -o '"value": [0-9.]*' $log) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
