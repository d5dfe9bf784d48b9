#!/bin/bash
# (experiment record: MAMBA_AMD_SSF_LDS_PAD was a temporary launcher switch -- dynamic LDS padding of selscan_fwd_sg_k --
#  removed after the measurement, profiles/r5/selscan_fwd_whole_rounds_rejected.txt)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
mkdir -p gpurun_out/ssf
for r in 1 2; do
for pad in 0 12288; do
  out=$PWD/gpurun_out/ssf/p${pad}_$r
  MAMBA_AMD_SSF_LDS_PAD=$pad timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o k -- python3 bench.py --model mamba1-280m --steps 1 --warmup 1 > $out.log 2>&1 || { tail -5 $out.log; exit 1; }
  csv=$(find $out -name "*kernel_stats.csv" | head -1)
  echo "pad=$pad r=$r $(grep selscan_fwd $csv | cut -d, -f1-6 | tr '\n' ' ') $(grep -o '"value": [0-9.]*' $out.log)"
  rm -rf $out
done
done
