cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/hg && i=0
for v in auto 12 8 auto 12 8; do
  i=$((i + 1)); log=gpurun_out/hg/${i}_hg$v.log
  if [ $v = auto ]; then unset MAMBA_AMD_SSD_HG; else export MAMBA_AMD_SSD_HG=$v; fi
  timeout -k 10 400 python bench.py --steps 4 --warmup 2 > $log 2>&1; rc=$?
  echo "hg=$v: $(grep -o '"value": [0-9.]*' $log) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
