cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/ka && i=0
for v in unset 1 unset 1; do
  i=$((i + 1)); log=gpurun_out/ka/${i}_$v.log
  if [ $v = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$v; fi
  timeout -k 10 400 python bench.py --steps 4 --warmup 2 > $log 2>&1; rc=$?
  echo "kernarg=$v: $(grep -o '"value": [0-9.]*' $log) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
