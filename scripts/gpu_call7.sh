cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "accumulation or mamba1 or Mamba1" > gpurun_out/t7.log 2>&1; rc=$?; tail -2 gpurun_out/t7.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_envab.sh 2 "MAMBA_AMD_DEFER_REDUCE=0" "MAMBA_AMD_M1_OUTPROJ_PIPE=0" "-" -- --model mamba1-280m --steps 4 --warmup 2 || exit 1
bash scripts/gpu_argab.sh 1 "--global-batch-tokens 65536 --B 64 --overlap off --steps 6 --warmup 3" "--B 64 --overlap off --steps 3 --warmup 1" || exit 1
MAMBA_AMD_DEFER_REDUCE=0 bash scripts/gpu_argab.sh 1 "@ab/6ffc845 --model mamba2-1.4b --steps 3 --warmup 1" "@ab/d8f4ba2 --model mamba2-1.4b --steps 3 --warmup 1"
