cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_varlen_gpu.py tests/test_mamba2_variants.py -k "accumulation or mamba1 or Mamba1 or selscan or selective or reducer_two_ranks or ssd or varlen or mamba2 or Mamba2" > gpurun_out/t4.log 2>&1; rc=$?; tail -3 gpurun_out/t4.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_envab.sh 2 "MAMBA_AMD_SSD_FUSE_DBC=0" "-" -- --steps 4 --warmup 2 || exit 1
bash scripts/gpu_envab.sh 2 "MAMBA_AMD_DEFER_REDUCE=0" "-" -- --model mamba1-280m --steps 4 --warmup 2 || exit 1
bash scripts/gpu_envab.sh 1 "MAMBA_AMD_WGRAD_DIRECT=0" "-" -- --model mamba2-1.4b --steps 3 --warmup 1
