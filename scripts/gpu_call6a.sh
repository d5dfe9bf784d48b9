cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_pipe_gpu.py -k "accumulation or mamba1 or Mamba1 or selscan or selective or model_native or fused_dbc or gp_bf16" > gpurun_out/t6.log 2>&1; rc=$?; tail -3 gpurun_out/t6.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_envab.sh 2 "MAMBA_AMD_DEFER_REDUCE=0" "MAMBA_AMD_M1_OUTPROJ_PIPE=0" "-" -- --model mamba1-280m --steps 4 --warmup 2 || exit 1
bash scripts/gpu_envab.sh 1 "MAMBA_AMD_WGRAD_DIRECT=0" "-" -- --model mamba2-1.4b --steps 3 --warmup 1 || exit 1
bash scripts/gpu_call6.sh
