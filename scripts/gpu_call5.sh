cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_pipe_gpu.py -k "accumulation or mamba1 or Mamba1 or selscan or selective or model_native or fused_dbc or gp_mm or gemm_pipe" > gpurun_out/t5.log 2>&1; rc=$?; tail -3 gpurun_out/t5.log; [ $rc -eq 0 ] || exit $rc
for v in old new old new; do cp ab/C_$v.so mamba_distributed_amd/_C.so; timeout -k 10 200 python scripts/kbench.py --only selscan --reps 20 > gpurun_out/kb_$v.log 2>&1 || { tail gpurun_out/kb_$v.log; exit 1; }; echo "$v $(grep -i selscan gpurun_out/kb_$v.log | tr '\n' ' ')"; done
cp ab/C_new.so mamba_distributed_amd/_C.so
bash scripts/gpu_envab.sh 2 "MAMBA_AMD_SSD_FUSE_DBC=0" "-" -- --steps 4 --warmup 2 || exit 1
bash scripts/gpu_envab.sh 2 "MAMBA_AMD_DEFER_REDUCE=0" "-" -- --model mamba1-280m --steps 4 --warmup 2 || exit 1
bash scripts/gpu_envab.sh 1 "MAMBA_AMD_WGRAD_DIRECT=0" "-" -- --model mamba2-1.4b --steps 3 --warmup 1
