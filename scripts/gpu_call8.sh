cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
bash scripts/gpu_envab.sh 1 "MAMBA_AMD_M1_DEFER=none" "MAMBA_AMD_M1_DEFER=selscan" "MAMBA_AMD_M1_DEFER=conv" "-" "MAMBA_AMD_DEFER_REDUCE=0" -- --model mamba1-280m --steps 4 --warmup 2 || exit 1
bash scripts/gpu_envab.sh 2 "MAMBA_AMD_PROJ_GEMM=lib" "MAMBA_AMD_PROJ_GEMM=dgrad_long" "MAMBA_AMD_PROJ_GEMM=fwd_short,dgrad" -- --steps 4 --warmup 2 || exit 1
bash scripts/gpu_argab.sh 1 "--model mamba2-1.4b --steps 3 --warmup 1" "--B 64 --overlap on --steps 3 --warmup 1" "--B 64 --overlap off --steps 3 --warmup 1"
