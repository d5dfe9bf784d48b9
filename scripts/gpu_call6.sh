# serialized kernel tables (no micro-batch overlap, no side stream) of Mamba-1 280M and Mamba-2 280M at HEAD,
# plus the launch-order kernel sequence of one Mamba-1 micro-batch (GEMM -> projection mapping)
cd $GRAFT_REPO_ROOT && R=$PWD && export TMPDIR=/tmp && mkdir -p gpurun_out/prof6
for m in mamba1-280m mamba2-280m; do
  cd /tmp
  MAMBA_AMD_WGRAD_STREAM=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof6/$m" -o run -- python3 "$R/bench.py" --model $m --steps 1 --warmup 1 --no-overlap > "$R/gpurun_out/prof6/$m.log" 2>&1 || { tail -5 "$R/gpurun_out/prof6/$m.log"; exit 1; }
  cd $R
  st=$(find gpurun_out/prof6/$m -name "*kernel_stats.csv" | head -1); tr=$(find gpurun_out/prof6/$m -name "*kernel_trace.csv" | head -1)
  python scripts/prof_summary.py "$st" 32 40 > gpurun_out/prof6/${m}_table.md
  [ $m = mamba1-280m ] && python scripts/prof_sequence.py "$tr" 20000 140 > gpurun_out/prof6/${m}_sequence.txt
  rm -f "$tr"
  head -12 gpurun_out/prof6/${m}_table.md
done
