cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp MAMBA_AMD_WGRAD_STREAM=0
out=$PWD/gpurun_out/nat
rm -rf $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o k -- python3 bench.py --model mamba1-280m --B 64 --T 1024 --steps 1 --warmup 0 > gpurun_out/nat.log 2>&1 || { tail -5 gpurun_out/nat.log; exit 1; }
csv=$(find $out -name "*kernel_stats.csv" | head -1)
python3 - "$csv" <<'PY' > gpurun_out/nat_names.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r.get("Name") or r.get("KernelName")
    if "at::native" in n or "rocprim" in n:
        print(r["Calls"], r["TotalDurationNs"], n[:400])
PY
rm -rf $out
