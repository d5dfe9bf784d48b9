#!/bin/bash
# GPU box: per-kernel average times of one microbenchmark command in the working tree and in a built
# worktree ab/<name>, interleaved (rocprofv3 --kernel-trace --stats only).
#   [KFILTER=substr] bash scripts/gpu_kstats_ab.sh <name> <rounds> <script.py args...>
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
name=$1; rounds=$2; shift 2
mkdir -p gpurun_out/kab
for r in $(seq 1 $rounds); do
  for side in cur $name; do
    d=$GRAFT_REPO_ROOT; [ $side = cur ] || d=$GRAFT_REPO_ROOT/ab/$name
    out=$GRAFT_REPO_ROOT/gpurun_out/kab/${side}_$r
    (cd $d && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o k -- python3 "$@") > $out.log 2>&1 || { tail -20 $out.log; exit 1; }
    python3 - "$out" "$side" <<'PY'
import glob, sqlite3, sys
db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
c = sqlite3.connect(db)
import os
f = os.environ.get("KFILTER", "")
q = "select name, count(*), avg(duration)/1000.0 from kernels group by name order by 3 desc"
for n, k, t in [r for r in c.execute(q) if f in r[0]][:8]:
    print(f"{sys.argv[2]:4s} {t:9.1f} us  x{k:<4d} {n[:90]}")
PY
    rm -rf "$out"  # the trace database: only the summary above is kept (gpurun_out/ returns <= 64 MiB)
  done
done
