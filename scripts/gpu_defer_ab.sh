#!/bin/bash
# Deferred once-per-step reductions (MAMBA_AMD_DEFER_REDUCE) re-measured after the stream-ordered keep-alive fix, on
# the configs where the auto policy keeps them off (d_model > 1024, Mamba-1); interleaved on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/defer
for r in 1 2; do
  for c in "mamba2-1.4b auto" "mamba2-1.4b 1" "mamba1-280m auto" "mamba1-280m 1"; do
    set -- $c
    log=gpurun_out/defer/$1_$2_$r.log
    if [ $2 = auto ]; then env_=""; else env_="MAMBA_AMD_DEFER_REDUCE=$2"; fi
    env $env_ timeout -k 10 400 python bench.py --model $1 --steps 2 --warmup 1 > $log 2>&1 || { tail -5 $log; exit 1; }
    echo "$1 defer=$2 round $r: $(grep -o '"value": [0-9.]*\|"peak_reserved_gb": [0-9.]*\|"alloc_retries": [0-9]*' $log | tr '\n' ' ')"
  done
done
