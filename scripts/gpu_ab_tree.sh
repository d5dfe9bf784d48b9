#!/bin/bash
# GPU box: interleaved whole-step A/B of the working tree against a built worktree under ab/<name>
# (git worktree add --detach ab/<name> <commit>; build it in place on the CPU first).
#   bash scripts/gpu_ab_tree.sh <name> <rounds> [bench.py args...]
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
name=$1; rounds=$2; shift 2
mkdir -p gpurun_out/ab
for r in $(seq 1 $rounds); do
  for side in cur $name; do
    d=$GRAFT_REPO_ROOT; [ $side = cur ] || d=$GRAFT_REPO_ROOT/ab/$name
    (cd $d && timeout -k 10 300 python bench.py "$@") > gpurun_out/ab/${side}_$r.log 2>&1 || { tail -20 gpurun_out/ab/${side}_$r.log; exit 1; }
    echo "$side $(tail -1 gpurun_out/ab/${side}_$r.log | cut -c1-200)"
  done
done
