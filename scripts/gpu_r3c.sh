#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/pk_bench.py --M 65536 --reps 10 --rounds 3 --only in_fwd,in_fwd_pad,in_dgrad,in_dgrad_pad,out_fwd 2>&1 | grep -v amdgpu.ids
