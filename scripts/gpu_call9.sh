cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu9.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu9.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1 || exit 1
bash scripts/gpu_argab.sh 1 "--steps 4 --warmup 2" "--B 32 --steps 4 --warmup 2" "--global-batch-tokens 65536 --steps 6 --warmup 3" "--model mamba1-280m --steps 4 --warmup 2" "--model mamba1-280m --B 32 --steps 4 --warmup 2" "--model mamba1-370m --steps 3 --warmup 1" "--model mamba1-370m --B 32 --steps 3 --warmup 1"
