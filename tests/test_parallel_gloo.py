"""Tensor / sequence / context parallelism on CPU (gloo): the parallel model must reproduce the
single-process loss, global gradient norm and full gradients.

Each case launches tests/parallel_worker.py under torchrun; every rank checks itself against the
unsharded reference it computes locally."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(nproc, *args):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", MAMBA_AMD_FORCE_REFERENCE="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "parallel_worker.py"), *args]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "PARALLEL_OK" in r.stdout, r.stdout[-2000:]


@pytest.mark.parametrize("ngroups", [1, 2])
def test_tensor_parallel_tp2(ngroups):
    """ngroups=1: replicated B/C + TP-spanning norm; ngroups=2: sharded groups, local norm."""
    _run(2, "--tp", "2", "--ngroups", str(ngroups))


def test_tensor_sequence_parallel_tp2():
    _run(2, "--tp", "2", "--sp")


def test_context_parallel_cp2():
    _run(2, "--cp", "2")


def test_tp2_cp2_sp_world4():
    _run(4, "--tp", "2", "--cp", "2", "--sp", "--ngroups", "2")


@pytest.mark.parametrize("mode", [["--tp", "2", "--sequence-parallel"], ["--cp", "2"]])
def test_train_py_parallel_matches_single_process(tmp_path, mode):
    """train.py end to end under TP+SP / CP (world 2, dp 1): same losses as one process on the same
    global batch, and the checkpoint (full upstream layout, reassembled over TP) matches too."""
    import torch
    from mamba_distributed_amd.data.loader import write_synthetic_shards
    from test_distributed_gloo import COMMON, _assert_close_sd, _env, _losses, _run_single
    data = str(tmp_path / "data")
    write_synthetic_shards(data, n_train=1, n_val=1, tokens_per_shard=1 << 14, vocab_size=50304)
    sd_single, out_single = _run_single(tmp_path, data, B=4)
    log = str(tmp_path / "par")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "train.py"), *COMMON,
           "--B", "4", "--data-root", data, "--log-dir", log, *mode]
    r = subprocess.run(cmd, capture_output=True, text=True, env=_env(), timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    la, lb = _losses(r.stdout), _losses(out_single)
    assert len(la) == 3 and all(abs(x - y) < 1e-4 * abs(y) for x, y in zip(la, lb)), (la, lb)
    _assert_close_sd(torch.load(os.path.join(log, "model_00002.pt"))["model"], sd_single)


def test_comm_bench_runs_on_gloo():
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "scripts", "comm_bench.py"),
           "--max-mb", "1", "--iters", "2", "--warmup", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert '"op": "all_reduce"' in r.stdout and '"busbw_GBs"' in r.stdout
