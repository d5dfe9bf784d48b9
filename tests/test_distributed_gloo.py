"""Multi-process data parallelism on CPU with gloo (SURVEY.md §4 'Distributed (fake multi-node)').

torchrun --nproc-per-node 2 (gloo) on the tiny Mamba-2 config (the BASELINE 'CPU/gloo world_size=2'
plumbing config) must produce the same parameters as a single process that sees the same global
batch (DDP averages gradients; DataLoaderLite's rank striding splits the global batch exactly).
A second test runs two torchrun "nodes" on localhost (--nnodes 2 --node-rank i).
"""
import math
import os
import socket
import subprocess
import sys

import pytest
import torch

from mamba_distributed_amd.data.loader import write_synthetic_shards

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


COMMON = ["--model", "mamba2-tiny", "--n-layer", "2", "--T", "32", "--total-batch-size", "256", "--steps", "3",
          "--val-every", "100", "--val-steps", "1", "--ckpt-every", "1000", "--sample-every", "1000",
          "--warmup-steps", "2", "--device-type", "cpu", "--backend", "gloo"]


def _env():
    return dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", MAMBA_AMD_FORCE_REFERENCE="1")


def _run_single(tmp, data, B):
    log = str(tmp / "single")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "train.py"), *COMMON, "--B", str(B),
                        "--data-root", data, "--log-dir", log], capture_output=True, text=True, env=_env(), timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return torch.load(os.path.join(log, "model_00002.pt"))["model"], r.stdout


def _assert_close_sd(a, b):
    # AdamW turns fp-roundoff-sized gradient differences on (near-)zero-gradient entries into
    # O(lr) updates, so parameters agree to a few lr (6e-4) after 3 steps, not to fp32 epsilon;
    # the loss trajectories (compared separately) agree to ~1e-5 relative.
    for k in a:
        torch.testing.assert_close(a[k], b[k], rtol=0, atol=3e-3, msg=k)


def _losses(stdout):
    return [float(l.split("loss: ")[1].split(" ")[0]) for l in stdout.splitlines() if l.startswith("step ")]


@pytest.mark.parametrize("dp_impl,bucket_mb", [("native", "100"), ("native", "0.05"), ("ddp", "100")])
def test_ddp_gloo_world2_matches_single_process(tmp_path, dp_impl, bucket_mb):
    """Both data-parallel implementations (parallel/reducer.py, torch DDP) -- and the native one with
    tiny buckets, so many in-order bucket launches happen during the backward -- match 1 process."""
    data = str(tmp_path / "data")
    write_synthetic_shards(data, n_train=1, n_val=1, tokens_per_shard=1 << 14, vocab_size=50304)
    sd_single, out_single = _run_single(tmp_path, data, B=4)
    log = str(tmp_path / "ddp")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "train.py"), *COMMON,
           "--B", "2", "--data-root", data, "--log-dir", log, "--dp-impl", dp_impl, "--bucket-cap-mb", bucket_mb]
    r = subprocess.run(cmd, capture_output=True, text=True, env=_env(), timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "=> calculated gradient accumulation steps: 2" in r.stdout
    sd_ddp = torch.load(os.path.join(log, "model_00002.pt"))["model"]
    _assert_close_sd(sd_ddp, sd_single)
    la, lb = _losses(r.stdout), _losses(out_single)
    assert len(la) == 3 and all(abs(x - y) < 1e-4 * abs(y) for x, y in zip(la, lb)), (la, lb)


def test_two_node_rendezvous_on_localhost(tmp_path):
    data = str(tmp_path / "data")
    write_synthetic_shards(data, n_train=1, n_val=1, tokens_per_shard=1 << 14, vocab_size=50304)
    port = _port()
    log = str(tmp_path / "nodes")
    procs = []
    for node in range(2):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "2", "--node-rank", str(node),
               "--nproc-per-node", "1", "--master-addr", "127.0.0.1", "--master-port", str(port),
               os.path.join(ROOT, "train.py"), *COMMON, "--B", "2", "--data-root", data, "--log-dir", log]
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=_env()))
    outs = [p.communicate(timeout=600) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    sd_single, _ = _run_single(tmp_path, data, B=4)
    _assert_close_sd(torch.load(os.path.join(log, "model_00002.pt"))["model"], sd_single)


def _loss_by_step(stdout):
    out = {}
    for l in stdout.splitlines():
        if l.startswith("step "):
            out[int(l.split("|")[0].split()[1])] = float(l.split("loss: ")[1].split(" ")[0])
    return out  # last occurrence wins (re-run steps after a restart)


def test_elastic_restart_resumes_from_checkpoint(tmp_path):
    """SURVEY.md §5.3 fault injection: rank 1 dies at the start of step 3 on the first attempt;
    torchrun (--max-restarts 1) restarts both workers, train.py --resume reloads model, optimizer,
    every rank's loader position and RNG from model_00002.pt (written at the start of step 2) and
    re-runs steps 2-5.  The losses must equal an uninterrupted run's."""
    data = str(tmp_path / "data")
    write_synthetic_shards(data, n_train=1, n_val=1, tokens_per_shard=1 << 14, vocab_size=50304)
    args = [a for a in COMMON]
    args[args.index("--steps") + 1] = "6"
    args[args.index("--val-every") + 1] = "2"
    args[args.index("--ckpt-every") + 1] = "2"

    def launch(log, restarts, fault):
        env = _env()
        if fault:
            env.update(MAMBA_AMD_FAULT_AT_STEP="3", MAMBA_AMD_FAULT_RANK="1")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
               "--max-restarts", str(restarts), "--master-addr", "127.0.0.1", "--master-port", str(_port()),
               os.path.join(ROOT, "train.py"), *args, "--B", "2", "--data-root", data, "--log-dir", log, "--resume"]
        # own session: the elastic agent signals its process group when it tears workers down
        return subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=900, start_new_session=True)

    ref = launch(str(tmp_path / "clean"), 0, False)
    assert ref.returncode == 0, ref.stderr[-3000:]
    ft = launch(str(tmp_path / "faulty"), 1, True)
    assert ft.returncode == 0, ft.stderr[-3000:]
    assert "[fault-injection] rank 1 exiting at step 3" in ft.stdout + ft.stderr
    assert "model_00002.pt at step 2" in ft.stdout
    la, lb = _loss_by_step(ref.stdout), _loss_by_step(ft.stdout)
    assert sorted(la) == list(range(6)) and sorted(lb) == list(range(6)), (la, lb)
    for s in (2, 3, 4, 5):
        assert abs(la[s] - lb[s]) <= 1e-6 * abs(la[s]), (s, la[s], lb[s])


@pytest.mark.parametrize("dp_impl", ["native", "ddp"])
def test_bench_multi_rank_flow_on_cpu(dp_impl):
    """bench.py exactly as the round driver launches it for N > 1 (torch.distributed.run, one rank
    per device, 127.0.0.1 rendezvous), rehearsed on CPU with gloo and the tiny model: every rank
    runs the same steps through the data-parallel wrapper, and rank 0 prints ONE JSON line."""
    import json
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--model", "mamba2-tiny", "--B", "2", "--T", "64", "--global-batch-tokens", "512",
           "--steps", "2", "--warmup", "1", "--dp-impl", dp_impl]
    r = subprocess.run(cmd, capture_output=True, text=True, env=_env(), timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["warmup"] == 1 and d["scaling"] == "strong"
    assert d["config"]["parallelism"] == "dp2" and d["config"]["dp_impl"] == dp_impl
    assert d["config"]["grad_accum"] == 2 and d["value"] > 0
    assert math.isfinite(d["config"]["final_loss"]), d
    # the post-timing all-reduce probe (bus bandwidth of one 100 MB gradient bucket and of 400 MB)
    assert d["config"]["comm"]["allreduce_100MB_busbw_GBps"] > 0 and d["config"]["comm"]["allreduce_400MB_ms"] > 0, d


def test_bench_gpus2_relaunches_under_torchrun():
    """``python bench.py --gpus 2`` outside torchrun must start 2 ranks itself (a child
    torch.distributed.run) and report n_gpus 2 from the real world size, never one rank."""
    import json
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--model", "mamba2-tiny", "--B", "2", "--T", "32", "--global-batch-tokens", "256"]
    env = dict(_env())
    env.pop("RANK", None)
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["config"]["comm"]["world_size"] == 2 and out["config"]["comm"]["n_buckets"] >= 1
    assert out["config"]["grad_accum"] == 2


def test_bench_refuses_world_mismatch():
    """Under torchrun, a --gpus that disagrees with WORLD_SIZE exits non-zero without a JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "0", "--model", "mamba2-tiny", "--B", "2", "--T", "32",
           "--global-batch-tokens", "128"]
    p = subprocess.run(cmd, env=_env(), stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600)
    assert p.returncode != 0
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
