"""Training-loop integration on CPU: overfit, logging formats, resume, CLI (SURVEY.md §4 'Integration')."""
import json
import os
import subprocess
import sys

import torch

from mamba_distributed_amd import LMHeadModel, MambaConfig
from mamba_distributed_amd.trainer import TrainArgs, Trainer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tiny_model_overfits_fixed_batch():
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=64, n_layer=2, vocab_size=128, ssm_cfg={"layer": "Mamba2", "headdim": 16, "d_state": 16})
    m = LMHeadModel(cfg, device="cpu", enc=object())
    opt = torch.optim.AdamW(m.parameters(), lr=3e-3)
    x = torch.randint(0, 128, (4, 32))
    y = torch.roll(x, -1, 1)
    losses = []
    for _ in range(60):
        opt.zero_grad()
        _, loss = m(x, y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < 0.5 * losses[0], losses[::10]


def _args(tmp, **kw):
    base = dict(model="mamba1-tiny", synthetic=True, B=2, T=32, total_batch_size=128, steps=4, val_every=2,
                val_steps=2, ckpt_every=3, sample_every=100, warmup_steps=2, max_steps=10, log_dir=str(tmp),
                metrics_jsonl=str(tmp / "m.jsonl"), device_type="cpu", n_layer=1)
    base.update(kw)
    return TrainArgs(**base)


def test_trainer_logs_checkpoints_and_resume(tmp_path, capsys):
    Trainer(_args(tmp_path)).run()
    out = capsys.readouterr().out
    assert "=> calculated gradient accumulation steps: 2" in out
    assert "step     0 | loss:" in out and "| tok/sec:" in out
    lines = open(tmp_path / "log.txt").read().splitlines()
    assert lines[0].startswith("0 val ") and lines[1].startswith("0 train ")
    assert any(l.startswith("3 train") for l in lines)
    assert os.path.exists(tmp_path / "model_00003.pt")
    rec = [json.loads(l) for l in open(tmp_path / "m.jsonl")]
    assert [r["step"] for r in rec] == [0, 1, 2, 3]
    # model_00003.pt is written at the START of step 3 (before its update, as in the reference), so
    # resuming from it re-runs step 3
    t = Trainer(_args(tmp_path, steps=6, resume=True))
    assert t.start_step == 3
    t.run()
    lines = open(tmp_path / "log.txt").read().splitlines()
    assert lines[-1].startswith("5 train")


def test_train_cli_help_and_tiny_run(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "train.py"), "--model", "mamba2-tiny", "--n-layer", "1",
                        "--synthetic", "--B", "1", "--T", "64", "--total-batch-size", "64", "--steps", "2",
                        "--val-steps", "1", "--log-dir", str(tmp_path), "--device-type", "cpu"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "step     1 | loss:" in r.stdout


def test_overlap_policy_by_width():
    """parallel/microbatch.py::resolve_overlap: auto = on for d_model <= 1024 (measured crossover)."""
    from mamba_distributed_amd import preset
    from mamba_distributed_amd.parallel.microbatch import resolve_overlap
    assert resolve_overlap("auto", preset("mamba2-280m")) is True
    assert resolve_overlap("auto", preset("mamba2-1.4b")) is False
    assert resolve_overlap("off", preset("mamba2-280m")) is False
    assert resolve_overlap("on", preset("mamba2-1.4b")) is True
    assert resolve_overlap(True, None) is True


def test_defer_reduce_policy_by_width(monkeypatch):
    """auto_defer_reduce: on for d_model <= 2048 (both mixers); accumulation_scope(defer_reduce=...) gates
    grad_accum.deferred, and MAMBA_AMD_DEFER_REDUCE=0/1 overrides it."""
    import torch
    from mamba_distributed_amd import preset
    from mamba_distributed_amd.ops import grad_accum
    from mamba_distributed_amd.parallel.microbatch import auto_defer_reduce
    assert auto_defer_reduce(preset("mamba2-280m")) is True
    assert auto_defer_reduce(preset("mamba1-280m")) is True
    assert auto_defer_reduce(preset("mamba2-1.4b")) is True
    assert auto_defer_reduce(preset("mamba2-2.8b")) is False
    p = torch.nn.Parameter(torch.zeros(4))
    monkeypatch.delenv("MAMBA_AMD_DEFER_REDUCE", raising=False)
    try:
        assert grad_accum.deferred(p, "t", (2, 4), p.device) is None  # outside a scope
        with grad_accum.accumulation_scope(defer_reduce=False):
            assert grad_accum.deferred(p, "t", (2, 4), p.device) is None
            monkeypatch.setenv("MAMBA_AMD_DEFER_REDUCE", "1")
            assert grad_accum.deferred(p, "t", (2, 4), p.device) is not None
        monkeypatch.delenv("MAMBA_AMD_DEFER_REDUCE")
        with grad_accum.accumulation_scope(defer_reduce=True):
            buf, mode = grad_accum.deferred(p, "t", (2, 4), p.device)
            assert buf.shape == (2, 4) and mode == 3  # sync micro-step (not direct): store + reduce
            monkeypatch.setenv("MAMBA_AMD_DEFER_REDUCE", "0")
            assert grad_accum.deferred(p, "t", (2, 4), p.device) is None
    finally:
        grad_accum.release_buffers()


def test_deferred_partials_refuse_silent_drops(monkeypatch):
    """a shape change of a (param, tag) partial buffer with pending partials, or partials added on a
    no-sync micro-step and never reduced, must raise instead of silently dropping gradient contributions."""
    import pytest
    from mamba_distributed_amd.ops import grad_accum
    monkeypatch.setenv("MAMBA_AMD_DEFER_REDUCE", "1")
    p = torch.nn.Parameter(torch.zeros(4))
    try:
        # equal shapes: no-sync store, no-sync add, sync add + reduce
        with grad_accum.accumulation_scope():
            grad_accum.set_direct(True)
            assert grad_accum.deferred(p, "t", (2, 4), p.device)[1] == 1
            assert grad_accum.deferred(p, "t", (2, 4), p.device)[1] == 2
            grad_accum.set_direct(False)
            assert grad_accum.deferred(p, "t", (2, 4), p.device)[1] == 4
        # a short micro-batch (different partial-row count) while partials are pending
        with pytest.raises(RuntimeError, match="shape changed"):
            with grad_accum.accumulation_scope():
                grad_accum.set_direct(True)
                grad_accum.deferred(p, "t", (2, 4), p.device)
                grad_accum.deferred(p, "t", (3, 4), p.device)
        # partials of a no-sync micro-step that the sync micro-step never reduces
        with pytest.raises(RuntimeError, match="never reduced"):
            with grad_accum.accumulation_scope():
                grad_accum.set_direct(True)
                grad_accum.deferred(p, "t", (2, 4), p.device)
                grad_accum.set_direct(False)
        # the next step starts clean
        with grad_accum.accumulation_scope():
            grad_accum.set_direct(False)
            assert grad_accum.deferred(p, "t", (3, 4), p.device)[1] == 3
    finally:
        grad_accum.release_buffers()
