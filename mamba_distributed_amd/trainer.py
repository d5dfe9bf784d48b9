"""The training loop of the reference (train.py:24-244) as a library.

Zero-flag ``TrainArgs()`` reproduces the reference hyper-parameters:
B=32, T=1024, 524,288 tokens/step, lr 6e-4 -> 6e-5 (warmup 715, cosine to 19,073), wd 0.1,
AdamW(0.9, 0.95, 1e-8, fused), clip 1.0, bf16 autocast, seed 1337, val 20x every 250 steps,
checkpoint every 1000, samples every 250, ``MambaConfig(d_model=768, vocab_size=50304)``.

Log formats are kept byte-compatible (train.py:151, 237-241): ``"{step} val {:.4f}"``,
``"{step} train {:.6f}"`` and the ``step {:5d} | loss: ... | tok/sec: ...`` stdout line.
Additions: flags (model preset, Mamba1/Mamba2, sizes, synthetic data, steps, DDP knobs), resume
(optimizer + every rank's loader position + RNG in the checkpoint), steady-state tok/s excluding
eval steps (A10), optional JSONL metrics, and a fault-injection hook for the elastic-restart test
(SURVEY.md §5.3): ``MAMBA_AMD_FAULT_AT_STEP=k`` [``MAMBA_AMD_FAULT_RANK=r``] kills rank r at the start
of step k on the first torchrun attempt; ``torchrun --max-restarts N ... train.py --resume`` then
restarts every worker from the latest checkpoint.

Checkpoint timing follows the reference: ``model_{step}.pt`` is written at the START of ``step``
(after validation, before that step's update), so resuming from it re-runs ``step``.
"""
from __future__ import annotations

import json
import os
import time
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn.functional as F

from .config import MambaConfig, preset
from .data.loader import DataLoaderLite, SyntheticTokens
from .ops import grad_accum
from .lm import LMHeadModel
from .parallel import ddp as ddp_mod
from .parallel.api import clip_grad_norm_ as par_clip_grad_norm_
from .parallel.api import full_state_dict, parallelize, sync_tp_grads
from .parallel.dist import all_gather_object, all_reduce_avg, barrier, destroy, init_distributed
from .parallel.groups import init_parallel_groups
from .parallel.microbatch import auto_defer_reduce, resolve_overlap, run_micro_batches
from .utils.checkpoint import latest_checkpoint, load_checkpoint, rng_state, save_checkpoint, set_rng_state
from .utils.lr import get_lr


@dataclass
class TrainArgs:
    total_batch_size: int = 524288
    B: int = 32
    T: int = 1024
    model: Optional[str] = None          # preset name; None -> reference MambaConfig(768, 50304)
    layer: Optional[str] = None          # override ssm_cfg["layer"]: Mamba1 | Mamba2
    n_layer: Optional[int] = None
    d_model: Optional[int] = None
    max_lr: float = 6e-4
    min_lr_ratio: float = 0.1
    warmup_steps: int = 715
    max_steps: int = 19073               # schedule length (reference)
    steps: Optional[int] = None          # stop after this many steps (default: max_steps)
    weight_decay: float = 0.1
    grad_clip: float = 1.0
    val_every: int = 250
    val_steps: int = 20
    ckpt_every: int = 1000
    sample_every: int = 250              # <= 0: never sample
    data_root: str = "edu_fineweb10B"
    synthetic: bool = False
    log_dir: str = "log"
    seed: int = 1337
    backend: str = "auto"
    bucket_cap_mb: float = 100.0
    grad_comm_dtype: str = "fp32"
    dp_impl: str = "native"              # "native" bucketed reducer (parallel/reducer.py) or "ddp"
    resume: bool = False
    fused_ce: bool = True
    save_optimizer: bool = True
    allow_optimizer_reset: bool = False  # resume even when the checkpoint holds no (matching) optimizer state
    metrics_jsonl: Optional[str] = None
    sample_prompt: str = "Hello, I'm a language model,"
    device_type: str = "auto"
    tuned_gemms: bool = True             # replay the shipped gfx950 hipBLASLt solution table (only consulted when a
                                         # library GEMM can run: the MAMBA_AMD_PROJ_GEMM / MAMBA_AMD_LMHEAD A/B switches)
    fp32_matmul_precision: str = "highest"  # reference train.py uses "high" (A100 TF32); gfx950 has no
                                            # xf32 and the tuned GEMM table needs "highest" (utils/gemm_tuning)
    tp: int = 1                          # tensor parallel degree (Mamba-2 heads; parallel/tensor_parallel.py)
    cp: int = 1                          # context parallel degree (sequence shards; parallel/context_parallel.py)
    sequence_parallel: bool = False      # with tp > 1: shard the residual stream over tokens as well
    activation_checkpointing: int = 0   # recompute every N-th block in the backward (0 = off)
    overlap_microbatches: str = "auto"   # next micro-batch's forward beside the current backward (GPU):
                                         # auto (d_model <= 1024, parallel/microbatch.py::auto_overlap) / on / off


def build_config(a: TrainArgs) -> MambaConfig:
    cfg = preset(a.model) if a.model else MambaConfig(d_model=768, vocab_size=50304)
    if a.layer:
        cfg.ssm_cfg = dict(cfg.ssm_cfg, layer=a.layer)
    if a.n_layer:
        cfg.n_layer = a.n_layer
    if a.d_model:
        cfg.d_model = a.d_model
    return cfg


class Trainer:
    def __init__(self, args: TrainArgs):
        self.a = a = args
        self.info = init_distributed(a.backend, a.device_type)
        self.device = self.info.device
        self.device_type = "cuda" if self.device.startswith("cuda") else "cpu"
        self.master = self.info.master
        torch.manual_seed(a.seed)
        if torch.cuda.is_available():
            torch.cuda.manual_seed(a.seed)
        self.groups = init_parallel_groups(a.tp, a.cp)
        # ranks of one TP x CP group consume the same batch: the data-parallel world is dp
        world, data_rank = self.groups.dp, self.groups.dp_rank
        self.data_world = world
        assert a.total_batch_size % (a.B * a.T * world) == 0, \
            "make sure total_batch_size is divisible by B * T * ddp_world_size"
        self.grad_accum_steps = a.total_batch_size // (a.B * a.T * world)
        if self.master:
            print(f"total desired batch size: {a.total_batch_size}")
            print(f"=> calculated gradient accumulation steps: {self.grad_accum_steps}")
        self.config = build_config(a)
        if a.synthetic:
            self.train_loader = SyntheticTokens(a.B, a.T, self.config.vocab_size, data_rank, world,
                                                device=self.device, seed=a.seed)
            self.val_loader = SyntheticTokens(a.B, a.T, self.config.vocab_size, data_rank, world,
                                              device=self.device, seed=a.seed + 1)
        else:
            self.train_loader = DataLoaderLite(a.B, a.T, data_rank, world, "train", self.master, a.data_root)
            self.val_loader = DataLoaderLite(a.B, a.T, data_rank, world, "val", self.master, a.data_root)
        if self.device_type == "cuda":
            torch.set_float32_matmul_precision(a.fp32_matmul_precision)
            from .ops.linear import library_gemms_possible
            if a.tuned_gemms and (library_gemms_possible(self.config) or os.environ.get("MAMBA_AMD_LMHEAD") == "lib"):
                from .utils.gemm_tuning import enable_tuned_gemms
                enable_tuned_gemms()
        self.raw_model = LMHeadModel(self.config, device=self.device)
        self.raw_model.to(self.device)
        if a.activation_checkpointing:
            self.raw_model.set_activation_checkpointing(a.activation_checkpointing)
        if self.master:
            total = int(sum(p.numel() for p in self.raw_model.parameters()) // 1e6)
            print(f"Total number of parameters: {total}M")
        os.makedirs(a.log_dir, exist_ok=True)
        self.log_file = os.path.join(a.log_dir, "log.txt")
        self.start_step = 0
        self.resumed_at = None
        ck = self._load_model_checkpoint() if a.resume else None   # full layout: before sharding
        self.parallel = a.tp > 1 or a.cp > 1
        if self.parallel:
            parallelize(self.raw_model, self.groups, a.sequence_parallel)
            grp = self.groups.dp_cp_group
            ddp_info = self.info if self.groups.dp * self.groups.cp > 1 else None
            self.model = (ddp_mod.wrap_data_parallel(self.raw_model, ddp_info, a.dp_impl, a.bucket_cap_mb,
                                                     a.grad_comm_dtype, process_group=grp)
                          if ddp_info is not None else self.raw_model)
        else:
            self.model = ddp_mod.wrap_data_parallel(self.raw_model, self.info, a.dp_impl, a.bucket_cap_mb,
                                                    a.grad_comm_dtype)
        self.optimizer = self.raw_model.configure_optimizers(a.weight_decay, a.max_lr, self.device_type, self.master)
        if not self.parallel:  # TP / CP: sync_tp_grads and the TP clip read .grad (the average stays in finish())
            ddp_mod.configure_grad_average(self.model, self.optimizer)
        if ck is not None:
            self._resume_rest(ck)
        if self.master and self.start_step == 0:
            with open(self.log_file, "w"):
                pass
        self.enc = self.raw_model.enc
        self.step_times = []

    # ------------------------------------------------------------------
    def lr(self, it):
        a = self.a
        return get_lr(it, a.max_lr, a.max_lr * a.min_lr_ratio, a.warmup_steps, a.max_steps)

    def _autocast(self):
        return torch.autocast(device_type=self.device_type, dtype=torch.bfloat16)

    def _batch(self, loader):
        x, y = loader.next_batch()
        return x.to(self.device, non_blocking=True), y.to(self.device, non_blocking=True)

    def _load_model_checkpoint(self):
        path = latest_checkpoint(self.a.log_dir)
        if path is None:
            return None
        ck = load_checkpoint(path, map_location=self.device)
        self.raw_model.load_state_dict(ck["model"])
        ck["_path"] = path
        return ck

    def _resume_rest(self, ck):
        path = ck["_path"]
        if "optimizer" in ck and self.a.tp == 1:
            self.optimizer.load_state_dict(ck["optimizer"])
        elif ck.get("optimizer_sharded"):
            shard = f"{path}.optim_rank{self.info.rank}.pt"
            if os.path.exists(shard) and int(ck.get("tp", 0)) == self.a.tp:
                self.optimizer.load_state_dict(load_checkpoint(shard, map_location=self.device)["optimizer"])
            elif not self.a.allow_optimizer_reset:
                raise RuntimeError(f"{shard} missing or saved at another TP degree: resuming would restart the "
                                   "AdamW moments (pass --allow-optimizer-reset to accept that)")
        elif self.a.save_optimizer and not self.a.allow_optimizer_reset:
            raise RuntimeError(f"{path} holds no optimizer state: resuming would restart the AdamW moments "
                               "(pass --allow-optimizer-reset to accept that)")
        if "loader" in ck and hasattr(self.train_loader, "load_state_dict"):
            loaders = ck["loader"]
            if isinstance(loaders, list) and len(loaders) != self.info.world_size and self.master:
                print(f"warning: checkpoint has {len(loaders)} loader states for world size {self.info.world_size}")
            r = self.info.rank
            st = loaders[r] if isinstance(loaders, list) and r < len(loaders) else None
            if st is not None:
                self.train_loader.load_state_dict(st)
        if "rng" in ck:  # per-rank list (older checkpoints: one dict, rank 0's)
            rngs = ck["rng"]
            r = self.info.rank
            set_rng_state(rngs[r] if isinstance(rngs, list) and r < len(rngs) else
                          (rngs[0] if isinstance(rngs, list) else rngs))
        # the checkpoint was taken at the start of ck["step"], before that step's update
        self.start_step = int(ck["step"])
        self.resumed_at = self.start_step
        if self.master:
            print(f"resumed from {path} at step {self.start_step}")

    # ------------------------------------------------------------------
    @torch.no_grad()
    def validate(self):
        self.model.eval()
        self.val_loader.reset()
        val_loss_accum = torch.zeros((), device=self.device)
        for _ in range(self.a.val_steps):
            x, y = self._batch(self.val_loader)
            with self._autocast():
                _, loss = self.model(x, y, return_logits=False)
            val_loss_accum += loss.detach().float() / self.a.val_steps
        all_reduce_avg(val_loss_accum)
        return val_loss_accum.item()

    @torch.no_grad()
    def sample(self, num_return_sequences=4, max_length=32):
        if self.a.cp > 1 or self.a.sequence_parallel:
            return  # the sharded forward needs full-length, divisible sequences
        self.model.eval()
        tokens = torch.tensor(self.enc.encode(self.a.sample_prompt), dtype=torch.long)
        xgen = tokens.unsqueeze(0).repeat(num_return_sequences, 1).to(self.device)
        sample_rng = torch.Generator(device=self.device)
        sample_rng.manual_seed(42 + self.info.rank)
        while xgen.size(1) < max_length:
            with self._autocast():
                logits, _ = self.model(xgen)
            last = logits[:, -1, :].float()
            if not bool(torch.isfinite(last).all()):  # multinomial would hit a device-side assert
                print(f"rank {self.info.rank} sample: non-finite logits, skipping")
                return
            probs = F.softmax(last, dim=-1)
            topk_probs, topk_indices = torch.topk(probs, 50, dim=-1)
            ix = torch.multinomial(topk_probs, 1, generator=sample_rng)
            xgen = torch.cat((xgen, torch.gather(topk_indices, -1, ix)), dim=1)
        for i in range(num_return_sequences):
            print(f"rank {self.info.rank} sample {i}: {self.enc.decode(xgen[i, :max_length].tolist())}")

    def train_step(self, step):
        self.model.train()
        ddp_mod.zero_grad(self.model, self.optimizer)
        def compute_loss(x, y):
            with self._autocast():
                _, loss = self.model(x, y, return_logits=not self.a.fused_ce)
            return loss / self.grad_accum_steps

        # overlap micro-batch k+1's forward with k's backward on a second stream (parallel/microbatch.py);
        # not under TP/CP, whose per-layer collectives must be issued on one stream per communicator
        overlap = (resolve_overlap(self.a.overlap_microbatches, self.raw_model.config, self.a.B * self.a.T)
                   and self.device_type == "cuda" and not self.parallel)
        with grad_accum.accumulation_scope(defer_reduce=auto_defer_reduce(self.raw_model.config)):  # weights are frozen until optimizer.step()
            loss_accum = run_micro_batches(self.model, lambda: self._batch(self.train_loader), self.grad_accum_steps,
                                           compute_loss, overlap=overlap)
        all_reduce_avg(loss_accum)
        lr = self.lr(step)
        for g in self.optimizer.param_groups:
            g["lr"] = lr
        if self.parallel:
            sync_tp_grads(self.model, self.groups)
            norm = par_clip_grad_norm_(self.model, self.a.grad_clip, self.groups)
            self.optimizer.step()
        else:
            # clip + AdamW (one norm pass and one update pass on the native optimizer, parallel/ddp.py)
            norm = ddp_mod.clip_and_step(self.model, self.optimizer, self.a.grad_clip)
        return loss_accum, norm, lr

    def save(self, step, val_loss):
        """Collective (every rank calls it): gathers all ranks' loader positions and RNG states,
        rank 0 writes the model checkpoint.  Under tensor parallelism every rank also writes its own
        optimizer shard next to it (``<ckpt>.optim_rank{r}.pt``): the AdamW moments live in the
        sharded layout, so resume restores them rank by rank."""
        st = self.train_loader.state_dict() if hasattr(self.train_loader, "state_dict") else None
        loader_states = all_gather_object(st)
        rngs = all_gather_object(rng_state())
        full_sd = full_state_dict(self.raw_model) if self.a.tp > 1 else None   # collective over TP
        path = os.path.join(self.a.log_dir, f"model_{step:05d}.pt")
        if self.a.tp > 1 and self.a.save_optimizer:
            os.makedirs(self.a.log_dir, exist_ok=True)
            shard = f"{path}.optim_rank{self.info.rank}.pt"
            torch.save({"optimizer": self.optimizer.state_dict(), "rank": self.info.rank,
                        "world_size": self.info.world_size, "tp": self.a.tp}, shard + ".tmp")
            os.replace(shard + ".tmp", shard)
        barrier()  # every shard is on disk before the model file that points at them
        if not self.master:
            return None
        opt = self.optimizer if (self.a.save_optimizer and self.a.tp == 1) else None
        save_checkpoint(path, self.raw_model, step, val_loss, optimizer=opt,
                        loader_state=loader_states if st is not None else None,
                        model_state=full_sd, extra={"rng": rngs, "tp": self.a.tp,
                                                    "optimizer_sharded": self.a.tp > 1 and self.a.save_optimizer})
        return path

    def _maybe_inject_fault(self, step):
        at = os.environ.get("MAMBA_AMD_FAULT_AT_STEP")
        if at is None or int(at) != step or os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") != "0":
            return
        if self.info.rank == int(os.environ.get("MAMBA_AMD_FAULT_RANK", "0")):
            print(f"[fault-injection] rank {self.info.rank} exiting at step {step}", flush=True)
            os._exit(17)

    def run(self):
        a = self.a
        last = (a.steps if a.steps is not None else a.max_steps)
        metrics = open(a.metrics_jsonl, "a") if (a.metrics_jsonl and self.master) else None
        for step in range(self.start_step, last):
            t0 = time.time()
            last_step = step == last - 1
            eval_step = False
            resumed_here = step == self.resumed_at  # its validation/checkpoint happened before the restart
            if (step % a.val_every == 0 or last_step) and not resumed_here:
                eval_step = True
                val_loss = self.validate()
                if self.master:
                    print(f"validation loss: {val_loss:.4f}")
                    with open(self.log_file, "a") as f:
                        f.write(f"{step} val {val_loss:.4f}\n")
                if step > 0 and (step % a.ckpt_every == 0 or last_step):
                    self.save(step, val_loss)
            if (a.sample_every > 0 and ((step > 0 and step % a.sample_every == 0) or last_step)
                    and not resumed_here):
                eval_step = True
                self.sample()
            self._maybe_inject_fault(step)
            loss_accum, norm, lr = self.train_step(step)
            if self.device_type == "cuda":
                torch.cuda.synchronize()
            dt = time.time() - t0
            tokens_processed = a.B * a.T * self.grad_accum_steps * self.data_world
            tps = tokens_processed / dt
            if not eval_step:
                self.step_times.append(dt)
            if self.master:
                print(f"step {step:5d} | loss: {loss_accum.item():.6f} | lr {lr:.4e} | norm: {norm:.4f} | "
                      f"dt: {dt*1000:.2f}ms | tok/sec: {tps:.2f}")
                with open(self.log_file, "a") as f:
                    f.write(f"{step} train {loss_accum.item():.6f}\n")
                if metrics:
                    metrics.write(json.dumps({"step": step, "loss": loss_accum.item(), "lr": lr,
                                              "norm": float(norm), "dt_ms": dt * 1000, "tok_s": tps,
                                              "eval_step": eval_step}) + "\n")
                    metrics.flush()
        if self.master and self.step_times:
            ts = sorted(self.step_times[1:] or self.step_times)
            med = ts[len(ts) // 2]
            print(f"steady-state median step {med*1000:.1f} ms, "
                  f"{a.B * a.T * self.grad_accum_steps * self.data_world / med:.1f} tok/s "
                  f"(excluding eval/sample steps)")
        if metrics:
            metrics.close()
        # the deferred-reduction slabs (~66 MB per 280M out_proj) and partial buffers are dead once training
        # ends: free them before any in-process eval / generation
        from .ops import grad_accum
        grad_accum.release_buffers()
        destroy()


