"""Native AdamW step (csrc/kernels/optim.hip): torch.optim.AdamW semantics, one multi-tensor launch.

Reference: /root/reference/model.py:146-148 (``torch.optim.AdamW(optim_groups, lr, betas=(0.9, 0.95), eps=1e-8,
fused=True)``), /root/reference/train.py:222 (``clip_grad_norm_(model.parameters(), 1.0)``) and :227
(``optimizer.step()``); SURVEY.md G8 / G9.

What it folds, per optimizer step:
  * the gradient clip: ONE sum-of-squares pass over every gradient and a one-block launch that turns it into the
    clip coefficient on the device (``clip_and_step``); the update multiplies each gradient by it as it reads it,
    so there is no separate scale pass over the gradients;
  * the data-parallel average: with the native reducer (parallel/reducer.py) the reducer can leave the summed
    gradients unscaled and the 1/world factor rides on the same coefficient (``clip_and_step(grad_divisor=...)``,
    passed explicitly per call from the reducer's state);
  * the bf16 weight images: the projection GEMMs of the next step read bf16 copies of the weights (plain casts, and
    the zero-padded in_proj rows of ops/linear.py).  The update pass writes them from the updated fp32 value it
    already holds (ops/grad_accum.py image_demand / provide_image), instead of a cast / zero-fill / copy per
    weight per step.

State layout: exp_avg / exp_avg_sq of every parameter are views into two flat fp32 buffers per device, so
``state_dict()`` has torch.optim.AdamW's format ({step, exp_avg, exp_avg_sq} per parameter) and a checkpoint moves
between the two optimizers.  Deterministic: every element has one writer, the norm is a fixed-order reduction.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch

from . import _ext, grad_accum

_SEG_DTYPE = np.dtype([("p", "<u8"), ("g", "<u8"), ("m", "<u8"), ("v", "<u8"), ("img", "<u8"), ("n", "<i8"),
                       ("step_size", "<f4"), ("bc2_rsqrt", "<f4"), ("decay", "<f4"), ("vec", "<i4")])
assert _SEG_DTYPE.itemsize == 64


def native_available(params) -> bool:
    ps = [p for p in params if isinstance(p, torch.Tensor)]
    return (bool(ps) and all(p.is_cuda and p.dtype == torch.float32 for p in ps) and not _ext.force_reference()
            and _ext.load())


def _images_enabled() -> bool:
    """MAMBA_AMD_OPT_IMAGES=0: the update writes no bf16 weight images (the GEMMs cast per step as before)."""
    import os
    return os.environ.get("MAMBA_AMD_OPT_IMAGES", "1") != "0"


class NativeAdamW(torch.optim.Optimizer):
    """AdamW (decoupled weight decay) over fp32 CUDA parameters on the native multi-tensor kernel."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2):
        if lr < 0 or eps < 0 or not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"invalid AdamW hyper-parameters lr={lr} betas={betas} eps={eps}")
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay))
        self._flat: Dict[torch.device, tuple] = {}  # device -> (m, v, {id(p): offset})
        self._imgs: Dict[tuple, torch.Tensor] = {}   # (id(p), kind) -> persistent bf16 image buffer
        self._blk_cache: Dict[tuple, torch.Tensor] = {}

    # ---- state -------------------------------------------------------------------------------------------------
    def _params(self) -> List[torch.Tensor]:
        return [p for g in self.param_groups for p in g["params"]]

    def _ensure_flat(self) -> None:
        """exp_avg / exp_avg_sq of every parameter as views of flat per-device buffers (zero for a fresh state,
        the loaded values after load_state_dict)."""
        by_dev: Dict[torch.device, List[torch.Tensor]] = {}
        for p in self._params():
            by_dev.setdefault(p.device, []).append(p)
        for dev, ps in by_dev.items():
            ent = self._flat.get(dev)
            if ent is not None and all(id(p) in ent[2] for p in ps) and all(
                    self.state[p].get("exp_avg") is not None and self.state[p]["exp_avg"].data_ptr() ==
                    ent[0].data_ptr() + 4 * ent[2][id(p)] for p in ps):
                continue
            total = sum(p.numel() for p in ps)
            m = torch.zeros(total, device=dev, dtype=torch.float32)
            v = torch.zeros(total, device=dev, dtype=torch.float32)
            offs, off = {}, 0
            for p in ps:
                n = p.numel()
                st = self.state[p]
                mv, vv = m[off:off + n].view_as(p), v[off:off + n].view_as(p)
                if "exp_avg" in st:  # loaded (or torch-AdamW) state: copy into the flat buffers
                    mv.copy_(st["exp_avg"].to(device=dev, dtype=torch.float32))
                    vv.copy_(st["exp_avg_sq"].to(device=dev, dtype=torch.float32))
                st["exp_avg"], st["exp_avg_sq"] = mv, vv
                s = st.get("step", 0.0)
                st["step"] = torch.tensor(float(s.item() if isinstance(s, torch.Tensor) else s), dtype=torch.float32)
                offs[id(p)] = off
                off += n
            self._flat[dev] = (m, v, offs)

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._flat.clear()
        self._ensure_flat()

    # ---- images ------------------------------------------------------------------------------------------------
    def _image_for(self, p: torch.Tensor, wanted: Dict[int, List[tuple]]) -> Optional[tuple]:
        """(buffer the update writes, [(kind, tensor to register)]) for parameter p, or None."""
        kinds = wanted.get(id(p))
        if not kinds or p.dim() != 2 or not p.is_contiguous():
            return None
        pad = [k for k in kinds if k[0] == "pad_rows" and k[1] == torch.bfloat16]
        cast = [k for k in kinds if k[0] == "cast" and k[1] == torch.bfloat16]
        if pad:
            k = pad[0]
            key = (id(p), k)
            buf = self._imgs.get(key)
            if buf is None or buf.shape != (k[2], p.shape[1]):
                buf = torch.zeros(k[2], p.shape[1], device=p.device, dtype=torch.bfloat16)  # pad rows stay zero
                self._imgs[key] = buf
            reg = [(k, buf)] + [(c, buf[:p.shape[0]]) for c in cast]
            return buf, reg
        if cast:
            k = cast[0]
            key = (id(p), k)
            buf = self._imgs.get(key)
            if buf is None or buf.shape != p.shape:
                buf = torch.empty(p.shape, device=p.device, dtype=torch.bfloat16)
                self._imgs[key] = buf
            return buf, [(k, buf)]
        return None

    # ---- tables ------------------------------------------------------------------------------------------------
    def _tables(self, group_filter=None):
        """Per device: (segment table (uint8 CUDA), block table (int64 CUDA, (nblk, 2)), [(param, registrations)],
        per-group block ranges)."""
        self._ensure_flat()
        chunk = int(_ext.ops().opt_chunk())
        wanted: Dict[int, List[tuple]] = {}
        if _images_enabled():
            for p, kind in grad_accum.image_demand():
                wanted.setdefault(id(p), []).append(kind)
        out = {}
        for gi, group in enumerate(self.param_groups):
            lr, wd = group["lr"], group["weight_decay"]
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("NativeAdamW does not support sparse gradients")
                dev = p.device
                ent = out.setdefault(dev, {"rows": [], "keep": [], "regs": [], "sizes": [], "groups": []})
                m, v, offs = self._flat[dev]
                st = self.state[p]
                step = float(st["step"].item()) + 1.0
                g = p.grad if p.grad.is_contiguous() and p.grad.dtype == torch.float32 else \
                    p.grad.contiguous().float()
                if not p.is_contiguous():
                    raise RuntimeError("NativeAdamW needs contiguous parameters")
                img = self._image_for(p, wanted)
                ip = img[0].data_ptr() if img is not None else 0
                mp = m.data_ptr() + 4 * offs[id(p)]
                vp = v.data_ptr() + 4 * offs[id(p)]
                n = p.numel()
                vec = int(all(x % 16 == 0 for x in (p.data_ptr(), g.data_ptr(), mp, vp)) and n % 4 == 0
                          and ip % 8 == 0)
                ent["rows"].append((p.data_ptr(), g.data_ptr(), mp, vp, ip, n, lr / (1.0 - b1 ** step),
                                    1.0 / math.sqrt(1.0 - b2 ** step), 1.0 - lr * wd, vec))
                ent["keep"].append(g)
                ent["regs"].append((p, img[1] if img is not None else []))
                ent["sizes"].append(n)
                ent["groups"].append(gi)
        res = {}
        for dev, ent in out.items():
            seg = np.array(ent["rows"], dtype=_SEG_DTYPE)
            tab = torch.from_numpy(seg.view(np.uint8).copy()).pin_memory().to(dev, non_blocking=True)
            bkey = (dev, tuple(ent["sizes"]), tuple(ent["groups"]))
            cached = self._blk_cache.get(bkey)
            if cached is None:  # (segment, offset) per chunk; depends only on the parameter sizes and groups
                rows, ranges = [], {}
                for i, (n, gi) in enumerate(zip(ent["sizes"], ent["groups"])):
                    lo = len(rows)
                    rows.extend((i, o) for o in range(0, n, chunk))
                    r = ranges.get(gi)
                    ranges[gi] = (r[0] if r else lo, len(rows))
                cached = (torch.tensor(rows, dtype=torch.int64).to(dev), ranges)
                self._blk_cache[bkey] = cached
            res[dev] = (tab, cached[0], ent["regs"], cached[1], ent["keep"])
        if len(res) > 1:
            raise RuntimeError("NativeAdamW: parameters on more than one device (one process per GPU)")
        return res

    # ---- step --------------------------------------------------------------------------------------------------
    @torch.no_grad()
    def clip_and_step(self, max_norm: float, grad_divisor: float = 1.0) -> torch.Tensor:
        """clip_grad_norm_(params, max_norm) followed by step(), as one norm pass + one update pass, on the gradients
        DIVIDED by ``grad_divisor`` (the native reducer's deferred 1/world average: parallel/ddp.py::clip_and_step
        passes reducer.grad_divisor).  Returns the total norm of the divided gradients."""
        return self._run(max_norm, float(grad_divisor))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._run(None, 1.0)
        return loss

    def _run(self, max_norm: Optional[float], grad_divisor: float):
        ops = _ext.ops()
        norm = None
        for dev, (tab, blk, regs, ranges, keep) in self._tables().items():
            gscale = None
            if max_norm is not None or grad_divisor != 1.0:
                gscale = ops.opt_grad_norm(tab, blk, float(max_norm) if max_norm is not None else 0.0, grad_divisor)
                norm = gscale[0]
            for gi, group in enumerate(self.param_groups):
                r = ranges.get(gi)
                if r is None:
                    continue
                b1, b2 = group["betas"]
                ops.opt_adamw(tab, blk[r[0]:r[1]], gscale, float(b1), float(b2), float(group["eps"]))
            for p, reg in regs:
                self.state[p]["step"] += 1.0
                for kind, t in reg:
                    grad_accum.provide_image(p, kind, t)
            del keep
        if norm is None:
            norm = torch.zeros((), device=self._params()[0].device)
        return norm
