"""torchrun worker for tests/test_parallel_gloo.py (not collected by pytest: no test_ prefix).

Every rank builds the same full model and batch, computes the single-process reference loss and
gradients locally, then runs the TP / SP / CP form of the same model on the same batch and checks
that loss, global grad norm and the reassembled full gradients (and parameters) match.
"""
import argparse
import copy
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mamba_distributed_amd import LMHeadModel, MambaConfig  # noqa: E402
from mamba_distributed_amd.parallel.api import (full_state_dict, grad_norm, parallelize,  # noqa: E402
                                                sync_tp_grads)
from mamba_distributed_amd.parallel.dist import init_distributed  # noqa: E402
from mamba_distributed_amd.parallel.groups import init_parallel_groups  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--cp", type=int, default=1)
    ap.add_argument("--sp", action="store_true")
    ap.add_argument("--ngroups", type=int, default=1)
    ap.add_argument("--T", type=int, default=64)
    a = ap.parse_args()
    info = init_distributed("gloo", "cpu")
    groups = init_parallel_groups(a.tp, a.cp)
    torch.manual_seed(0)
    cfg = MambaConfig(d_model=128, n_layer=2, vocab_size=512,
                      ssm_cfg={"layer": "Mamba2", "d_state": 16, "headdim": 16, "ngroups": a.ngroups})
    ref = LMHeadModel(cfg, device="cpu", enc=object())
    model = copy.deepcopy(ref)
    g = torch.Generator().manual_seed(1)
    x = torch.randint(0, 512, (2, a.T), generator=g)
    y = torch.randint(0, 512, (2, a.T), generator=g)

    _, lref = ref(x, y)
    lref.backward()
    ref_grads = {k: p.grad.clone() for k, p in ref.named_parameters()}
    ref_norm = torch.sqrt(sum(v.pow(2).sum() for v in ref_grads.values()))

    parallelize(model, groups, sequence_parallel=a.sp)
    _, loss = model(x, y)
    loss.backward()
    sync_tp_grads(model, groups)
    if groups.cp > 1:  # what DDP over the DP x CP group does
        loss = loss.detach().clone()
        dist.all_reduce(loss, group=groups.cp_group)
        loss /= groups.cp
        for p in model.parameters():
            if p.grad is not None:
                dist.all_reduce(p.grad, group=groups.cp_group)
                p.grad /= groups.cp
    torch.testing.assert_close(loss.detach(), lref.detach(), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(grad_norm(model), ref_norm, rtol=1e-4, atol=1e-6)

    sd = full_state_dict(model)
    ref_sd = ref.state_dict()
    assert sorted(sd) == sorted(ref_sd), set(sd) ^ set(ref_sd)
    for k in ref_sd:
        torch.testing.assert_close(sd[k], ref_sd[k], rtol=0, atol=0, msg=k)
    # gradients in the upstream layout: swap grads into the params and reassemble
    params = list(model.parameters())
    saved = [p.data for p in params]
    for p in params:
        p.data = p.grad if p.grad is not None else torch.zeros_like(p)
    gsd = full_state_dict(model)
    for p, d in zip(params, saved):
        p.data = d
    name_of = {id(p): k for k, p in ref.named_parameters()}
    for k, t in ref.state_dict(keep_vars=True).items():
        kk = name_of.get(id(t), k)
        torch.testing.assert_close(gsd[k], ref_grads[kk], rtol=2e-4, atol=2e-6, msg=k)
    if info.rank == 0:
        print(f"PARALLEL_OK tp={a.tp} cp={a.cp} sp={a.sp} ngroups={a.ngroups} loss={loss.item():.6f}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
