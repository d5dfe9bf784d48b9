"""mamba-ssm-compatible generation (upstream ``mamba_ssm/utils/generation.py``: ``GenerationMixin.generate``
-> ``decode``), so code written against ``MambaLMHeadModel.generate(input_ids, max_length, top_k, top_p,
min_p, temperature, repetition_penalty, eos_token_id, cg=...)`` runs unchanged.

The token loop is ours: the prompt runs through the chunked native kernels (one prefill pass filling the
conv / SSM caches), and every later token is one cached decode step -- with ``cg=True`` the whole-stack
step replayed as a HIP graph (``inference.GraphedDecoder``, fused per-layer decode kernels for Mamba-2
stacks), otherwise eager.  Sampling follows upstream's rules (top-k first, then top-p / min-p on what is
left, temperature on the kept logits; top_k=1 is greedy).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple


import torch


@dataclass
class DecodeOutput:
    sequences: torch.Tensor                     # (b, prompt + generated)
    scores: Optional[Tuple[torch.Tensor, ...]] = None  # per generated token: (b, V) logits before the penalty


def modify_logits_for_top_p_filtering(logits: torch.Tensor, top_p: float) -> None:
    """In place: keep the smallest set of tokens whose probability mass reaches top_p."""
    if top_p <= 0.0 or top_p >= 1.0:
        return
    sorted_logits, sorted_idx = torch.sort(logits, descending=False)
    cum = sorted_logits.softmax(dim=-1).cumsum(dim=-1)
    remove_sorted = cum <= (1 - top_p)
    remove = remove_sorted.scatter(1, sorted_idx, remove_sorted)
    logits.masked_fill_(remove, float("-inf"))


def modify_logits_for_min_p_filtering(logits: torch.Tensor, min_p: float) -> None:
    """In place: drop tokens whose probability is below min_p times the most likely one's."""
    if min_p <= 0.0 or min_p >= 1.0:
        return
    probs = logits.softmax(dim=-1)
    logits.masked_fill_(probs < min_p * probs.max(dim=-1, keepdim=True).values, float("-inf"))


def modify_logit_for_repetition_penalty(logits: torch.Tensor, prev_tokens: torch.Tensor, penalty: float = 1.0):
    """Upstream / CTRL rule: a seen token's logit is divided by the penalty if positive, else multiplied."""
    if penalty == 1.0:
        return logits
    score = torch.gather(logits, 1, prev_tokens)
    score = torch.where(score < 0, score * penalty, score / penalty)
    logits.scatter_(1, prev_tokens, score)
    return logits


def sample(logits: torch.Tensor, top_k: int = 1, top_p: float = 0.0, min_p: float = 0.0,
           temperature: float = 1.0) -> torch.Tensor:
    """(b, V) logits -> (b,) token ids."""
    if top_k == 1:
        return logits.argmax(dim=-1)
    if top_p > 0.0:
        assert top_p <= 1.0, "top_p must be <= 1.0"
    if top_k > 0:
        top_k = min(top_k, logits.size(-1))
        top, idx = torch.topk(logits, top_k, dim=-1)
        if temperature != 1.0:
            top = top / temperature
        modify_logits_for_top_p_filtering(top, top_p)
        pick = torch.multinomial(torch.softmax(top, dim=-1), num_samples=1).squeeze(-1)
        return idx[torch.arange(idx.shape[0], device=idx.device), pick]
    work = logits / temperature if temperature != 1.0 else logits.clone()
    modify_logits_for_min_p_filtering(work, min_p)
    modify_logits_for_top_p_filtering(work, top_p)
    return torch.multinomial(torch.softmax(work, dim=-1), num_samples=1).squeeze(-1)


def _param_signature(model) -> tuple:
    """Storage pointers and dtypes of every parameter: a captured graph reads these addresses, so a decoder is
    only reused while none of them changed (``.to(dtype)``, ``.cuda()``, ``load_state_dict(assign=True)``)."""
    return tuple((p.data_ptr(), p.dtype) for p in model.parameters())


def _decoder_cache(model) -> dict:
    """The model's decoder cache {(b, max_length, cg, dev): (signature, decoder)}, kept as a plain attribute of
    the model itself: the model -> cache -> decoder -> model cycle is collected with the model (a module-level
    WeakKeyDictionary whose values hold the model strongly never released it)."""
    cache = model.__dict__.get("_amd_decoders")
    if cache is None:
        cache = {}
        object.__setattr__(model, "_amd_decoders", cache)
    return cache


@torch.no_grad()
def decode(input_ids: torch.Tensor, model, max_length: int, top_k: int = 1, top_p: float = 0.0,
           min_p: float = 0.0, temperature: float = 1.0, repetition_penalty: float = 1.0,
           eos_token_id: Optional[int] = None, teacher_outputs: Optional[torch.Tensor] = None,
           vocab_size: Optional[int] = None, cg: bool = False, output_scores: bool = False,
           **_ignored) -> DecodeOutput:
    """Generate until ``max_length`` total tokens (prompt included) or until every row emitted
    ``eos_token_id``.  ``teacher_outputs`` (b, >= max_length) forces those tokens (testing), and
    ``vocab_size`` masks the padded vocabulary rows of the logits."""
    from ..inference import GraphedDecoder
    b, l0 = input_ids.shape
    dev = input_ids.device
    # one decoder (caches + captured graph) per (batch, max_length, cg), kept on the model like upstream's
    # graph cache; reused calls reset the states and re-derive the fused step's weight copies
    cache = _decoder_cache(model)
    key = (b, max_length, bool(cg), dev)
    sig = _param_signature(model)
    ent = cache.get(key)
    if ent is None or ent[0] != sig:
        cache.pop(key, None)  # parameters moved or changed dtype: the captured graph reads stale addresses
        # NB every rebuild re-captures the decode graph, and each persistent-GEMM launch captured into a graph
        # holds one of a fixed number of tile-claim counter pairs for the life of the process
        # (gemm_pipe.hip PK_CAPTURED = 8192; the capture fails with a clear error once they are spent)
        dec = GraphedDecoder(model, batch_size=b, max_seqlen=max_length, use_graph=None if cg else False)
        cache[key] = (sig, dec)
    else:
        dec = ent[1]
        dec.refresh()
    seqs = [input_ids]
    scores = []
    logits = dec.prefill(input_ids)
    done = torch.zeros(b, dtype=torch.bool, device=dev)
    while True:
        logits = logits.float()
        if vocab_size is not None:
            logits = logits[:, :vocab_size]
        if output_scores:  # the raw logits, like upstream (the penalty only shapes the sampling copy)
            scores.append(logits.clone())
        work = logits
        if repetition_penalty != 1.0:
            work = modify_logit_for_repetition_penalty(logits.clone(), torch.cat(seqs, 1), repetition_penalty)
        pos = sum(s.shape[1] for s in seqs)
        if teacher_outputs is not None and pos < teacher_outputs.shape[1]:
            tok = teacher_outputs[:, pos]
        else:
            tok = sample(work, top_k=top_k, top_p=top_p, min_p=min_p, temperature=temperature)
        seqs.append(tok.unsqueeze(1))
        if eos_token_id is not None:
            done |= tok == eos_token_id
        if pos + 1 >= max_length or bool(done.all()):
            break
        logits = dec.step(tok)
    return DecodeOutput(sequences=torch.cat(seqs, 1), scores=tuple(scores) if output_scores else None)


class GenerationMixin:
    """``generate`` with upstream's signature, for ``MambaLMHeadModel``."""

    def generate(self, input_ids, max_length, top_k=1, top_p=0.0, min_p=0.0, temperature=1.0,
                 return_dict_in_generate=False, output_scores=False, **kwargs):
        out = decode(input_ids, self, max_length, top_k=top_k, top_p=top_p, min_p=min_p,
                     temperature=temperature, output_scores=output_scores, **kwargs)
        return out if return_dict_in_generate else out.sequences
