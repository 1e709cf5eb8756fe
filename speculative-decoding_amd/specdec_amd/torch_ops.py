"""torch.library registration of the hot-path entry points ("wrapped by
torch.library ops"), so the sampler and the verify step are dispatcher-visible operators —
traceable by torch.compile / torch.export (fake implementations give output shapes without a
GPU), and callable as ``torch.ops.specdec.*``.

    torch.ops.specdec.sample(logits [R, V], kind, temperature, top_k, top_p, seed, offset, row_base)
        -> (tokens int64 [R], row_stats fp32 [R, 2], row_status int32 [R])
        LogitsProcessor.__call__ + .sample per row (utils/logits_processor.py:13-103), Philox noise.
    torch.ops.specdec.verify(target [B, T, V], draft [B, γ, V], draft_tokens int64 [B, >=γ], stop_tokens int64 [n],
                             rule, kind, temperature, top_k, top_p, seed, offset, row_base)
        -> (n_accepted int32 [B], next_token int64 [B], resample_mass fp32 [B], prune_drafter int32 [B],
            prune_target int32 [B], stop_index int32 [B], row_status int32 [B])
        One verify step: rule 0 = sampling/speculative_decoding.py:129-187 (T = γ+1 target rows),
        rule 1 = engine/infer_engine.py:276-336 (T = γ, plain softmax), Philox noise.

Both run the same C-ABI calls as ``specdec_amd.ops`` (libspecdec.so); the parity STREAM noise
mode keeps generator state on the host side and stays on the Python API.
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch import Tensor

from . import _lib, ops
from .noise import PhiloxNoise

_KINDS = {v: k for k, v in ops.KIND.items()}


def _spec(kind: int, temperature: float, top_k: int, top_p: float) -> ops.ProcSpec:
    if kind not in _KINDS:
        raise ValueError(f"unknown processor kind {kind}")
    return ops.ProcSpec(_KINDS[kind], float(temperature), int(top_k), float(top_p))


@torch.library.custom_op("specdec::sample", mutates_args=())
def sample(logits: Tensor, kind: int, temperature: float, top_k: int, top_p: float, seed: int, offset: int,
           row_base: int) -> Tuple[Tensor, Tensor, Tensor]:
    R = logits.shape[0]
    stats = torch.empty(R, 2, dtype=torch.float32, device=logits.device)
    tokens, _, status = ops.sample_rows(logits, _spec(kind, temperature, top_k, top_p),
                                        PhiloxNoise(seed, offset), row_base=row_base, row_stats_out=stats)
    return tokens, stats, status


@sample.register_fake
def _(logits, kind, temperature, top_k, top_p, seed, offset, row_base):
    R = logits.shape[0]
    return (logits.new_empty(R, dtype=torch.long), logits.new_empty(R, 2, dtype=torch.float32),
            logits.new_empty(R, dtype=torch.int32))


@torch.library.custom_op("specdec::verify", mutates_args=())
def verify(target: Tensor, draft: Tensor, draft_tokens: Tensor, stop_tokens: Tensor, rule: int, kind: int,
           temperature: float, top_k: int, top_p: float, seed: int, offset: int,
           row_base: int) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    gamma = draft.shape[1]
    spec = _spec(kind, temperature, top_k, top_p) if rule == _lib.SD_RULE_SPEC else ops.PLAIN_SOFTMAX
    out = ops.verify([target[:, t] for t in range(target.shape[1])], [draft[:, d] for d in range(gamma)],
                     draft_tokens, rule, spec, spec, PhiloxNoise(seed, offset), stop_tokens, row_base=row_base)
    # ops.verify hands back views of one device buffer; a custom op's outputs may not alias each other
    return tuple(t.clone() for t in (out.n_accepted, out.next_token, out.resample_mass, out.prune_drafter,
                                     out.prune_target, out.stop_index, out.row_status))


@verify.register_fake
def _(target, draft, draft_tokens, stop_tokens, rule, kind, temperature, top_k, top_p, seed, offset, row_base):
    B = target.shape[0]
    i32 = dict(dtype=torch.int32)
    return (target.new_empty(B, **i32), target.new_empty(B, dtype=torch.long),
            target.new_empty(B, dtype=torch.float32), target.new_empty(B, **i32), target.new_empty(B, **i32),
            target.new_empty(B, **i32), target.new_empty(B, **i32))
