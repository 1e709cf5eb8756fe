"""Verify windows of more than SD_MAX_GAMMA drafts.

The reference takes any γ (sampling/speculative_decoding.py:106, engine/infer_engine.py:216,
ngram_assisted/ngram_assisted.py:98); the C ABI verifies at most SD_MAX_GAMMA drafts per call.  A
longer window runs as consecutive chunks of <= SD_MAX_GAMMA drafts, and the chunks' outputs are
combined on the device so that the result — accept count, token, stop position, KV prune lengths,
engine state, words of the torch generator consumed — is the one call over the whole window:

* ENGINE (rule A10, :287-336).  The walk is serial in the drafts and the reference draws row after
  row (one uniform per visited draft, 2V words for a residual), so a row's chunk k+1 continues
  exactly where its chunk k stopped: it runs only for rows that accepted every draft of chunk k
  without finishing (``active``), with the engine state's ``step`` advanced by the chunk start.
  Under STREAM noise the calls go row by row (each row's chunks in order, the generator moved by
  each call's device count), so the words are consumed in the reference's row-serial order — B·⌈γ/32⌉
  calls, each ending in a device→host read of the words used: exact, but slow at engine batch sizes
  (a chunked STREAM window is a parity tool; Philox windows of any length are one call per chunk); under
  Philox every chunk runs on all rows at once.  Afterwards the window's tail past each stopped row's
  last accepted draft is zeroed, as :332-336 does for the whole window.
* SPEC (rule A8, :139-171).  ``r = rand(γ)`` is drawn for the whole window before anything else,
  then the residual / bonus row is sampled from the 2V words after it.  Chunk k gets the uniforms
  of its drafts followed by those sample words (STREAM: a small gathered buffer per chunk); its
  bonus row is the next chunk's first target row, so when a chunk accepts everything its sample is
  simply not used.  The decision is the first chunk that rejects (or the last one); the stop scan
  over the accepted drafts is the first chunk, in order, that reports a stop — the accept count
  still includes the later chunks' accepts, as :147 counts them before :150 returns.
* A11 (ngram_assisted.py:111-164).  Compare draw i uses words [2Vi, 2V(i+1)) and only rows before
  the first mismatch are visited, so chunk k's words start at 2V·c_k; the final draw x comes from
  the chunk that mismatches (or the last chunk's bonus row); filler ids are per row.

Under STREAM the SPEC chunks run row by row (each row's words where the one-call layout puts them);
A11 under STREAM needs one sequence (the reference's n-gram loop is batch 1; the kernel's per-row
word windows are sized by the call's γ).  Philox takes any batch.  Every chunk is an ordinary ``ops.verify`` /
``ops.ngram_verify`` call on the HIP library.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib
from .noise import StreamNoise


def chunks(gamma: int) -> List[Tuple[int, int]]:
    """(first draft, drafts) of each chunk of a γ-draft window."""
    m = _lib.SD_MAX_GAMMA
    return [(c, min(m, gamma - c)) for c in range(0, gamma, m)]


class _Words(StreamNoise):
    """A fixed device word buffer for one chunk call: the words the reference consumes at that point.
    The generator itself is moved once per sequence, by the combined count (StreamNoise.consumed)."""

    def __init__(self, words: torch.Tensor):
        super().__init__(None)
        self._words = words

    def prepare(self, n_words: int, device) -> torch.Tensor:
        return self._words

    def consumed(self, count=None, used_dev=None) -> None:
        return None


def _or_errors(status_or: Optional[torch.Tensor], status: torch.Tensor) -> None:
    """status_or |= the SD_ROW_ERROR_MASK bits of any row (device ops, no sync)."""
    if status_or is None or status.numel() == 0:
        return
    for bit in (_lib.SD_ROW_INVALID_DIST, _lib.SD_ROW_NOISE_OVERRUN, _lib.SD_ROW_EXCHANGE_TIMEOUT):
        status_or.bitwise_or_(((status & bit) != 0).any().to(torch.int32) * bit)


def _stop_rank(stop_tokens: Optional[torch.Tensor], tok: torch.Tensor) -> torch.Tensor:
    """Position of each token in the stop list (its first occurrence), 2^30 for none: the loops
    return at the first-LISTED stop token among the accepted drafts (the row-major nonzero of
    eq(drafts[1, n], stop_tokens[S, 1]), sampling/speculative_decoding.py:150-152), so chunks that
    each found a stop are compared by that rank, then by position."""
    big = torch.full_like(tok, 1 << 30)
    if stop_tokens is None or stop_tokens.numel() == 0:
        return big
    eq = stop_tokens.to(tok.device).view(1, -1) == tok.view(-1, 1)
    return torch.where(eq.any(1), eq.to(torch.int32).argmax(1).to(tok.dtype), big)


def _take_stop(stop_tokens, draft_tokens, c, o, t, best, stop_index, seen):
    """Fold chunk (start c, outputs o) into the window's stop scan for the rows open in it (t)."""
    new = t & ((o.row_status & _lib.SD_ROW_STOP_IN_DRAFTS) != 0)
    pos = (c + o.stop_index.clamp(min=0)).long()
    tok = draft_tokens.gather(1, pos.view(-1, 1).clamp(max=draft_tokens.shape[1] - 1)).view(-1)
    r = _stop_rank(stop_tokens, tok)
    better = new & (r < best)   # equal ranks: the same token, the earlier chunk's position first
    return (torch.where(better, r, best), torch.where(better, c + o.stop_index, stop_index), seen | new)


def _groups(noise, B: int, per_row: bool) -> List[Tuple[int, int]]:
    return [(b, b + 1) for b in range(B)] if per_row else [(0, B)]


def verify_chunked(target_rows, draft_rows, draft_tokens, rule, target_proc, draft_proc, noise, stop_tokens,
                   skip_sample_adjustment, draft_is_probs, active, engine_state, sync_noise, row_base,
                   draft_row_stats, draft_row_keep, status_or, row_counts):
    """ops.verify for γ > SD_MAX_GAMMA (module docstring).  Under STREAM noise the generator is
    always moved (per sequence, by the words the window consumed): chunks of later rows start
    where earlier rows stopped, so the count cannot be left to the caller (sync_noise is implied)."""
    from .ops import VerifyOut, proc_spec, verify
    g = len(draft_rows)
    n_t = g + 1 if rule == _lib.SD_RULE_SPEC else g
    if len(target_rows) != n_t:
        raise ValueError(f"expected {n_t} target rows, got {len(target_rows)}")
    B, V = target_rows[0].shape
    dev = target_rows[0].device
    if draft_tokens.dim() != 2 or draft_tokens.shape[0] != B or draft_tokens.shape[1] < g:
        raise ValueError(f"draft_tokens must be int64 [B, >={g}]")
    stream = isinstance(noise, StreamNoise)
    i32 = dict(dtype=torch.int32, device=dev)
    n = torch.zeros(B, **i32)
    nxt = torch.full((B,), -1, dtype=torch.long, device=dev)
    mass = torch.full((B,), float("nan"), device=dev)
    status = torch.zeros(B, **i32)
    prune_d = torch.zeros(B, **i32)
    prune_t = torch.zeros(B, **i32)
    stop_index = torch.full((B,), -1, **i32)
    words = torch.zeros(1, dtype=torch.long, device=dev)
    inexact = _lib.SD_ROW_NUCLEUS_INEXACT

    def sub(x, c, gk, b0, b1):   # the chunk's slice of an optional [γ, S, k] drafter-row tensor
        return None if x is None else x[c:c + gk, b0:b1]

    if rule == _lib.SD_RULE_ENGINE:
        act0 = (active != 0) if active is not None else torch.ones(B, dtype=torch.bool, device=dev)
        for b0, b1 in _groups(noise, B, stream):
            act = act0[b0:b1].clone()
            for c, gk in chunks(g):
                es = None
                if engine_state is not None:
                    es = dict(generated=engine_state["generated"][b0:b1], step=int(engine_state["step"]) + c,
                              finished=engine_state["finished"][b0:b1], accepted=engine_state["accepted"][b0:b1])
                o = verify([t[b0:b1] for t in target_rows[c:c + gk]], [d[b0:b1] for d in draft_rows[c:c + gk]],
                           draft_tokens[b0:b1, c:c + gk], rule, target_proc, draft_proc, noise, stop_tokens,
                           skip_sample_adjustment, draft_is_probs, act.to(torch.uint8), es, True, None,
                           row_base + b0, sub(draft_row_stats, c, gk, b0, b1), sub(draft_row_keep, c, gk, b0, b1),
                           status_or, None if row_counts is None else row_counts[b0:b1])
                stopped = act & ((o.n_accepted < gk) | ((o.row_status & _lib.SD_ROW_FINISHED) != 0))
                n[b0:b1] += torch.where(act, o.n_accepted, 0)
                nxt[b0:b1] = torch.where(stopped, o.next_token, nxt[b0:b1])
                mass[b0:b1] = torch.where(stopped, o.resample_mass, mass[b0:b1])
                status[b0:b1] = torch.where(act, o.row_status | (status[b0:b1] & inexact), status[b0:b1])
                words += o.words_used
                act &= ~stopped
        if engine_state is not None:   # :332-336 over the whole window: zero past the last accepted draft
            step = int(engine_state["step"])
            win = engine_state["generated"][:, step:step + g]
            pos = torch.arange(g, device=dev)
            win.masked_fill_(act0[:, None] & (pos[None, :] > n[:, None].long()), 0)
        return VerifyOut(n, nxt, mass, prune_d, prune_t, stop_index, status, words)

    # SPEC: under STREAM row by row (the kernels' own row-serial layout: each row's γ uniforms, then
    # its sample words), each row's chunks reading its window's words
    stoch = proc_spec(target_proc).stochastic
    for b0, b1 in _groups(noise, B, stream):
        nb = b1 - b0
        W = None
        if stream:
            need = g + (2 * V if stoch else 0)
            W = noise.prepare(need, dev)
        open_ = torch.ones(nb, dtype=torch.bool, device=dev)
        seen = torch.zeros(nb, dtype=torch.bool, device=dev)
        best = torch.full((nb,), 1 << 30, dtype=torch.long, device=dev)
        sidx = torch.full((nb,), -1, **i32)
        nn = torch.zeros(nb, **i32)
        for c, gk in chunks(g):
            last = c + gk == g
            nz = noise
            if stream:   # this chunk's uniforms, then the window's sample words
                nz = _Words(torch.cat([W[c:c + gk], W[g:g + (2 * V if stoch else 0)]]))
            o = verify([t[b0:b1] for t in target_rows[c:c + gk + 1]], [d[b0:b1] for d in draft_rows[c:c + gk]],
                       draft_tokens[b0:b1, c:c + gk], rule, target_proc, draft_proc, nz, stop_tokens,
                       skip_sample_adjustment, draft_is_probs, None, None, True, None, row_base + b0,
                       sub(draft_row_stats, c, gk, b0, b1), sub(draft_row_keep, c, gk, b0, b1), None, None)
            t = open_
            nn += torch.where(t, o.n_accepted, 0)
            best, sidx, seen = _take_stop(stop_tokens, draft_tokens[b0:b1], c, o, t, best, sidx, seen)
            ended = t & ((o.n_accepted < gk) | last)
            use = ended & ~seen
            nxt[b0:b1] = torch.where(use, o.next_token, nxt[b0:b1])
            mass[b0:b1] = torch.where(use, o.resample_mass, mass[b0:b1])
            status[b0:b1] = torch.where(use, o.row_status, status[b0:b1]) | torch.where(t, o.row_status & inexact, 0)
            open_ = t & ~ended
        stop_flags = _lib.SD_ROW_DONE | _lib.SD_ROW_STOP_IN_DRAFTS
        stop_index[b0:b1] = sidx
        status[b0:b1] = torch.where(seen, (status[b0:b1] & inexact) | stop_flags, status[b0:b1])
        n[b0:b1] = nn
        pruned = (nn < g) & ~seen                     # :163-165 (the stop return comes first, :150-155)
        prune_d[b0:b1] = torch.where(pruned, g - nn, 0)
        prune_t[b0:b1] = torch.where(pruned, g - nn + 1, 0)
        if stream:   # r = rand(γ), then the sample's 2V words unless the stop return came first
            used = (g + torch.where(seen, 0, 2 * V if stoch else 0)).to(torch.long).reshape(1)
            words += used
            noise.consumed(used_dev=used)
    _or_errors(status_or, status)
    if row_counts is not None:
        emitted = n.long() + (((status & _lib.SD_ROW_STOP_IN_DRAFTS) == 0) & (nxt >= 0)).long()
        row_counts += torch.stack([n.long(), emitted], dim=1)
    return VerifyOut(n, nxt, mass, prune_d, prune_t, stop_index, status, words)


def ngram_verify_chunked(target_rows, draft_tokens, proc, noise, stop_tokens, filler_k, sync_noise, row_base,
                         status_or):
    """ops.ngram_verify for γ' > SD_MAX_GAMMA (module docstring); STREAM needs one sequence (the
    reference's loop is batch 1) and always moves the generator."""
    from .ops import NgramOut, ngram_verify, proc_spec
    g = len(target_rows) - 1
    B, V = target_rows[0].shape
    dev = target_rows[0].device
    stream = isinstance(noise, StreamNoise)
    if stream and B != 1:
        raise ValueError(f"ngram_verify: STREAM noise over more than {_lib.SD_MAX_GAMMA} drafts needs batch 1 "
                         "(the reference's n-gram loop is batch 1; Philox takes any batch)")
    stoch = proc_spec(proc).stochastic
    i32 = dict(dtype=torch.int32, device=dev)
    dtok = draft_tokens.to(dev)
    if stop_tokens is not None:
        stop_tokens = stop_tokens.to(device=dev, dtype=torch.long)
    W = noise.prepare((g + 1) * 2 * V if stoch else 1, dev) if stream else None
    open_ = torch.ones(B, dtype=torch.bool, device=dev)
    seen = torch.zeros(B, dtype=torch.bool, device=dev)
    best = torch.full((B,), 1 << 30, dtype=torch.long, device=dev)
    n = torch.zeros(B, **i32)
    nxt = torch.full((B,), -1, dtype=torch.long, device=dev)
    status = torch.zeros(B, **i32)
    stop_index = torch.full((B,), -1, **i32)
    filler = torch.empty(B, g + 1, filler_k, dtype=torch.long, device=dev) if filler_k else None
    inexact = _lib.SD_ROW_NUCLEUS_INEXACT
    for c, gk in chunks(g):
        last = c + gk == g
        nz = _Words(W[c * 2 * V:] if stoch else W) if stream else noise
        o = ngram_verify(target_rows[c:c + gk + 1], dtok[:, c:c + gk], proc, nz, stop_tokens, filler_k,
                         True, row_base, None)
        t = open_
        n += torch.where(t, o.n_accepted, 0)
        best, stop_index, seen = _take_stop(stop_tokens, dtok, c, o, t, best, stop_index, seen)
        ended = t & ((o.n_accepted < gk) | last)
        use = ended & ~seen
        nxt = torch.where(use, o.next_token, nxt)
        status = torch.where(use, o.row_status, status) | torch.where(t, o.row_status & inexact, 0)
        open_ = t & ~ended
        if filler is not None:   # every row's own top-k; the chunk's bonus row is the next chunk's row 0
            filler[:, c:c + gk + (1 if last else 0)] = o.filler_ids[:, :gk + (1 if last else 0)]
    stop_flags = _lib.SD_ROW_DONE | _lib.SD_ROW_STOP_IN_DRAFTS
    status = torch.where(seen, (status & inexact) | stop_flags, status)
    nxt = torch.where(seen, -1, nxt)
    prune_t = torch.where(~seen & (n < g), g - n + 1, 0).to(torch.int32)   # :139-141
    words = torch.zeros(1, dtype=torch.long, device=dev)
    if stream and stoch:   # compare draws up to the first mismatch, then x unless the stop return came first
        draws = torch.where(n < g, n + 1, g).long() + torch.where(seen, 0, 1)
        words = (draws * 2 * V).reshape(1)
        noise.consumed(used_dev=words)
    elif stream:
        noise.consumed(count=0)
    _or_errors(status_or, status)
    return NgramOut(n, nxt, prune_t, stop_index, status, filler, words)
