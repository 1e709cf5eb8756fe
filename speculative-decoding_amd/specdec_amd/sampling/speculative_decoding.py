"""Batch-1 speculative sampling loop on the fused HIP path.

Drop-in for sampling/speculative_decoding.py:22-189 (``speculative_generate``): same
signature, defaults and return value ``(List[int], float)``.  Per step the drafter runs γ'
forwards (PyTorch-ROCm); each draft row is processed + sampled by ``sd_sample`` straight into
``input_ids`` on the device; the target runs once; then ONE ``sd_verify`` call does the
processor softmax over the γ'+1 target and γ' drafter rows, the ``r <= p/q`` accept test, the
stop-token scan, the bonus / (p-q)+ residual sample and the prune lengths.  The host reads
back four integers per step.

Differences from the reference, all on paths where it is broken: ``use_cache``
works on transformers 5.x (only uncached positions are fed, caches are cropped on reject), and
``debug`` printing is reduced to one line per step.
"""
from __future__ import annotations

from typing import List, Tuple

import torch
from torch.nn import Module

from .. import _lib
from ..noise import StreamNoise, default_noise, noise_session
from ..ops import _user_process, proc_spec, sample_rows, verify
from ..utils.caching import prune_cache
from ..utils.logits_processor import GreedyProcessor, LogitsProcessor


def max_fn(x: torch.Tensor) -> torch.Tensor:
    """sampling/speculative_decoding.py:10-19 (x⁺ / Σx⁺).  The verify kernel fuses this; kept
    as a tensor utility for callers of the reference API."""
    x_max = torch.where(x > 0, x, torch.zeros_like(x))
    return x_max / torch.sum(x_max, dim=-1, keepdim=True)


def _cache_len(cache) -> int:
    if cache is None:
        return 0
    if isinstance(cache, tuple):
        return cache[0][0].shape[2]
    if hasattr(cache, "get_seq_length"):
        return int(cache.get_seq_length())
    return int(cache.length)


def _forward(model, ids: torch.Tensor, end: int, cache, use_cache: bool, static_len=None):
    """Run `model` on positions [cached, end) of ids; returns (logits, new cache, first position).
    static_len: the host's copy of a StaticCache's length (its own is a device tensor, and the
    positions are passed explicitly, so nothing is read back)."""
    kw = {}
    if not use_cache:
        start = 0
    elif static_len is not None:
        start = static_len
        kw["cache_position"] = torch.arange(start, end, device=ids.device)
    else:
        start = _cache_len(cache)
    out = model(input_ids=ids[..., start:end], past_key_values=cache if use_cache else None, use_cache=use_cache,
                **kw)
    return out.logits, (cache if static_len is not None else out.past_key_values), start


@torch.no_grad()
def speculative_generate(
    inputs: List[int],
    drafter: Module,
    target: Module,
    tokenizer=None,
    gamma: int = 5,
    logits_processor: LogitsProcessor = GreedyProcessor(),
    max_gen_len: int = 40,
    eos_tokens_id: int | List[int] = 1,
    pad_token_id: int = 0,
    use_cache: bool = False,
    skip_sample_adjustment: bool = False,
    first_target: bool = True,
    debug: bool = False,
    static_cache: bool = False,
) -> Tuple[List[int], float]:
    """sampling/speculative_decoding.py:22-189.  One keyword beyond the reference's:
    static_cache (with use_cache): both models decode into a transformers-5 StaticCache sized for
    the whole sequence, cropped ON THE DEVICE by the verify kernel's prune outputs (§8f-2)."""
    noise = default_noise()
    with noise_session(noise):   # STREAM: the generator state stays on the device for the loop
        return _speculative_generate(noise, inputs, drafter, target, gamma, logits_processor, max_gen_len,
                                     eos_tokens_id, pad_token_id, use_cache, skip_sample_adjustment, first_target,
                                     debug, static_cache)


def _static_caches(drafter, target, total_len):
    from transformers.cache_utils import StaticCache
    return (StaticCache(config=drafter.config, max_cache_len=total_len),
            StaticCache(config=target.config, max_cache_len=total_len))


def _speculative_generate(noise, inputs, drafter, target, gamma, logits_processor, max_gen_len, eos_tokens_id,
                          pad_token_id, use_cache, skip_sample_adjustment, first_target, debug, static_cache=False):
    spec = proc_spec(logits_processor)
    # what the kernels are handed: the spec, or the processor itself when it has its own _process
    # (ops.processed_rows runs it on the rows first)
    kproc = logits_processor if _user_process(logits_processor) is not None else spec
    dev = target.device
    if torch.device(dev).type != "cuda":
        raise RuntimeError("specdec_amd.speculative_generate runs on the GPU (HIP); the target is on "
                           f"{dev}. There is no CPU path.")
    stops = eos_tokens_id if isinstance(eos_tokens_id, list) else [eos_tokens_id]
    stop_t = torch.tensor(stops, dtype=torch.long, device=dev)
    drafts_accepted, drafts_speculated = 0.0, 0.0                # :71
    cfg = target.config
    max_seq = getattr(cfg, "max_position_embeddings", None) or getattr(cfg, "max_context_length", None) or 1024
    prompt_len = len(inputs)
    total_len = min(max_seq, prompt_len + max_gen_len)           # :77-78
    input_ids = torch.full((1, total_len), pad_token_id, dtype=torch.long, device=dev)
    input_ids[0, :prompt_len] = torch.tensor(inputs, dtype=torch.long, device=dev)
    cur = prompt_len
    drafter_cache = target_cache = None
    static = bool(static_cache and use_cache)
    dlen = tlen = 0                                              # host copies of the static lengths
    if static:
        drafter_cache, target_cache = _static_caches(drafter, target, total_len)
    # every draw's and verify's failed rows (SD_ROW_ERROR_MASK) OR into one device word, read with the
    # integers each step already reads back: where torch.multinomial raises in the reference
    # (:96,123,171), this loop raises too — a draw's -1 is clamped to 0 first, so no forward ever
    # indexes an embedding with it before the error is seen
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    err_d = err if torch.device(drafter.device) == torch.device(dev) else \
        torch.zeros(1, dtype=torch.int32, device=drafter.device)

    def check_err():
        bits = int(err.item()) | (int(err_d.item()) if err_d is not err else 0)
        _lib.raise_row_error(bits, "speculative_generate")

    if first_target:                                             # :84-103
        logits, target_cache, _ = _forward(target, input_ids, cur, target_cache, use_cache, tlen if static else None)
        tlen = cur
        sample_rows(logits[:, -1, :], kproc, noise, tokens_out=input_ids[0, cur:cur + 1], status_or=err)
        t, bits = torch.stack([input_ids[0, cur], err[0].long()]).tolist()
        _lib.raise_row_error(bits, "speculative_generate")
        cur += 1
        if t in stops:
            return input_ids[0, prompt_len:cur].tolist(), 0

    # each draw also returns its row's (max, Σexp) (both noise modes), so verify reads only target
    # rows.  Not for top-k / nucleus processors: their stats would need the draw's threshold search,
    # which the nucleus draw skips (k_draw_nuc, rejection against the nucleus); the verify
    # thresholds all its rows in one launch anyway.
    stash = torch.device(drafter.device) == torch.device(dev) and not spec.keeps
    dstats = torch.empty(max(gamma, 1), 1, 2, dtype=torch.float32, device=dev) if stash else None
    while cur < total_len:                                       # :105
        g = min(gamma, total_len - cur - 1)                      # :106
        ids_d = input_ids.to(drafter.device)
        draft_rows = []
        for k in range(g):                                       # :112-124
            logits, drafter_cache, _ = _forward(drafter, ids_d, cur + k, drafter_cache, use_cache,
                                                dlen if static else None)
            dlen = cur + k
            row = logits[:, -1, :]
            if k == 0 and isinstance(noise, StreamNoise) and spec.stochastic and row.device == torch.device(dev):
                # the step's words in one generation: g draws of 2V, the verify's g + 2V
                V = row.shape[-1]
                noise.reserve(g * 2 * V + g + 2 * V, dev, known=g * 2 * V)
            tok = ids_d[0, cur + k:cur + k + 1]
            sample_rows(row, kproc, noise, tokens_out=tok, row_stats_out=dstats[k] if stash else None, status_or=err_d)
            tok.clamp_(0, row.shape[-1] - 1)   # a failed row's -1 never reaches a forward
            draft_rows.append(row if row.device == torch.device(dev) else row.to(dev))
        drafts_speculated += g
        input_ids = ids_d.to(dev)
        logits, target_cache, start = _forward(target, input_ids, cur + g, target_cache, use_cache,
                                               tlen if static else None)
        tlen = cur + g
        if g == 0:
            # last position: rand(0) draws nothing, n = 0 = γ', the bonus row is sampled (:158-171)
            sample_rows(logits[:, cur - 1 - start, :], kproc, noise, tokens_out=input_ids[0, cur:cur + 1],
                        status_or=err)
            check_err()
            x = int(input_ids[0, cur].item())
            cur += 1
            if x in stops:
                return input_ids[0, prompt_len:cur].tolist(), drafts_accepted / drafts_speculated
            continue
        trows = [logits[:, cur - 1 + t - start, :] for t in range(g + 1)]   # :135 and bonus row :159
        out = verify(trows, draft_rows, input_ids[:, cur:cur + g], _lib.SD_RULE_SPEC, kproc, kproc, noise,
                     stop_t, skip_sample_adjustment=skip_sample_adjustment,
                     draft_row_stats=dstats[:g] if stash else None, status_or=err)
        if err_d is not err:
            err.bitwise_or_(err_d.to(dev))
        n, x, status, stop_index, bits = (int(v) for v in torch.stack([
            out.n_accepted[0].long(), out.next_token[0], out.row_status[0].long(), out.stop_index[0].long(),
            err[0].long()]).tolist())
        _lib.raise_row_error(bits | status, "speculative_generate")   # a draft draw's or this verify's
        drafts_accepted += n                                     # :147
        if status & _lib.SD_ROW_STOP_IN_DRAFTS:                  # :150-155
            return input_ids[0, prompt_len:cur + stop_index + 1].tolist(), drafts_accepted / drafts_speculated
        if static:                                               # :163-165 on the device (0 = no-op)
            prune_cache(drafter_cache, out.prune_drafter)
            prune_cache(target_cache, out.prune_target)
            if n < g:
                dlen, tlen = dlen - (g - n), tlen - (g - n + 1)
        elif n < g and use_cache:                                # :163-165
            drafter_cache = prune_cache(drafter_cache, g - n)
            target_cache = prune_cache(target_cache, g - n + 1)
        input_ids[0, cur + n:cur + g] = pad_token_id             # :176-177
        input_ids[0, cur + n] = x
        if debug:
            print(f"[specdec] pos {cur}: accepted {n}/{g}, next {x}")
        cur += n + 1
        if x in stops:                                           # :184-187
            return input_ids[0, prompt_len:cur].tolist(), drafts_accepted / drafts_speculated
    return input_ids[0, prompt_len:].tolist(), drafts_accepted / drafts_speculated
