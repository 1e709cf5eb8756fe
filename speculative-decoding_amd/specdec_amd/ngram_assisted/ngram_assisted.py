"""N-gram-assisted speculative loop (ngram_assisted/ngram_assisted.py:11-164) on the HIP path.

Same signature, defaults and return value.  Per step the n-gram store drafts γ' tokens on the
host, the target runs once, and ONE ``sd_ngram_verify`` call processes the γ'+1 target rows and
runs the sample-and-compare walk, the stop scan, the independent draw of x and the filler
top-k; the host reads back n, x, the stop position and the filler ids to update the store.
With ``torch.manual_seed`` and the default STREAM noise the tokens equal the reference's.
"""
from __future__ import annotations

from typing import List, Tuple

import torch
from torch.nn import Module

from .. import _lib
from ..noise import default_noise
from ..ops import _user_process, ngram_verify, proc_spec, sample_rows
from ..sampling.speculative_decoding import _forward
from ..utils.caching import prune_cache
from ..utils.logits_processor import GreedyProcessor, LogitsProcessor
from .ngram_storage import INgramStorage


@torch.no_grad()
def ngram_assisted_speculative_generate(
    inputs: List[int],
    ngramstorage: INgramStorage,
    target: Module,
    tokenizer=None,
    gamma: int = 5,
    filler_top_k: int = 3,
    logits_processor: LogitsProcessor = GreedyProcessor(),
    max_gen_len: int = 40,
    eos_tokens_id: int | List[int] = 1,
    pad_token_id: int = 0,
    use_cache: bool = False,
    first_target: bool = True,
    stop_if_unknown: bool = False,
    debug: bool = False,
) -> Tuple[List[int], float]:
    spec = proc_spec(logits_processor)
    # what the kernels are handed: the spec, or the processor itself when it has its own _process
    # (ops.processed_rows runs it on the rows first)
    kproc = logits_processor if _user_process(logits_processor) is not None else spec
    noise = default_noise()
    dev = target.device
    if torch.device(dev).type != "cuda":
        raise RuntimeError("specdec_amd.ngram_assisted_speculative_generate runs on the GPU (HIP); the target "
                           f"is on {dev}. There is no CPU path.")
    if filler_top_k < 0:   # any k up to the vocabulary (p.topk(k), ngram_assisted.py:152-155); ops checks V
        raise ValueError("filler_top_k must be >= 0")
    stops = eos_tokens_id if isinstance(eos_tokens_id, list) else [eos_tokens_id]
    stop_t = torch.tensor(stops, dtype=torch.long, device=dev)
    accepted, speculated = 0.0, 0.0
    prompt_len = len(inputs)
    total_len = min(target.config.max_position_embeddings, prompt_len + max_gen_len)
    ids = [pad_token_id] * total_len                              # host mirror of input_ids
    ids[:prompt_len] = list(inputs)
    cur = prompt_len
    cache = None
    ngramstorage.initialize(torch.tensor([ids[:prompt_len]], dtype=torch.long))
    filler = filler_top_k if filler_top_k > 1 else 0

    def rate():
        return accepted / speculated if speculated > 0 else 0.0

    def as_2d(tokens):
        return torch.tensor([tokens], dtype=torch.long)

    if first_target:                                              # :78-93 (no stop check here)
        ids_d = torch.tensor([ids], dtype=torch.long, device=dev)
        logits, cache, _ = _forward(target, ids_d, cur, cache, use_cache)
        tok, _, st = sample_rows(logits[:, -1, :], kproc, noise)
        t, bits = torch.stack([tok[0], st[0].long()]).tolist()
        _lib.raise_row_error(bits, "ngram_assisted_speculative_generate")   # torch raises (:89-90)
        ids[prompt_len] = t
        cur += 1
        ngramstorage.update(as_2d(ids[:prompt_len]), as_2d([t]))

    while cur < total_len:                                        # :95
        g = min(gamma, total_len - cur - 1)
        drafted = list(ids)
        if hasattr(ngramstorage, "draft_chain"):                  # device store: one launch, one read-back
            toks, knowns = ngramstorage.draft_chain(as_2d(drafted[:cur]), g, stop_if_unknown)
            toks, knowns = toks[0].tolist(), knowns[0].tolist()
        for k in range(g):                                        # :101-105
            if hasattr(ngramstorage, "draft_chain"):
                tok_k, known_k = toks[k], knowns[k]
            else:
                tok, known = ngramstorage.next_token(as_2d(drafted[:cur + k]))
                tok_k, known_k = int(tok[0]), bool(known[0])
            drafted[cur + k] = tok_k
            if not known_k and stop_if_unknown:
                g = k
                break
        speculated += g
        ids_d = torch.tensor([drafted], dtype=torch.long, device=dev)
        logits, cache, start = _forward(target, ids_d, cur + g, cache, use_cache)   # :108-115
        rows = [logits[:, cur - 1 + t - start, :] for t in range(g + 1)]           # p rows and the bonus row
        out = ngram_verify(rows, ids_d[:, cur:cur + g] if g else None, kproc, noise, stop_t, filler_k=filler)
        head = torch.stack([out.n_accepted[0].long(), out.next_token[0], out.row_status[0].long(),
                            out.stop_index[0].long()]).tolist()
        n, x, status, stop_index = (int(v) for v in head)
        fill = out.filler_ids[0].tolist() if filler else None
        _lib.raise_row_error(status, "ngram_assisted_speculative_generate")   # torch raises (:117,141)
        accepted += n
        if status & _lib.SD_ROW_STOP_IN_DRAFTS:                   # :126-131
            return drafted[prompt_len:cur + stop_index + 1], rate()
        if n < g and use_cache:                                   # :139-141
            cache = prune_cache(cache, g - n + 1)
        ids[cur:cur + n] = drafted[cur:cur + n]
        ids[cur + n] = x
        if debug:
            print(f"[specdec ngram] pos {cur}: accepted {n}/{g}, next {x}")
        for i in range(n):                                        # :151-155
            ngramstorage.update(as_2d(ids[:cur + i]), as_2d([ids[cur + i]]))
            if filler:
                ngramstorage.update(as_2d(ids[:cur + i]), as_2d(fill[i]))
        ngramstorage.update(as_2d(ids[:cur + n]), as_2d([x]))
        if filler:
            ngramstorage.update(as_2d(ids[:cur + n]), as_2d(fill[n if n < g else g]))
        cur += n + 1
        if x in stops:                                            # :161-164
            return ids[prompt_len:cur], rate()
    return ids[prompt_len:], rate()
