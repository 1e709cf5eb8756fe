"""KV-cache prune (utils/caching.py:6-77).

The prune is metadata-only: drop the last k positions of every K/V tensor.  The verify kernel
returns k per sequence (prune_drafter = γ'-n, prune_target = γ'-n+1,
sampling/speculative_decoding.py:163-165).  Unlike the reference, the DynamicCache branch works
on transformers 5.x (the reference reads the removed ``key_cache``/``_seen_tokens``):
it calls ``DynamicCache.crop(-k)``, the transformers-5 way to drop the last k positions.

Reference semantics kept on purpose: the tuple path slices ``[:, :, :-k, :]`` (:51), so k = 0
returns EMPTY K/V views, exactly as the reference does (its loops never prune 0 positions:
the prune only runs after a reject, k_drafter >= 1, k_target >= 2).
"""
from __future__ import annotations

from typing import Tuple, Union

from torch import Tensor

try:  # transformers is optional for the tuple path
    from transformers.cache_utils import DynamicCache
except Exception:  # pragma: no cover
    DynamicCache = None


def prune_cache(cache, num_tokens_to_discard: int):
    """utils/caching.py:6-24: tuple caches -> views, cache objects -> cropped in place."""
    if cache is None:
        return None
    if isinstance(cache, tuple):
        return prune_tuple_cache(cache, num_tokens_to_discard)
    if (DynamicCache is not None and isinstance(cache, DynamicCache)) or hasattr(cache, "crop"):
        return prune_dynamic_cache(cache, num_tokens_to_discard)
    raise ValueError("Unsupported cache type.")


def prune_tuple_cache(cache: Tuple[Tuple[Tensor, Tensor]], num_tokens_to_discard: int):
    """utils/caching.py:27-55: views without the last k positions (dim 2) of every K/V tensor."""
    if cache is None:
        return None
    out = []
    for layer in cache:
        if layer is None:
            out.append(None)
            continue
        out.append(tuple(t[:, :, :-num_tokens_to_discard, :] for t in layer))
    return tuple(out)


def prune_dynamic_cache(cache, num_tokens_to_discard: int):
    """utils/caching.py:58-77, on the transformers-5 API: drop the last k positions of every layer
    in place (``crop(-k)``; the reference's ``key_cache`` / ``_seen_tokens`` no longer exist)."""
    if cache is None:
        return None
    if num_tokens_to_discard > 0:
        cache.crop(-int(num_tokens_to_discard))
    return cache
