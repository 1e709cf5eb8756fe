"""KV-cache prune (utils/caching.py:6-77).

The prune is metadata-only: drop the last k positions of every K/V tensor.  A transformers-5
StaticCache is cropped ON THE DEVICE by the verify kernel's prune output (prune_static_cache).  The verify kernel
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

import torch
from torch import Tensor

try:  # transformers is optional for the tuple path
    from transformers.cache_utils import DynamicCache
except Exception:  # pragma: no cover
    DynamicCache = None


def _static_lengths(cache):
    """The per-layer device length tensors of a transformers-5 StaticCache (StaticLayer keeps the
    cached length as a device tensor, ``cumulative_length``, and writes new keys at it), or None."""
    layers = getattr(cache, "layers", None)
    if not layers:
        return None
    lens = [getattr(layer, "cumulative_length", None) for layer in layers]
    if not all(torch.is_tensor(t) for t in lens):
        return None
    return lens


def prune_cache(cache, num_tokens_to_discard: Union[int, Tensor]):
    """utils/caching.py:6-24: tuple caches -> views, cache objects -> cropped in place.

    num_tokens_to_discard may be a device tensor (the verify kernel's ``prune_*`` output) for a
    StaticCache: the crop then runs on the device, driven by the kernel, with no host read."""
    if cache is None:
        return None
    if _static_lengths(cache) is not None:
        return prune_static_cache(cache, num_tokens_to_discard)
    if torch.is_tensor(num_tokens_to_discard):
        num_tokens_to_discard = int(num_tokens_to_discard.reshape(-1)[0].item())   # host crop: one read
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


def prune_static_cache(cache, num_tokens_to_discard: Union[int, Tensor]):
    """Device-side crop of a transformers-5 StaticCache: the K/V buffers keep
    their addresses and the stale positions are overwritten by the next write (the causal mask
    built from ``cache_position`` hides them meanwhile), so dropping the last k positions is
    ``cumulative_length -= k`` in every layer — one multi-tensor launch.  k is an int, or a device
    tensor of one element (batch 1, as the reference's prune; ``prune_*[0]`` of a verify), which
    keeps the crop on the device without a host read.  k = 0 is a no-op, so a loop can apply the
    kernel's prune output every step without branching on it."""
    lens = _static_lengths(cache)
    if lens is None:
        raise ValueError("not a StaticCache")
    if torch.is_tensor(num_tokens_to_discard):
        k = num_tokens_to_discard.reshape(-1)[:1].reshape(())
        torch._foreach_sub_(lens, k.to(device=lens[0].device, dtype=lens[0].dtype))
    elif num_tokens_to_discard:
        torch._foreach_sub_(lens, int(num_tokens_to_discard))
    return cache

