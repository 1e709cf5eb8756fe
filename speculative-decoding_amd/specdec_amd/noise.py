"""Noise sources for the verify / sample kernels.

StreamNoise  (parity mode)  feeds the kernels the raw mt19937 words of torch's CPU generator
             (torch.default_generator unless one is given), so every torch.rand / multinomial
             draw the reference makes is reproduced bit-exactly, in the reference's order, on
             the GPU.  Words are generated on the host by libspecdec (sd_mt19937_fill) and the
             generator is advanced by exactly the words the kernels consumed.
PhiloxNoise  (perf mode)    counter-based Philox4x32-10 inside the kernels: no host work, no
             noise bytes in HBM; statistically equivalent, not stream-identical.

The mode used by the drop-in entry points is chosen by ``set_noise_mode`` or the
SPECDEC_NOISE environment variable (``stream`` | ``philox``; default ``stream``).
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch

from . import _lib
from ._lib import lib


class StreamNoise:
    mode = _lib.SD_NOISE_STREAM

    def __init__(self, generator: Optional[torch.Generator] = None):
        self.generator = generator

    @property
    def gen(self) -> torch.Generator:
        return self.generator if self.generator is not None else torch.default_generator

    def draw(self, n_words: int, device) -> torch.Tensor:
        """The next n_words generator words (the generator is NOT advanced), on `device`."""
        n = max(int(n_words), 1)
        st = self.gen.get_state().contiguous()
        host = np.empty(n, dtype=np.uint32)
        _lib.check(lib.sd_mt19937_fill(st.data_ptr(), st.numel(), host.ctypes.data, n), "sd_mt19937_fill")
        return torch.from_numpy(host.view(np.int32)).to(device)

    def advance(self, n_words: int) -> None:
        if n_words <= 0:
            return
        st = self.gen.get_state().clone()
        _lib.check(lib.sd_mt19937_advance(st.data_ptr(), st.numel(), int(n_words)), "sd_mt19937_advance")
        self.gen.set_state(st)


class PhiloxNoise:
    mode = _lib.SD_NOISE_PHILOX

    def __init__(self, seed: Optional[int] = None, offset: int = 0):
        if seed is None:   # deterministic under torch.manual_seed
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self.seed = seed & 0xFFFFFFFFFFFFFFFF
        self.offset = offset

    def next_offset(self) -> int:
        o = self.offset
        self.offset += 1
        return o


_mode = os.environ.get("SPECDEC_NOISE", "stream").lower()
_philox: Optional[PhiloxNoise] = None


def set_noise_mode(mode: str, seed: Optional[int] = None) -> None:
    global _mode, _philox
    if mode not in ("stream", "philox"):
        raise ValueError(f"noise mode must be 'stream' or 'philox', got {mode!r}")
    _mode = mode
    _philox = PhiloxNoise(seed) if mode == "philox" else None


def default_noise():
    global _philox
    if _mode == "philox":
        if _philox is None:
            _philox = PhiloxNoise()
        return _philox
    return StreamNoise()
