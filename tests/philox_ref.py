"""Philox4x32-10 (Salmon, Moraes, Dror, Shaw — "Parallel random numbers: as easy as 1, 2, 3",
SC'11) in numpy, for checking the perf-mode (SD_NOISE_PHILOX) kernels.  Mirrors
csrc/sd_device.h: philox4x32_10, philox_block's counter layout, uniform_from_word,
cdf_uniform.  Test infrastructure only.
"""
from __future__ import annotations

import numpy as np

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF
SITE_ACCEPT, SITE_SAMPLE, SITE_CDF = 1, 2, 3


def philox4x32_10(ctr, key):
    """ctr: 4 uint32 (ints or uint64 arrays), key: 2 uint32 -> 4 uint32 (same shape)."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) for c in ctr)
    k0, k1 = (np.asarray(k, dtype=np.uint64) for k in key)
    for _ in range(10):
        p0 = c0 * np.uint64(M0)
        p1 = c2 * np.uint64(M1)
        hi0, lo0 = p0 >> np.uint64(32), p0 & np.uint64(MASK)
        hi1, lo1 = p1 >> np.uint64(32), p1 & np.uint64(MASK)
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        k0 = (k0 + np.uint64(W0)) & np.uint64(MASK)
        k1 = (k1 + np.uint64(W1)) & np.uint64(MASK)
    return c0, c1, c2, c3


def block(seed: int, offset: int, row, site: int, idx):
    ctr = (idx, (np.asarray(row, dtype=np.uint64) & np.uint64(0xFFFFFF)) | np.uint64(site << 24),
           offset & MASK, (offset >> 32) & MASK)
    return philox4x32_10(ctr, (seed & MASK, (seed >> 32) & MASK))


def accept_uniform(seed: int, offset: int, row: int, i: int) -> float:
    """The accept-test uniform of draft i of row `row`: word i % 4 of block i // 4 (torch.rand's fp32
    from one word)."""
    w = int(block(seed, offset, row, SITE_ACCEPT, i >> 2)[i & 3])
    return np.float32((w & 0xFFFFFF) * 2.0 ** -24)


def cdf_uniform(seed: int, offset: int, row: int) -> float:
    x, y, _, _ = block(seed, offset, row, SITE_CDF, 0)
    return float(((int(x) << 32) | int(y)) >> 11) * 2.0 ** -53
