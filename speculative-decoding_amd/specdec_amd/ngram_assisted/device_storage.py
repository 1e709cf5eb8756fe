"""Device-resident n-gram drafters with the reference's interface
(ngram_assisted/ngram_storage.py:5-68): ``DeviceOneLevelNGramStorage`` and ``DeviceNGramStorage``
behave as ``OneLevelNGramStorage`` / ``NGramStorage`` (ngram_storage.py:71-249) but keep their
tables in HBM (``csrc/ngram_store.hip``, C ABI ``sd_ngram_store_*``).

What stays on the host is what the reference's observable behaviour needs without a device
round trip: the record clock (every record's position in the reference's processing order, so
the device can apply a batch in any order), the orders NGramStorage has created (its
``next_token`` raises ``KeyError`` for an order never recorded, ngram_storage.py:171), and the
``torch.randint`` fallback draws from the default generator (ngram_storage.py:77,163), drawn
first so the generator stream lines up with the reference's.

``next_token`` returns device tensors (tokens int64 [B], known bool [B]) on the store's device;
``has_gram`` returns a Python bool (one sync, as the reference's ``.item()``).  Inputs may be CPU
or device tensors.  There is no host fallback: the store needs the HIP library and a GPU.
"""
from __future__ import annotations

import ctypes as C
from typing import Tuple

import torch

from .. import _lib
from .ngram_storage import INgramStorage


def _stream(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


class _DeviceStore(INgramStorage):
    _one_level = 0

    def __init__(self, n: int, vocab_size: int, device=None, gram_capacity: int = 1 << 20,
                 pair_capacity: int = 1 << 21):
        super().__init__(n, vocab_size)
        if n > _lib.SD_NGRAM_MAX_N:
            raise ValueError(f"device n-gram store supports n <= {_lib.SD_NGRAM_MAX_N}")
        if vocab_size > 1 << 17:
            raise ValueError("device n-gram store supports vocab_size <= 2^17")
        for c in (gram_capacity, pair_capacity):
            if c <= 0 or c & (c - 1):
                raise ValueError("capacities must be powers of two")
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise RuntimeError("the device n-gram store runs on the GPU (HIP); there is no CPU path")
        self._gcap, self._pcap = gram_capacity, pair_capacity
        self.reset()

    # ---------------------------------------------------------------- state
    def reset(self):
        d = self.device
        self._gram_keys = torch.zeros(self._gcap, dtype=torch.int64, device=d)
        self._gram_best = torch.zeros(self._gcap, dtype=torch.int64, device=d)
        self._pair_keys = torch.zeros(self._pcap, dtype=torch.int64, device=d)
        self._pair_count = torch.zeros(self._pcap, dtype=torch.int32, device=d)
        self._pair_ts = torch.zeros(self._pcap, dtype=torch.int32, device=d)
        self._status = torch.zeros(1, dtype=torch.int32, device=d)
        self._ts = 0
        self._orders = set()
        self._s = _lib.sd_ngram_store(self._gram_keys.data_ptr(), self._gram_best.data_ptr(), self._gcap,
                                      self._pair_keys.data_ptr(), self._pair_count.data_ptr(),
                                      self._pair_ts.data_ptr(), self._pcap, self._status.data_ptr(),
                                      self.n, self._one_level, self.vocab_size)

    def status(self) -> int:
        """SD_NGRAM_* bits raised on the device (table full, token out of range); syncs."""
        return int(self._status.item())

    def _ids(self, x) -> torch.Tensor:
        t = x if isinstance(x, torch.Tensor) else torch.tensor(x, dtype=torch.long)
        if t.dim() == 1:
            t = t.unsqueeze(0)
        return t.to(device=self.device, dtype=torch.long).contiguous()

    # ---------------------------------------------------------------- interface
    def initialize(self, input_ids: torch.Tensor):
        ids = self._ids(input_ids)
        B, L = ids.shape
        self._created_by_initialize(L)
        _lib.check(_lib.lib.sd_ngram_store_initialize(C.byref(self._s), ids.data_ptr(), B, L, ids.stride(0),
                                                      self._ts, _stream(self.device)), "sd_ngram_store_initialize")
        self._ts += B * L

    def update(self, input_ids: torch.Tensor, next_tokens: torch.Tensor):
        ids = self._ids(input_ids)
        nxt = self._ids(next_tokens)
        B, L = ids.shape
        if nxt.shape[0] != B:
            raise ValueError("next_tokens must have one row per sequence")
        k = nxt.shape[1]
        if k == 0:   # the reference records nothing (or raises IndexError for a new gram): no-op
            return
        self._created_by_update(L)
        _lib.check(_lib.lib.sd_ngram_store_update(C.byref(self._s), ids.data_ptr(), B, L, ids.stride(0),
                                                  nxt.data_ptr(), k, nxt.stride(0), self._ts,
                                                  _stream(self.device)), "sd_ngram_store_update")
        self._ts += B * k

    def next_token(self, input_ids: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        ids = self._ids(input_ids)
        B, L = ids.shape
        out = torch.randint(self.vocab_size, size=(B,)).to(self.device)   # the reference's fallback draws
        known = torch.zeros(B, dtype=torch.bool, device=self.device)
        self._check_orders(L)
        _lib.check(_lib.lib.sd_ngram_store_next_token(C.byref(self._s), ids.data_ptr(), B, L, ids.stride(0),
                                                      out.data_ptr(), known.data_ptr(), _stream(self.device)),
                   "sd_ngram_store_next_token")
        return out, known

    def draft_chain(self, input_ids: torch.Tensor, gamma: int,
                    stop_if_unknown: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
        """The n-gram loop's drafting (ngram_assisted/ngram_assisted.py:94-101) in one launch:
        gamma chained ``next_token`` calls, call k on the history extended by drafts 0..k-1.
        Returns (drafts [B, gamma], known [B, gamma]) on the device.  The fallback draws are the
        calls' ``torch.randint(V, (B,))`` draws, taken together ((gamma, B) in one call is the
        same stream).  With ``stop_if_unknown`` the reference stops calling after the first
        unknown draft, so the generator is rewound and advanced by exactly the calls made (one
        read-back, which the loop needs anyway for the drafted ids)."""
        ids = self._ids(input_ids)
        B, L = ids.shape
        for k in range(gamma):
            self._check_orders(L + k)
        state = torch.get_rng_state() if stop_if_unknown else None
        fb = torch.randint(self.vocab_size, size=(gamma, B)).t().contiguous().to(self.device)
        drafts = torch.empty(B, gamma, dtype=torch.long, device=self.device)
        known = torch.zeros(B, gamma, dtype=torch.bool, device=self.device)
        _lib.check(_lib.lib.sd_ngram_store_draft(C.byref(self._s), ids.data_ptr(), B, L, ids.stride(0), gamma,
                                                 fb.data_ptr(), fb.stride(0), drafts.data_ptr(), drafts.stride(0),
                                                 known.data_ptr(), _stream(self.device)), "sd_ngram_store_draft")
        if stop_if_unknown and gamma:
            kn = known.all(0).cpu()   # batch 1 in the reference's loop
            calls = gamma if bool(kn.all()) else int((~kn).nonzero()[0]) + 1
            torch.set_rng_state(state)
            torch.randint(self.vocab_size, size=(calls, B))
        return drafts, known

    def has_gram(self, ngram: torch.Tensor) -> bool:
        g = self._ids(ngram)[0]
        res = torch.zeros(1, dtype=torch.uint8, device=self.device)
        _lib.check(_lib.lib.sd_ngram_store_has_gram(C.byref(self._s), g.data_ptr(), g.numel(), res.data_ptr(),
                                                    _stream(self.device)), "sd_ngram_store_has_gram")
        return bool(res.item())

    # ---------------------------------------------------------------- order bookkeeping
    def _created_by_initialize(self, L: int):
        pass

    def _created_by_update(self, L: int):
        pass

    def _check_orders(self, L: int):
        pass


class DeviceOneLevelNGramStorage(_DeviceStore):
    """OneLevelNGramStorage (ngram_storage.py:71-150) with its tables on the device."""
    _one_level = 1


class DeviceNGramStorage(_DeviceStore):
    """NGramStorage (ngram_storage.py:154-249) with its tables on the device."""
    _one_level = 0

    def _created_by_initialize(self, L: int):
        # ngram_storage.py:229-231: position i creates orders 2 .. min(n-1, i)
        self._orders.update(range(2, min(self.n - 1, L - 1) + 1))

    def _created_by_update(self, L: int):
        self._orders.update(range(2, min(self.n - 1, L) + 1))   # :202-205

    def _check_orders(self, L: int):
        # ngram_storage.py:171 indexes self.ngrams[j] from the longest order down; orders are
        # created as a contiguous range 2..m, so the reference raises KeyError exactly when the
        # longest order is missing
        hi = min(self.n - 1, L)
        if hi >= 2 and hi not in self._orders:
            raise KeyError(hi)
