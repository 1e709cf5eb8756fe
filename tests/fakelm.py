"""Weight-free stand-in models for driving the speculative loops in tests.

No checkpoints exist offline, so the loops are driven by FakeLM:
logits at position t are a row of a seeded logit bank picked by (token, t).  It has
the surface the reference's loops touch: ``model(input_ids, past_key_values=…,
use_cache=…, attention_mask=…)`` returning ``.logits``/``.past_key_values``, plus
``.config.vocab_size``, ``.config.max_position_embeddings`` and ``.device``.

The drafter bank is the target bank plus N(0, sigma^2) noise, so acceptance is
realistic (≈0.5 at sigma=1).  Banks are generated on CPU from a seed, then moved.
"""
from __future__ import annotations

import hashlib
from types import SimpleNamespace

import torch


class FakeCache:
    """Stands in for past_key_values: only the number of cached positions matters."""

    def __init__(self, length: int):
        self.length = length

    def get_seq_length(self) -> int:
        return self.length

    def crop(self, max_length: int) -> None:   # transformers-5 DynamicCache.crop (negative: drop -k)
        self.length = self.length + max_length if max_length < 0 else min(self.length, max_length)


class FakeLM:
    def __init__(self, bank: torch.Tensor, max_position_embeddings: int = 4096, pos_mult: int = 7):
        self.bank = bank
        self.pos_mult = pos_mult   # 0: logits depend on the token only
        self.config = SimpleNamespace(vocab_size=bank.shape[1],
                                      max_position_embeddings=max_position_embeddings)

    @property
    def device(self):
        return self.bank.device

    def to(self, device):
        return FakeLM(self.bank.to(device), self.config.max_position_embeddings, self.pos_mult)

    def __call__(self, input_ids=None, past_key_values=None, use_cache=False, attention_mask=None, **_):
        ids = input_ids.to(self.bank.device)
        B, L = ids.shape
        off = past_key_values.length if isinstance(past_key_values, FakeCache) else 0
        pos = torch.arange(off, off + L, device=ids.device, dtype=torch.long)
        idx = (ids * 31 + pos * self.pos_mult) % self.bank.shape[0]
        logits = self.bank[idx]                                   # [B, L, V]
        return SimpleNamespace(logits=logits,
                               past_key_values=FakeCache(off + L) if use_cache else None)


def make_banks(vocab: int, rows: int = 64, sigma: float = 1.0, seed: int = 0,
               scale: float = 3.0, dtype=torch.bfloat16, peak: float = 0.0):
    """Target / drafter logit banks.  peak > 0 boosts one token per bank row by `peak` (a peaked,
    LM-like distribution: sampled continuations repeat, so n-gram drafters get accepted)."""
    g = torch.Generator().manual_seed(seed)
    t = torch.randn(rows, vocab, generator=g) * scale
    d = t + sigma * torch.randn(rows, vocab, generator=g)
    if peak > 0:
        hot = torch.randint(0, vocab, (rows,), generator=torch.Generator().manual_seed(seed + 555))
        t[torch.arange(rows), hot] += peak
        d[torch.arange(rows), hot] += peak
    return t.to(dtype), d.to(dtype)


def make_pair(vocab: int, rows: int = 64, sigma: float = 1.0, seed: int = 0, dtype=torch.bfloat16,
              device="cpu", max_position_embeddings: int = 4096, pos_mult: int = 7, peak: float = 0.0):
    t, d = make_banks(vocab, rows, sigma, seed, dtype=dtype, peak=peak)
    return (FakeLM(t.to(device), max_position_embeddings, pos_mult),
            FakeLM(d.to(device), max_position_embeddings, pos_mult))


def bank_digest(lm: FakeLM) -> str:
    b = lm.bank.detach().cpu().contiguous()
    return hashlib.sha256(b.view(torch.uint8).numpy().tobytes()).hexdigest()[:16]


def likely_tokens(lm: FakeLM, rows: int = 12, top: int = 2, offset: int = 5):
    """Tokens that the bank makes likely (top-`top` of `rows` bank rows): eos lists that really fire."""
    b = lm.bank.float().cpu()
    picks = torch.topk(b[offset:offset + rows], top, dim=-1).indices.reshape(-1).tolist()
    return sorted(set(int(t) for t in picks))


class TupleFakeLM(FakeLM):
    """FakeLM whose past_key_values is the legacy tuple-of-(K, V) layout [B, 1, L, 1] (one layer):
    what the reference's target-only loop gathers / scatters per active row
    (engine/infer_engine.py:430-467).  The cached length L sets the position offset.
    no_cache=True: the model returns no cache at all (past_key_values None)."""

    def __init__(self, bank, max_position_embeddings: int = 4096, pos_mult: int = 7, no_cache: bool = False):
        super().__init__(bank, max_position_embeddings, pos_mult)
        self.no_cache = no_cache

    def __call__(self, input_ids=None, past_key_values=None, use_cache=False, attention_mask=None, **_):
        ids = input_ids.to(self.bank.device)
        B, L = ids.shape
        off = 0
        if isinstance(past_key_values, (tuple, list)) and len(past_key_values):
            off = past_key_values[0][0].shape[2]
        elif isinstance(past_key_values, FakeCache):
            off = past_key_values.length
        pos = torch.arange(off, off + L, device=ids.device, dtype=torch.long)
        logits = self.bank[(ids * 31 + pos * self.pos_mult) % self.bank.shape[0]]
        kv = torch.zeros(B, 1, off + L, 1, device=ids.device)
        keep = use_cache and not self.no_cache
        return SimpleNamespace(logits=logits, past_key_values=((kv, kv.clone()),) if keep else None)
