"""N-gram drafters (ngram_assisted/ngram_storage.py), host side.

The drafter is a small dictionary updated between verify steps; it stays on the host here, as in
the reference (a device-resident store is SURVEY.md §8f, rank 4).  Behaviour is the reference's,
including its draws: ``next_token`` always draws ``torch.randint(vocab_size, (B,))`` from the
default generator first (the fallback for unknown grams), so under ``torch.manual_seed`` the
random stream — and with it every later multinomial draw — lines up with the reference.

A ``_Table`` keeps, for one gram order, the per-gram token counts and the current best token:
the first token ever recorded for a gram is its best until another token's count becomes
STRICTLY larger than the best's.
"""
from __future__ import annotations

import abc
from typing import Dict, List, Sequence, Tuple

import torch


def _ids(x) -> List[int]:
    return x.tolist() if isinstance(x, torch.Tensor) else list(x)


class _Table:
    __slots__ = ("counts", "best")

    def __init__(self):
        self.counts: Dict[tuple, Dict[int, int]] = {}
        self.best: Dict[tuple, int] = {}

    def record(self, gram: tuple, tokens: Sequence[int]) -> None:
        per = self.counts.setdefault(gram, {})
        if gram not in self.best:
            self.best[gram] = tokens[0]
        for tok in tokens:
            c = per.get(tok, 0) + 1
            per[tok] = c
            if c > 1 and c > per[self.best[gram]]:
                self.best[gram] = tok


class INgramStorage(abc.ABC):
    """Interface (ngram_storage.py:5-68): a dynamic n-gram model returning the most likely next token."""

    def __init__(self, n: int, vocab_size: int):
        assert n > 1, "n should be greater than 1"
        self.n = n
        self.vocab_size = vocab_size

    @abc.abstractmethod
    def next_token(self, input_ids: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(tokens [B], known [B]) for the sequences input_ids [B, L]."""

    @abc.abstractmethod
    def has_gram(self, ngram: torch.Tensor) -> bool:
        """Whether the n-gram (its last token after its prefix) has been seen."""

    @abc.abstractmethod
    def update(self, input_ids: torch.Tensor, next_tokens: torch.Tensor):
        """Record next_tokens [B, k] after the sequences input_ids [B, L]."""

    @abc.abstractmethod
    def initialize(self, input_ids: torch.Tensor):
        """Record every n-gram of the prompts input_ids [B, L]."""

    @abc.abstractmethod
    def reset(self):
        """Forget everything."""


class OneLevelNGramStorage(INgramStorage):
    """Only (n-1)-token grams (ngram_storage.py:71-150)."""

    def __init__(self, n: int, vocab_size: int):
        super().__init__(n, vocab_size)
        self._t = _Table()

    @property
    def counts(self):
        return self._t.counts

    @property
    def ngrams(self):
        return self._t.best

    def next_token(self, input_ids):
        out = torch.randint(self.vocab_size, size=(input_ids.shape[0],))
        known = torch.zeros(input_ids.shape[0], dtype=torch.bool, device=input_ids.device)
        k = self.n - 1
        for i, seq in enumerate(input_ids):
            if seq.shape[0] < k:
                continue
            best = self._t.best.get(tuple(_ids(seq[-k:])))
            if best is not None:
                out[i] = best
                known[i] = True
        return out, known

    def has_gram(self, ngram):
        if ngram.shape[0] < self.n:
            return False
        per = self._t.counts.get(tuple(_ids(ngram[-(self.n - 1):])))
        return per is not None and int(ngram[-1]) in per

    def update(self, input_ids, next_tokens):
        k = self.n - 1
        for i, seq in enumerate(input_ids):
            if seq.shape[0] < self.n:
                continue
            self._t.record(tuple(_ids(seq[-k:])), _ids(next_tokens[i]))

    def initialize(self, input_ids):
        k = self.n - 1
        for seq in input_ids:
            s = _ids(seq)
            for i in range(len(s) - k):
                self._t.record(tuple(s[i:i + k]), [s[i + k]])

    def reset(self):
        self._t = _Table()


class NGramStorage(INgramStorage):
    """All gram orders j = 2 .. n-1; the longest known suffix predicts (ngram_storage.py:154-249)."""

    def __init__(self, n: int, vocab_size: int):
        super().__init__(n, vocab_size)
        self._tables: Dict[int, _Table] = {}

    @property
    def counts(self):
        return {j: t.counts for j, t in self._tables.items()}

    @property
    def ngrams(self):
        return {j: t.best for j, t in self._tables.items()}

    def _orders(self, length: int):
        return range(min(self.n - 1, length), 1, -1)

    def next_token(self, input_ids):
        out = torch.randint(self.vocab_size, size=(input_ids.shape[0],))
        known = torch.zeros(input_ids.shape[0], dtype=torch.bool, device=input_ids.device)
        for i, seq in enumerate(input_ids):
            s = _ids(seq)
            for j in self._orders(len(s)):
                best = self._tables[j].best.get(tuple(s[-j:]))   # KeyError for an unseen order, as the reference
                if best is not None:
                    out[i] = best
                    known[i] = True
                    break
        return out, known

    def has_gram(self, ngram):
        s = _ids(ngram)
        for j in self._orders(len(s)):
            per = self._tables[j].counts.get(tuple(s[-j:])) if j in self._tables else None
            if per is not None and s[-1] in per:
                return True
        return False

    def update(self, input_ids, next_tokens):
        for i, seq in enumerate(input_ids):
            s = _ids(seq)
            toks = _ids(next_tokens[i])
            for j in self._orders(len(s)):
                self._tables.setdefault(j, _Table()).record(tuple(s[-j:]), toks)

    def initialize(self, input_ids):
        for seq in input_ids:
            s = _ids(seq)
            for i in range(len(s)):
                for j in range(min(self.n - 1, i), 1, -1):
                    self._tables.setdefault(j, _Table()).record(tuple(s[i - j:i]), [s[i]])

    def reset(self):
        self._tables = {}
