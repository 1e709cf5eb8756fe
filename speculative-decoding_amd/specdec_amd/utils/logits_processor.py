"""Logits processors with the reference's names and constructor signatures
(utils/logits_processor.py:7-103), backed by the HIP kernels.

In the drop-in loops a processor is only a parameter carrier: its (kind, temperature, top_k,
top_p) are handed to the fused verify / sample kernels, which apply
``softmax(_process(logits) / T)`` and the sampling rule inside one pass over the row.  Calling
a processor directly (``proc(logits)``) materialises the probabilities with the sd_probs
kernel; tensors must live on the GPU (there is no CPU path).
"""
from __future__ import annotations

import abc

import torch
from torch import Tensor

from ..ops import ProcSpec, probs_rows


class LogitsProcessor(abc.ABC):
    """Logits processors for sampling (utils/logits_processor.py:7-23)."""

    kind = "multinomial"

    def __init__(self, temperature: float):
        self.temperature = temperature

    def spec(self) -> ProcSpec:
        return ProcSpec(self.kind, float(self.temperature), int(getattr(self, "top_k", 0)),
                        float(getattr(self, "top_p", 1.0)))

    def __call__(self, logits: Tensor) -> Tensor:
        return probs_rows(logits, self.spec())

    def _process(self, logits: Tensor) -> Tensor:   # kept for API parity; the kernels fuse it
        raise NotImplementedError("processing is fused into the sd_probs / sd_verify kernels")

    @abc.abstractmethod
    def sample(self, probs: Tensor) -> Tensor:
        pass


class GreedyProcessor(LogitsProcessor):
    """Greedy: most probable token (utils/logits_processor.py:26-36)."""

    kind = "greedy"

    def __init__(self, temperature: float = 1):
        super().__init__(temperature)

    def sample(self, probs: Tensor) -> Tensor:
        return torch.argmax(probs, dim=-1).unsqueeze(-1)


class MultinomialProcessor(LogitsProcessor):
    """Multinomial: random sampling (utils/logits_processor.py:39-49)."""

    kind = "multinomial"

    def __init__(self, temperature: float):
        super().__init__(temperature)

    def sample(self, probs: Tensor) -> Tensor:
        """The reference's own call (utils/logits_processor.py:48-49), for callers that sample
        ``proc(logits)`` outside the loops.  On a GPU tensor it draws from torch's device
        generator, so it is NOT the bit-exact draw of the CPU reference; the drop-in loops never
        call it — their draws go through ``sd_sample`` / ``sd_verify`` (STREAM mode for
        torch-generator bit-exactness, ``specdec_amd.noise``)."""
        return torch.multinomial(probs, num_samples=1)


class TopKProcessor(MultinomialProcessor):
    """Top-k sampling (utils/logits_processor.py:52-63)."""

    kind = "topk"

    def __init__(self, temperature: float, top_k: int):
        super().__init__(temperature)
        self.top_k = top_k


class NucleusProcessor(MultinomialProcessor):
    """Nucleus / top-p sampling (utils/logits_processor.py:66-81)."""

    kind = "nucleus"

    def __init__(self, temperature: float, top_p: float):
        super().__init__(temperature)
        self.top_p = top_p


class TopKNucleusProcessor(MultinomialProcessor):
    """Top-k then nucleus (utils/logits_processor.py:84-103)."""

    kind = "topknucleus"

    def __init__(self, temperature: float, top_k: int, top_p: float):
        super().__init__(temperature)
        self.top_k = top_k
        self.top_p = top_p
