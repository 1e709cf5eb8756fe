"""Logits processors with the reference's names and constructor signatures
(utils/logits_processor.py:7-103), backed by the HIP kernels.

In the drop-in loops one of these five processors is only a parameter carrier: its (kind,
temperature, top_k, top_p) are handed to the fused verify / sample kernels, which apply
``softmax(_process(logits) / T)`` and the sampling rule inside one pass over the row.  Calling
a processor directly (``proc(logits)``) materialises the probabilities with the sd_probs
kernel; tensors must live on the GPU (there is no CPU path).

``_process`` is the reference's extension point (utils/logits_processor.py:18-20): a user subclass
that overrides it (often ``super()._process(logits)`` plus its own edit) has it run as written, in
torch ops on the device rows, and the kernels apply the softmax and the base class's sampling rule
to its output (``specdec_amd.ops.processed_rows``).  So each class's ``_process`` below is the
reference's own rule in torch (used only by such subclasses; the five classes themselves never run
it — the kernels fuse it).
"""
from __future__ import annotations

import abc

import torch
from torch import Tensor
from torch.nn import functional as F

from ..ops import ProcSpec, probs_rows

NEG_FILL = -1e20   # utils/logits_processor.py:62,79: the value written over removed logits


def _mask_below_kth(logits: Tensor, top_k: int) -> Tensor:
    """utils/logits_processor.py:59-63 (in place, as the reference)."""
    k = min(top_k, logits.size(-1))
    logits[logits < torch.topk(logits, k, dim=-1)[0][..., -1, None]] = NEG_FILL
    return logits


def _mask_outside_nucleus(logits: Tensor, top_p: float) -> Tensor:
    """utils/logits_processor.py:73-81: sort, cumulative softmax, keep through the first crossing."""
    sorted_logits, sorted_indices = torch.sort(logits, descending=True)
    cum = torch.cumsum(F.softmax(sorted_logits, dim=-1), dim=-1)
    drop = cum > top_p
    drop[..., 1:] = drop[..., :-1].clone()
    drop[..., 0] = False
    sorted_logits[drop] = NEG_FILL
    return torch.gather(sorted_logits, -1, sorted_indices.argsort(-1))


class LogitsProcessor(abc.ABC):
    """Logits processors for sampling (utils/logits_processor.py:7-23)."""

    kind = "multinomial"

    def __init__(self, temperature: float):
        self.temperature = temperature

    def spec(self) -> ProcSpec:
        return ProcSpec(self.kind, float(self.temperature), int(getattr(self, "top_k", 0)),
                        float(getattr(self, "top_p", 1.0)))

    def __call__(self, logits: Tensor) -> Tensor:
        return probs_rows(logits, self)

    def _process(self, logits: Tensor) -> Tensor:
        """The reference's processing in torch (utils/logits_processor.py:31-33, 44-46): identity.
        Run only for user subclasses that build on it; the kernels fuse the five classes' own."""
        return logits

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

    def _process(self, logits: Tensor) -> Tensor:
        return _mask_below_kth(logits, self.top_k)


class NucleusProcessor(MultinomialProcessor):
    """Nucleus / top-p sampling (utils/logits_processor.py:66-81)."""

    kind = "nucleus"

    def __init__(self, temperature: float, top_p: float):
        super().__init__(temperature)
        self.top_p = top_p

    def _process(self, logits: Tensor) -> Tensor:
        return _mask_outside_nucleus(logits, self.top_p)


class TopKNucleusProcessor(MultinomialProcessor):
    """Top-k then nucleus (utils/logits_processor.py:84-103)."""

    kind = "topknucleus"

    def __init__(self, temperature: float, top_k: int, top_p: float):
        super().__init__(temperature)
        self.top_k = top_k
        self.top_p = top_p

    def _process(self, logits: Tensor) -> Tensor:
        return _mask_outside_nucleus(_mask_below_kth(logits, self.top_k), self.top_p)
