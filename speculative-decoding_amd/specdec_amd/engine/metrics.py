"""Bookkeeping the engine feeds (engine/metrics.py:10-129), restated as plain dataclasses.

Only the fields and properties the speculative path fills or the benchmark reads are kept;
their meaning is the reference's: generated_tokens = len(output) - Σattention_mask (it counts
padding, :124-126 of engine/infer_engine.py), throughput = tokens / batch latency, and the
average acceptance rate skips rows whose rate is 0 (:123-129).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List


@dataclass
class RequestMetrics:
    prompt_tokens: int = 0
    generated_tokens: int = 0
    total_tokens: int = 0
    ttft: float = 0.0
    time_per_token: List[float] = field(default_factory=list)
    total_latency: float = 0.0
    acceptance_rate: float = 0.0
    drafts_generated: int = 0
    drafts_accepted: int = 0
    start_time: float = 0.0
    first_token_time: float = 0.0
    end_time: float = 0.0


@dataclass
class BatchMetrics:
    batch_size: int = 0
    requests: List[RequestMetrics] = field(default_factory=list)
    batch_start_time: float = 0.0
    batch_end_time: float = 0.0

    @property
    def batch_latency(self) -> float:
        return self.batch_end_time - self.batch_start_time

    @property
    def total_tokens(self) -> int:
        return sum(r.generated_tokens for r in self.requests)

    @property
    def throughput(self) -> float:
        lat = self.batch_latency
        return self.total_tokens / lat if lat > 0 else 0.0

    @property
    def avg_acceptance_rate(self) -> float:
        rs = [r.acceptance_rate for r in self.requests if r.acceptance_rate > 0]
        return sum(rs) / len(rs) if rs else 0.0


@dataclass
class BenchmarkResults:
    method: str
    batches: List[BatchMetrics] = field(default_factory=list)
    start_time: float = 0.0
    end_time: float = 0.0

    @property
    def total_duration(self) -> float:
        return self.end_time - self.start_time

    @property
    def total_tokens(self) -> int:
        return sum(b.total_tokens for b in self.batches)

    @property
    def overall_throughput(self) -> float:
        d = self.total_duration
        return self.total_tokens / d if d > 0 else 0.0

    @property
    def avg_acceptance_rate(self) -> float:
        rs = [r.acceptance_rate for b in self.batches for r in b.requests if r.acceptance_rate > 0]
        return sum(rs) / len(rs) if rs else 0.0
