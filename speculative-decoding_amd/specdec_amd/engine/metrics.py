"""Bookkeeping the engine feeds — the full surface of engine/metrics.py:10-230.

The benchmark harness (engine/benchmark_runner.py:200-340, benchmark_old.py:383-560) builds
``BenchmarkResults`` from the ``BatchMetrics`` that ``infer_batch`` returns and calls
``to_dict`` / ``save_json`` / ``print_benchmark_summary`` / ``print_comparison`` on them, so
every field, property and key is the reference's, with the reference's formulas:

* ``generated_tokens = len(output) − Σattention_mask`` (it counts padding,
  engine/infer_engine.py:124-126);
* batch and overall throughput = tokens / latency (0 when the latency is not positive);
* ``avg_ttft`` / ``avg_latency`` are plain means over requests (metrics.py:52-64,107-121);
* ``avg_acceptance_rate`` averages only requests whose rate is > 0 (:123-129).

The printers write the same lines as the reference without colour codes (the reference's
``termcolor`` is not a dependency here).
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from typing import Dict, List


@dataclass
class RequestMetrics:
    """engine/metrics.py:10-30."""
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
    """engine/metrics.py:33-71."""
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
    def avg_ttft(self) -> float:
        if not self.requests:
            return 0.0
        return sum(r.ttft for r in self.requests) / len(self.requests)

    @property
    def avg_latency(self) -> float:
        if not self.requests:
            return 0.0
        return sum(r.total_latency for r in self.requests) / len(self.requests)

    @property
    def throughput(self) -> float:
        if self.batch_latency <= 0:
            return 0.0
        return self.total_tokens / self.batch_latency

    @property
    def avg_acceptance_rate(self) -> float:
        # not in the reference's BatchMetrics; kept for callers of round 1's drop-in
        rs = [r.acceptance_rate for r in self.requests if r.acceptance_rate > 0]
        return sum(rs) / len(rs) if rs else 0.0


@dataclass
class BenchmarkResults:
    """engine/metrics.py:74-175."""
    method: str
    total_requests: int = 0
    total_batches: int = 0
    batches: List[BatchMetrics] = field(default_factory=list)
    start_time: float = 0.0
    end_time: float = 0.0

    def _requests(self, positive_rate: bool = False) -> List[RequestMetrics]:
        return [r for b in self.batches for r in b.requests if not positive_rate or r.acceptance_rate > 0]

    @property
    def total_duration(self) -> float:
        return self.end_time - self.start_time

    @property
    def total_tokens(self) -> int:
        return sum(b.total_tokens for b in self.batches)

    @property
    def total_prompt_tokens(self) -> int:
        return sum(r.prompt_tokens for r in self._requests())

    @property
    def overall_throughput(self) -> float:
        if self.total_duration <= 0:
            return 0.0
        return self.total_tokens / self.total_duration

    @property
    def avg_ttft(self) -> float:
        rs = self._requests()
        return sum(r.ttft for r in rs) / len(rs) if rs else 0.0

    @property
    def avg_latency(self) -> float:
        rs = self._requests()
        return sum(r.total_latency for r in rs) / len(rs) if rs else 0.0

    @property
    def avg_acceptance_rate(self) -> float:
        rs = self._requests(positive_rate=True)
        return sum(r.acceptance_rate for r in rs) / len(rs) if rs else 0.0

    def to_dict(self) -> Dict:
        """engine/metrics.py:131-168: the same keys, in the same nesting."""
        return {
            "method": self.method,
            "total_requests": self.total_requests,
            "total_batches": self.total_batches,
            "total_duration": self.total_duration,
            "total_tokens": self.total_tokens,
            "total_prompt_tokens": self.total_prompt_tokens,
            "overall_throughput": self.overall_throughput,
            "avg_ttft": self.avg_ttft,
            "avg_latency": self.avg_latency,
            "avg_acceptance_rate": self.avg_acceptance_rate,
            "batches": [_batch_dict(b) for b in self.batches],
        }

    def save_json(self, filepath: str) -> None:
        """engine/metrics.py:170-175."""
        with open(filepath, "w") as f:
            json.dump(self.to_dict(), f, indent=2)
        print(f"✅ Results saved to {filepath}")


def _batch_dict(b: BatchMetrics) -> Dict:
    return {
        "batch_size": b.batch_size,
        "batch_latency": b.batch_latency,
        "total_tokens": b.total_tokens,
        "avg_ttft": b.avg_ttft,
        "avg_latency": b.avg_latency,
        "throughput": b.throughput,
        "requests": [
            {
                "prompt_tokens": r.prompt_tokens,
                "generated_tokens": r.generated_tokens,
                "total_tokens": r.total_tokens,
                "ttft": r.ttft,
                "total_latency": r.total_latency,
                "acceptance_rate": r.acceptance_rate,
                "drafts_generated": r.drafts_generated,
                "drafts_accepted": r.drafts_accepted,
            }
            for r in b.requests
        ],
    }


def print_benchmark_summary(results: BenchmarkResults) -> None:
    """engine/metrics.py:178-203 (same lines, no colour)."""
    print("\n" + "=" * 70)
    print(f"📊 Benchmark Results: {results.method.upper()}")
    print("=" * 70)
    print("\n🎯 Overall Statistics:")
    print(f"  Total Requests:     {results.total_requests}")
    print(f"  Total Batches:      {results.total_batches}")
    print(f"  Total Duration:     {results.total_duration:.2f} s")
    print(f"  Total Tokens:       {results.total_tokens:,}")
    print(f"  Prompt Tokens:      {results.total_prompt_tokens:,}")
    print(f"  Generated Tokens:   {results.total_tokens - results.total_prompt_tokens:,}")
    print("\n⚡ Performance Metrics:")
    print(f"  Overall Throughput: {results.overall_throughput:.2f} tokens/s")
    print(f"  Average TTFT:       {results.avg_ttft * 1000:.2f} ms")
    print(f"  Average Latency:     {results.avg_latency * 1000:.2f} ms")
    if results.method == "speculative":
        print("\n🎲 Speculative Decoding Metrics:")
        print(f"  Average Acceptance Rate: {results.avg_acceptance_rate:.3f}")
    print("\n" + "=" * 70)


def print_comparison(spec_results: BenchmarkResults, target_results: BenchmarkResults) -> None:
    """engine/metrics.py:206-230 (same ratios, same guards, no colour)."""
    s, t = spec_results, target_results
    speedup = t.avg_latency / s.avg_latency if s.avg_latency > 0 else 0
    gain = (s.overall_throughput / t.overall_throughput - 1) * 100 if t.overall_throughput > 0 else 0
    print("\n" + "=" * 70)
    print("📈 Performance Comparison")
    print("=" * 70)
    print("\n⚡ Speed Metrics:")
    print(f"  Throughput Speedup:  {speedup:.2f}x")
    print(f"  Throughput Gain:     {gain:+.1f}%")
    if t.avg_latency > 0:
        print(f"  Latency Reduction:   {(1 - s.avg_latency / t.avg_latency) * 100:.1f}%")
    else:
        print("  Latency Reduction:   N/A")
    print("\n📊 Detailed Comparison:")
    print(f"{'Metric':<25} {'Speculative':<15} {'Target AR':<15} {'Ratio':<10}")
    print("-" * 70)
    print(f"{'Throughput (tok/s)':<25} {s.overall_throughput:<15.2f} {t.overall_throughput:<15.2f} {speedup:<10.2f}x")
    if t.avg_ttft > 0:
        print(f"{'Avg TTFT (ms)':<25} {s.avg_ttft * 1000:<15.2f} {t.avg_ttft * 1000:<15.2f} "
              f"{s.avg_ttft / t.avg_ttft:<10.2f}x")
    else:
        print(f"{'Avg TTFT (ms)':<25} {s.avg_ttft * 1000:<15.2f} {t.avg_ttft * 1000:<15.2f} {'N/A':<10}")
    print(f"{'Avg Latency (ms)':<25} {s.avg_latency * 1000:<15.2f} {t.avg_latency * 1000:<15.2f} {speedup:<10.2f}x")
    print("\n" + "=" * 70)
