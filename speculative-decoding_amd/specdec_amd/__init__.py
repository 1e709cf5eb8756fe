"""specdec_amd — MI355X-native speculative verify/accept path (drop-in for the hot path of
dadiaokua/speculative-decoding).

Module layout mirrors the reference's import paths for the hot path:

    specdec_amd.utils.logits_processor   <- utils/logits_processor.py
    specdec_amd.utils.caching            <- utils/caching.py
    specdec_amd.sampling                 <- sampling/speculative_decoding.py (speculative_generate, max_fn)
    specdec_amd.engine.infer_engine      <- engine/infer_engine.py (infer_batch, run_batch_speculative,
                                            batch_speculative_generate)
    specdec_amd.engine.metrics           <- engine/metrics.py (the bookkeeping dataclasses it feeds)

All compute goes through libspecdec.so (HIP, gfx950); importing fails if it is missing.
"""
from . import _lib  # noqa: F401  (loads libspecdec.so or raises)
from ._lib import RowError, get_poll_policy, set_poll_policy  # noqa: F401
from .noise import PhiloxNoise, StreamNoise, default_noise, set_noise_mode  # noqa: F401
from .ops import ProcSpec, proc_spec, probs_rows, sample_rows, verify  # noqa: F401
from . import torch_ops  # noqa: F401,E402  (registers torch.ops.specdec.sample / .verify)

__all__ = ["RowError", "get_poll_policy", "set_poll_policy", "PhiloxNoise", "StreamNoise", "default_noise", "set_noise_mode", "ProcSpec", "proc_spec",
           "probs_rows", "sample_rows", "verify"]
