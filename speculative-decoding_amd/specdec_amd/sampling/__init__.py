from .speculative_decoding import max_fn, speculative_generate  # noqa: F401
