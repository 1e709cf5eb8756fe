"""User logits processors that override only ``_process`` — the reference's extension point
(/root/reference/utils/logits_processor.py:7-23: ``__call__`` = softmax(_process(logits) / T)) —
written once and built on any of three processor modules, so every side runs the same user code:

* the reference's ``utils.logits_processor`` (tests/golden/make_golden.py: the goldens);
* the drop-in ``specdec_amd.utils.logits_processor`` (GPU tests: the kernels sample its output);
* the oracle (``oracle.specdec_ref``: a ``Processor`` whose ``pre`` runs the same edit on the
  oracle's restatement of the base processing).

Edits use only operations that round the same on the CPU and the GPU (bf16 add / multiply by a
power of two, topk selection, fills), so the GPU loops can equal the CPU reference bit for bit;
``nucleus_bias`` (a torch sort + softmax + cumsum on the device) is checked on the CPU only.
"""
import torch

IDS = (3, 17, 101, 257, 1024, 2047, 3000, 4000)   # token ids the edits touch (V >= 4096)


def _edit(name, y):
    if name == "penalty":          # a fixed penalty on a few tokens (a no-repeat-style bias)
        y[..., list(IDS)] -= 4.0
    elif name == "banned_topk":    # top-k (the base's own _process), then ban a few tokens
        y[..., list(IDS[:4])] = -1e20
    elif name == "sharpen_greedy":
        y = y * 2.0
    elif name == "nucleus_bias":   # nucleus, then a bias on a few tokens
        y[..., list(IDS[4:])] += 0.5
    return y


BASE = {"penalty": "multinomial", "banned_topk": "topk", "sharpen_greedy": "greedy", "nucleus_bias": "nucleus"}


def make_custom(lp, name, T, k=20, p=0.9):
    """The user processor `name` at temperature T (k, p: the base's top-k / top-p) on module lp."""
    base = BASE[name]
    if hasattr(lp, "processed_logits"):   # the oracle: Processor(sampling kind, T, pre=edit after the base)
        inner = lp.Processor(base, 1.0, k, p)

        def pre(x):
            return _edit(name, lp.processed_logits(x, inner))
        return lp.Processor("greedy" if base == "greedy" else "multinomial", T, pre=pre)
    if base == "multinomial":
        class Penalty(lp.MultinomialProcessor):
            def _process(self, logits):
                return _edit(name, logits.clone())
        return Penalty(T)
    if base == "topk":
        class BannedTopK(lp.TopKProcessor):
            def _process(self, logits):
                return _edit(name, super()._process(logits))
        return BannedTopK(T, k)
    if base == "greedy":
        class Sharpen(lp.GreedyProcessor):
            def _process(self, logits):
                return _edit(name, logits)
        return Sharpen(T)

    class NucleusBias(lp.NucleusProcessor):
        def _process(self, logits):
            return _edit(name, super()._process(logits))
    return NucleusBias(T, p)


def golden_processor(mod, pp):
    """The processor of a golden record's {kind, temperature, top_k, top_p} on module `mod` (the
    oracle or a processor module): custom:* kinds through make_custom."""
    kind, T, k, p = pp["kind"], pp["temperature"], pp["top_k"], pp["top_p"]
    if kind.startswith("custom:"):
        return make_custom(mod, kind.split(":", 1)[1], T, k, p)
    if hasattr(mod, "processed_logits"):
        return mod.Processor(kind, T, k, p)
    return {"greedy": lambda: mod.GreedyProcessor(T), "multinomial": lambda: mod.MultinomialProcessor(T),
            "topk": lambda: mod.TopKProcessor(T, k), "nucleus": lambda: mod.NucleusProcessor(T, p),
            "topknucleus": lambda: mod.TopKNucleusProcessor(T, k, p)}[kind]()
