"""End-to-end share of the verify/accept hot path in the drop-in engine (GPU box).

Random-init transformers models with the Llama-3-8B (target) and Llama-3.2-1B (drafter) shapes,
bf16, on one GPU (no download: LlamaConfig only), drive the drop-in
``specdec_amd.engine.infer_engine.batch_speculative_generate`` (engine/infer_engine.py:149-359)
at B = 32, γ = 4 — configs[2] on one GPU — in both noise modes.  Every call of the hot path
(sd_sample draws, sd_verify, the STREAM word reservations) is bracketed by HIP events on the launch
stream, so the report gives the device time of the hot path against the loop's wall time, and the
end-to-end output tokens/s.  With random weights the acceptance rate means nothing (near-uniform
logits); the token count and the time split are what this measures.

    python scripts/e2e_timing.py [--batch 32 --prompt 128 --gen 64 --layers-8b 32 --layers-1b 16]
Prints one JSON object (written to profiles/ by the caller).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "speculative-decoding_amd"), ROOT]

import torch  # noqa: E402


def llama(hidden, inter, layers, heads, kv_heads, vocab=128256):
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(vocab_size=vocab, hidden_size=hidden, intermediate_size=inter, num_hidden_layers=layers,
                      num_attention_heads=heads, num_key_value_heads=kv_heads, max_position_embeddings=8192,
                      rope_theta=500000.0, tie_word_embeddings=False)
    torch.manual_seed(0)
    prev = torch.get_default_dtype()
    torch.set_default_dtype(torch.bfloat16)
    try:
        with torch.device("cuda"):
            m = LlamaForCausalLM(cfg)
    finally:
        torch.set_default_dtype(prev)
    return m.eval()


class HotPathTimer:
    """Wraps the ops the engine calls with HIP event pairs on the current stream."""

    def __init__(self, modules):
        self.pairs, self.saved = [], []
        for mod in modules:
            for name in ("sample_rows", "verify"):
                if hasattr(mod, name):
                    fn = getattr(mod, name)
                    self.saved.append((mod, name, fn))
                    setattr(mod, name, self._wrap(fn))

    def _wrap(self, fn):
        def inner(*a, **k):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            out = fn(*a, **k)
            e.record()
            self.pairs.append((s, e))
            return out
        return inner

    def device_ms(self):
        torch.cuda.synchronize()
        return sum(s.elapsed_time(e) for s, e in self.pairs)

    def restore(self):
        for mod, name, fn in self.saved:
            setattr(mod, name, fn)


def run(batch=32, prompt=128, gen=64, gamma=4, layers_8b=32, layers_1b=16,
        modes=("philox", "stream", "philox_cached", "stream_cached")):
    """Build the two random-init models, run the drop-in engine once per noise mode (after a warm-up
    run) and return the report dict."""
    from specdec_amd import set_noise_mode
    from specdec_amd.engine import infer_engine
    t0 = time.time()
    target = llama(4096, 14336, layers_8b, 32, 8)      # Llama-3-8B shape
    drafter = llama(2048, 8192, layers_1b, 32, 8)      # Llama-3.2-1B shape
    torch.cuda.synchronize()
    build_s = time.time() - t0
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(1000, 120000, (batch, prompt), generator=g).cuda()
    mask = torch.ones_like(ids)
    from types import SimpleNamespace
    ctx = SimpleNamespace(drafter=drafter, target=target, gamma=gamma, gen_len=gen,
                          end_tokens=[128001, 128009])
    res = {"target": "Llama-3-8B shape (random init, 32 layers)" if layers_8b == 32 else f"Llama-3-8B shape, {layers_8b} layers",
           "drafter": "Llama-3.2-1B shape (random init, 16 layers)" if layers_1b == 16 else f"Llama-3.2-1B shape, {layers_1b} layers",
           "dtype": "bf16", "batch": batch, "prompt_len": prompt, "gen_len": gen,
           "gamma": gamma, "model_build_s": build_s,
           "note": "random weights: the acceptance rate is meaningless (near-uniform logits); the tokens/s and the "
                   "hot path's share of the wall time are the measurement. philox / stream: the target runs "
                   "uncached over the whole sequence every window, as the reference does "
                   "(engine/infer_engine.py:270-273); *_cached: the opt-in cached target window "
                   "(ctx.cached_target: KV cache cropped to the previous window's start, same tokens)."}
    for mode in modes:
        noise_mode = mode.split("_")[0]
        ctx.cached_target = mode.endswith("_cached")
        set_noise_mode(noise_mode, seed=5) if noise_mode == "philox" else set_noise_mode("stream")
        torch.manual_seed(3)
        infer_engine.batch_speculative_generate(ctx, ids, mask, batch)   # warm-up
        torch.cuda.synchronize()
        from specdec_amd import noise as nz
        timer = HotPathTimer([infer_engine])
        timer.saved.append((nz.StreamNoise, "reserve", nz.StreamNoise.reserve))   # the STREAM word pool
        nz.StreamNoise.reserve = timer._wrap(nz.StreamNoise.reserve)
        torch.manual_seed(3)
        t0 = time.perf_counter()
        try:
            outs, rates = infer_engine.batch_speculative_generate(ctx, ids, mask, batch)
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            hot = timer.device_ms() / 1e3
            n_calls = len(timer.pairs)
        finally:
            timer.restore()
        gen_tokens = sum(len(o) - prompt for o in outs)
        res[mode] = {"wall_s": wall, "hot_path_device_s": hot, "hot_path_share": hot / wall,
                     "hot_path_calls": n_calls, "output_tokens": gen_tokens, "tokens_per_s": gen_tokens / wall,
                     "acceptance_rate_meaningless": sum(rates) / len(rates)}
        print(json.dumps({mode: res[mode]}), file=sys.stderr, flush=True)
    set_noise_mode("stream")
    del target, drafter
    torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--gen", type=int, default=64)
    ap.add_argument("--gamma", type=int, default=4)
    ap.add_argument("--layers-8b", type=int, default=32)
    ap.add_argument("--layers-1b", type=int, default=16)
    args = ap.parse_args()
    print(json.dumps(run(args.batch, args.prompt, args.gen, args.gamma, args.layers_8b, args.layers_1b)), flush=True)


if __name__ == "__main__":
    main()
