"""The engine's opt-in cached target window (ctx.cached_target, specdec_amd/engine/infer_engine.py).

The reference re-encodes the whole sequence with the target every window (engine/infer_engine.py:
269-273).  With ``cached_target`` the drop-in keeps the target's KV cache, crops it back to the start of
the previous window (whose rejected drafts the verify zeroed, :332-336) and feeds only that window's
final tokens and the new drafts: the same tokens at the same positions, so on a random-init Llama
(fp32: the cached and the full forward agree to rounding) the decoded tokens equal the uncached loop's
in both noise modes."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def tiny_llama(seed, layers, vocab=4096):
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(vocab_size=vocab, hidden_size=256, intermediate_size=512, num_hidden_layers=layers,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512,
                      tie_word_embeddings=False)
    torch.manual_seed(seed)
    m = LlamaForCausalLM(cfg).to(DEV).eval()
    # sharpen the output distribution so drafts are sometimes accepted (random weights are near-uniform)
    with torch.no_grad():
        m.lm_head.weight.mul_(40.0)
    return m


@pytest.mark.parametrize("mode", ["philox", "stream"])
def test_cached_target_window_equals_uncached(mode):
    from types import SimpleNamespace
    from specdec_amd import set_noise_mode
    from specdec_amd.engine.infer_engine import batch_speculative_generate
    # the drafter: the target with a perturbed output layer, so drafts are accepted AND rejected (the
    # rejected ones zeroed in place, whose cached keys / values the next window must recompute)
    target, drafter = tiny_llama(1, 2), tiny_llama(1, 2)
    with torch.no_grad():
        g = torch.Generator(device=DEV).manual_seed(9)
        drafter.lm_head.weight.add_(torch.randn(drafter.lm_head.weight.shape, generator=g, device=DEV) * 0.3)
    B, L = 4, 12
    ids = torch.randint(3, 4096, (B, L), generator=torch.Generator().manual_seed(4)).to(DEV)
    mask = torch.ones_like(ids)
    res = []
    for cached in (False, True):
        set_noise_mode(mode, seed=11) if mode == "philox" else set_noise_mode("stream")
        ctx = SimpleNamespace(drafter=drafter, target=target, gamma=4, gen_len=24, end_tokens=[1],
                              cached_target=cached)
        torch.manual_seed(7)
        outs, rates = batch_speculative_generate(ctx, ids, mask, B)
        res.append(([o.tolist() for o in outs], rates))
    set_noise_mode("stream")
    assert res[0][0] == res[1][0]
    assert res[0][1] == res[1][1]
    assert 0 < sum(res[0][1]) / len(res[0][1]) < 1   # accepts and rejects: the crop was exercised
