"""§8f-2 / §8f-3 on the GPU:

* ``PhiloxNoise.offset_dev``: the device-resident counter base is added to the call's offset;
* the engine window as one hipGraph (specdec_amd.engine.graph_window.EngineWindow): replays
  equal the eager windows bit for bit, and both equal the eager drop-in
  ``batch_speculative_generate`` on the same FakeLM banks and Philox seed (the window graph
  draws the noise the eager loop draws);
* device-side KV crop: ``speculative_generate(use_cache=True, static_cache=True)`` on a small
  random-init transformers Llama decodes into a StaticCache cropped by the verify kernel's
  prune outputs on the device, and returns what the uncached loop returns;
* workspaces are per stream: calls interleaved on two streams equal the same calls on one.
"""
from types import SimpleNamespace

import pytest
import torch

from fakelm import make_pair

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_offset_dev_shifts_the_philox_counter():
    from specdec_amd import PhiloxNoise, ops
    g = torch.Generator(device=DEV).manual_seed(5)
    x = (torch.randn(16, 32000, generator=g, device=DEV) * 3).to(torch.bfloat16)
    a = torch.empty(16, dtype=torch.long, device=DEV)
    b = torch.empty_like(a)
    sa = torch.empty(16, 2, device=DEV)
    sb = torch.empty_like(sa)
    ops.sample_rows(x, ops.PLAIN_SOFTMAX, PhiloxNoise(77, offset=12), tokens_out=a, row_stats_out=sa)
    od = torch.tensor([9], dtype=torch.long, device=DEV)
    ops.sample_rows(x, ops.PLAIN_SOFTMAX, PhiloxNoise(77, offset=3, offset_dev=od), tokens_out=b, row_stats_out=sb)
    assert torch.equal(a, b) and torch.equal(sa, sb)
    # a different base draws differently (a 16-row draw over 32000 tokens repeats with prob ~0)
    ops.sample_rows(x, ops.PLAIN_SOFTMAX, PhiloxNoise(77, offset=4, offset_dev=od), tokens_out=b)
    assert not torch.equal(a, b)
    with pytest.raises(ValueError):
        ops.sample_rows(x, ops.PLAIN_SOFTMAX, PhiloxNoise(77, offset_dev=od.int()), tokens_out=b)


def _window_setup(V=4096, B=8, gamma=4, gen_len=22, sigma=1.0):
    target, drafter = make_pair(V, dtype=torch.bfloat16, device=DEV, pos_mult=0, sigma=sigma)
    g = torch.Generator().manual_seed(2468)
    ids = torch.randint(3, V, (B, 6), generator=g).to(DEV)
    # end tokens that fire: the most likely continuations of a few bank rows
    ends = torch.topk(target.bank[:6].float(), 1, dim=-1).indices.flatten().tolist()
    K = target.bank.shape[0]

    def drafter_step(prev, d, step_dev):        # FakeLM(pos_mult=0) on one token: bank[(tok*31) % K]
        return drafter.bank[(prev * 31) % K]

    def target_rows(tokens, step_dev):
        return target.bank[(tokens * 31) % K]

    ctx = SimpleNamespace(drafter=drafter, target=target, gamma=gamma, gen_len=gen_len, end_tokens=ends)
    gctx = SimpleNamespace(drafter=drafter, target=target, gamma=gamma, gen_len=gen_len, end_tokens=ends,
                           drafter_step=drafter_step, target_rows=target_rows)
    return ctx, gctx, ids


@pytest.mark.parametrize("gen_len,sigma", [(22, 1.0), (40, 0.3), (8, 1.0)])
def test_window_graph_equals_the_eager_dropin(gen_len, sigma):
    from specdec_amd import set_noise_mode
    from specdec_amd.engine.infer_engine import batch_speculative_generate
    ctx, gctx, ids = _window_setup(gen_len=gen_len, sigma=sigma)
    mask = torch.ones_like(ids)
    set_noise_mode("philox", seed=31337)
    want, wrates = batch_speculative_generate(ctx, ids, mask, ids.shape[0])
    set_noise_mode("philox", seed=31337)
    got, rates = batch_speculative_generate(gctx, ids, mask, ids.shape[0])
    set_noise_mode("stream")
    assert [o.tolist() for o in got] == [o.tolist() for o in want]
    assert rates == wrates
    assert any(len(o) > ids.shape[1] for o in got)


def test_window_replays_equal_eager_windows_bit_for_bit():
    from specdec_amd import PhiloxNoise
    from specdec_amd.engine.graph_window import EngineWindow
    _, gctx, ids = _window_setup(gen_len=40, sigma=0.5)
    res = []
    for use_graph in (True, False, True):
        w = EngineWindow(gctx.drafter_step, gctx.target_rows, ids[:, -1], gctx.gamma, gctx.gen_len,
                         gctx.end_tokens, PhiloxNoise(4242))
        gen, dr, acc = w.run(use_graph=use_graph)
        torch.cuda.synchronize()
        res.append((gen.cpu(), dr.cpu(), acc.cpu(), w.finished.cpu()))
        if use_graph:
            assert w.graph is not None or w.windows_run <= 1
    for r in res[1:]:
        assert all(torch.equal(a, b) for a, b in zip(res[0], r))
    assert int(res[0][2].sum()) > 0


def test_window_offsets_move_on_the_device():
    """Two replays of the same captured window draw different noise (the base advanced)."""
    from specdec_amd import PhiloxNoise
    from specdec_amd.engine.graph_window import EngineWindow
    _, gctx, ids = _window_setup(gen_len=8, sigma=1.0, B=32, V=8192)
    w = EngineWindow(gctx.drafter_step, gctx.target_rows, ids[:, -1], 4, 8, [-1], PhiloxNoise(99))
    w.run()
    torch.cuda.synchronize()
    assert int(w.noise.offset_dev.item()) == 2 * 5
    assert int(w.step_dev.item()) == 8
    first, second = w.generated[:, :4], w.generated[:, 4:]
    assert not torch.equal(first, second)


def _tiny_llama(seed, vocab=512, layers=2):
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(vocab_size=vocab, hidden_size=128, intermediate_size=256, num_hidden_layers=layers,
                      num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256)
    torch.manual_seed(seed)
    return LlamaForCausalLM(cfg).to(DEV).eval()


@pytest.mark.parametrize("proc", ["greedy", "multinomial"])
def test_static_cache_device_crop_equals_the_uncached_loop(proc):
    pytest.importorskip("transformers")
    from specdec_amd import set_noise_mode
    from specdec_amd.sampling import speculative_generate
    from specdec_amd.utils.logits_processor import GreedyProcessor, MultinomialProcessor
    target, drafter = _tiny_llama(1), _tiny_llama(2)
    p = GreedyProcessor() if proc == "greedy" else MultinomialProcessor(temperature=1.0)
    prompt = [5, 17, 99, 3, 250, 41]
    outs = []
    for kw in (dict(use_cache=False), dict(use_cache=True, static_cache=True), dict(use_cache=True)):
        set_noise_mode("philox", seed=555)
        outs.append(speculative_generate(prompt, drafter, target, gamma=4, logits_processor=p, max_gen_len=30,
                                         eos_tokens_id=[-1], **kw))
    set_noise_mode("stream")
    assert outs[1][0] == outs[0][0] and outs[2][0] == outs[0][0]
    assert outs[1][1] == outs[0][1]
    assert len(outs[0][0]) == 30


def test_prune_static_cache_on_the_device():
    pytest.importorskip("transformers")
    from transformers.cache_utils import StaticCache
    from specdec_amd.utils.caching import prune_cache
    m = _tiny_llama(3)
    c = StaticCache(config=m.config, max_cache_len=32)
    ids = torch.randint(0, 512, (1, 10), device=DEV)
    with torch.no_grad():
        m(ids, past_key_values=c, use_cache=True)
    k = torch.tensor([3], dtype=torch.int32, device=DEV)
    prune_cache(c, k)
    assert all(int(layer.cumulative_length) == 7 for layer in c.layers)
    prune_cache(c, torch.zeros(1, dtype=torch.int32, device=DEV))
    prune_cache(c, 2)
    assert all(int(layer.cumulative_length) == 5 for layer in c.layers)


def test_workspaces_are_per_stream():
    from specdec_amd import PhiloxNoise, ops
    from specdec_amd import _lib
    g = torch.Generator(device=DEV).manual_seed(8)
    B, gam, V = 16, 4, 32000
    tl = (torch.randn(B, gam, V, generator=g, device=DEV) * 3).to(torch.bfloat16)
    dl = (tl.float() + torch.randn(B, gam, V, generator=g, device=DEV)).to(torch.bfloat16)
    draft = torch.randint(0, V, (B, gam), generator=g, device=DEV)

    def call(seed):
        return ops.verify([tl[:, t] for t in range(gam)], [dl[:, t] for t in range(gam)], draft,
                          _lib.SD_RULE_ENGINE, ops.PLAIN_SOFTMAX, ops.PLAIN_SOFTMAX, PhiloxNoise(seed))

    want = [call(s) for s in range(6)]
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    got = []
    for s in range(6):
        with torch.cuda.stream(s1 if s % 2 == 0 else s2):
            got.append(call(s))
    torch.cuda.synchronize()
    for a, b in zip(want, got):
        assert torch.equal(a.n_accepted, b.n_accepted) and torch.equal(a.next_token, b.next_token)
        assert torch.equal(a.row_status, b.row_status)


def test_torch_library_ops_equal_the_python_api():
    from specdec_amd import PhiloxNoise, _lib, ops
    g = torch.Generator(device=DEV).manual_seed(12)
    B, gam, V = 8, 4, 50257
    tl = (torch.randn(B, gam + 1, V, generator=g, device=DEV) * 3).to(torch.bfloat16)
    dl = (tl[:, :gam].float() + torch.randn(B, gam, V, generator=g, device=DEV)).to(torch.bfloat16)
    tok, stats, st = torch.ops.specdec.sample(dl[:, 0], 1, 1.0, 0, 1.0, 5, 3, 0)
    want_stats = torch.empty(B, 2, device=DEV)
    want, _, _ = ops.sample_rows(dl[:, 0], ops.ProcSpec("multinomial"), PhiloxNoise(5, 3), row_stats_out=want_stats)
    assert torch.equal(tok, want) and torch.equal(stats, want_stats)
    draft = torch.randint(0, V, (B, gam), generator=g, device=DEV)
    stops = torch.tensor([1, 2], dtype=torch.long, device=DEV)
    got = torch.ops.specdec.verify(tl, dl, draft, stops, _lib.SD_RULE_SPEC, 3, 0.8, 0, 0.9, 9, 1, 0)
    spec = ops.ProcSpec("nucleus", 0.8, 0, 0.9)
    ref = ops.verify([tl[:, t] for t in range(gam + 1)], [dl[:, d] for d in range(gam)], draft, _lib.SD_RULE_SPEC,
                     spec, spec, PhiloxNoise(9, 1), stops)
    for a, b in zip(got, (ref.n_accepted, ref.next_token, ref.resample_mass, ref.prune_drafter, ref.prune_target,
                          ref.stop_index, ref.row_status)):
        assert torch.equal(a, b) or (a.dtype == torch.float32 and torch.equal(a.isnan(), b.isnan()))

    # traced by torch.compile (aot_eager: fake-tensor tracing through register_fake, no inductor)
    def engine_verify(t, d, ids):
        return torch.ops.specdec.verify(t, d, ids, stops, _lib.SD_RULE_ENGINE, 1, 1.0, 0, 1.0, 21, 0, 0)[0]
    eager = engine_verify(tl[:, :gam], dl, draft)
    compiled = torch.compile(engine_verify, backend="aot_eager", fullgraph=True)(tl[:, :gam], dl, draft)
    assert torch.equal(eager, compiled)
