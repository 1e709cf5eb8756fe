"""The device n-gram store (csrc/ngram_store.hip, sd_ngram_store_*) against
the oracle's restatement of ngram_assisted/ngram_storage.py (pinned by tests/golden/ngram_loops.json
through tests/test_ngram_storage_cpu.py): identical predictions, known flags, default-generator
draws and has_gram answers along random histories, and identical best-token tables after batched
initialize / update calls with many ties (small alphabets)."""
import pytest
import torch

from oracle import specdec_ref as ref
from specdec_amd import _lib
from specdec_amd.ngram_assisted import DeviceNGramStorage, DeviceOneLevelNGramStorage

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _make(kind, n, V, **kw):
    return (DeviceOneLevelNGramStorage if kind == "one" else DeviceNGramStorage)(n, V, device=DEV, **kw)


def _tables_equal(dev, theirs, kind, n):
    """Every gram the oracle knows predicts its best token on the device (one batched lookup per
    order: a history of exactly j tokens is looked up in order j first)."""
    for j, best in theirs.best.items():
        if not best:
            continue
        grams = list(best)
        out, known = dev.next_token(torch.tensor(grams, dtype=torch.long))
        assert bool(known.all()), j
        assert out.cpu().tolist() == [best[g] for g in grams], j


@pytest.mark.parametrize("kind,n", [("one", 2), ("one", 3), ("one", 4), ("multi", 2), ("multi", 3), ("multi", 4)])
def test_device_store_matches_oracle_along_a_history(kind, n):
    V = 50
    g = torch.Generator().manual_seed(n * 11 + len(kind))
    prompt = torch.randint(0, 8, (1, 12), generator=g)
    ours = _make(kind, n, V)
    theirs = ref.NgramStore(kind, n, V, ref.TorchNoise(None))
    ours.initialize(prompt)
    theirs.initialize(prompt[0].tolist())
    seq = prompt[0].tolist()
    for step in range(120):
        torch.manual_seed(1000 + step)
        a_tok, a_known = ours.next_token(torch.tensor([seq]))
        state_a = torch.get_rng_state()
        torch.manual_seed(1000 + step)
        b_tok, b_known = theirs.next_token(seq)
        assert torch.equal(state_a, torch.get_rng_state())          # same randint draws
        assert (int(a_tok[0]), bool(a_known[0])) == (b_tok, b_known), step
        nxt = [int(torch.randint(0, 8, (1,), generator=g))] + ([int(v) for v in torch.randint(0, V, (2,), generator=g)]
                                                                if step % 3 == 0 else [])
        ours.update(torch.tensor([seq]), torch.tensor([nxt]))
        theirs.update(seq, nxt)
        seq.append(nxt[0])
        for q in (seq[-n:], seq[-n + 1:] + [int(torch.randint(0, 8, (1,), generator=g))]):
            if kind == "one":
                per = theirs.counts.get(n - 1, {}).get(tuple(q[-(n - 1):]), {})
                want = len(q) >= n and q[-1] in per
            else:
                want = any(q[-1] in theirs.counts.get(j, {}).get(tuple(q[-j:]), {}) for j in theirs._orders(len(q)))
            assert ours.has_gram(torch.tensor(q)) == want
    _tables_equal(ours, theirs, kind, n)
    assert ours.status() == 0


@pytest.mark.parametrize("kind,n", [("one", 3), ("multi", 4)])
def test_batched_initialize_and_update_match_sequential_oracle(kind, n):
    """B histories in one initialize and one update per step: the device applies every record of
    a call at once; the oracle applies them in the reference's order (sequence by sequence)."""
    V, B, L = 64, 8, 300
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, 6, (B, L), generator=g)   # 6 symbols: dense grams, many count ties
    ours = _make(kind, n, V)
    theirs = ref.NgramStore(kind, n, V, ref.TorchNoise(None))
    ours.initialize(ids.to(DEV))
    for b in range(B):
        theirs.initialize(ids[b].tolist())
    _tables_equal(ours, theirs, kind, n)
    hist = ids.clone()
    for step in range(6):
        nxt = torch.randint(0, 6, (B, 3), generator=g)
        ours.update(hist.to(DEV), nxt.to(DEV))
        for b in range(B):
            theirs.update(hist[b].tolist(), nxt[b].tolist())
        hist = torch.cat([hist, nxt[:, :1]], 1)
        torch.manual_seed(step)
        a_tok, a_known = ours.next_token(hist)
        torch.manual_seed(step)
        want = [theirs.next_token(hist[b].tolist()) for b in range(B)]
        assert a_tok.cpu().tolist() == [w[0] for w in want]
        assert a_known.cpu().tolist() == [w[1] for w in want]
    _tables_equal(ours, theirs, kind, n)
    assert ours.status() == 0


def test_llama_vocab_ids_and_reset():
    V = 128256
    s = _make("multi", 3, V)
    s.initialize(torch.tensor([[128000, 9906, 1917, 128000, 9906, 1917, 128001]]))
    tok, known = s.next_token(torch.tensor([[128000, 9906]]))
    assert bool(known[0]) and int(tok[0]) == 1917
    s.reset()
    with pytest.raises(KeyError):          # NGramStorage: no order recorded yet (ngram_storage.py:171)
        s.next_token(torch.tensor([[128000, 9906]]))
    s.initialize(torch.tensor([[4, 5, 6]]))
    tok, known = s.next_token(torch.tensor([[4, 5]]))
    assert bool(known[0]) and int(tok[0]) == 6


def test_full_table_is_reported():
    s = _make("one", 3, 100, gram_capacity=8, pair_capacity=8)
    s.initialize(torch.arange(64).view(1, 64) % 97)
    assert s.status() & _lib.SD_NGRAM_FULL
