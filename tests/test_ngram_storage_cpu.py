"""The shipped n-gram drafters (specdec_amd.ngram_assisted, host side) against the oracle's
restatement of ngram_assisted/ngram_storage.py, itself pinned by tests/golden/ngram_loops.json:
identical predictions, known flags and default-generator draws on random token histories."""
import pytest
import torch

from oracle import specdec_ref as ref
from specdec_amd.ngram_assisted import NGramStorage, OneLevelNGramStorage


@pytest.mark.parametrize("kind,n", [("one", 2), ("one", 3), ("multi", 2), ("multi", 3), ("multi", 5)])
def test_storage_matches_oracle(kind, n):
    V = 50
    g = torch.Generator().manual_seed(n * 7 + len(kind))
    prompt = torch.randint(0, 8, (1, 12), generator=g)
    ours = (OneLevelNGramStorage if kind == "one" else NGramStorage)(n, V)
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
        assert (int(a_tok[0]), bool(a_known[0])) == (b_tok, b_known)
        nxt = [int(torch.randint(0, 8, (1,), generator=g))] + ([int(v) for v in torch.randint(0, V, (2,), generator=g)]
                                                                if step % 3 == 0 else [])
        ours.update(torch.tensor([seq]), torch.tensor([nxt]))
        theirs.update(seq, nxt)
        seq.append(nxt[0])
        # has_gram, with the reference's lookup: the gram is the LAST n-1 (or j) tokens, the queried
        # token included (ngram_storage.py:90-99, :177-188)
        for q in (seq[-n:], seq[-n + 1:] + [int(torch.randint(0, 8, (1,), generator=g))]):
            qt = torch.tensor(q)
            if kind == "one":
                per = theirs.counts.get(n - 1, {}).get(tuple(q[-(n - 1):]), {})
                want = len(q) >= n and q[-1] in per
            else:
                want = any(q[-1] in theirs.counts.get(j, {}).get(tuple(q[-j:]), {}) for j in theirs._orders(len(q)))
            assert ours.has_gram(qt) == want
    # identical best-token tables
    ob = ours.ngrams if kind == "one" else ours.ngrams
    tb = theirs.best[n - 1] if kind == "one" else theirs.best
    assert ob == tb


def test_reset_forgets():
    s = NGramStorage(3, 10)
    s.initialize(torch.tensor([[1, 2, 3, 1, 2, 3]]))
    assert s.next_token(torch.tensor([[1, 2]]))[1][0]
    s.reset()
    s.initialize(torch.tensor([[4, 5, 6]]))
    tok, known = s.next_token(torch.tensor([[4, 5]]))
    assert known[0] and int(tok[0]) == 6


def _best_by_stamps(records):
    """The device store's rule (csrc/ngram_store.hip): best = argmax over tokens of (count, -latest
    ts), with ts the record's position in the reference's processing order."""
    cnt, last = {}, {}
    for ts, (gram, tok) in enumerate(records):
        cnt[(gram, tok)] = cnt.get((gram, tok), 0) + 1
        last[(gram, tok)] = ts
    best = {}
    for (gram, tok), c in cnt.items():
        key = (c, -last[(gram, tok)])
        if gram not in best or key > best[gram][0]:
            best[gram] = (key, tok)
    return {gram: tok for gram, (key, tok) in best.items()}


@pytest.mark.parametrize("seed", range(6))
def test_order_free_best_rule_equals_the_reference_rule(seed):
    """Pins the device store's algorithm on the CPU: for random record streams (few grams, few
    tokens: many ties), argmax (count, -latest ts) equals the reference's incremental rule."""
    g = torch.Generator().manual_seed(seed)
    recs = [((int(a),), int(t)) for a, t in zip(torch.randint(0, 4, (400,), generator=g),
                                                 torch.randint(0, 5, (400,), generator=g))]
    store = ref.NgramStore("one", 2, 10, ref.TorchNoise(None))
    for gram, tok in recs:
        store._add(1, gram, [tok])
    assert _best_by_stamps(recs) == store.best[1]
