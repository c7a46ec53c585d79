"""ba.py's coin source replayed in C++ (libba_hip ba_mt_*, host only, no device).

Pinned against tests/golden/om1_cases.json, which recorded -- from ba.py itself
under the canonical schedule -- every random.randint(0, 1) coin of a round in
draw order and the next getrandbits(32) word after it (gen_golden.py)."""
import json
import os
import random

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _cases():
    return json.load(open(os.path.join(GOLD, "om1_cases.json")))["cases"]


def _masks(c):
    fm = sum(1 << i for i, f in enumerate(c["faulty"]) if f)
    pm = sum(1 << i for i, f in enumerate(c["polls_commander"]) if f)
    return fm, pm


def test_mt_matches_cpython_random():
    from ba_amd import lib as L
    for seed in (0, 1, 5, 0xBA5EED, (1 << 32) - 1, 1 << 32, (1 << 64) - 1, 123456789012345):
        mt = L.MT(seed)
        ref = random.Random(seed)
        assert [mt.next32() for _ in range(1500)] == [ref.getrandbits(32) for _ in range(1500)]


def test_coins_match_randint():
    from ba_amd import lib as L
    mt = L.MT(2024)
    ref = random.Random(2024)
    packed = mt.coins(1000)
    got = [(int(packed[c >> 5]) >> (c & 31)) & 1 for c in range(1000)]
    assert got == [1 if ref.randint(0, 1) == 0 else 0 for _ in range(1000)]
    assert mt.next32() == ref.getrandbits(32)


def test_coin_count_and_draws_match_ba_py_rounds():
    """Every fixture round: the count, the coins and the MT state after it."""
    from ba_amd import lib as L
    cases = _cases()
    assert len(cases) >= 400
    for c in cases:
        n = len(c["ids"])
        fm, pm = _masks(c)
        cnt = L.om1_coin_count(n, 1, fm, pm)
        assert cnt == len(c["coins"]), c["case"]
        mt = L.MT(c["seed"])
        packed = mt.coins(cnt, L.table_stride(n))
        got = [(int(packed[i >> 5]) >> (i & 31)) & 1 for i in range(cnt)]
        assert got == c["coins"], c["case"]
        assert mt.next32() == c["next_mt_word"], c["case"]


def test_batched_table_matches_fixtures():
    from ba_amd import lib as L
    by_n = {}
    for c in _cases():
        by_n.setdefault(len(c["ids"]), []).append(c)
    for n, cs in by_n.items():
        fms, pms = zip(*[_masks(c) for c in cs])
        tab, nxt = L.mt_table(n, 1, [c["seed"] for c in cs], fms, pms, threads=4)
        assert np.array_equal(tab, L.pack_coins([c["coins"] for c in cs], n)), n
        assert nxt.tolist() == [c["next_mt_word"] for c in cs], n


def test_table_threads_invariant():
    from ba_amd import lib as L
    rng = np.random.default_rng(1)
    B, n = 5000, 13
    seeds = rng.integers(0, 1 << 62, B, dtype=np.uint64)
    fm = rng.integers(0, 1 << n, B, dtype=np.uint64).astype(np.uint32)
    pm = rng.integers(0, 1 << n, B, dtype=np.uint64).astype(np.uint32)
    a = L.mt_table(n, 1, seeds, fm, pm, threads=1)
    b = L.mt_table(n, 1, seeds, fm, pm, threads=7)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_mt_errors():
    from ba_amd import lib as L
    with pytest.raises(ValueError):
        L.MT(-1)
    assert L.om1_coin_count(0, 1, 0, 0) == 0
    assert L.om1_coin_count(4, 0, 0b1111, 0) == 3  # OM(0): commander coins only
    mt = L.MT(1)
    with pytest.raises(L.BAError):
        mt.coins(100, 2)  # 64 bits cannot hold 100 coins
