"""k_cascade (ba_cascade.hip): the LEVELS tree in one launch -- leaf-up units plus
the in-launch fan-in cascade of the majority levels above them, the roots and
the quorum epilogue (ba.py:159-255 generalised to OM(m)).  Bit-exact against the
C oracle on decisions, outcome bytes and counters, for every instantiated
(n, m_eff) shape, ragged batches, given and drawn inputs, several chunks per
call; and identical to the multi-launch LEVELS pipeline it replaces
(BA_NO_CASCADE=1, read per call)."""
import numpy as np
import pytest

import oracle_c
from test_gpu import same

pytestmark = pytest.mark.gpu

# the shapes k_cascade is compiled for (ba_cascade.hip BA_CASC_SHAPES): (n, m)
SHAPES = [(16, 5), (16, 4), (16, 3), (10, 3), (9, 4), (8, 5)]


def _check(res, n, m, B, **kw):
    od, oo, oc = oracle_c.sliced_run(n, m, B, **kw)
    same(res.decisions, od, "decisions")
    same(res.outcome, oo, "outcome")
    assert {k: res.counters[k] for k in oc} == oc


@pytest.mark.parametrize("n,m", SHAPES)
@pytest.mark.parametrize("B", [1, 70, 700])
def test_cascade_matches_oracle(engine, n, m, B):
    from ba_amd import lib as L
    kw = dict(seed=0xBA5EED + B, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3 + 1,
              order_mode=L.ORDER_RANDOM, first_trial=64 * 3)
    res = engine.run(n, m, B, engine=L.ENGINE_LEVELS, **kw)
    _check(res, n, m, B, **kw)


@pytest.mark.parametrize("n,m", [(16, 5), (10, 3), (9, 4)])
def test_cascade_given_inputs_and_other_orders(engine, n, m):
    """GIVEN faulty sets (dense, up to all generals faulty) and orders including
    a non-attack/retreat one (ba.py:214-215)."""
    from ba_amd import lib as L
    rng = np.random.default_rng(n * 100 + m)
    B = 200
    fm = rng.integers(0, 1 << n, B, dtype=np.uint64).astype(np.uint32)
    fm[:5] = (1 << n) - 1
    oc = rng.integers(0, 3, B).astype(np.uint8)
    res = engine.run(n, m, B, seed=7, engine=L.ENGINE_LEVELS, faulty=fm, order=oc)
    od, oo, ocnt = oracle_c.run(n, m, B, seed=7, faulty=fm, order=oc)
    same(res.decisions, od, "decisions")
    same(res.outcome, oo, "outcome")
    assert {k: res.counters[k] for k in ocnt} == ocnt


def test_cascade_chunks(monkeypatch):
    """A scratch budget of a few words per chunk: many k_cascade launches per call,
    each with its own word range, counters and fan-in counters."""
    from ba_amd import lib as L
    monkeypatch.setenv("BA_SCRATCH_BYTES", str(5 * 72 * 8))  # n=10, m=3: 5 words per chunk
    eng = L.Engine(0)
    try:
        kw = dict(seed=99, faulty_mode=L.FAULTY_RANDOM, f=3, order_mode=L.ORDER_RANDOM,
                  first_trial=64 * 11)
        res = eng.run(10, 3, 64 * 23 + 5, engine=L.ENGINE_LEVELS, **kw)
        _check(res, 10, 3, 64 * 23 + 5, **kw)
    finally:
        eng.close()


@pytest.mark.parametrize("n,m,B", [(16, 5, 1024), (16, 5, 1), (10, 3, 65536), (9, 4, 3000)])
def test_cascade_equals_multi_launch_pipeline(engine, monkeypatch, n, m, B):
    """Config 5's full batch (and others): the one-launch cascade and the
    multi-launch LEVELS pipeline give the same bits; repeated calls on one ctx
    (counters reset by their last arrivers) too."""
    from ba_amd import lib as L
    kw = dict(seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3, order_mode=L.ORDER_RANDOM)
    a = engine.run(n, m, B, engine=L.ENGINE_LEVELS, **kw)
    a2 = engine.run(n, m, B, engine=L.ENGINE_LEVELS, **kw)
    monkeypatch.setenv("BA_NO_CASCADE", "1")
    b = engine.run(n, m, B, engine=L.ENGINE_LEVELS, **kw)
    monkeypatch.delenv("BA_NO_CASCADE")
    for r in (a2, b):
        same(r.decisions, a.decisions, "decisions")
        same(r.outcome, a.outcome, "outcome")
        assert r.counters == a.counters

