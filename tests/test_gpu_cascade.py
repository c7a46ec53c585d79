"""k_cascade (ba_cascade.hip): the LEVELS tree in one launch -- leaf-up units plus
the in-launch fan-in cascade of the majority levels above them, the roots and
the quorum epilogue (ba.py:159-255 generalised to OM(m)).  Bit-exact against the
C oracle on decisions, outcome bytes and counters, for every instantiated
(n, m_eff) shape, ragged batches, given and drawn inputs, several chunks per
call; and identical to the multi-launch LEVELS pipeline it replaces
(BA_NO_CASCADE=1, read per call)."""
import os

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
    multi-launch LEVELS pipeline give the same bits; a second cascade call on the
    same ctx with DIFFERENT inputs (seed, first_trial) too -- a hand-off that read
    the previous call's R words would show here, where identical inputs would hide
    it -- with the fan-in counters reset by their last arrivers in between."""
    from ba_amd import lib as L
    kw1 = dict(seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3, order_mode=L.ORDER_RANDOM)
    kw2 = dict(seed=0x5EED5, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3, order_mode=L.ORDER_RANDOM,
               first_trial=64 * 1001)
    a1 = engine.run(n, m, B, engine=L.ENGINE_LEVELS, **kw1)
    a2 = engine.run(n, m, B, engine=L.ENGINE_LEVELS, **kw2)
    monkeypatch.setenv("BA_NO_CASCADE", "1")
    b1 = engine.run(n, m, B, engine=L.ENGINE_LEVELS, **kw1)
    b2 = engine.run(n, m, B, engine=L.ENGINE_LEVELS, **kw2)
    monkeypatch.delenv("BA_NO_CASCADE")
    for a, b in ((a1, b1), (a2, b2)):
        same(a.decisions, b.decisions, "decisions")
        same(a.outcome, b.outcome, "outcome")
        assert a.counters == b.counters
    if B >= 64:
        assert not np.array_equal(a1.decisions, a2.decisions)  # the inputs did change


# --- hand-off check build (BA_CASC_CHECK, ba_cascade.hip CHECK) ---------------------
def _check_calls(engine, n, m, batches, calls, mode):
    """`calls` cascade calls on one ctx, batch sizes cycling through `batches`, each
    with its own seed and first_trial (inputs drawn in-kernel), in the check build;
    returns (mismatch count of every call, results of the calls kept for the oracle)."""
    import torch
    from ba_amd import lib as L
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    bmax = max(batches)
    dec = torch.empty(bmax, dtype=torch.int64, device=dev)
    out = torch.empty(bmax, dtype=torch.uint8, device=dev)
    cnt = torch.zeros((calls, 16), dtype=torch.int64, device=dev)
    kept = []
    for i in range(calls):
        B = batches[i % len(batches)]
        kw = dict(seed=0xC0DE + 7919 * i, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3 + i % 2,
                  order_mode=L.ORDER_RANDOM, first_trial=64 * (13 * i + 1))
        engine.run_device(L.make_params(n, m, engine=L.ENGINE_LEVELS, **kw), B,
                          d_decisions=dec.data_ptr(), d_outcome=out.data_ptr(),
                          d_counters=cnt[i].data_ptr(), stream=s)
        if i < 2 or i == calls - 1:
            torch.cuda.synchronize()
            kept.append((B, kw, dec[:B].cpu().numpy().view(np.uint64).copy(), out[:B].cpu().numpy().copy(),
                         cnt[i].cpu().tolist()))
    torch.cuda.synchronize()
    c = cnt.cpu().numpy()
    return c[:, 14], c, kept


@pytest.mark.parametrize("n,m,batches,calls", [(16, 5, (1, 1024), 120), (8, 5, (1, 700, 64), 60),
                                               (10, 3, (1, 4096), 60)])
def test_cascade_handoff_tags(engine, monkeypatch, n, m, batches, calls):
    """Every child word a cascade step reads carries this launch's epoch tag: over
    >= 100 calls that alternate batch 1 and 1024 at n=16, m=5 (and other shapes),
    with new inputs on every call, no step ever reads a word that a hand-off of
    the same launch had not yet written (0 mismatches); the check build's results
    are the oracle's."""
    from ba_amd import lib as L
    monkeypatch.setenv("BA_CASC_CHECK", "1")
    mism, cnt, kept = _check_calls(engine, n, m, batches, calls, 1)
    assert int(mism.sum()) == 0, f"stale hand-off reads: {mism.nonzero()}"
    assert (cnt[:, 0] > 0).all()
    for B, kw, d, o, c in kept:
        od, oo, oc = (oracle_c.sliced_run if B > 64 else oracle_c.run)(n, m, B, **kw)
        same(d, od, "decisions")
        same(o, oo, "outcome")
        assert c[:len(L.COUNTER_NAMES)] == list(oc.values())


@pytest.mark.parametrize("n,m", [(16, 5), (8, 5), (10, 3)])
def test_cascade_handoff_detector_fires(engine, monkeypatch, n, m):
    """BA_CASC_CHECK=2: the launch's first unit stores a stale tag beside its R word;
    the step that reads it must count exactly one mismatch per launch (the
    detector of test_cascade_handoff_tags can see a stale read)."""
    monkeypatch.setenv("BA_CASC_CHECK", "2")
    mism, _, _ = _check_calls(engine, n, m, (1, 130), 6, 2)
    assert mism.tolist() == [1] * 6


@pytest.mark.parametrize("n,m,budget_words", [(8, 5, 3), (9, 4, 2), (16, 5, 1)])
def test_cascade_scratch_budget_counts_counters(monkeypatch, n, m, budget_words):
    """BA_SCRATCH_BYTES bounds the cascade's scratch AND its fan-in counter lines
    together (round-3 advisor finding: the counters were allocated on top): with a
    budget of a few words' worth, scratch + counters stay within it, the batch runs
    in several chunks, and the results are the oracle's."""
    from ba_amd import lib as L
    # per 64-instance word: R_1..R_{me-2} (line-padded) + one 128-B counter per fan-in slot
    lib = L.load()
    me = L.effective_depth(n, m)
    S = [lib.ba_level_slots(n, m, k) for k in range(me + 1)]
    Lh = n - 1

    def pad(k):
        g = (Lh - k + 1) * (Lh - k)
        # R_1 (the roots' hand-off) is stored as granules: two words per value
        return ((g + 15) // 16) * 16 * (S[k - 2] if k >= 2 else 2)
    per_word = 8 * sum(pad(k) for k in range(1, me - 1)) + 128 * (1 + sum(S[k] for k in range(me - 3)))
    budget = per_word * budget_words + per_word // 2
    monkeypatch.setenv("BA_SCRATCH_BYTES", str(budget))
    eng = L.Engine(0)
    try:
        B = 64 * (budget_words * 3 + 1) + 17
        kw = dict(seed=0xB0D6E7 + n, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3,
                  order_mode=L.ORDER_RANDOM, first_trial=64 * 2)
        eng.profile(True)
        res = eng.run(n, m, B, engine=L.ENGINE_LEVELS, **kw)
        prof = eng.profile_read()
        mem = eng.memory()
        assert mem["budget"] == budget
        assert 0 < mem["scratch"] + mem["counters"] <= budget, mem
        units = [v[0] for k, v in prof.items() if k in ("k_cascade", "k_cascade_units", "k_cascade_units_lat")]
        assert units and units[0] >= 3, prof  # chunked
        _check(res, n, m, B, **kw)
    finally:
        eng.close()


@pytest.mark.parametrize("n,m,B", [(16, 5, 1024), (16, 5, 70), (16, 4, 600), (9, 4, 3000), (8, 5, 700),
                                   (8, 5, 1)])
def test_two_launch_equals_one_launch(engine, monkeypatch, n, m, B):
    """BA_CASC_TWO=1 (units in one launch, the fan-in from level me-3 up in a second,
    k_cascade_top) and BA_CASC_TWO=0 (the one-launch cascade) give the same bits,
    and the oracle's; the profile shows which kernels ran."""
    from ba_amd import lib as L
    kw = dict(seed=0x2A + B, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3 + 1, order_mode=L.ORDER_RANDOM,
              first_trial=64 * 9)
    out = {}
    for two in ("1", "0"):
        monkeypatch.setenv("BA_CASC_TWO", two)
        monkeypatch.setenv("BA_CASC_CO", "0")
        engine.profile(True)
        out[two] = engine.run(n, m, B, engine=L.ENGINE_LEVELS, **kw)
        prof = engine.profile_read()
        engine.profile(False)
        assert any(k in prof for k in ("k_cascade_top", "k_cascade_wtop", "k_cascade_mtop")) == (two == "1"), prof
    monkeypatch.delenv("BA_CASC_TWO")
    a, b = out["1"], out["0"]
    same(a.decisions, b.decisions, "decisions")
    same(a.outcome, b.outcome, "outcome")
    assert a.counters == b.counters
    if B <= 700:
        _check(a, n, m, B, **kw)


CO_SHAPES = [(16, 5), (16, 4), (9, 4), (8, 5)]  # ba_cascade.hip BA_CASC_TWO_SHAPES


@pytest.mark.parametrize("n,m", CO_SHAPES)
@pytest.mark.parametrize("B", [1, 64, 70, 128])
def test_co_launch_equals_two_launch(engine, monkeypatch, n, m, B):
    """The CO launch (units + co-resident fan-in blocks polling the units'
    granules, casc_co_top; the default up to 4 words) and the two-launch cascade
    (units, then k_cascade_mtop) give the same bits, and the oracle's; the profile
    shows which ran."""
    from ba_amd import lib as L
    kw = dict(seed=0xC0 + B + n, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3 + 1, order_mode=L.ORDER_RANDOM,
              first_trial=64 * 5)
    out = {}
    for co in ("1", "0"):
        monkeypatch.setenv("BA_CASC_CO", co)
        engine.profile(True)
        out[co] = engine.run(n, m, B, engine=L.ENGINE_LEVELS, **kw)
        prof = engine.profile_read()
        engine.profile(False)
        assert ("k_cascade_co" in prof) == (co == "1") and ("k_cascade_mtop" in prof) == (co == "0"), prof
    monkeypatch.delenv("BA_CASC_CO")
    engine.profile(True)
    engine.run(n, m, B, engine=L.ENGINE_LEVELS, **kw)
    assert "k_cascade_co" in engine.profile_read()  # the default at <= 4 words
    engine.profile(False)
    same(out["1"].decisions, out["0"].decisions, "decisions")
    same(out["1"].outcome, out["0"].outcome, "outcome")
    assert out["1"].counters == out["0"].counters
    _check(out["1"], n, m, B, **kw)


@pytest.mark.parametrize("B,co", [(255, True), (256, True), (257, False), (320, False)])
def test_co_launch_limit(engine, B, co):
    """The CO launch is the default up to 4 words (256 instances) and the two-launch
    cascade above; both sides of the limit equal the oracle (the sliced port)."""
    from ba_amd import lib as L
    n, m = 16, 5
    kw = dict(seed=0x11A7 + B, faulty_mode=L.FAULTY_RANDOM, f=5, order_mode=L.ORDER_RANDOM, first_trial=64 * 2)
    engine.profile(True)
    res = engine.run(n, m, B, engine=L.ENGINE_LEVELS, **kw)
    prof = engine.profile_read()
    engine.profile(False)
    assert ("k_cascade_co" in prof) == co and ("k_cascade_mtop" in prof) == (not co), prof
    _check(res, n, m, B, **kw)


def test_co_launch_handoff_tags(engine, monkeypatch):
    """The CO launch in the check build, 60 calls alternating batch 1 and 128 (new
    inputs each): every granule the fan-in blocks accept carries this launch's
    tag (0 mismatches), and replays never see the previous launch's granules."""
    monkeypatch.setenv("BA_CASC_CO", "1")
    monkeypatch.setenv("BA_CASC_CHECK", "1")
    mism, cnt, _ = _check_calls(engine, 16, 5, (1, 128), 60, 1)
    assert int(mism.sum()) == 0
    assert (cnt[:, 0] > 0).all()


@pytest.mark.parametrize("mtop", ["1", "0"])
def test_two_launch_handoff_tags(engine, monkeypatch, mtop):
    """The two-launch mode in the check build: the fan-in launch reads every child
    the units launch wrote with this call's epoch (60 calls, batch 1024 and 512),
    fan-in by k_cascade_mtop and by k_cascade_top."""
    monkeypatch.setenv("BA_CASC_TWO", "1")
    monkeypatch.setenv("BA_CASC_CO", "0")
    monkeypatch.setenv("BA_CASC_MTOP", mtop)
    monkeypatch.setenv("BA_CASC_CHECK", "1")
    mism, cnt, _ = _check_calls(engine, 16, 5, (1024, 512), 60, 1)
    assert int(mism.sum()) == 0
    assert (cnt[:, 0] > 0).all()


FANIN = {"wtop": {"BA_CASC_WTOP": "1", "BA_CASC_MTOP": "0"},
         "top": {"BA_CASC_WTOP": "0", "BA_CASC_MTOP": "0"},
         "mtop": {"BA_CASC_WTOP": "0", "BA_CASC_MTOP": "1"}}


@pytest.mark.parametrize("n,m,B", [(16, 5, 1024), (16, 5, 1), (16, 4, 130), (9, 4, 700), (8, 5, 200)])
def test_fanin_variants_agree(engine, monkeypatch, n, m, B):
    """The two-launch fan-in three ways -- one block per word (k_cascade_wtop), one
    wave per level-(me-4) slot with hand-offs (k_cascade_top), one block per
    level-(me-5) slot with one hand-off fewer (k_cascade_mtop, the default) --
    gives the same bits; and the oracle's."""
    from ba_amd import lib as L
    kw = dict(seed=0x77 + B, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3 + 1, order_mode=L.ORDER_RANDOM,
              first_trial=64 * 4)
    monkeypatch.setenv("BA_CASC_TWO", "1")
    monkeypatch.setenv("BA_CASC_CO", "0")
    out = {}
    for name, env in FANIN.items():
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        engine.profile(True)
        out[name] = engine.run(n, m, B, engine=L.ENGINE_LEVELS, **kw)
        prof = engine.profile_read()
        engine.profile(False)
        assert {x for x in FANIN if f"k_cascade_{x}" in prof} == {name}, prof
    for name in ("top", "mtop"):
        same(out["wtop"].decisions, out[name].decisions, f"decisions {name}")
        same(out["wtop"].outcome, out[name].outcome, f"outcome {name}")
        assert out["wtop"].counters == out[name].counters, name
    if B <= 200:
        _check(out["mtop"], n, m, B, **kw)


@pytest.mark.parametrize("n,m,B", [(16, 5, 1), (16, 5, 64), (16, 5, 130), (9, 4, 1), (9, 4, 700), (8, 5, 1),
                                   (8, 5, 333)])
def test_latency_mode_units_agree(engine, monkeypatch, n, m, B):
    """The units launch in latency mode (BA_CASC_LAT=1: two lanes per leaf block,
    the second in mirrored member labels, partial counts combined across the lane
    pair) and in the normal mode (one lane per leaf block) give the same bits, and
    the oracle's; the profile shows which units kernel ran."""
    from ba_amd import lib as L
    kw = dict(seed=0x1A7 + B, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3 + 1, order_mode=L.ORDER_RANDOM,
              first_trial=64 * 11)
    monkeypatch.setenv("BA_CASC_TWO", "1")
    monkeypatch.setenv("BA_CASC_CO", "0")
    out = {}
    for lat in ("1", "0"):
        monkeypatch.setenv("BA_CASC_LAT", lat)
        engine.profile(True)
        out[lat] = engine.run(n, m, B, engine=L.ENGINE_LEVELS, **kw)
        prof = engine.profile_read()
        engine.profile(False)
        assert ("k_cascade_units_lat" in prof) == (lat == "1") and ("k_cascade_units" in prof) == (lat == "0"), prof
    same(out["1"].decisions, out["0"].decisions, "decisions")
    same(out["1"].outcome, out["0"].outcome, "outcome")
    assert out["1"].counters == out["0"].counters
    if B <= 130:
        _check(out["1"], n, m, B, **kw)


def test_latency_mode_handoff_tags(engine, monkeypatch):
    """The latency-mode units in the check build: the fan-in reads every child with
    this call's epoch (40 calls, batch 1 and 64)."""
    monkeypatch.setenv("BA_CASC_TWO", "1")
    monkeypatch.setenv("BA_CASC_CO", "0")
    monkeypatch.setenv("BA_CASC_LAT", "1")
    monkeypatch.setenv("BA_CASC_CHECK", "1")
    mism, cnt, _ = _check_calls(engine, 16, 5, (1, 64), 40, 1)
    assert int(mism.sum()) == 0
    assert (cnt[:, 0] > 0).all()


def _fuzz_cases(k=24, seed=None):
    # BA_FUZZ_SEED="s1,s2,..." draws k cases per seed instead (a wider sweep on a lease)
    if seed is None:
        seeds = os.environ.get("BA_FUZZ_SEED", str(0xF022)).split(",")
        return [c for j, s in enumerate(seeds)
                for c in ((i + j * k,) + c[1:] for i, c in enumerate(_fuzz_cases(k, int(s))))]
    rng = np.random.default_rng(seed)
    shapes = SHAPES
    out = []
    for i in range(k):
        n, m = shapes[rng.integers(len(shapes))]
        B = int(rng.choice([1, 63, 64, 65, int(rng.integers(2, 900))]))
        mode = int(rng.integers(3))  # 0 random faulty sets, 1 exact f, 2 given inputs
        two = str(rng.integers(2))
        fanin = list(FANIN)[int(rng.integers(len(FANIN)))]
        fanin += "+lat" if rng.integers(2) else ""
        out.append((i, n, m, B, mode, two, fanin, int(rng.integers(0, 50)), int(rng.integers(1 << 30))))
    # the CO launch (units + co-resident fan-in blocks) drawn per case too
    co = np.random.default_rng(seed + 1).integers(2, size=k)
    return [c[:5] + (c[5] + ("+co" if co[j] else ""),) + c[6:] for j, c in enumerate(out)]


@pytest.mark.parametrize("i,n,m,B,mode,two,fanin,ft,sd", _fuzz_cases())
def test_cascade_fuzz_vs_oracle(engine, monkeypatch, i, n, m, B, mode, two, fanin, ft, sd):
    """Seeded random cascade calls: every shape k_cascade is compiled for, batch 1 to
    900 (ragged, one word, word edges), random / exact-f / given faulty sets and
    orders (incl. non-attack/retreat), random first_trial and seed, one- or two-launch
    (BA_CASC_TWO), the two-launch fan-in by any of the three kernels: bit-exact with the
    oracle on decisions, outcome bytes and counters."""
    from ba_amd import lib as L
    monkeypatch.setenv("BA_CASC_TWO", two.split("+")[0])
    monkeypatch.setenv("BA_CASC_CO", "1" if two.endswith("+co") else "0")
    for k, v in FANIN[fanin.split("+")[0]].items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("BA_CASC_LAT", "1" if fanin.endswith("+lat") else "0")
    if mode == 2:
        rng = np.random.default_rng(sd)
        fm = (rng.integers(0, 1 << n, B, dtype=np.uint64) & rng.integers(0, 1 << n, B, dtype=np.uint64)
              ).astype(np.uint32)
        oc = rng.integers(0, 3, B).astype(np.uint8)
        kw = dict(seed=sd, faulty=fm, order=oc, first_trial=64 * ft)
    else:
        kw = dict(seed=sd, faulty_mode=L.FAULTY_RANDOM if mode == 0 else L.FAULTY_EXACT,
                  f=(n - 1) // 3 + (sd % 2), order_mode=L.ORDER_RANDOM, first_trial=64 * ft)
    res = engine.run(n, m, B, engine=L.ENGINE_LEVELS, **kw)
    od, oo, oc_ = oracle_c.run(n, m, B, **kw) if B <= 128 or n < 16 else oracle_c.sliced_run(n, m, B, **kw)
    same(res.decisions, od, f"decisions case {i}")
    same(res.outcome, oo, f"outcome case {i}")
    assert {k: res.counters[k] for k in oc_} == oc_, i


def test_cascade_chunk_capped_at_sink_capacity(engine):
    """The counter sink takes < 2^16 units per replica (one unit = one word in
    k_cascade, 64 replicas): a LEVELS call of 268.4M trials (64 x 65535 + 37 words,
    more than one launch may carry) runs as two k_cascade chunks, its counters
    add up (IC1 holds for every trial in bound), and the sink replicas are left
    at zero -- the next small call is exact against the oracle."""
    from ba_amd import lib as L
    words = 64 * 65535 + 37
    B = 64 * words
    p = L.make_params(10, 3, 5, L.LIE_PHILOX, L.FAULTY_RANDOM, 3, L.ORDER_RANDOM, L.ATTACK,
                      L.ENGINE_LEVELS, 0)
    import torch
    cnt = torch.zeros(16, dtype=torch.int64, device="cuda")
    engine.profile(True)
    engine.run_device(p, B, d_counters=cnt.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    prof = engine.profile_read()
    engine.profile(False)
    c = dict(zip(L.COUNTER_NAMES, cnt.cpu().tolist()))
    assert prof["k_cascade"][0] == 2, prof
    assert c["trials"] == B and c["agreement"] == B and c["in_bound"] == B
    assert c["quorum_retreat"] + c["quorum_attack"] + c["quorum_undetermined"] == B
    kw = dict(seed=6, faulty_mode=L.FAULTY_RANDOM, f=4, order_mode=L.ORDER_RANDOM)
    _check(engine.run(10, 3, 700, engine=L.ENGINE_LEVELS, **kw), 10, 3, 700, **kw)


def test_split_falls_back_to_levels_when_cascade_scratch_does_not_fit(monkeypatch):
    """Range mode sizes the cascade's scratch for the whole tree per word; when
    that does not fit the budget in one chunk, the split runs the per-range LEVELS
    kernels (scratch shrinks with the rank's range) instead of failing with
    ETOOBIG, and the root pass (k_cascade_wtop) grows no scratch at all.  At a
    1 MiB budget, n=16, m=5, batch 1024: every second-hop unit's votes one unit at
    a time, then the root pass, equal the oracle."""
    import torch

    from ba_amd import lib as L
    monkeypatch.setenv("BA_SCRATCH_BYTES", str(1 << 20))
    eng = L.Engine(0)
    try:
        n, m, B = 16, 5, 1024
        kw = dict(seed=21, faulty_mode=L.FAULTY_RANDOM, f=5, order_mode=L.ORDER_RANDOM,
                  first_trial=64)
        p = L.make_params(n, m, **kw)
        units, per, W = L.split_units(n, m, 2), n - 3, (B + 63) // 64
        votes = torch.zeros((units * per, W), dtype=torch.int64, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        eng.profile(True)
        for u in range(units):
            eng.split_votes_device(p, B, 2, u, u + 1, votes[u * per:].data_ptr(), stream=s)
        torch.cuda.synchronize()
        prof = eng.profile_read()
        eng.profile(False)
        assert not any("k_cascade" in k for k in prof), prof  # the LEVELS kernels ran
        dec = torch.empty(B, dtype=torch.int64, device="cuda")
        out = torch.empty(B, dtype=torch.uint8, device="cuda")
        cnt = torch.zeros(16, dtype=torch.int64, device="cuda")
        scratch_before = eng.memory()["scratch"]
        eng.root_from_split_votes_device(p, B, 2, votes.data_ptr(), cnt.data_ptr(),
                                         d_decisions=dec.data_ptr(), d_outcome=out.data_ptr(),
                                         stream=s)
        torch.cuda.synchronize()
        assert eng.memory()["scratch"] == scratch_before
        od, oo, oc = oracle_c.sliced_run(n, m, B, **kw)
        same(dec.cpu().numpy().view(np.uint64), od, "decisions")
        same(out.cpu().numpy(), oo, "outcome")
        assert cnt.cpu().tolist()[:12] == list(oc.values())
    finally:
        eng.close()
