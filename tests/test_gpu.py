"""GPU parity tests: libba_hip.so (through its C ABI) against the oracle.

Bit-exact on decisions, per-trial outcome bytes and run counters.  The oracle
runs on the same seeded inputs at sizes it finishes in seconds; at the bench's
full size (n=10, m=3, 1M trials) the checks are size-independent properties
plus oracle spot-checks of sampled trial words."""
import json
import os

import numpy as np
import pytest

import oracle_c

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
CODE = {"attack": 1, "retreat": 0, "undefined": 2}
def _engines(n=None, m=None):
    """Every engine that supports (n, m): LEVELS always, FUSED where it plans."""
    from ba_amd import lib as L
    out = [L.ENGINE_LEVELS]
    if n is not None and L.load().ba_engine_for(n, m) == L.ENGINE_FUSED:
        out.insert(0, L.ENGINE_FUSED)
    return out


def same(a, b, what=""):
    """Compact bit-exact comparison (first mismatches only, not whole arrays)."""
    a, b = np.asarray(a), np.asarray(b)
    if a.shape == b.shape and np.array_equal(a, b):
        return
    if a.shape != b.shape:
        raise AssertionError(f"{what}: shape {a.shape} != {b.shape}")
    idx = np.nonzero(a != b)[0]
    raise AssertionError(f"{what}: {len(idx)} mismatches, first at {idx[:5].tolist()}: "
                         f"got {a[idx[:5]].tolist()} want {b[idx[:5]].tolist()}")


def dec_codes(word, n):
    return [(int(word) >> (2 * r)) & 3 for r in range(n - 1)]


# --- bit-exact vs ba.py (canonical schedule, MT19937 coins in draw order) ----------
def test_table_mode_matches_ba_py(engine):
    from ba_amd import lib as L
    cases = json.load(open(os.path.join(GOLD, "om1_cases.json")))["cases"]
    by_n = {}
    for c in cases:
        by_n.setdefault(len(c["ids"]), []).append(c)
    checked = 0
    for n, cs in sorted(by_n.items()):
        fm = [sum(1 << i for i, f in enumerate(c["faulty"]) if f) for c in cs]
        pm = [sum(1 << i for i, f in enumerate(c["polls_commander"]) if f) for c in cs]
        oc = [CODE.get(c["order"], 2) for c in cs]
        tab = L.pack_coins([c["coins"] for c in cs], n)
        res = engine.run(n, 1, len(cs), lie_mode=L.LIE_TABLE, faulty=fm, order=oc, table=tab,
                         poll=pm)
        od, oo, ocnt = oracle_c.run(n, 1, len(cs), lie_mode=1, faulty=fm, order=oc, table=tab,
                                    poll=pm)
        for j, c in enumerate(cs):
            assert dec_codes(res.decisions[j], n) == [CODE[x] for x in c["majorities"][1:]], c["case"]
            q = c["quorum_line"]
            eq = 0 if "order: retreat!" in q else (1 if "order: attack!" in q else 2)
            assert int(res.outcome[j]) & 3 == eq, c["case"]
            checked += 1
        same(res.outcome, oo, '')
        assert {k: res.counters[k] for k in ocnt} == ocnt
    assert checked == len(cases)


# --- Philox mode vs the C oracle ------------------------------------------------
CONFIGS = [(1, 1), (2, 1), (3, 1), (4, 1), (4, 2), (5, 2), (6, 3), (7, 2), (7, 3), (8, 0),
           (9, 3), (10, 1), (10, 2), (10, 3), (11, 2), (13, 2), (16, 1), (17, 1), (32, 1),
           (20, 2), (12, 4)]


@pytest.mark.parametrize("n,m", CONFIGS)
def test_philox_random_sets_bit_exact(engine, n, m):
    from ba_amd import lib as L
    B = 777 if n <= 13 else 200
    kw = dict(seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=max(1, (n - 1) // 3 + 1),
              order_mode=L.ORDER_RANDOM, first_trial=64 * 1000)
    od, oo, ocnt = oracle_c.run(n, m, B, **kw)
    for eng in _engines(n, m):
        res = engine.run(n, m, B, engine=eng, **kw)
        same(res.decisions, od, f"decisions n={n} m={m} engine={eng}")
        same(res.outcome, oo, f"outcome n={n} m={m} engine={eng}")
        assert {k: res.counters[k] for k in ocnt} == ocnt


@pytest.mark.parametrize("n,m", [(4, 1), (10, 3), (16, 2), (32, 1), (5, 3)])
def test_given_inputs_and_other_orders(engine, n, m):
    rng = np.random.default_rng(n * 100 + m)
    B = 333
    fm = rng.integers(0, 1 << n, B, dtype=np.uint64).astype(np.uint32)
    fm &= rng.integers(0, 1 << n, B, dtype=np.uint64).astype(np.uint32)  # sparser sets
    oc = rng.choice([0, 1, 2], B).astype(np.uint8)
    od, oo, ocnt = oracle_c.run(n, m, B, seed=42, faulty=fm, order=oc, first_trial=128)
    for eng in _engines(n, m):
        res = engine.run(n, m, B, seed=42, faulty=fm, order=oc, first_trial=128, engine=eng)
        same(res.decisions, od, '')
        same(res.outcome, oo, '')
        assert {k: res.counters[k] for k in ocnt} == ocnt


def test_faulty_fraction_sweep_counters(engine):
    """Config 4 shape (n=10, m=3, exactly f faulty) at oracle-checkable size."""
    from ba_amd import lib as L
    for f in range(0, 5):
        kw = dict(seed=0xBA5EED, faulty_mode=L.FAULTY_EXACT, f=f, order_mode=L.ORDER_RANDOM)
        _, _, ocnt = oracle_c.run(10, 3, 1024, **kw)
        res = engine.run(10, 3, 1024, want_decisions=False, want_outcome=False, **kw)
        assert {k: res.counters[k] for k in ocnt} == ocnt
        if f <= 3:
            assert ocnt["bound_violations"] == 0


def test_sharding_invariance(engine):
    """Trials are keyed by global index: any split over calls/ranks gives the same bits."""
    from ba_amd import lib as L
    kw = dict(seed=7, faulty_mode=L.FAULTY_RANDOM, f=3, order_mode=L.ORDER_RANDOM)
    full = engine.run(10, 3, 64 * 40, **kw)
    parts = [engine.run(10, 3, 64 * 10, first_trial=64 * 10 * i, **kw) for i in range(4)]
    assert np.array_equal(full.decisions, np.concatenate([p.decisions for p in parts]))
    tot = {k: sum(p.counters[k] for p in parts) for k in full.counters}
    assert tot == full.counters


def test_levels_chunking(monkeypatch):
    """A small scratch budget forces many chunks; results must not change."""
    from ba_amd import lib as L
    kw = dict(seed=3, faulty_mode=L.FAULTY_RANDOM, f=3, order_mode=L.ORDER_RANDOM,
              engine=L.ENGINE_LEVELS)
    e1 = L.Engine(0)
    ref = e1.run(10, 3, 5000, **kw)
    e1.close()
    monkeypatch.setenv("BA_SCRATCH_BYTES", str(40 * 1024 * 8 * 5))  # ~5 words per chunk
    e2 = L.Engine(0)
    got = e2.run(10, 3, 5000, **kw)
    e2.close()
    same(ref.decisions, got.decisions, '')
    assert ref.counters == got.counters


def test_single_huge_instance_n16_m5(engine):
    """Config 5 shape: one OM(5) instance over 16 generals (4M tree slots)."""
    from ba_amd import lib as L
    fm = np.array([0b0000100000100110], np.uint32)  # generals 1, 2, 5, 11 faulty (f=4 <= 5)
    od, oo, ocnt = oracle_c.run(16, 5, 1, seed=99, faulty=fm, order=[1], first_trial=0)
    res = engine.run(16, 5, 1, seed=99, faulty=fm, order=[1], engine=L.ENGINE_LEVELS)
    same(res.decisions, od, '')
    same(res.outcome, oo, '')


def test_n13_m4_batch(engine):
    from ba_amd import lib as L
    kw = dict(seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=4, order_mode=L.ORDER_RANDOM,
              first_trial=64 * 77)
    od, oo, ocnt = oracle_c.run(13, 4, 130, **kw)
    for eng in _engines(13, 4):
        res = engine.run(13, 4, 130, engine=eng, **kw)
        same(res.decisions, od, '')
        assert {k: res.counters[k] for k in ocnt} == ocnt


def test_bench_size_properties(engine):
    """n=10, m=3, 1M trials (BASELINE config 2): size-independent invariants +
    oracle spot-checks of three sampled 64-trial words."""
    from ba_amd import lib as L
    B = 1 << 20
    kw = dict(seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=3, order_mode=L.ORDER_RANDOM)
    res = engine.run(10, 3, B, **kw)
    c = res.counters
    assert c["trials"] == B
    assert c["quorum_retreat"] + c["quorum_attack"] + c["quorum_undetermined"] == B
    assert c["in_bound"] == B and c["bound_violations"] == 0  # f <= 3 = m, n = 10 > 9
    assert c["agreement"] == B
    assert c["validity"] == c["validity_applicable"]
    assert c["undefined_decisions"] == 0
    # f ~ U{0..3}: mean 1.5 +- 5 sigma
    assert abs(c["faulty_total"] / B - 1.5) < 5 * np.sqrt(1.25 / B)
    for w in (0, 7777, B // 64 - 1):
        od, oo, _ = oracle_c.run(10, 3, 64, first_trial=64 * w, **kw)
        same(res.decisions[64 * w:64 * w + 64], od, f"word {w}")
        same(res.outcome[64 * w:64 * w + 64], oo, f"word {w}")


def test_device_api_accumulates(engine):
    import torch
    from ba_amd import lib as L
    B = 4096
    p = L.make_params(10, 3, seed=1, faulty_mode=L.FAULTY_RANDOM, f=3, order_mode=L.ORDER_RANDOM)
    dec = torch.zeros(B, dtype=torch.int64, device="cuda")
    cnt = torch.zeros(16, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    engine.run_device(p, B, d_decisions=dec.data_ptr(), d_counters=cnt.data_ptr(), stream=s.cuda_stream)
    engine.run_device(p, B, d_decisions=dec.data_ptr(), d_counters=cnt.data_ptr(), stream=s.cuda_stream)
    torch.cuda.synchronize()
    ref = engine.run(10, 3, B, seed=1, faulty_mode=L.FAULTY_RANDOM, f=3, order_mode=L.ORDER_RANDOM)
    same(dec.cpu().numpy().view(np.uint64), ref.decisions, '')
    got = cnt.cpu().numpy()
    assert int(got[0]) == 2 * B and int(got[1]) == 2 * ref.counters["agreement"]


def test_errors(engine):
    from ba_amd import lib as L
    with pytest.raises(L.BAError) as ei:
        engine.run(5, 2, 4, lie_mode=L.LIE_TABLE, faulty=[0] * 4, order=[1] * 4,
                   table=np.zeros((4, 1), np.uint32))
    assert ei.value.code == L.ENOTSUP
    with pytest.raises(L.BAError) as ei:
        engine.run(5, 1, 4, first_trial=5, faulty=[0] * 4, order=[1] * 4)
    assert ei.value.code == L.EINVAL
    with pytest.raises(L.BAError) as ei:
        engine.run(0, 1, 4, faulty=[0] * 4, order=[1] * 4)
    assert ei.value.code == L.EINVAL
    with pytest.raises(L.BAError) as ei:
        engine.run(5, 1, 4, faulty_mode=L.FAULTY_GIVEN, order=[1] * 4)
    assert ei.value.code == L.EINVAL
    res = engine.run(5, 1, 0, faulty=[], order=[])
    assert res.counters["trials"] == 0


@pytest.mark.parametrize("n,m", [(10, 3), (7, 2), (13, 4), (9, 4), (16, 3)])
def test_engines_agree_with_and_without_leaf_fusion(monkeypatch, n, m):
    """FUSED, LEVELS+k_leaf and LEVELS with the leaf level materialised
    (BA_NO_LEAF_FUSION=1) are three code paths for one function."""
    from ba_amd import lib as L
    kw = dict(seed=0xC0FFEE, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3 + 1,
              order_mode=L.ORDER_RANDOM, first_trial=64 * 5)
    B = 64 * 37 + 5
    outs = []
    e1 = L.Engine(0)
    for eng in _engines(n, m):
        outs.append((f"engine {eng}", e1.run(n, m, B, engine=eng, **kw)))
    e1.close()
    monkeypatch.setenv("BA_NO_LEAF_FUSION", "1")
    e2 = L.Engine(0)
    outs.append(("levels, leaf materialised", e2.run(n, m, B, engine=L.ENGINE_LEVELS, **kw)))
    e2.close()
    ref_name, ref = outs[-1]
    for name, r in outs[:-1]:
        same(r.decisions, ref.decisions, f"{name} vs {ref_name}")
        same(r.outcome, ref.outcome, f"{name} vs {ref_name}")
        assert r.counters == ref.counters, name
    od, oo, _ = oracle_c.run(n, m, 128, **kw)
    same(ref.decisions[:128], od, "vs oracle")


def test_fused_engine_selected_for_bench_config():
    from ba_amd import lib as L
    assert L.load().ba_engine_for(10, 3) == L.ENGINE_FUSED


@pytest.mark.parametrize("n", [4, 10, 16])
def test_philox_om1_equals_table_mode_gpu(engine, n):
    """On the device: OM(1) with Philox lies (LEVELS kernels) equals the ba.py
    table-mode kernel fed the same lies in ba.py's canonical draw order."""
    import ctypes
    from test_oracle import philox_as_ba_py_table
    from ba_amd import lib as L
    B, seed, f = 500, 23, n // 3 + 1
    res_p = engine.run(n, 1, B, seed=seed, faulty_mode=L.FAULTY_RANDOM, f=f,
                       order_mode=L.ORDER_RANDOM)
    lib = oracle_c.load()
    fms, ocs = [], []
    for t in range(B):
        fm, oc = ctypes.c_uint32(), ctypes.c_uint8()
        lib.ba_oracle_gen(n, seed, 1, f, 1, 1, t, ctypes.byref(fm), ctypes.byref(oc))
        fms.append(fm.value)
        ocs.append(oc.value)
    tab = L.pack_coins([philox_as_ba_py_table(n, seed, t, fms[t]) for t in range(B)], n)
    res_t = engine.run(n, 1, B, lie_mode=L.LIE_TABLE, faulty=fms, order=ocs, table=tab)
    same(res_p.decisions, res_t.decisions, "decisions")
    same(res_p.outcome, res_t.outcome, "outcome")
    assert res_p.counters == res_t.counters


# --- effective depth 3: the WAVE kernel vs the block and generic FUSED kernels --
OM3_CASES = [(5, 3, 1, 1), (5, 4, 2, 1), (6, 3, 1, 2), (7, 3, 2, 1), (8, 3, 3, 1), (9, 3, 3, 2),
             (10, 3, 0, 1), (10, 3, 3, 1), (10, 3, 5, 2), (10, 3, 10, 1), (11, 3, 4, 1),
             (12, 3, 7, 2), (13, 3, 4, 1), (14, 3, 14, 2), (14, 3, 4, 0)]


@pytest.mark.parametrize("n,m,f,fmode", OM3_CASES)
def test_om3_wave_block_generic_vs_oracle(monkeypatch, n, m, f, fmode):
    """k_om3w (default) and the generic block kernel k_fused (BA_FUSED_KIND=2)
    against the oracle, over every synthetic-input path of the WAVE
    kernels' branch-free generator (f <= 2, 3, <= 6 and the generic fallback;
    random / exact / given faulty sets), a ragged batch, and the persistent
    loop (BA_WAVE_MAX_BLOCKS=1: one block walks every task)."""
    from ba_amd import lib as L
    B = 64 * 8 * 5 + 37
    if fmode == 0:
        rng = np.random.default_rng(n * 31 + f)
        fm = (rng.integers(0, 1 << n, B, dtype=np.uint64) & rng.integers(0, 1 << n, B, dtype=np.uint64)
              ).astype(np.uint32)
        oc = rng.choice([0, 1, 2], B).astype(np.uint8)
        kw = dict(seed=7, faulty=fm, order=oc, first_trial=64 * 3)
        ref = oracle_c.run(n, m, B, seed=7, faulty=fm, order=oc, first_trial=64 * 3)
    else:
        kw = dict(seed=0xBA5EED + n, faulty_mode=fmode, f=f, order_mode=L.ORDER_RANDOM if f % 2 else
                  L.ORDER_CONST, order_value=1, first_trial=64 * 77)
        ref = oracle_c.run(n, m, B, **kw)
    od, oo, ocnt = ref
    for kind, cap in (("0", None), ("0", "1"), ("2", None)):
        monkeypatch.setenv("BA_FUSED_KIND", kind)
        if cap:
            monkeypatch.setenv("BA_WAVE_MAX_BLOCKS", cap)
        else:
            monkeypatch.delenv("BA_WAVE_MAX_BLOCKS", raising=False)
        e = L.Engine(0)
        try:
            res = e.run(n, m, B, engine=L.ENGINE_FUSED, **kw)
        finally:
            e.close()
        tag = f"kind={kind} cap={cap} n={n} m={m} f={f} fmode={fmode}"
        same(res.decisions, od, "decisions " + tag)
        same(res.outcome, oo, "outcome " + tag)
        assert {k: res.counters[k] for k in ocnt} == ocnt, tag


@pytest.mark.parametrize("n,B", [(10, 64 * 8 * 700 + 5), (13, 64 * 5 * 600 + 63), (7, 64 * 16 * 300)])
def test_om3_mid_batches_vs_oracle(engine, n, B):
    """The depth-3 WAVE kernel k_om3w at mid-size batches (several tasks per wave in
    its persistent loop, ragged last task), staged and drawn inputs, against the
    oracle."""
    import torch
    from ba_amd import lib as L
    kw = dict(seed=0xC0FFEE + n, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3 + 1,
              order_mode=L.ORDER_RANDOM, first_trial=64 * 11)
    od, oo, ocnt = oracle_c.run(n, 3, B, **kw)
    res = engine.run(n, 3, B, **kw)
    same(res.decisions, od, "drawn inputs")
    same(res.outcome, oo, "drawn inputs")
    assert {k: res.counters[k] for k in ocnt} == ocnt
    fb = torch.empty(B, dtype=torch.int32, device="cuda")
    ob = torch.empty(B, dtype=torch.uint8, device="cuda")
    dec = torch.empty(B, dtype=torch.int64, device="cuda")
    out = torch.empty(B, dtype=torch.uint8, device="cuda")
    cnt = torch.zeros(16, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    engine.gen_inputs_device(L.make_params(n, 3, **kw), B, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(),
                             stream=s)
    p = L.make_params(n, 3, seed=kw["seed"], first_trial=kw["first_trial"])
    engine.run_device(p, B, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(), d_decisions=dec.data_ptr(),
                      d_outcome=out.data_ptr(), d_counters=cnt.data_ptr(), stream=s)
    torch.cuda.synchronize()
    same(dec.cpu().numpy().view(np.uint64), od, "staged inputs")
    same(out.cpu().numpy(), oo, "staged inputs")
    assert cnt.cpu().tolist()[:12] == list(ocnt.values())


@pytest.mark.parametrize("n,m,fmode,f,omode", [(10, 3, 1, 3, 1), (10, 3, 2, 4, 2), (13, 4, 1, 4, 1),
                                               (4, 1, 2, 1, 1), (16, 2, 1, 5, 1), (7, 3, 1, 7, 2)])
def test_staged_inputs_equal_in_kernel_draws(engine, n, m, fmode, f, omode):
    """ba_gen_inputs_device + GIVEN-mode run == the run that draws its own
    inputs (bench.py stages inputs this way), on every engine; the staged
    inputs themselves equal the oracle's generator."""
    import ctypes
    import torch
    from ba_amd import lib as L
    B, first = 64 * 41 + 9, 64 * 123
    kw = dict(seed=0x5EED + n, faulty_mode=fmode, f=f, order_mode=omode, order_value=1,
              first_trial=first)
    fm = torch.zeros(B, dtype=torch.int32, device="cuda")
    oc = torch.zeros(B, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    p = L.make_params(n, m, kw["seed"], L.LIE_PHILOX, fmode, f, omode, 1, L.ENGINE_AUTO, first)
    engine.gen_inputs_device(p, B, d_faulty=fm.data_ptr(), d_order=oc.data_ptr(), stream=s.cuda_stream)
    torch.cuda.synchronize()
    fm_h = fm.cpu().numpy().view(np.uint32)
    oc_h = oc.cpu().numpy()
    lib = oracle_c.load()
    for t in (0, 1, 63, 64, B - 1):
        a, b = ctypes.c_uint32(), ctypes.c_uint8()
        lib.ba_oracle_gen(n, kw["seed"], fmode, f, omode, 1, first + t, ctypes.byref(a), ctypes.byref(b))
        assert (int(fm_h[t]), int(oc_h[t])) == (a.value, b.value), t
    for eng in _engines(n, m):
        drawn = engine.run(n, m, B, engine=eng, **kw)
        given = engine.run(n, m, B, seed=kw["seed"], faulty=fm_h, order=oc_h, first_trial=first,
                           engine=eng)
        same(given.decisions, drawn.decisions, f"decisions engine={eng}")
        same(given.outcome, drawn.outcome, f"outcome engine={eng}")
        assert given.counters == drawn.counters
    with pytest.raises(L.BAError):
        engine.gen_inputs_device(L.make_params(n, m, 1), B, d_faulty=fm.data_ptr())


# --- effective depth 4: the WAVE kernel k_om4w vs the oracle -----------------------
OM4_CASES = [(6, 4, 1), (6, 5, 2), (7, 4, 2), (8, 4, 2), (9, 4, 3), (10, 4, 3), (11, 4, 3),
             (12, 4, 4), (13, 4, 4), (14, 4, 5)]


@pytest.mark.parametrize("n,m,f", OM4_CASES)
def test_om4_wave_vs_oracle(monkeypatch, n, m, f):
    """k_om4w (rounds over second-level subtrees, R1 counters per first hop)
    against the oracle on a ragged batch, with and without the persistent task
    loop (BA_WAVE_MAX_BLOCKS=1 or 2: one or two blocks take tasks from the ctx's
    dynamic counter; BA_WAVE_STATIC_TASKS=1: the static stride), random faulty
    sets and given inputs."""
    from ba_amd import lib as L
    assert L.load().ba_engine_for(n, m) == L.ENGINE_FUSED
    B = 64 * 13 + 37
    kw = dict(seed=0x4A11 + n, faulty_mode=L.FAULTY_RANDOM, f=f, order_mode=L.ORDER_RANDOM,
              first_trial=64 * 55)
    od, oo, ocnt = oracle_c.run(n, m, B, **kw)
    rng = np.random.default_rng(n)
    fm = (rng.integers(0, 1 << n, B, dtype=np.uint64) & rng.integers(0, 1 << n, B, dtype=np.uint64)
          ).astype(np.uint32)
    oc = rng.choice([0, 1, 2], B).astype(np.uint8)
    gd, go, gcnt = oracle_c.run(n, m, B, seed=3, faulty=fm, order=oc)
    for cap, stat in ((None, "0"), ("1", "0"), ("2", "0"), ("2", "1")):
        monkeypatch.setenv("BA_WAVE_STATIC_TASKS", stat)
        if cap:
            monkeypatch.setenv("BA_WAVE_MAX_BLOCKS", cap)
        else:
            monkeypatch.delenv("BA_WAVE_MAX_BLOCKS", raising=False)
        e = L.Engine(0)
        try:
            res = e.run(n, m, B, engine=L.ENGINE_FUSED, **kw)
            given = e.run(n, m, B, seed=3, faulty=fm, order=oc, engine=L.ENGINE_FUSED)
        finally:
            e.close()
        tag = f"n={n} m={m} cap={cap} static={stat}"
        same(res.decisions, od, "decisions " + tag)
        same(res.outcome, oo, "outcome " + tag)
        assert {k: res.counters[k] for k in ocnt} == ocnt, tag
        same(given.decisions, gd, "given decisions " + tag)
        same(given.outcome, go, "given outcome " + tag)
        assert {k: given.counters[k] for k in gcnt} == gcnt, tag


def test_random_configs_fuzz(engine):
    """30 seeded random (n, m, f, modes, batch, first_trial) cases on the AUTO
    engine, each bit-exact against the oracle (decisions, outcomes, counters).
    BA_FUZZ_SEED="s1,s2,..." draws 30 per seed instead (a wider sweep on a lease;
    the default seed is the one the round-end run uses)."""
    from ba_amd import lib as L
    for s in os.environ.get("BA_FUZZ_SEED", "20261016").split(","):
        _random_configs(L, engine, np.random.default_rng(int(s)), s)


def _random_configs(L, engine, rng, s):
    for case in range(30):
        n = int(rng.integers(2, 17))
        m = int(rng.integers(0, 5))
        me = min(m, max(0, n - 2))
        if n > 13 and me >= 4:
            m = 3
        B = int(rng.integers(1, 700))
        first = 64 * int(rng.integers(0, 1 << 20))
        fmode = int(rng.integers(0, 3))
        omode = int(rng.integers(0, 3))
        f = int(rng.integers(0, n + 1))
        seed = int(rng.integers(0, 1 << 62))
        kw = dict(seed=seed, first_trial=first)
        if fmode == 0:
            kw["faulty"] = rng.integers(0, 1 << n, B, dtype=np.uint64).astype(np.uint32)
        else:
            kw.update(faulty_mode=fmode, f=f)
        if omode == 0:
            kw["order"] = rng.choice([0, 1, 2], B).astype(np.uint8)
        else:
            kw.update(order_mode=omode, order_value=int(rng.integers(0, 3)))
        od, oo, ocnt = oracle_c.run(n, m, B, **kw)
        res = engine.run(n, m, B, **kw)
        tag = f"seed {s} case {case}: n={n} m={m} B={B} fmode={fmode} omode={omode} f={f}"
        same(res.decisions, od, "decisions " + tag)
        same(res.outcome, oo, "outcome " + tag)
        assert {k: res.counters[k] for k in ocnt} == ocnt, tag


@pytest.mark.parametrize("n,m", [(4, 1), (7, 2), (10, 3), (16, 2), (13, 1), (15, 3)])
@pytest.mark.parametrize("epi_w", ["1", "0"])
def test_levels_bitsliced_epilogue_vs_oracle(monkeypatch, n, m, epi_w):
    """LEVELS at a batch of >= 64 groups of 64 words takes the big-batch epilogue
    (k_epilogue_w; BA_NO_EPILOGUE_W=1: the previous k_epilogue_bs): bit-exact
    with the oracle, given inputs including non-attack/retreat ("other") orders
    and dense faulty sets, ragged tail."""
    from ba_amd import lib as L
    monkeypatch.setenv("BA_NO_EPILOGUE_W", "0" if epi_w == "1" else "1")
    engine = L.Engine(0)
    rng = np.random.default_rng(n * 7 + m)
    B = 64 * 64 * 64 + 37
    fm = rng.integers(0, 1 << n, B, dtype=np.uint64).astype(np.uint32)
    fm &= rng.integers(0, 1 << n, B, dtype=np.uint64).astype(np.uint32)
    oc = rng.choice([0, 1, 2], B, p=[0.45, 0.45, 0.1]).astype(np.uint8)
    od, oo, ocnt = oracle_c.run(n, m, B, seed=9, faulty=fm, order=oc, first_trial=64 * 3)
    try:
        res = engine.run(n, m, B, seed=9, faulty=fm, order=oc, first_trial=64 * 3,
                         engine=L.ENGINE_LEVELS)
    finally:
        engine.close()
    same(res.decisions, od, f"decisions n={n} m={m}")
    same(res.outcome, oo, f"outcome n={n} m={m}")
    assert {k: res.counters[k] for k in ocnt} == ocnt


def test_run_trials_multi_world1_rccl(engine):
    """ba_run_trials_multi over a one-rank RCCL communicator owned by the C ABI:
    the all-reduced counters equal one ba_run_trials_device call, and the
    share's decisions equal the oracle's (world-N sharding is the same code
    path with a different ba_trial_share; N>1 runs on the driver's node)."""
    import torch
    from ba_amd import lib as L
    uid = L.comm_unique_id()
    comm = L.Comm(engine, 1, 0, uid)
    try:
        n, m, B = 10, 3, 64 * 50 + 9
        p = L.make_params(n, m, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_RANDOM, 3, L.ORDER_RANDOM,
                          L.ATTACK, L.ENGINE_AUTO, 64 * 7)
        dec = torch.empty(B, dtype=torch.int64, device="cuda")
        out = torch.empty(B, dtype=torch.uint8, device="cuda")
        cnt, first, count = comm.run_trials(p, B, dec.data_ptr(), out.data_ptr())
        assert (first, count) == (0, B)
        od, oo, oc = oracle_c.run(n, m, B, seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=3,
                                  order_mode=L.ORDER_RANDOM, first_trial=64 * 7)
        same(dec.cpu().numpy().view(np.uint64), od, "decisions")
        same(out.cpu().numpy(), oo, "outcome")
        assert {k: cnt[k] for k in oc} == oc
        with pytest.raises(L.BAError) as ei:  # given inputs are not sharded by this entry
            comm.run_trials(L.make_params(n, m, 1), B)
        assert ei.value.code == L.EINVAL
    finally:
        comm.close()


@pytest.mark.parametrize("n,m,B", [(16, 5, 100), (16, 5, 1), (10, 3, 64 * 64), (10, 3, 64 * 64 + 1),
                                   (7, 2, 5), (13, 4, 64 * 20 + 9), (9, 5, 130), (16, 5, 1024),
                                   (16, 3, 300), (16, 2, 70), (12, 4, 200)])
def test_levels_small_batch_fusions_vs_oracle(monkeypatch, n, m, B):
    """LEVELS launch fusions on and off -- the inputs bit-sliced inside
    k_relay_top (batches up to 2 words) vs the k_input launch, k_leaf taking
    the level me-2 majority itself (leaf-up, m_eff >= 3) vs writing R_{me-1} for
    a k_majority launch, and the small-batch k_tail (level 1 + roots + quorum,
    up to 16 words) vs k_majority + k_epilogue (BA_NO_INPUT_FUSION /
    BA_NO_LEAF_UP / BA_NO_TAIL = 1): every combination equals the oracle, for
    drawn and given inputs.  (16, 3) and (16, 2) run without leaf fusion (the
    tail then reads R_2 / the leaves L_2); (12, 4) and (9, 5) have relay pairs
    that straddle two parents in k_relay_top."""
    from ba_amd import lib as L
    kw = dict(seed=0xFACE + n, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3 + 1,
              order_mode=L.ORDER_RANDOM, first_trial=64 * 9)
    od, oo, ocnt = oracle_c.run(n, m, B, **kw)
    rng = np.random.default_rng(B)
    fm = rng.integers(0, 1 << n, B, dtype=np.uint64).astype(np.uint32)
    oc = rng.choice([0, 1, 2], B).astype(np.uint8)
    gd, go, gcnt = oracle_c.run(n, m, B, seed=3, faulty=fm, order=oc)
    for off_in, off_up, off_tail in (("0", "0", "0"), ("1", "1", "1"), ("0", "1", "0"),
                                     ("1", "0", "1"), ("0", "0", "1"), ("1", "1", "0")):
        off = off_in + off_up + off_tail
        monkeypatch.setenv("BA_NO_INPUT_FUSION", off_in)
        monkeypatch.setenv("BA_NO_LEAF_UP", off_up)
        monkeypatch.setenv("BA_NO_TAIL", off_tail)
        e = L.Engine(0)
        try:
            res = e.run(n, m, B, engine=L.ENGINE_LEVELS, **kw)
            same(res.decisions, od, f"drawn, no_fusion={off}")
            same(res.outcome, oo, f"drawn, no_fusion={off}")
            assert {k: res.counters[k] for k in ocnt} == ocnt
            res = e.run(n, m, B, seed=3, faulty=fm, order=oc, engine=L.ENGINE_LEVELS)
            same(res.decisions, gd, f"given, no_fusion={off}")
            assert {k: res.counters[k] for k in gcnt} == gcnt
        finally:
            e.close()


def test_two_ctxs_in_flight_equal_one_stream():
    """bench.py's schedule: calls alternate over two ctxs, each on its own ctx stream
    (ba_ctx_stream), so two run at once; every call's outputs and the summed counters
    equal the same calls made one at a time, and equal the oracle."""
    import torch
    from ba_amd import lib as L
    n, m, B, K = 10, 3, 64 * 257 + 5, 6
    engs = [L.Engine(0), L.Engine(0)]
    try:
        sts = [e.stream() for e in engs]
        assert sts[0] and sts[1] and sts[0] != sts[1]
        cnt = torch.zeros(16, dtype=torch.int64, device="cuda")
        decs = [torch.empty(B, dtype=torch.int64, device="cuda") for _ in range(K)]
        outs = [torch.empty(B, dtype=torch.uint8, device="cuda") for _ in range(K)]
        for i in range(K):
            p = L.make_params(n, m, 0xBA5EED, L.LIE_PHILOX, L.FAULTY_RANDOM, 3, L.ORDER_RANDOM,
                              L.ATTACK, L.ENGINE_AUTO, i * 64 * 300)
            engs[i % 2].run_device(p, B, d_decisions=decs[i].data_ptr(), d_outcome=outs[i].data_ptr(),
                                   d_counters=cnt.data_ptr(), stream=sts[i % 2])
        torch.cuda.synchronize()
        total = {k: 0 for k in L.COUNTER_NAMES}
        for i in range(K):
            od, oo, oc = oracle_c.run(n, m, B, seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=3,
                                      order_mode=L.ORDER_RANDOM, first_trial=i * 64 * 300)
            same(decs[i].cpu().numpy().view(np.uint64), od, f"decisions call {i}")
            same(outs[i].cpu().numpy(), oo, f"outcome call {i}")
            for k, v in oc.items():
                total[k] += v
        got = dict(zip(L.COUNTER_NAMES, [int(x) for x in cnt.cpu().tolist()]))
        assert {k: got[k] for k in total} == total
    finally:
        for e in engs:
            e.close()
