"""CPU tests: the oracle pinned against ba.py's own outputs (tests/golden/), its
C and Python restatements against each other, Philox known-answer vectors, OM
theory properties, and the closed-form slot arithmetic of the GPU engines."""
import json
import os
import random
import re

import numpy as np
import pytest

import ba_oracle as O
import levels_model
import oracle_c

GOLD = os.path.join(os.path.dirname(__file__), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = {"attack": 1, "retreat": 0, "undefined": 2}


def load_cases():
    with open(os.path.join(GOLD, "om1_cases.json")) as fh:
        return json.load(fh)["cases"]


def case_inputs(c):
    n = len(c["ids"])
    fm = sum(1 << i for i, f in enumerate(c["faulty"]) if f)
    pm = sum(1 << i for i, f in enumerate(c["polls_commander"]) if f)
    oc = CODE.get(c["order"], 2)
    exp = [CODE[x] for x in c["majorities"][1:]]
    q = c["quorum_line"]
    eq = 0 if q.startswith("Execute order: retreat!") else (1 if q.startswith("Execute order: attack!") else 2)
    return n, fm, pm, oc, exp, eq


# --- Philox4x32-10 known-answer vectors (Random123 kat_vectors) ------------
KAT = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
       ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
       ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
        (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_philox_kat(ctr, key, want):
    assert O.philox4x32_10(ctr, key) == want
    lib = oracle_c.load()
    c = np.array(ctr, np.uint32)
    k = np.array(key, np.uint32)
    o = np.zeros(4, np.uint32)
    lib.ba_oracle_philox(c.ctypes.data, k.ctypes.data, o.ctypes.data)
    assert tuple(int(x) for x in o) == want


def test_lie_c_matches_python():
    lib = oracle_c.load()
    rng = random.Random(1)
    for _ in range(300):
        seed, t, k, x = rng.getrandbits(64), rng.getrandbits(40), rng.randrange(8), rng.getrandbits(31)
        assert lib.ba_oracle_lie(seed, t, k, x) == O.lie(seed, t, k, x)


# --- pinned against ba.py ----------------------------------------------------
def test_golden_python_restatement():
    cases = load_cases()
    assert len(cases) >= 400
    for c in cases:
        n, fm, pm, oc, exp, eq = case_inputs(c)
        dec = O.om1_table_decisions(n, 1, fm, int(oc == 1), c["coins"], pm)
        assert dec == exp, c["case"]
        assert O.quorum(n, oc, dec)[0] == eq, c["case"]


def test_golden_mt_replay():
    """random.Random(seed) drawing the canonical coin count reproduces ba.py's
    coins and leaves the MT19937 stream where ba.py left it."""
    for c in load_cases():
        n, fm, pm, oc, exp, eq = case_inputs(c)
        rng = random.Random(c["seed"])
        assert O.mt_coins(rng, n, fm, 1, pm) == c["coins"], c["case"]
        assert rng.getrandbits(32) == c["next_mt_word"], c["case"]


def test_golden_c_oracle_table_mode():
    by_n = {}
    for c in load_cases():
        by_n.setdefault(len(c["ids"]), []).append(c)
    for n, cs in by_n.items():
        from ba_amd.lib import pack_coins
        tab = pack_coins([c["coins"] for c in cs], n)
        ins = [case_inputs(c) for c in cs]
        dec, out, cnt = oracle_c.run(n, 1, len(cs), lie_mode=1, faulty=[i[1] for i in ins],
                                     order=[i[3] for i in ins], table=tab,
                                     poll=[i[2] for i in ins])
        for j, (c, i) in enumerate(zip(cs, ins)):
            got = [(int(dec[j]) >> (2 * r)) & 3 for r in range(n - 1)]
            assert got == i[4], c["case"]
            assert int(out[j]) & 3 == i[5], c["case"]


# --- C vs Python restatement (Philox mode) ------------------------------------
@pytest.mark.parametrize("n,m", [(1, 1), (2, 1), (3, 1), (4, 1), (4, 2), (5, 2), (7, 3), (10, 2),
                                 (6, 4), (8, 0), (13, 1)])
def test_c_matches_python_philox(n, m):
    B = 96
    d1, o1, c1 = oracle_c.run(n, m, B, seed=0xBA5EED, faulty_mode=1, f=max(1, n // 3),
                              order_mode=1, first_trial=64 * 3)
    d2, o2, c2 = O.run(n, m, seed=0xBA5EED, faulty_mode=1, f=max(1, n // 3), order_mode=1,
                       first_trial=64 * 3, batch=B)
    assert [int(x) for x in d1] == d2
    assert [int(x) for x in o1] == o2
    assert c1 == c2


def test_c_gen_matches_python():
    lib = oracle_c.load()
    fm = np.zeros(1, np.uint32)
    oc = np.zeros(1, np.uint8)
    for n in (1, 4, 10, 16, 32):
        for mode, f in ((1, n // 3), (2, min(n, 5)), (2, n)):
            for t in (0, 1, 63, 64, 12345, 1 << 33):
                lib.ba_oracle_gen(n, 77, mode, f, 1, 0, t, fm.ctypes.data, oc.ctypes.data)
                pm, po = O.gen(n, 77, mode, f, 1, 0, t)
                assert (int(fm[0]), int(oc[0])) == (pm, po)
                if mode == 2:
                    assert bin(pm).count("1") == min(n, f)


# --- OM theory properties ------------------------------------------------------
@pytest.mark.parametrize("n,m", [(4, 1), (7, 2), (10, 3), (13, 4)])
def test_om_guarantee_within_bound(n, m):
    """Lamport: with n > 3m generals and at most m traitors OM(m) satisfies IC1+IC2."""
    B = 256 if n < 13 else 64
    _, out, cnt = oracle_c.run(n, m, B, seed=5, faulty_mode=1, f=m, order_mode=1)
    assert cnt["in_bound"] == B
    assert cnt["bound_violations"] == 0
    assert cnt["agreement"] == B


def test_om_breaks_beyond_bound():
    """n=4, 2 traitors: OM(1) loses agreement on some trials (IC1 is not free)."""
    _, _, cnt = oracle_c.run(4, 1, 2048, seed=9, faulty_mode=2, f=2, order_mode=1)
    assert cnt["in_bound"] == 0
    assert cnt["agreement"] < 2048


def test_counter_identities():
    _, out, cnt = oracle_c.run(10, 3, 512, seed=3, faulty_mode=1, f=4, order_mode=1)
    assert cnt["quorum_retreat"] + cnt["quorum_attack"] + cnt["quorum_undetermined"] == 512
    assert cnt["validity"] <= cnt["validity_applicable"]
    assert cnt["attack_decisions"] + cnt["undefined_decisions"] <= 512 * 9
    assert cnt["undefined_decisions"] == 0  # 9 inputs at the root never tie


def test_sharding_invariance_oracle():
    full = oracle_c.run(7, 2, 256, seed=11, faulty_mode=1, f=2, order_mode=1)
    a = oracle_c.run(7, 2, 128, seed=11, faulty_mode=1, f=2, order_mode=1)
    b = oracle_c.run(7, 2, 128, seed=11, faulty_mode=1, f=2, order_mode=1, first_trial=128)
    assert np.array_equal(full[0], np.concatenate([a[0], b[0]]))
    assert {k: a[2][k] + b[2][k] for k in a[2]} == full[2]


# --- closed-form slot arithmetic of the GPU engines (CPU model) ----------------
@pytest.mark.parametrize("n,m", [(4, 1), (5, 2), (6, 3), (7, 2), (10, 1)])
def test_levels_model_matches_oracle(n, m):
    seed, gw = 0xBA5EED, 5
    fm, oc = [], []
    for t in range(64 * gw, 64 * gw + 64):
        a, b = O.gen(n, seed, 1, max(1, (n - 1) // 3 + 1), 1, 0, t)
        fm.append(a)
        oc.append(b)
    dec = levels_model.run_word(n, m, seed, gw, fm, oc)
    d2, _, _ = oracle_c.run(n, m, 64, seed=seed, faulty=fm, order=oc, first_trial=64 * gw)
    for t in range(64):
        assert dec[t] == [(int(d2[t]) >> (2 * r)) & 3 for r in range(n - 1)], t


# --- numeric contract between include/ba.h, the oracle and the binding ---------
def test_header_constants_agree():
    hdr = open(os.path.join(ROOT, "include", "ba.h")).read()
    defs = dict(re.findall(r"#define (BA_\w+) \(?(-?\d+)\)?", hdr))
    from ba_amd import lib as L
    pairs = {"BA_LIE_PHILOX": L.LIE_PHILOX, "BA_LIE_TABLE": L.LIE_TABLE,
             "BA_FAULTY_GIVEN": L.FAULTY_GIVEN, "BA_FAULTY_RANDOM": L.FAULTY_RANDOM,
             "BA_FAULTY_EXACT": L.FAULTY_EXACT, "BA_ORDER_GIVEN": L.ORDER_GIVEN,
             "BA_ORDER_RANDOM": L.ORDER_RANDOM, "BA_ORDER_CONST": L.ORDER_CONST,
             "BA_RETREAT": O.RETREAT, "BA_ATTACK": O.ATTACK, "BA_OTHER": O.OTHER,
             "BA_UNDEFINED": O.UNDEFINED, "BA_Q_RETREAT": O.Q_RETREAT, "BA_Q_ATTACK": O.Q_ATTACK,
             "BA_Q_UNDETERMINED": O.Q_UNDET, "BA_NCOUNTERS": L.NCOUNTERS,
             "BA_ABI_VERSION": L.ABI_VERSION, "BA_MAX_GENERALS": L.MAX_GENERALS,
             "BA_EINVAL": L.EINVAL, "BA_EDEVICE": L.EDEVICE, "BA_ENOTSUP": L.ENOTSUP,
             "BA_ENGINE_FUSED": L.ENGINE_FUSED, "BA_ENGINE_LEVELS": L.ENGINE_LEVELS}
    for k, v in pairs.items():
        assert int(defs[k]) == v, k
    names = re.findall(r"#define BA_C_(\w+) (\d+)", hdr)
    run = [int(x) for k, x in names if k != "CHECK_MISMATCH"]
    assert run == list(range(len(L.COUNTER_NAMES)))
    # the test-only hand-off check slot sits past the run counters, below the error flag
    assert dict(names)["CHECK_MISMATCH"] == str(L.NCOUNTERS - 2)
    assert L.COUNTER_NAMES == O.COUNTERS == oracle_c.COUNTER_NAMES


def philox_as_ba_py_table(n, seed, t, fm):
    """The Philox lies of an OM(1) trial, laid out as ba.py's canonical coin
    sequence: the commander's coins for lieutenants 1..n-1 (ba.py:263-273), then
    receiver-major: for r = 1..n-1, for j != r faulty, the coin j tells r
    (ba.py:169-186).  Level-1 slot of (j, r) = j'(L-1) + r' - [r' > j']."""
    L = n - 1
    coins = []
    if fm & 1:
        coins += [O.lie(seed, t, 0, r) for r in range(L)]
    for r in range(L):
        for j in range(L):
            if j != r and (fm >> (j + 1)) & 1:
                coins.append(O.lie(seed, t, 1, j * (L - 1) + r - (r > j)))
    return coins


@pytest.mark.parametrize("n", [3, 4, 7, 10, 13])
def test_om_recursion_at_m1_is_ba_py_rule(n):
    """Links the OM(m) recursion (Philox lies) to ba.py: at m=1 it equals the
    table-mode restatement -- pinned on ba.py's own fixtures above -- fed the
    same lies in ba.py's draw order."""
    from ba_amd.lib import pack_coins
    B = 300
    kw = dict(seed=17, faulty_mode=1, f=n // 2, order_mode=1)
    dec_p, out_p, cnt_p = oracle_c.run(n, 1, B, **kw)
    fms, ocs = [], []
    lib = oracle_c.load()
    import ctypes
    for t in range(B):
        fm, oc = ctypes.c_uint32(), ctypes.c_uint8()
        lib.ba_oracle_gen(n, 17, 1, n // 2, 1, 1, t, ctypes.byref(fm), ctypes.byref(oc))
        fms.append(fm.value)
        ocs.append(oc.value)
    tab = pack_coins([philox_as_ba_py_table(n, 17, t, fms[t]) for t in range(B)], n)
    dec_t, out_t, cnt_t = oracle_c.run(n, 1, B, lie_mode=1, faulty=fms, order=ocs, table=tab)
    assert np.array_equal(dec_p, dec_t)
    assert np.array_equal(out_p, out_t)
    assert cnt_p == cnt_t


# --- the word-sliced OpenMP port (oracle/ba_sliced.c) equals the recursion ----------
SLICED_CASES = [(2, 1), (3, 1), (4, 1), (4, 2), (5, 3), (6, 6), (7, 2), (8, 5), (9, 4), (10, 0),
                (10, 1), (10, 3), (11, 3), (12, 2), (13, 4), (16, 2), (20, 2), (32, 1)]


@pytest.mark.parametrize("n,m", SLICED_CASES)
def test_sliced_port_equals_recursion(n, m):
    """bench.py's CPU baseline and the large-size checker (ba_sliced.c) against the
    textbook recursion, on random, exact (beyond the bound) and dense faulty sets,
    ragged batches, a non-zero first trial and 'other' orders."""
    import oracle_c
    B = 300 if n < 13 else 100
    for fm, f, om in [(1, (n - 1) // 3, 1), (2, min(n, m + 1), 2), (1, n, 1)]:
        kw = dict(seed=12345 + n, faulty_mode=fm, f=f, order_mode=om, order_value=2,
                  first_trial=64 * 7)
        d1, o1, c1 = oracle_c.run(n, m, B, **kw)
        d2, o2, c2 = oracle_c.sliced_run(n, m, B, **kw)
        assert np.array_equal(d1, d2) and np.array_equal(o1, o2) and c1 == c2, (n, m, fm, f, om)


def test_sliced_port_given_inputs_and_n16_m5():
    """Given inputs (sliced_gen staging) equal in-port draws; config 5's tree (n=16,
    m=5) on three instances equals the recursion."""
    import oracle_c
    kw = dict(seed=0xBA5EED, faulty_mode=1, f=3, order_mode=1, first_trial=64 * 5)
    fm, oc = oracle_c.sliced_gen(10, 1000, **kw)
    a = oracle_c.sliced_run(10, 3, 1000, **kw)
    b = oracle_c.sliced_run(10, 3, 1000, faulty=fm, order=oc, first_trial=64 * 5, seed=0xBA5EED)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) and a[2] == b[2]
    kw = dict(seed=0xBA5EED, faulty_mode=1, f=5, order_mode=1, first_trial=64 * 3)
    d1, o1, c1 = oracle_c.run(16, 5, 3, **kw)
    d2, o2, c2 = oracle_c.sliced_run(16, 5, 3, **kw)
    assert np.array_equal(d1, d2) and np.array_equal(o1, o2) and c1 == c2
