"""A lost in-launch hand-off of the LEVELS cascade is an error, never a wrong
answer; and the CO launch's forward-progress bound (ba_api.cpp co_admit).

The cascade's workgroups hand R_1 (and, in CO launches, R_{me-2}) to each other
through tagged granules whose polls are bounded in time (ba_cascade.hip).  A
poll that runs out of time counts into counter slot 14; ba_run_trials and the
multi-rank jobs then return BA_EDEVICE, and device-path callers see slot 14
(include/ba.h).  BA_TEST_GRANULE_TICKS shrinks the bound to force it.  ba.py
swallows errors (ba.py:185-186, 219-221); this path must not turn them into
silent wrong decisions.
"""
import numpy as np
import pytest

import oracle_c
from test_gpu import same

pytestmark = pytest.mark.gpu

N, M = 16, 5


def _kw(B, i):
    from ba_amd import lib as L
    return dict(seed=0x7A11 + 31 * i + B, faulty_mode=L.FAULTY_RANDOM, f=5, order_mode=L.ORDER_RANDOM,
                first_trial=64 * (i + 1))


def _check(res, B, **kw):
    od, oo, oc = oracle_c.sliced_run(N, M, B, **kw)
    same(res.decisions, od, "decisions")
    same(res.outcome, oo, "outcome")
    assert {k: res.counters[k] for k in oc} == oc


def test_handoff_timeout_returns_edevice(engine, monkeypatch):
    """A CO launch whose granule polls may wait 1 tick (10 ns): its fan-in blocks
    reach the polls long before the units are done, so the call fails with
    BA_EDEVICE ("hand-off timed out") where it used to return BA_OK with stale
    decisions; a call whose polls happened to find their granules returns the
    oracle's bits; the ctx is sound afterwards."""
    from ba_amd import lib as L
    monkeypatch.setenv("BA_CASC_CO", "1")
    monkeypatch.setenv("BA_TEST_GRANULE_TICKS", "1")
    errs = 0
    for i in range(5):
        kw = _kw(1, i)
        engine.profile(True)
        try:
            res = engine.run(N, M, 1, engine=L.ENGINE_LEVELS, **kw)
        except L.BAError as e:
            assert e.code == L.EDEVICE and "hand-off timed out" in str(e), e
            errs += 1
        else:
            _check(res, 1, **kw)
        assert "k_cascade_co" in engine.profile_read()
        engine.profile(False)
    assert errs >= 1
    monkeypatch.delenv("BA_TEST_GRANULE_TICKS")
    for i in (7, 8):  # the default bound: correct results on the same ctx
        kw = _kw(1, i)
        _check(engine.run(N, M, 1, engine=L.ENGINE_LEVELS, **kw), 1, **kw)


def test_handoff_timeout_device_path_slot14(engine, monkeypatch):
    """ba_run_trials_device is asynchronous: the timed-out call's counters carry
    slot 14, which check_handoff turns into BA_EDEVICE."""
    import torch
    from ba_amd import lib as L
    monkeypatch.setenv("BA_CASC_CO", "1")
    monkeypatch.setenv("BA_TEST_GRANULE_TICKS", "1")
    dev = torch.device("cuda", 0)
    cnt = torch.zeros((5, 16), dtype=torch.int64, device=dev)
    dec = torch.empty(64, dtype=torch.int64, device=dev)
    for i in range(5):
        p = L.make_params(N, M, 0x5107 + i, L.LIE_PHILOX, L.FAULTY_RANDOM, 5, L.ORDER_RANDOM, L.ATTACK,
                          L.ENGINE_LEVELS, 0)
        engine.run_device(p, 64, d_decisions=dec.data_ptr(), d_counters=cnt[i].data_ptr(),
                          stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    c = cnt.cpu().numpy()
    assert (c[:, 0] == 64).all()
    bad = [i for i in range(5) if c[i, L.C_HANDOFF_LOST] != 0]
    assert bad
    with pytest.raises(L.BAError) as ei:
        L.check_handoff(cnt[bad[0]].cpu())
    assert ei.value.code == L.EDEVICE
    for i in set(range(5)) - set(bad):
        L.check_handoff(c[i])


def test_handoff_timeout_multi_rank_job(engine, monkeypatch):
    """ba_run_trials_multi all-reduces slot 14 with the counters, so every rank of
    the job returns BA_EDEVICE (one-rank RCCL communicator here)."""
    from ba_amd import lib as L
    monkeypatch.setenv("BA_CASC_CO", "1")
    monkeypatch.setenv("BA_TEST_GRANULE_TICKS", "1")
    comm = L.Comm(engine, 1, 0, L.comm_unique_id())
    try:
        errs = 0
        for i in range(4):
            p = L.make_params(N, M, 0x3A11 + i, L.LIE_PHILOX, L.FAULTY_RANDOM, 5, L.ORDER_RANDOM, L.ATTACK,
                              L.ENGINE_LEVELS, 0)
            try:
                comm.run_trials(p, 64)
            except L.BAError as e:
                assert e.code == L.EDEVICE and "hand-off timed out" in str(e), e
                errs += 1
        assert errs >= 1
        monkeypatch.delenv("BA_TEST_GRANULE_TICKS")
        cnt, _, _ = comm.run_trials(p, 64)  # the communicator is still usable
        assert cnt["trials"] == 64
    finally:
        comm.close()


def _stall_and_co(engines, B, stall_trials):
    """One CO-eligible n=16, m=5 call of B instances (same inputs) on each engine's
    own stream, all held behind one gate: a long k_om3w call on a separate ctx's
    stream, which every engine's stream waits for (an event), so that no CO call
    can start -- or finish -- while the calls are being queued.  Returns the
    per-engine profiles and the decisions / outcomes / counters."""
    import torch
    from ba_amd import lib as L
    dev = torch.device("cuda", 0)
    k = len(engines)
    sp = L.make_params(10, 3, 1, L.LIE_PHILOX, L.FAULTY_RANDOM, 3, L.ORDER_RANDOM, L.ATTACK, L.ENGINE_AUTO, 0)
    p = L.make_params(N, M, 0xC0AD, L.LIE_PHILOX, L.FAULTY_RANDOM, 5, L.ORDER_RANDOM, L.ATTACK,
                      L.ENGINE_LEVELS, 64 * 3)
    scnt = torch.zeros(16, dtype=torch.int64, device=dev)
    dec = torch.empty((k, B), dtype=torch.int64, device=dev)
    out = torch.empty((k, B), dtype=torch.uint8, device=dev)
    cnt = torch.zeros((k, 16), dtype=torch.int64, device=dev)
    for i, e in enumerate(engines):  # warm-up: geometry, scratch, fan-in counters
        e.run_device(p, B, d_decisions=dec[i].data_ptr(), d_outcome=out[i].data_ptr(),
                     d_counters=cnt[i].data_ptr(), stream=e.stream())
        torch.cuda.synchronize()
    # the admission counts another ctx's last CO launch until a later admission
    # sees that ctx's stream idle (co_admit, conservative: only the slow path
    # queries, and a stream kept busy by other work keeps counting).  One more
    # CO call on a scratch ctx with a one-launch budget takes the slow path,
    # sees every warm-up done, and closing that ctx drops its own launch
    import os
    os.environ["BA_TEST_CO_BUDGET"] = str(4 * 15)
    try:
        ew = L.Engine(0)
        ew.run_device(p, B, d_counters=scnt.data_ptr(), stream=ew.stream())
        torch.cuda.synchronize()
        ew.close()
    finally:
        del os.environ["BA_TEST_CO_BUDGET"]
    cnt.zero_()
    gate = L.Engine(0)  # never launches a CO cascade: counts nothing itself
    gs = torch.cuda.ExternalStream(gate.stream(), device=dev)
    torch.cuda.synchronize()
    try:
        gate.run_device(sp, stall_trials, d_counters=scnt.data_ptr(), stream=gate.stream())
        ev = torch.cuda.Event()
        ev.record(gs)
        for e in engines:
            e.profile(True)
            torch.cuda.ExternalStream(e.stream(), device=dev).wait_event(ev)
        for i, e in enumerate(engines):
            e.run_device(p, B, d_decisions=dec[i].data_ptr(), d_outcome=out[i].data_ptr(),
                         d_counters=cnt[i].data_ptr(), stream=e.stream())
        torch.cuda.synchronize()
    finally:
        gate.close()
    profs = [e.profile_read() for e in engines]
    for e in engines:
        e.profile(False)
    return profs, dec.cpu().numpy().view(np.uint64), out.cpu().numpy(), cnt.cpu().numpy()


def test_co_admission_falls_back_past_the_bound():
    """Concurrent CO launches on one device are bounded by their polling blocks
    (half of 3 blocks per CU): with one 256-instance CO call (4 words x 15
    fan-in blocks) queued behind a long kernel on each of several ctxs/streams,
    the first budget // 60 are CO launches and the rest take the two-launch
    cascade (k_cascade_mtop); every call's bits are the oracle's."""
    import torch
    from ba_amd import lib as L
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    budget = cus * 3 // 2
    B = 256
    admit = budget // (4 * 15)
    engines = [L.Engine(0) for _ in range(admit + 2)]
    try:
        profs, dec, out, cnt = _stall_and_co(engines, B, 64 << 20)
    finally:
        for e in engines:
            e.close()
    co = ["k_cascade_co" in pr for pr in profs]
    mtop = ["k_cascade_mtop" in pr for pr in profs]
    assert co == [True] * admit + [False] * 2, profs
    assert mtop == [False] * admit + [True] * 2, profs
    kw = dict(seed=0xC0AD, faulty_mode=L.FAULTY_RANDOM, f=5, order_mode=L.ORDER_RANDOM, first_trial=64 * 3)
    od, oo, oc = oracle_c.sliced_run(N, M, B, **kw)
    for i in range(len(engines)):
        same(dec[i], od, f"decisions {i}")
        same(out[i], oo, f"outcome {i}")
        assert dict(zip(L.COUNTER_NAMES, cnt[i][:len(L.COUNTER_NAMES)].tolist())) == oc
        assert cnt[i][L.C_HANDOFF_LOST] == 0


def test_co_admission_one_ctx_is_serial(engine):
    """One ctx's calls are ordered, so its CO launches never overlap: ten CO calls
    queued behind a long kernel on one ctx all stay CO launches."""
    import torch
    from ba_amd import lib as L
    dev = torch.device("cuda", 0)
    s = engine.stream()
    sp = L.make_params(10, 3, 1, L.LIE_PHILOX, L.FAULTY_RANDOM, 3, L.ORDER_RANDOM, L.ATTACK, L.ENGINE_AUTO, 0)
    p = L.make_params(N, M, 0xC0AE, L.LIE_PHILOX, L.FAULTY_RANDOM, 5, L.ORDER_RANDOM, L.ATTACK,
                      L.ENGINE_LEVELS, 0)
    scnt = torch.zeros(16, dtype=torch.int64, device=dev)
    cnt = torch.zeros(16, dtype=torch.int64, device=dev)
    engine.run_device(p, 256, d_counters=cnt.data_ptr(), stream=s)
    torch.cuda.synchronize()
    cnt.zero_()
    torch.cuda.synchronize()
    engine.profile(True)
    engine.run_device(sp, 16 << 20, d_counters=scnt.data_ptr(), stream=s)
    for _ in range(10):
        engine.run_device(p, 256, d_counters=cnt.data_ptr(), stream=s)
    torch.cuda.synchronize()
    prof = engine.profile_read()
    engine.profile(False)
    assert prof.get("k_cascade_co", (0, 0))[0] == 10 and "k_cascade_mtop" not in prof, prof
    c = cnt.cpu().numpy()
    assert c[0] == 2560 and c[L.C_HANDOFF_LOST] == 0


def test_forced_co_is_clamped(engine, monkeypatch):
    """BA_CASC_CO=1 at a batch whose fan-in blocks alone exceed the bound takes the
    two-launch cascade (advisor finding: a forced CO launch at any batch would
    put more polling blocks than block slots on the chip)."""
    import torch
    from ba_amd import lib as L
    monkeypatch.setenv("BA_CASC_CO", "1")
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    words = (cus * 3 // 2) // 15 + 1  # > budget polling blocks
    B = 64 * words
    kw = dict(seed=0xF0C0, faulty_mode=L.FAULTY_RANDOM, f=5, order_mode=L.ORDER_RANDOM, first_trial=0)
    engine.profile(True)
    res = engine.run(N, M, B, engine=L.ENGINE_LEVELS, **kw)
    prof = engine.profile_read()
    engine.profile(False)
    assert "k_cascade_co" not in prof and "k_cascade_mtop" in prof, prof
    assert res.counters["trials"] == B
