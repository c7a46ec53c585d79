"""Full-size parity: every configuration the bench and tools/run_configs.py claim,
checked trial by trial against the textbook oracle (oracle/ba_oracle.c, run on
this job's host threads) -- not sampled.

  config 2  n=10, m=3: all 1,048,576 trials of the bench's first step stream
            (seed 0xBA5EED, f ~ U{0..3}, random orders), staged and in-kernel inputs
  config 3  n=13, m=4: 65,536 trials (f ~ U{0..4}) vs the textbook oracle, and
            2,097,152 trials vs the word-sliced C port (itself pinned on the oracle)
  config 4  n=10, m=3 sweep f = 0..4 exactly faulty, the committed curve's 1,048,576
            trials per point (tools/run_configs.py's trial ranges) vs the sliced port
  config 5  n=16, m=5: the full batch of 1024 instances, unsplit and through the
            first-hop split (world 1), plus the word-sliced C port as a second check

Bit-exact on the decision words, the outcome bytes and the run counters."""
import os

import numpy as np
import pytest

import oracle_c

pytestmark = pytest.mark.gpu


def host_threads():
    env = os.environ.get("OMP_NUM_THREADS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


def check(res_dec, res_out, res_cnt, od, oo, ocnt, what):
    bad = np.nonzero(res_dec != od)[0]
    assert bad.size == 0, f"{what}: {bad.size} decision mismatches, first {bad[:5].tolist()}"
    bad = np.nonzero(res_out != oo)[0]
    assert bad.size == 0, f"{what}: {bad.size} outcome mismatches, first {bad[:5].tolist()}"
    assert {k: res_cnt[k] for k in ocnt} == ocnt, what


def test_config2_all_1m_trials_vs_oracle(engine):
    import torch
    from ba_amd import lib as L
    B = 1 << 20
    kw = dict(seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=3, order_mode=L.ORDER_RANDOM)
    od, oo, ocnt = oracle_c.run(10, 3, B, threads=host_threads(), **kw)
    assert ocnt["trials"] == B and ocnt["bound_violations"] == 0
    res = engine.run(10, 3, B, **kw)  # inputs drawn in the kernel
    check(res.decisions, res.outcome, res.counters, od, oo, ocnt, "in-kernel inputs")
    # the bench's staged path: ba_gen_inputs_device, then GIVEN inputs on device buffers
    dev = torch.device("cuda", 0)
    fb = torch.empty(B, dtype=torch.int32, device=dev)
    ob = torch.empty(B, dtype=torch.uint8, device=dev)
    dec = torch.empty(B, dtype=torch.int64, device=dev)
    out = torch.empty(B, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(16, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    engine.gen_inputs_device(L.make_params(10, 3, **kw), B, d_faulty=fb.data_ptr(),
                             d_order=ob.data_ptr(), stream=s)
    p = L.make_params(10, 3, seed=0xBA5EED, faulty_mode=L.FAULTY_GIVEN, f=3,
                      order_mode=L.ORDER_GIVEN)
    engine.run_device(p, B, d_faulty=fb.data_ptr(), d_order=ob.data_ptr(), d_decisions=dec.data_ptr(),
                      d_outcome=out.data_ptr(), d_counters=cnt.data_ptr(), stream=s)
    torch.cuda.synchronize()
    c = dict(zip(L.COUNTER_NAMES, [int(x) for x in cnt.cpu().tolist()]))
    check(dec.cpu().numpy().view(np.uint64), out.cpu().numpy(), c, od, oo, ocnt, "staged inputs")


def test_config3_65536_trials_vs_oracle(engine):
    from ba_amd import lib as L
    B = 1 << 16
    kw = dict(seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=4, order_mode=L.ORDER_RANDOM)
    od, oo, ocnt = oracle_c.run(13, 4, B, threads=host_threads(), **kw)
    res = engine.run(13, 4, B, **kw)
    check(res.decisions, res.outcome, res.counters, od, oo, ocnt, "config 3 (auto engine)")
    sd, so, sc = oracle_c.sliced_run(13, 4, B, threads=host_threads(), **kw)
    check(sd, so, sc, od, oo, ocnt, "C port vs oracle")


def test_config3_2m_trials_vs_sliced_port(engine):
    from ba_amd import lib as L
    B = 1 << 21
    kw = dict(seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=4, order_mode=L.ORDER_RANDOM,
              first_trial=1 << 22)
    sd, so, sc = oracle_c.sliced_run(13, 4, B, threads=host_threads(), **kw)
    assert sc["trials"] == B
    res = engine.run(13, 4, B, **kw)
    check(res.decisions, res.outcome, res.counters, sd, so, sc, "config 3, 2M trials")


def test_config4_curve_1m_per_point_vs_sliced_port(engine):
    """The f-sweep of tools/run_configs.py (exactly f faulty, point f on trials
    [f*T, (f+1)*T)) at its committed size, T = 1,048,576 per point."""
    from ba_amd import lib as L
    T = 1 << 20
    for f in range(0, 5):
        kw = dict(seed=0xBA5EED, faulty_mode=L.FAULTY_EXACT, f=f, order_mode=L.ORDER_RANDOM,
                  first_trial=T * f)
        sd, so, sc = oracle_c.sliced_run(10, 3, T, threads=host_threads(), **kw)
        res = engine.run(10, 3, T, **kw)
        check(res.decisions, res.outcome, res.counters, sd, so, sc, f"config 4, f={f}")
        assert sc["faulty_total"] == f * T
        if f <= 3:
            assert sc["bound_violations"] == 0 and sc["agreement"] == T


def test_config5_full_batch_vs_oracle(engine):
    import torch
    from ba_amd import dist as D
    from ba_amd import lib as L
    B = 1024
    kw = dict(seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=5, order_mode=L.ORDER_RANDOM)
    od, oo, ocnt = oracle_c.run(16, 5, B, threads=host_threads(), **kw)
    sd, so, sc = oracle_c.sliced_run(16, 5, B, threads=host_threads(), **kw)
    check(sd, so, sc, od, oo, ocnt, "C port vs oracle")
    res = engine.run(16, 5, B, engine=L.ENGINE_LEVELS, **kw)
    check(res.decisions, res.outcome, res.counters, od, oo, ocnt, "config 5 unsplit")
    comm = L.Comm(engine, 1, 0, L.comm_unique_id())
    try:
        dec, out, cnt = D.run_instance_split(comm, L.make_params(16, 5, **kw), B,
                                             torch.device("cuda", 0))
    finally:
        comm.close()
    check(dec.cpu().numpy().view(np.uint64), out.cpu().numpy(), cnt, od, oo, ocnt,
          "config 5 first-hop split")


@pytest.mark.parametrize("n", [4, 10])
def test_config1_table_mode_1m_trials_vs_oracle(engine, n):
    """ba.py-exact mode at batch scale (tools/run_configs.py --only 1): 1,048,576
    OM(1) rounds, each its own random.seed(seed_t) and coins in ba.py's draw order
    (ba_mt_table, the C++ MT19937 replay pinned on ba.py's 400 fixture rounds),
    random faulty sets (commander included, beyond the bound too), random
    stale-primary polls (ba.py:171) and orders (attack / retreat / other):
    k_table's decisions, outcome bytes and counters equal the oracle's table mode
    (the recursion of ba.py:159-195 fed the same coins)."""
    from ba_amd import lib as L
    T = 1 << 20
    rng = np.random.default_rng(77 + n)
    seeds = rng.integers(0, 1 << 63, T, dtype=np.uint64)
    faulty = rng.integers(0, 1 << n, T).astype(np.uint32)
    faulty[rng.random(T) < 0.5] &= 0  # half the trials loyal throughout
    poll = (rng.integers(0, 1 << n, T) & ~1).astype(np.uint32)
    order = rng.choice(np.array([0, 1, 2], np.uint8), T, p=[0.45, 0.45, 0.1])
    tab, _ = L.mt_table(n, 1, seeds, faulty, poll, threads=host_threads())
    res = engine.run(n, 1, T, lie_mode=L.LIE_TABLE, faulty=faulty, order=order, table=tab,
                     poll=poll)
    od, oo, ocnt = oracle_c.run(n, 1, T, lie_mode=1, faulty=faulty, order=order, table=tab,
                                poll=poll, threads=host_threads())
    check(res.decisions, res.outcome, res.counters, od, oo, ocnt, f"table mode n={n}")
    assert ocnt["trials"] == T and 0 < ocnt["bound_violations"] < T
