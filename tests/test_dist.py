"""Multi-GPU layer: the C ABI's sharding (ba_trial_share, ba_subtree_share),
the torch.distributed rendezvous of ba_amd.dist, and -- on CPU with gloo,
world sizes 2, 3 and 8 -- the composition of the shards the library's
collectives perform (counter all-reduce, vote all-gather), with the C oracle
doing each rank's device work and gloo standing in for RCCL.  The GPU tests at
the bottom run the real libba_hip entries over a one-rank RCCL communicator
(RCCL refuses two ranks on one GPU; N>1 runs on the driver's 8-GPU node)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_c

COUNTERS = 12


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    finally:
        dist.destroy_process_group()


def spawn(fn, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return [res[r] for r in range(world)]


# --- partition arithmetic of the C ABI (host-only entries, no device) -------------
def test_trial_share_partitions():
    from ba_amd import lib as L
    for total in (0, 1, 63, 64, 65, 1000, 64 * 1001 + 3, 64 << 20):
        for world in (1, 2, 3, 8):
            parts = [L.trial_share(total, world, r) for r in range(world)]
            pos = 0
            for first, count in parts:
                assert first % 64 == 0 and (count == 0 or first == pos)
                pos = first + count if count else pos
            assert sum(c for _, c in parts) == total
            words = [(c + 63) // 64 for _, c in parts]
            assert max(words) - min(words) <= 1  # balanced to one word


def test_subtree_share_partitions():
    from ba_amd import dist as D
    from ba_amd import lib as L
    for n in (3, 4, 10, 13, 16, 32):
        for world in (1, 2, 3, 8, 40):
            ranges = [L.subtree_share(n, world, r) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n - 1
            for (a, b), (c, d) in zip(ranges, ranges[1:]):
                assert b == c and a <= b  # contiguous, in rank order
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1
    assert D.subtree_ranges(15, 8) == [(0, 1), (1, 3), (3, 5), (5, 7), (7, 9), (9, 11), (11, 13),
                                       (13, 15)]
    assert L.subtree_share(4, 4, 0) == (0, 0)  # more ranks than subtrees: idle ranks
    with pytest.raises(L.BAError):
        L.subtree_share(2, 1, 0)


def test_split_share_levels():
    """ba_split_share: level 1 is ba_subtree_share; level 2 splits the (n-1)(n-2)
    second-hop subtrees evenly (n=16 over 8 ranks: 26/27 of 210, against 1-2 of 15
    first hops); the second-hop split needs m_eff >= 3."""
    from ba_amd import dist as D
    from ba_amd import lib as L
    for n in (4, 10, 13, 16):
        for world in (1, 2, 3, 8):
            assert D.split_ranges(n, 3, 1, world) == [L.subtree_share(n, world, r)
                                                     for r in range(world)]
    assert L.split_units(16, 5, 2) == 210 and L.split_units(16, 5, 1) == 15
    r8 = D.split_ranges(16, 5, 2, 8)
    assert r8[0][0] == 0 and r8[-1][1] == 210
    assert all(b == c for (_, b), (c, _) in zip(r8, r8[1:]))
    assert sorted({b - a for a, b in r8}) == [26, 27]
    assert L.split_vote_slots(16, 5, 2, 0, 210) == 210 * 13  # R_2: n-3 per unit
    assert L.split_vote_slots(16, 5, 1, 0, 15) == 15 * 14 == L.vote_slots(16, 5, 0, 15)
    assert L.split_units(10, 2, 2) == 0 and L.split_units(10, 3, 2) == 72
    assert L.split_units(10, 2, 3) == 0
    with pytest.raises(L.BAError):
        L.split_share(10, 2, 2, 2, 0)


def test_oracle_votes2_reproduce_votes():
    """Pins ba_oracle_votes2 on ba_oracle_votes: R_1[j.r] is the inner majority of
    L_1[j.r] and the level-2 results R_2[j.a.r] of every other second hop a."""
    import ctypes
    n, m, B = 8, 4, 40
    kw = dict(seed=7, faulty_mode=1, f=3, order_mode=1)
    v1 = oracle_c.votes(n, m, B, **kw)
    v2 = oracle_c.votes2(n, m, B, **kw)
    lib = oracle_c.load()
    L_ = n - 1
    for t in range(B):
        fm, oc = ctypes.c_uint32(), ctypes.c_uint8()
        lib.ba_oracle_gen(n, 7, 1, 3, 1, 1, t, ctypes.byref(fm), ctypes.byref(oc))
        for j in range(L_):
            l0 = lib.ba_oracle_lie(7, t, 0, j) if fm.value & 1 else int(oc.value == 1)
            for k in range(L_ - 1):
                r = k + (k >= j)
                # L_1[j.r]: lieutenant j relays L_0[j] (slot j*(L-1) + k at level 1)
                l1 = lib.ba_oracle_lie(7, t, 1, j * (L_ - 1) + k) if (fm.value >> (j + 1)) & 1 else l0
                a_cnt, c_cnt = l1, 1
                for ka in range(L_ - 1):
                    a = ka + (ka >= j)
                    if a == r:
                        continue
                    others = [x for x in range(L_) if x not in (j, a)]
                    a_cnt += int(v2[t, j * (L_ - 1) + ka, others.index(r)])
                    c_cnt += 1
                assert int(v1[t, j, k]) == int(2 * a_cnt > c_cnt), (t, j, r)


# --- gloo rehearsals of the collectives' composition ------------------------------
def _rendezvous(rank, world):
    from ba_amd import dist as D
    return D.rendezvous_uid()


@pytest.mark.parametrize("world", [2, 3])
def test_rendezvous_delivers_rank0_uid(world):
    """ba_amd.dist.rendezvous_uid: RCCL's unique id (ncclGetUniqueId works without a
    GPU) made on rank 0 reaches every rank byte for byte."""
    got = spawn(_rendezvous, world)
    assert all(len(u) == 128 and u == got[0] for u in got)


def _dp(rank, world):
    """Each rank resolves its ba_trial_share with the oracle; gloo sums the
    counters as ba_comm_allreduce_device does."""
    from ba_amd import lib as L
    total = 64 * 37 + 11
    first, count = L.trial_share(total, world, rank)
    cnt = torch.zeros(16, dtype=torch.int64)
    if count:
        _, _, c = oracle_c.run(10, 3, count, seed=5, faulty_mode=1, f=3, order_mode=1,
                               first_trial=first)
        cnt[:COUNTERS] = torch.tensor(list(c.values()), dtype=torch.int64)
    dist.all_reduce(cnt)
    return cnt[:COUNTERS].tolist()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_trial_dp_counters_allreduced(world):
    got = spawn(_dp, world)
    _, _, want = oracle_c.run(10, 3, 64 * 37 + 11, seed=5, faulty_mode=1, f=3, order_mode=1)
    for r in range(world):
        assert got[r] == list(want.values())


def _split(rank, world):
    """Each rank computes the vote rows of its ba_subtree_share (oracle votes in the
    library's layout), the rows are exchanged (gloo all-gather in place of the
    grouped broadcast), and the assembled array must equal the whole instance's."""
    from ba_amd import lib as L
    n, m, B = 10, 3, 70
    kw = dict(seed=9, faulty_mode=1, f=4, order_mode=1, first_trial=128)
    jb, je = L.subtree_share(n, world, rank)
    v = oracle_c.votes(n, m, B, **kw)
    mine = oracle_c.pack_votes(v, jb, je) if je > jb else np.zeros((0, (B + 63) // 64), np.uint64)
    parts = [None] * world
    dist.all_gather_object(parts, (jb, je, mine.tobytes()))
    W = (B + 63) // 64
    full = np.zeros(((n - 1) * (n - 2), W), np.uint64)
    for a, b, raw in parts:
        if b > a:
            full[a * (n - 2):b * (n - 2)] = np.frombuffer(raw, np.uint64).reshape(-1, W)
    return full.tobytes()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_instance_split_assembles_votes(world):
    got = spawn(_split, world)
    v = oracle_c.votes(10, 3, 70, seed=9, faulty_mode=1, f=4, order_mode=1, first_trial=128)
    want = oracle_c.pack_votes(v).tobytes()
    assert all(g == want for g in got)


def _split2(rank, world):
    """The second-hop split's exchange: every rank's ba_split_share rows of the
    level-2 votes, assembled by gloo in place of the grouped broadcast."""
    from ba_amd import lib as L
    n, m, B = 9, 4, 70
    kw = dict(seed=9, faulty_mode=1, f=3, order_mode=1, first_trial=128)
    ub, ue = L.split_share(n, m, 2, world, rank)
    v = oracle_c.votes2(n, m, B, **kw)
    W = (B + 63) // 64
    mine = oracle_c.pack_votes(v, ub, ue) if ue > ub else np.zeros((0, W), np.uint64)
    parts = [None] * world
    dist.all_gather_object(parts, (ub, ue, mine.tobytes()))
    full = np.zeros((L.split_vote_slots(n, m, 2, 0, L.split_units(n, m, 2)), W), np.uint64)
    for a, b, raw in parts:
        if b > a:
            full[a * (n - 3):b * (n - 3)] = np.frombuffer(raw, np.uint64).reshape(-1, W)
    return full.tobytes()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_second_hop_split_assembles_votes(world):
    got = spawn(_split2, world)
    v = oracle_c.votes2(9, 4, 70, seed=9, faulty_mode=1, f=3, order_mode=1, first_trial=128)
    want = oracle_c.pack_votes(v).tobytes()
    assert all(g == want for g in got)


def test_oracle_votes_reproduce_root_decisions():
    """Pins ba_oracle_votes on ba_oracle_run: the root majority of L_0[r] and the
    votes about every other first hop j is the lieutenant's decision."""
    n, m, B = 9, 3, 100
    kw = dict(seed=3, faulty_mode=1, f=3, order_mode=1)
    v = oracle_c.votes(n, m, B, **kw)
    dec, _, _ = oracle_c.run(n, m, B, **kw)
    lib = oracle_c.load()
    import ctypes
    for t in range(B):
        fm, oc = ctypes.c_uint32(), ctypes.c_uint8()
        lib.ba_oracle_gen(n, 3, 1, 3, 1, 1, t, ctypes.byref(fm), ctypes.byref(oc))
        for r in range(n - 1):
            l0 = lib.ba_oracle_lie(3, t, 0, r) if fm.value & 1 else int(oc.value == 1)
            a = l0 + sum(int(v[t, j, r - (r > j)]) for j in range(n - 1) if j != r)
            code = 1 if 2 * a > n - 1 else (0 if 2 * a < n - 1 else 2)
            assert (int(dec[t]) >> (2 * r)) & 3 == code


# --- GPU: the real entries ---------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("nocasc", ["0", "1"])
@pytest.mark.parametrize("n,m,B,nr", [(10, 3, 200, 4), (7, 1, 100, 4), (9, 2, 130, 4), (16, 5, 2, 4),
                                      # odd n at depth 3: a first-hop subtree holds an odd
                                      # number of level-1 slots, so with 3 ranks a range
                                      # starts mid slot pair (k_relay_top's range edges)
                                      (9, 3, 150, 3), (5, 3, 70, 3), (13, 3, 65, 5),
                                      (16, 5, 70, 8), (9, 4, 200, 3), (16, 4, 66, 6)])
def test_subtree_votes_match_oracle_gpu(engine, monkeypatch, n, m, B, nr, nocasc):
    """Every rank's ba_subtree_votes_device rows (ranges from ba_subtree_share) equal
    the oracle's, and the root pass over the assembled rows equals the oracle's run
    (the cascade's range and root modes on its shapes; BA_NO_CASCADE=1: the
    multi-launch LEVELS kernels)."""
    from ba_amd import lib as L
    monkeypatch.setenv("BA_NO_CASCADE", nocasc)
    dev = torch.device("cuda", 0)
    kw = dict(seed=11, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3 + 1, order_mode=L.ORDER_RANDOM,
              first_trial=64 * 3)
    p = L.make_params(n, m, **kw)
    W = (B + 63) // 64
    v_or = oracle_c.votes(n, m, B, **kw)
    full = torch.zeros(((n - 1) * (n - 2), W), dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    for r in range(nr):
        jb, je = L.subtree_share(n, nr, r)
        if je > jb:
            engine.subtree_votes_device(p, B, jb, je, full[jb * (n - 2):].data_ptr(), stream=s)
            got = full[jb * (n - 2):je * (n - 2)].cpu().numpy().view(np.uint64)
            assert np.array_equal(got, oracle_c.pack_votes(v_or, jb, je)), (jb, je)
    dec = torch.empty(B, dtype=torch.int64, device=dev)
    out = torch.empty(B, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(16, dtype=torch.int64, device=dev)
    engine.root_from_votes_device(p, B, full.data_ptr(), cnt.data_ptr(), d_decisions=dec.data_ptr(),
                                  d_outcome=out.data_ptr(), stream=s)
    torch.cuda.synchronize()
    od, oo, oc = oracle_c.run(n, m, B, **kw)
    assert np.array_equal(dec.cpu().numpy().view(np.uint64), od)
    assert np.array_equal(out.cpu().numpy(), oo)
    assert cnt.cpu().tolist()[:COUNTERS] == list(oc.values())


@pytest.mark.gpu
@pytest.mark.parametrize("nocasc", ["0", "1", "wave"])
@pytest.mark.parametrize("n,m,B,nr", [(10, 3, 200, 4), (9, 4, 130, 3), (13, 4, 65, 5),
                                      (7, 3, 100, 3), (16, 5, 2, 8), (16, 5, 70, 8), (8, 5, 300, 5)])
def test_second_hop_votes_match_oracle_gpu(engine, monkeypatch, n, m, B, nr, nocasc):
    """Second-hop split (ba_split_votes_device, level 2): every rank's R_2 rows
    (ranges from ba_split_share, starting mid first-hop subtree) equal the
    oracle's, and the root pass over the assembled rows equals the oracle's run --
    through the cascade (range-mode votes, k_cascade_root) where the shape has it,
    and through the multi-launch LEVELS kernels (BA_NO_CASCADE=1)."""
    from ba_amd import lib as L
    monkeypatch.setenv("BA_NO_CASCADE", "1" if nocasc == "1" else "0")
    monkeypatch.setenv("BA_CASC_WTOP", "0" if nocasc == "wave" else "1")  # root pass by waves / blocks
    dev = torch.device("cuda", 0)
    kw = dict(seed=13, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3 + 1, order_mode=L.ORDER_RANDOM,
              first_trial=64 * 5)
    p = L.make_params(n, m, **kw)
    W = (B + 63) // 64
    v_or = oracle_c.votes2(n, m, B, **kw)
    units = L.split_units(n, m, 2)
    full = torch.zeros((L.split_vote_slots(n, m, 2, 0, units), W), dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    per = n - 3
    for r in range(nr):
        ub, ue = L.split_share(n, m, 2, nr, r)
        if ue > ub:
            engine.split_votes_device(p, B, 2, ub, ue, full[ub * per:].data_ptr(), stream=s)
            got = full[ub * per:ue * per].cpu().numpy().view(np.uint64)
            assert np.array_equal(got, oracle_c.pack_votes(v_or, ub, ue)), (ub, ue)
    dec = torch.empty(B, dtype=torch.int64, device=dev)
    out = torch.empty(B, dtype=torch.uint8, device=dev)
    cnt = torch.zeros(16, dtype=torch.int64, device=dev)
    engine.root_from_split_votes_device(p, B, 2, full.data_ptr(), cnt.data_ptr(),
                                        d_decisions=dec.data_ptr(), d_outcome=out.data_ptr(),
                                        stream=s)
    torch.cuda.synchronize()
    od, oo, oc = oracle_c.run(n, m, B, **kw)
    assert np.array_equal(dec.cpu().numpy().view(np.uint64), od)
    assert np.array_equal(out.cpu().numpy(), oo)
    assert cnt.cpu().tolist()[:COUNTERS] == list(oc.values())
    with pytest.raises(L.BAError) as ei:  # m_eff < 3: no second-hop split
        engine.split_votes_device(L.make_params(10, 2, **kw), B, 2, 0, 1, full.data_ptr())
    assert ei.value.code == L.ENOTSUP


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,level,units", [(16, 5, 1, (0, 7, 14)), (16, 5, 2, (0, 1, 13, 100, 209)),
                                             (8, 5, 1, (0, 6)), (8, 5, 2, (0, 5, 41)),
                                             (16, 4, 1, (0, 9))])
def test_split_votes_single_units_through_cascade(engine, monkeypatch, n, m, level, units):
    """The subtree split through k_cascade's range mode (ba_split_votes_device on a
    cascade shape with h <= m_eff - 3): ranges of ONE h-hop subtree (the fewest
    units per word, so a block's units span several words), two-subtree ranges, at
    batch 1 and 130; rows equal the oracle's, equal the multi-launch pipeline's
    (BA_NO_CASCADE=1), and the profile shows k_cascade ran: in one launch
    (BA_CASC_TWO=0), and in two -- the units, then k_cascade_mtop ending at the vote
    level -- with the units in the normal and in the latency mode (BA_CASC_LAT)."""
    from ba_amd import lib as L
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    per = n - 1 - level
    modes = {"one": ("0", "0", "0"), "two": ("0", "1", "0"), "two_lat": ("0", "1", "1"), "multi": ("1", "0", "0")}
    lat_shape = (n, m) in ((16, 5), (9, 4), (8, 5))
    for B in (1, 130):
        kw = dict(seed=17 + B, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3 + 1,
                  order_mode=L.ORDER_RANDOM, first_trial=64 * 9)
        p = L.make_params(n, m, **kw)
        W = (B + 63) // 64
        v_or = (oracle_c.votes if level == 1 else oracle_c.votes2)(n, m, B, **kw)
        for ub in units:
            for ue in (ub + 1, min(ub + 2, L.split_units(n, m, level))):
                got = {}
                for mode, (nocasc, two, lat) in modes.items():
                    monkeypatch.setenv("BA_NO_CASCADE", nocasc)
                    monkeypatch.setenv("BA_CASC_TWO", two)
                    monkeypatch.setenv("BA_CASC_LAT", lat)
                    v = torch.zeros(((ue - ub) * per, W), dtype=torch.int64, device=dev)
                    engine.profile(True)
                    engine.split_votes_device(p, B, level, ub, ue, v.data_ptr(), stream=s)
                    torch.cuda.synchronize()
                    prof = engine.profile_read()
                    engine.profile(False)
                    assert any("k_cascade" in k for k in prof) == (mode != "multi"), prof
                    assert ("k_cascade_mtop" in prof) == mode.startswith("two"), (mode, prof)
                    assert ("k_cascade_units_lat" in prof) == (mode == "two_lat" and lat_shape), (mode, prof)
                    got[mode] = v.cpu().numpy().view(np.uint64)
                assert np.array_equal(got["one"], oracle_c.pack_votes(v_or, ub, ue)), (B, ub, ue)
                for mode in modes:
                    assert np.array_equal(got[mode], got["one"]), (mode, B, ub, ue)
    for k in ("BA_NO_CASCADE", "BA_CASC_TWO", "BA_CASC_LAT"):
        monkeypatch.delenv(k)


@pytest.mark.gpu
def test_split_multi_world1_equals_unsplit_n16_m5(engine):
    """Config 5 through ba_run_instance_split_multi on a one-rank RCCL communicator
    equals ba_run_trials on the same params, and equals the C port on the full
    1024-instance batch.  At one rank the entry takes the unsplit pass (no vote
    array, no broadcast); test_forced_split_world1_* below runs the exchange."""
    from ba_amd import dist as D
    from ba_amd import lib as L
    dev = torch.device("cuda", 0)
    comm = L.Comm(engine, 1, 0, L.comm_unique_id())
    try:
        p = L.make_params(16, 5, seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=5,
                          order_mode=L.ORDER_RANDOM)
        B = 1024
        dec, out, cnt = D.run_instance_split(comm, p, B, dev)
        ref = engine.run(16, 5, B, seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=5,
                         order_mode=L.ORDER_RANDOM, engine=L.ENGINE_LEVELS)
        assert np.array_equal(dec.cpu().numpy().view(np.uint64), ref.decisions)
        assert np.array_equal(out.cpu().numpy(), ref.outcome)
        assert cnt == ref.counters
        od, oo, oc = oracle_c.sliced_run(16, 5, B, seed=0xBA5EED, faulty_mode=1, f=5,
                                         order_mode=1)
        assert np.array_equal(ref.decisions, od) and np.array_equal(ref.outcome, oo)
        assert {k: cnt[k] for k in oc} == oc
    finally:
        comm.close()


@pytest.fixture
def force_split(monkeypatch):
    """BA_FORCE_SPLIT=1 (test-only, read by libba_hip on every call): the split
    entry takes the vote-array path at one rank -- the vote buffer, the
    pre-exchange error agreement, the grouped ncclBroadcast all-gather and the
    error all-reduce of finish_job all run on the real one-rank communicator."""
    monkeypatch.setenv("BA_FORCE_SPLIT", "1")
    yield


@pytest.mark.gpu
@pytest.mark.parametrize("B", [1, 70])
@pytest.mark.parametrize("level", [1, 2])
def test_forced_split_world1_matches_oracle(engine, force_split, level, B):
    """Config 5 (n=16, m=5), batch 1 and 70, through ba_run_instance_split_level_multi
    with the split forced at world 1 (the votes through k_cascade's range mode): decisions, outcome bytes and counters equal the
    oracle (every rank's rows are its own, so the broadcast's layout -- rows
    [ub*row, ue*row) of rank 0 -- must be the one the root pass reads)."""
    from ba_amd import dist as D
    from ba_amd import lib as L
    dev = torch.device("cuda", 0)
    kw = dict(seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=5, order_mode=L.ORDER_RANDOM,
              first_trial=64 * 7)
    p = L.make_params(16, 5, **kw)
    comm = L.Comm(engine, 1, 0, L.comm_unique_id())
    try:
        for _ in range(2):  # the second call reuses the grown vote buffer
            dec, out, cnt = D.run_instance_split(comm, p, B, dev, level=level)
            od, oo, oc = oracle_c.run(16, 5, B, **kw)
            assert np.array_equal(dec.cpu().numpy().view(np.uint64), od)
            assert np.array_equal(out.cpu().numpy(), oo)
            assert {k: cnt[k] for k in oc} == oc
    finally:
        comm.close()


@pytest.mark.gpu
def test_forced_split_world1_failure_before_exchange(engine, force_split, monkeypatch):
    """A rank that cannot allocate its vote buffer (BA_TEST_VOTE_ENOMEM=1 injects
    it) returns ENOMEM after the pre-exchange agreement instead of skipping the
    broadcast its peers wait in; an invalid split level fails the same way; the
    communicator stays usable and the next call is exact."""
    from ba_amd import dist as D
    from ba_amd import lib as L
    dev = torch.device("cuda", 0)
    kw = dict(seed=3, faulty_mode=L.FAULTY_RANDOM, f=3, order_mode=L.ORDER_RANDOM)
    p = L.make_params(10, 3, **kw)
    comm = L.Comm(engine, 1, 0, L.comm_unique_id())
    try:
        monkeypatch.setenv("BA_TEST_VOTE_ENOMEM", "1")
        with pytest.raises(L.BAError) as ei:
            D.run_instance_split(comm, p, 100, dev, level=2)
        assert ei.value.code == L.ENOMEM
        monkeypatch.delenv("BA_TEST_VOTE_ENOMEM")
        with pytest.raises(L.BAError) as ei:
            D.run_instance_split(comm, p, 100, dev, level=3)
        assert ei.value.code == L.EINVAL
        dec, out, cnt = D.run_instance_split(comm, p, 100, dev, level=2)
        od, oo, oc = oracle_c.run(10, 3, 100, **kw)
        assert np.array_equal(dec.cpu().numpy().view(np.uint64), od)
        assert {k: cnt[k] for k in oc} == oc
    finally:
        comm.close()


@pytest.mark.gpu
def test_comm_allreduce_and_split_errors(engine):
    """ba_comm_allreduce_device over one rank is the identity; a bad split request
    fails on the rank (after joining the error all-reduce) instead of hanging."""
    from ba_amd import lib as L
    comm = L.Comm(engine, 1, 0, L.comm_unique_id())
    try:
        x = torch.arange(16, dtype=torch.int64, device="cuda")
        comm.allreduce_device(x.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert x.cpu().tolist() == list(range(16))
        p0 = L.make_params(10, 0, seed=1, faulty_mode=L.FAULTY_RANDOM, f=3,
                           order_mode=L.ORDER_RANDOM)
        with pytest.raises(L.BAError) as ei:
            comm.run_instance_split(p0, 64)
        assert ei.value.code == L.ENOTSUP
        # the communicator stays usable after a failed call
        p = L.make_params(10, 3, seed=1, faulty_mode=L.FAULTY_RANDOM, f=3, order_mode=L.ORDER_RANDOM)
        c = comm.run_instance_split(p, 100)
        assert c["trials"] == 100
    finally:
        comm.close()


@pytest.mark.gpu
def test_split_api_errors(engine):
    from ba_amd import lib as L
    p = L.make_params(10, 3, seed=1, faulty_mode=L.FAULTY_RANDOM, f=3, order_mode=L.ORDER_RANDOM)
    v = torch.empty((100, 1), dtype=torch.int64, device="cuda")
    with pytest.raises(L.BAError) as ei:
        engine.subtree_votes_device(p, 64, 3, 3, v.data_ptr())
    assert ei.value.code == L.EINVAL
    with pytest.raises(L.BAError) as ei:
        engine.subtree_votes_device(p, 64, 0, 10, v.data_ptr())
    assert ei.value.code == L.EINVAL
    p0 = L.make_params(10, 0, seed=1, faulty_mode=L.FAULTY_RANDOM, f=3, order_mode=L.ORDER_RANDOM)
    with pytest.raises(L.BAError) as ei:
        engine.subtree_votes_device(p0, 64, 0, 2, v.data_ptr())
    assert ei.value.code == L.ENOTSUP


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,B", [(16, 5, 300), (10, 3, 1000), (9, 3, 150)])
def test_instance_split_graphs_equal_eager(engine, n, m, B):
    """The hipGraph-captured split (InstanceSplitGraphs, its own ctx) replays to the
    same decisions / outcome bytes / counters as the eager C-ABI split, on every
    replay (the counters are re-zeroed inside the graph)."""
    from ba_amd import dist as D
    from ba_amd import lib as L
    dev = torch.device("cuda", 0)
    p = L.make_params(n, m, seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3,
                      order_mode=L.ORDER_RANDOM, first_trial=64 * 5)
    comm = L.Comm(engine, 1, 0, L.comm_unique_id())
    try:
        ref_dec, ref_out, ref_cnt = D.run_instance_split(comm, p, B, dev)
    finally:
        comm.close()
    g = D.InstanceSplitGraphs(dev, p, B)
    try:
        for _ in range(3):
            dec, out, cnt = g.replay()
            torch.cuda.synchronize()
            assert torch.equal(dec, ref_dec)
            assert torch.equal(out, ref_out)
            assert cnt.cpu().tolist()[:COUNTERS] == [ref_cnt[k] for k in L.COUNTER_NAMES]
    finally:
        g.close()


@pytest.mark.gpu
def test_ctx_orders_calls_across_streams(engine):
    """Calls of one ctx issued back to back on two different streams (no host sync)
    share its scratch and counter sink safely: the library orders the second call
    after the first (include/ba.h).  Both results equal the oracle."""
    from ba_amd import lib as L
    dev = torch.device("cuda", 0)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    B = 1 << 16
    jobs = []
    for seed, s in ((3, s1), (4, s2), (5, s1)):
        p = L.make_params(16, 5, seed, L.LIE_PHILOX, L.FAULTY_RANDOM, 5, L.ORDER_RANDOM,
                          L.ATTACK, L.ENGINE_LEVELS, 0) if seed == 4 else \
            L.make_params(10, 3, seed, L.LIE_PHILOX, L.FAULTY_RANDOM, 3, L.ORDER_RANDOM)
        b = 64 if seed == 4 else B
        dec = torch.empty(b, dtype=torch.int64, device=dev)
        cnt = torch.zeros(16, dtype=torch.int64, device=dev)
        jobs.append((p, b, s, dec, cnt))
    torch.cuda.synchronize()
    outs = []
    for p, b, s, dec, cnt in jobs:  # back to back, no host sync in between
        engine.run_device(p, b, d_decisions=dec.data_ptr(), d_counters=cnt.data_ptr(),
                          stream=s.cuda_stream)
        outs.append((p.n, p.m, p.seed, b, dec, cnt))
    torch.cuda.synchronize()
    for n, m, seed, b, dec, cnt in outs:
        od, _, oc = oracle_c.sliced_run(n, m, b, seed=seed, faulty_mode=1, f=(5 if n == 16 else 3),
                                        order_mode=1)
        assert np.array_equal(dec.cpu().numpy().view(np.uint64), od), seed
        assert cnt.cpu().tolist()[:COUNTERS] == list(oc.values()), seed
