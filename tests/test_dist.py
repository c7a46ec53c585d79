"""Multi-GPU layer (ba_amd.dist) on CPU with gloo, world sizes 2 and 3.

The device work is done by a stand-in backend that answers from the C oracle
(test infrastructure), so these tests pin the host logic: word-aligned trial
shards, the counter all-reduce, the first-hop subtree partition, vote padding,
the all-gather and the reassembly order.  The GPU tests at the bottom run the
real libba_hip split entry points."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_c

COUNTERS = 12


class OracleBackend:
    device = torch.device("cpu")

    def counters(self):
        return torch.zeros(16, dtype=torch.int64)

    def run_trials(self, p, batch, counters, decisions=None, outcome=None):
        _, _, c = oracle_c.run(p.n, p.m, batch, seed=p.seed, faulty_mode=p.faulty_mode, f=p.f,
                               order_mode=p.order_mode, order_value=p.order_value,
                               first_trial=p.first_trial)
        counters[:COUNTERS] += torch.tensor(list(c.values()), dtype=torch.int64)

    def _kw(self, p):
        return dict(seed=p.seed, faulty_mode=p.faulty_mode, f=p.f, order_mode=p.order_mode,
                    order_value=p.order_value, first_trial=p.first_trial)

    def subtree_votes(self, p, batch, jb, je):
        v = oracle_c.votes(p.n, p.m, batch, **self._kw(p))
        return torch.from_numpy(oracle_c.pack_votes(v, jb, je).view(np.int64).copy())

    def root_from_votes(self, p, batch, votes):
        want = oracle_c.pack_votes(oracle_c.votes(p.n, p.m, batch, **self._kw(p)))
        assert np.array_equal(votes.numpy().view(np.uint64), want), "gathered votes misassembled"
        dec, out, c = oracle_c.run(p.n, p.m, batch, **self._kw(p))
        cnt = self.counters()
        cnt[:COUNTERS] = torch.tensor(list(c.values()), dtype=torch.int64)
        return torch.from_numpy(dec.view(np.int64)), torch.from_numpy(out), cnt


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
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return [res[r] for r in range(world)]


def test_word_shard_partitions():
    from ba_amd.dist import subtree_ranges, word_shard
    for total in (0, 1, 63, 64, 65, 1000, 64 * 1001 + 3):
        for world in (1, 2, 3, 8):
            parts = [word_shard(total, r, world) for r in range(world)]
            pos = 0
            for first, count in parts:
                assert first % 64 == 0 and (count == 0 or first == pos)
                pos = first + count if count else pos
            assert sum(c for _, c in parts) == total
    assert subtree_ranges(15, 8) == [(0, 1), (1, 3), (3, 5), (5, 7), (7, 9), (9, 11), (11, 13),
                                     (13, 15)]
    assert subtree_ranges(3, 4)[0] == (0, 0)  # more ranks than subtrees: idle ranks


def _dp(rank, world):
    from ba_amd import dist as D
    cnt = D.run_trials_dp(OracleBackend(), 10, 3, 64 * 37 + 11, seed=5, f=3, chunk=64 * 5)
    return cnt[:COUNTERS].tolist()


@pytest.mark.parametrize("world", [2, 3])
def test_trial_dp_counters_allreduced(world):
    got = spawn(_dp, world)
    _, _, want = oracle_c.run(10, 3, 64 * 37 + 11, seed=5, faulty_mode=1, f=3, order_mode=1)
    for r in range(world):
        assert got[r] == list(want.values())


def _split(rank, world):
    from ba_amd import dist as D
    from ba_amd import lib as L
    p = L.make_params(10, 3, seed=9, faulty_mode=L.FAULTY_RANDOM, f=4, order_mode=L.ORDER_RANDOM,
                      first_trial=128)
    dec, out, cnt = D.run_instance_split(OracleBackend(), p, 70)
    return dec.tolist(), out.tolist(), cnt[:COUNTERS].tolist()


@pytest.mark.parametrize("world", [2, 3])
def test_instance_split_gathers_votes(world):
    got = spawn(_split, world)
    dec, out, c = oracle_c.run(10, 3, 70, seed=9, faulty_mode=1, f=4, order_mode=1,
                               first_trial=128)
    for r in range(world):
        assert got[r][0] == dec.view(np.int64).tolist()
        assert got[r][1] == out.tolist()
        assert got[r][2] == list(c.values())


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


@pytest.mark.gpu
@pytest.mark.parametrize("n,m,B,nr", [(10, 3, 200, 4), (7, 1, 100, 4), (9, 2, 130, 4), (16, 5, 2, 4),
                                      # odd n at depth 3: a first-hop subtree holds an odd
                                      # number of level-1 slots, so with 3 ranks a range
                                      # starts mid slot pair (k_relay_top's range edges)
                                      (9, 3, 150, 3), (5, 3, 70, 3), (13, 3, 65, 5)])
def test_subtree_votes_match_oracle_gpu(engine, n, m, B, nr):
    from ba_amd import dist as D
    from ba_amd import lib as L
    dev = torch.device("cuda", 0)
    be = D.DeviceBackend(engine, dev)
    kw = dict(seed=11, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3 + 1, order_mode=L.ORDER_RANDOM,
              first_trial=64 * 3)
    p = L.make_params(n, m, **{k: v for k, v in kw.items()})
    v_or = oracle_c.votes(n, m, B, **kw)
    ranges = D.subtree_ranges(n - 1, nr)
    parts = []
    for jb, je in ranges:
        if je > jb:
            got = be.subtree_votes(p, B, jb, je).cpu().numpy().view(np.uint64)
            assert np.array_equal(got, oracle_c.pack_votes(v_or, jb, je)), (jb, je)
            parts.append(got)
    full = torch.from_numpy(np.concatenate(parts).view(np.int64)).to(dev)
    dec, out, cnt = be.root_from_votes(p, B, full)
    torch.cuda.synchronize()
    od, oo, oc = oracle_c.run(n, m, B, **kw)
    assert np.array_equal(dec.cpu().numpy().view(np.uint64), od)
    assert np.array_equal(out.cpu().numpy(), oo)
    assert cnt.cpu().tolist()[:COUNTERS] == list(oc.values())


@pytest.mark.gpu
def test_split_equals_unsplit_n16_m5_gpu(engine):
    """Config 5: one batch of n=16, m=5 instances through run_instance_split
    (world 1) equals ba_run_trials on the same params."""
    from ba_amd import dist as D
    from ba_amd import lib as L
    dev = torch.device("cuda", 0)
    be = D.DeviceBackend(engine, dev)
    p = L.make_params(16, 5, seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=5,
                      order_mode=L.ORDER_RANDOM)
    B = 300
    dec, out, cnt = D.run_instance_split(be, p, B)
    ref = engine.run(16, 5, B, seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=5,
                     order_mode=L.ORDER_RANDOM, engine=L.ENGINE_LEVELS)
    torch.cuda.synchronize()
    assert np.array_equal(dec.cpu().numpy().view(np.uint64), ref.decisions)
    assert np.array_equal(out.cpu().numpy(), ref.outcome)
    assert cnt.cpu().tolist()[:COUNTERS] == [ref.counters[k] for k in L.COUNTER_NAMES]


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
    """The hipGraph-captured split (InstanceSplitGraphs) replays to the same
    decisions / outcome bytes / counters as eager run_instance_split, on every
    replay (the counters are re-zeroed inside the graph)."""
    from ba_amd import dist as D
    from ba_amd import lib as L
    dev = torch.device("cuda", 0)
    p = L.make_params(n, m, seed=0xBA5EED, faulty_mode=L.FAULTY_RANDOM, f=(n - 1) // 3,
                      order_mode=L.ORDER_RANDOM, first_trial=64 * 5)
    ref_dec, ref_out, ref_cnt = D.run_instance_split(D.DeviceBackend(engine, dev), p, B)
    g = D.InstanceSplitGraphs(engine, dev, p, B)
    for _ in range(3):
        dec, out, cnt = g.replay()
        torch.cuda.synchronize()
        assert torch.equal(dec, ref_dec)
        assert torch.equal(out, ref_out)
        assert torch.equal(cnt, ref_cnt)
