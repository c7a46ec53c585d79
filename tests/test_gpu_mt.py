"""ba.py's coin table on the device (ba_mt_table_device, csrc/ba_mtdev.hip) against
the host replay (ba_mt_table, pinned on ba.py's fixtures and on CPython's own
random module by test_mt.py) -- row for row, next word for next word -- and, for
a few seeds, directly against CPython: random.seed(seed) then ba.py's coins
(random.randint(0, 1) == 0 -> "attack", ba.py:45, 269).  Shapes cover one
limb and two limb seeds, rounds that draw past the first 227 twisted words (the
in-place twist reads its own new words) and past 624 (a second twist)."""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _inputs(n, T, rng):
    seeds = rng.integers(0, 1 << 63, T, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, T, dtype=np.uint64)
    seeds[:8] = np.array([0, 1, 2, (1 << 32) - 1, 1 << 32, (1 << 64) - 1, 0xBA5EED, 1 << 63], np.uint64)
    seeds[8:T // 4] &= np.uint64(0xFFFFFFFF)  # one-limb keys
    faulty = rng.integers(0, 1 << min(n, 31), T, dtype=np.int64).astype(np.uint32)
    faulty[T // 2:] = np.where(rng.random(T - T // 2) < 0.5, 0, faulty[T // 2:])
    poll = (rng.integers(0, 1 << min(n, 31), T, dtype=np.int64) & ~1).astype(np.uint32)
    return seeds, faulty, poll


def _device_table(engine, n, seeds, faulty, poll, stride):
    import torch
    dev = torch.device("cuda", 0)
    T = len(seeds)
    d_s = torch.from_numpy(seeds.view(np.int64)).to(dev)
    d_f = torch.from_numpy(faulty.view(np.int32)).to(dev)
    d_p = torch.from_numpy(poll.view(np.int32)).to(dev)
    tab = torch.full((T, stride), -1, dtype=torch.int32, device=dev)  # every word must be written
    nxt = torch.zeros(T, dtype=torch.int32, device=dev)
    engine.mt_table_device(n, 1, T, d_s.data_ptr(), d_f.data_ptr(), stride, tab.data_ptr(),
                           d_poll=d_p.data_ptr(), d_next_word=nxt.data_ptr(),
                           stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return tab.cpu().numpy().view(np.uint32), nxt.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("n,T", [(4, 65536), (10, 262144), (16, 20000), (32, 3000)])
def test_device_table_equals_host_replay(engine, n, T):
    from ba_amd import lib as L
    rng = np.random.default_rng(n * 31 + 7)
    seeds, faulty, poll = _inputs(n, T, rng)
    stride = L.table_stride(n)
    htab, hnxt = L.mt_table(n, 1, seeds, faulty, poll)
    dtab, dnxt = _device_table(engine, n, seeds, faulty, poll, stride)
    bad = np.nonzero((dtab != htab).any(axis=1))[0]
    assert bad.size == 0, f"{bad.size} rows differ, first {bad[:5].tolist()}"
    assert np.array_equal(dnxt, hnxt)
    if n == 32:  # rounds long enough for a second twist (> 624 words) were in the batch
        counts = [L.om1_coin_count(n, 1, int(f), int(p)) for f, p in zip(faulty, poll)]
        assert max(counts) > 400


def test_device_table_equals_cpython(engine):
    """random.seed(seed); the round's coins are randint(0, 1) == 0 in draw order;
    the next word is getrandbits(32) -- CPython itself, no replay in between."""
    from ba_amd import lib as L
    n = 10
    seeds = np.array([0, 7, 0xBA5EED, (1 << 32) + 5, (1 << 64) - 1], np.uint64)
    faulty = np.array([0b1111111111, 0b0000000111, 0b1000100011, 0b0111111110, 0b1], np.uint32)
    poll = np.array([0b1010101010, 0, 0b0000001110, 0b1111111110, 0b10], np.uint32)
    stride = L.table_stride(n)
    dtab, dnxt = _device_table(engine, n, seeds, faulty, poll, stride)
    for t in range(len(seeds)):
        r = random.Random(int(seeds[t]))
        cnt = L.om1_coin_count(n, 1, int(faulty[t]), int(poll[t]))
        coins = [int(r.randint(0, 1) == 0) for _ in range(cnt)]
        got = [(int(dtab[t, c >> 5]) >> (c & 31)) & 1 for c in range(cnt)]
        assert got == coins, t
        assert int(dnxt[t]) == r.getrandbits(32), t
