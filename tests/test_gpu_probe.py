"""GPU test of the engine-clock probe (ba_clock_probe_device, include/ba.h): the rows
bench.py turns into `sclk_mhz_timed`."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.gpu
def test_clock_probe_rows_and_clock(engine):
    """Two probes around a few hundred microseconds of work: every row names an XCD
    0-7, s_memtime and s_memrealtime advance between the probes, and the per-XCD
    clock bench.py derives lies in a plausible engine-clock range."""
    import torch

    import bench
    from ba_amd import lib as L
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    probes = torch.zeros((2, L.PROBE_BLOCKS, 4), dtype=torch.int64, device=dev)
    engine.clock_probe_device(probes[0].data_ptr(), stream=s)
    for i in range(20):
        engine.run(10, 3, 1 << 16, seed=i, faulty_mode=L.FAULTY_RANDOM, f=3, order_mode=L.ORDER_RANDOM)
    engine.clock_probe_device(probes[1].data_ptr(), stream=s)
    torch.cuda.synchronize()
    rows = probes.cpu().tolist()
    for p in rows:
        assert all(0 <= r[0] < 8 for r in p), p
        assert all(r[2] > 0 and r[3] > 0 for r in p), p
    assert min(r[3] for r in rows[1]) > max(r[3] for r in rows[0])  # s_memrealtime: one clock
    med, per = bench.clock_from_probes(rows[0], rows[1])
    assert med is not None and 300 <= med <= 3000, (med, per)
    assert per and all(100 <= v <= 3500 for v in per.values()), (per, rows)
