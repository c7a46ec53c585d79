"""bench.py's host-side accounting (no GPU): the roofline byte and Philox-call
models, the committed PMC lookup, and the CPU-baseline thread count.  The GPU
numbers themselves come from the box (profiles/)."""
from __future__ import annotations

import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

bench = pytest.importorskip("bench")


def test_philox_call_floor_n10_m3():
    # ceil(|L_k| / 2) per level: 9, 72, 504, 3024 slots -> 5 + 36 + 252 + 1512
    assert bench.philox_calls_per_trial_word(10, 3) == 1805


def test_level_synchronous_bytes_n10_m3():
    # 8 B of per-trial I/O + 2 x ceil(3609 tree bits / 8)
    assert bench.level_synchronous_bytes_per_trial(10, 3) == 8 + 2 * 452


def test_kernel_io_bytes_wave_engine():
    B = 1 << 20
    assert bench.kernel_io_bytes("k_om3w", 10, 3, B, staged=True) == 14 * B
    assert bench.kernel_io_bytes("k_om3w", 10, 3, B, staged=False) == 9 * B


def test_pmc_lookup_finds_committed_wave_counters():
    e, path, same = bench.pmc_for(10, 3, 1 << 20, "auto", "k_om3w", "no-such-digest")
    assert e is not None and path.startswith("profiles/")
    assert not same  # a digest no build has
    assert e["traffic_bytes"] > 0 and e["counters"]["SQ_INSTS_VALU"] > 0
    # the newest summary wins; the same digest makes it a same-build match
    d = json.load(open(os.path.join(ROOT, path)))
    e2, path2, same2 = bench.pmc_for(10, 3, 1 << 20, "auto", "k_om3w", d["lib_sha16"])
    assert same2 and path2 == path


def test_philox_peaks_cover_kernel_occupancy():
    peaks = bench.philox_peaks()
    assert 2 in peaks and 8 in peaks and peaks[8] >= peaks[2] > 0


def test_cpu_threads_follows_omp(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    assert bench.cpu_threads() == 3
    monkeypatch.delenv("OMP_NUM_THREADS")
    assert bench.cpu_threads() >= 1


def test_kernel_io_bytes_levels():
    W = (1 << 20) // 64
    assert bench.kernel_io_bytes("k_leaf_up", 10, 3, 1 << 20, staged=True) == 8 * W * 2 * 72
    assert bench.kernel_io_bytes("k_relay_top", 10, 3, 1 << 20, staged=True) == 8 * W * (9 + 72)
    assert bench.kernel_io_bytes("k_epilogue", 10, 3, 1 << 20, staged=True) == \
        8 * W * (9 + 72 + 13) + 9 * (1 << 20)


def test_world_check_and_launch_command(monkeypatch):
    """--gpus N: under a launcher the WORLD_SIZE must equal N (else exit code 2);
    without one, N == 1 runs in-process and N > 1 starts torch.distributed.run on
    N local ranks (127.0.0.1 rendezvous) as a child and returns its exit code."""
    assert bench.check_or_launch_world(1, [], {}) is None
    assert bench.check_or_launch_world(4, [], {"WORLD_SIZE": "4"}) is None
    assert bench.check_or_launch_world(2, [], {"WORLD_SIZE": "3"}) == 2
    assert bench.check_or_launch_world(1, [], {"WORLD_SIZE": "8"}) == 2
    assert bench.check_or_launch_world(0, [], {}) == 2
    cmd = bench.launch_cmd(8, ["--gpus", "8", "--steps", "5"], 29500)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd
    assert "--master-port=29500" in cmd and cmd[-4:] == ["--gpus", "8", "--steps", "5"]
    assert cmd[-5].endswith("bench.py")
    seen = {}

    def fake_call(c, env):
        seen["cmd"], seen["env"] = c, env
        return 7
    import subprocess
    monkeypatch.setattr(subprocess, "call", fake_call)
    assert bench.check_or_launch_world(2, ["--gpus", "2"], {"PATH": "/bin"}) == 7
    assert "--nproc-per-node=2" in seen["cmd"] and seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_bench_exits_nonzero_on_world_mismatch():
    """The script itself, before importing torch or touching a GPU."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=3" in r.stderr


def test_cpu_baseline_checks_counters_against_gpu():
    """The CPU leg runs the GPU's timed trial range first and compares all 12
    counters; a mismatch is a hard failure (SystemExit)."""
    import oracle_c
    n, m, first, count = 10, 3, 64 * 1000, 64 * 50
    _, _, want = oracle_c.run(n, m, count, seed=5, faulty_mode=1, f=3, order_mode=1,
                              first_trial=first)
    cpu = bench.run_cpu_baseline(n, m, 5, 3, 0.0, [(first, count)], dict(want), 64 * 5000)
    assert cpu["counters_match"] is True and cpu["counters_checked"]["trials"] == count
    assert cpu["value"] > 0 and cpu["kind"] == "port"
    bad = dict(want, agreement=want["agreement"] + 1)
    with pytest.raises(SystemExit):
        bench.run_cpu_baseline(n, m, 5, 3, 0.0, [(first, count)], bad, 64 * 5000)


def test_rank_ranges_shard_the_timed_trials():
    """Every rank's timed ranges are disjoint, B trials per step, and together
    cover exactly the job's timed slots."""
    B, base, K = 128, 5, 4
    assert bench.rank_ranges(base, K, 0, 1, B) == [(base * B, K * B)]
    for world in (2, 3, 8):
        seen = set()
        for r in range(world):
            rr = bench.rank_ranges(base, K, r, world, B)
            assert len(rr) == K and all(c == B for _, c in rr)
            for f0, c in rr:
                seen.update(range(f0, f0 + c))
        assert seen == set(range(base * world * B, (base + K) * world * B))


def _cpu_baseline_rank(rank, world, port, q):
    """One gloo rank of the N>1 bench flow with the C oracle as the GPU stand-in:
    its local counters over rank_ranges, the all-reduce, then rank 0's CPU leg
    checked against its PRE-all-reduce counters (the job's totals must fail it)."""
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_c
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        import torch
        n, m, B, base, K, seed, fmax = 10, 3, 192, 3, 3, 0x77, 3
        local = None
        for f0, c in bench.rank_ranges(base, K, rank, world, B):
            _, _, cc = oracle_c.run(n, m, c, seed=seed, faulty_mode=1, f=fmax, order_mode=1,
                                    first_trial=f0)
            local = cc if local is None else {k: local[k] + cc[k] for k in local}
        t = torch.tensor(list(local.values()), dtype=torch.int64)
        dist.all_reduce(t)
        total = dict(zip(local, t.tolist()))
        if rank == 0:
            cpu = bench.run_cpu_baseline(n, m, seed, fmax, 0.0, bench.rank_ranges(base, K, 0, world, B),
                                         local, bench.first_trial(base + K + 2, 0, world, B))
            ok = cpu["counters_match"] and cpu["counters_checked"]["ranges"] == K
            try:
                bench.run_cpu_baseline(n, m, seed, fmax, 0.0, bench.rank_ranges(base, K, 0, world, B),
                                       total, 0)
                ok = False
            except SystemExit:
                pass
            q.put(ok and total["trials"] == world * K * B)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_cpu_baseline_world2_gloo():
    """bench.py's N>1 CPU leg: rank 0 checks the port against its own timed ranges
    with its pre-all-reduce counters (world 2, gloo, CPU)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = bench.free_port()
    ps = [ctx.Process(target=_cpu_baseline_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    assert all(p.exitcode == 0 for p in ps)
    assert q.get(timeout=5) is True


def test_clock_from_probes_pairs_rows_by_cu():
    """The engine clock per XCD comes from rows of the same XCD, shader engine and CU
    (HW_ID bits 8-15) in the two probes; an unrelated CU's counter (another engine's
    s_memtime) never enters a difference, and an XCD with no CU in both probes is
    left out."""
    p0 = [(0, 0x0100, 1000, 10), (0, 0x0200, 900000, 10), (1, 0x0100, 5000, 10), (2, 0x0100, 7, 10)]
    p1 = [(0, 0x0100, 1000 + 2400, 110), (0, 0x0300, 10, 110), (1, 0x0100, 5000 + 2300, 110),
          (2, 0x0200, 7 + 2200, 110)]
    med, per = bench.clock_from_probes(p0, p1)
    assert per == {0: 2400.0, 1: 2300.0}
    assert med == 2350.0


def test_lds_bank_model_matches_the_ablation_pmc():
    """tools/lds_bank_model.py's per-task prediction for k_om3w<10> is what the
    ablation builds measured (profiles/r06c_bank/: dropping the R2T leaf stores
    removed 589,824 conflict cycles per 2,048-task launch, dropping the R1T
    store 73,728 -- exactly 288 and 36 per task)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import lds_bank_model as M
    m = M.model(10)
    assert m["r2t_stores"] == 288 and m["r1t_stores"] == 36
    assert m["r2t_columns"] == 0 and m["r1t_roots"] == 0 and m["e_gathers"] == 0
    pmc = {}
    for name in ("base", "nor2t", "nor1t"):
        d = json.load(open(os.path.join(ROOT, "profiles", "r06c_bank", f"bank_om3_{name}_summary.json")))
        (e,) = [v for k, v in d["kernels"].items() if "k_om3w<10, 0, true>" in k]
        pmc[name] = e["counters"]["SQ_LDS_BANK_CONFLICT"]
    assert pmc["base"] - pmc["nor2t"] == m["r2t_stores"] * 2048
    assert pmc["base"] - pmc["nor1t"] == m["r1t_stores"] * 2048


def test_config3_rooflines_from_committed_pmc():
    """tools/config3_prof.rooflines finds the committed same-build-keyed PMC of
    k_om4w<13> at 8M trials (profiles/r06zb_pmc_om4w_*.json) and prices the three
    rooflines; the HBM one is on the 14 B/trial of per-trial I/O."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import config3_prof as C
    roof, valu, comp = C.rooflines(13, 4, 8 << 20, 10e-3, True, engine="auto/staged")
    assert roof["algorithmic_bytes_per_trial"] == 14.0 and roof["traffic"] > 0
    assert valu and valu["valu_insts_per_launch"] > 0
    assert comp["calls_per_launch"] == 54192 * (8 << 20) // 64
