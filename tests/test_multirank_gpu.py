"""The library's N>1 paths executed on one GPU: N processes on cuda:0, each with
a libba_hip communicator over tests/native's shared-memory RCCL stand-in
(BA_RCCL_LIB; RCCL itself refuses two ranks on one GPU).  What runs is the
library's own multi-GPU code (csrc/ba_multi.cpp): ba_run_trials_multi's
counter all-reduce, ba_run_instance_split_level_multi's pre-exchange error
agreement, grouped-broadcast vote all-gather and error all-reduce,
InstanceSplitGraphs' eager all-gather between its two graphs, the watchdog and
ncclCommAbort -- against the oracle, at world sizes 2, 3 and 8
(tests/multirank.py runs the ranks).  ba.py analogue: the per-general polling
of get_majorities (ba.py:197-223) and the relay exchange (ba.py:169-186)."""
import numpy as np
import pytest

import multirank as MR
import oracle_c

pytestmark = pytest.mark.gpu

ENOMEM, EDEVICE, EABORTED = -2, -3, -6
_cache = {}


def ranks(world, tmp_path_factory, scen=("dp", "split", "graphs", "enomem")):
    key = (world, tuple(scen))
    if key not in _cache:
        _cache[key] = MR.launch(world, list(scen), str(tmp_path_factory.mktemp(f"w{world}")))
    return _cache[key]


def oracle(n, m, B, f, first, seed=MR.SEED):
    return oracle_c.run(n, m, B, seed=seed, faulty_mode=1, f=f, order_mode=1, first_trial=first)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_trial_dp_multi_matches_oracle(world, tmp_path_factory):
    """ba_run_trials_multi: each rank's share (ba_trial_share) of decisions and
    outcome bytes, assembled, equals the oracle's whole job, and every rank's
    all-reduced counters equal the oracle's (= one unsharded run)."""
    res = ranks(world, tmp_path_factory)
    for k, (n, m, total, f, first) in enumerate(MR.DP_CASES):
        od, oo, oc = oracle(n, m, total, f, first)
        dec = np.zeros(total, np.uint64)
        out = np.zeros(total, np.uint8)
        covered = 0
        for r in res:
            g = r["dp"][k]
            assert g["case"] == [n, m, total, f, first]
            assert {c: g["counters"][c] for c in oc} == oc, (world, r["rank"], n, m)
            s, c = g["first"], g["count"]
            dec[s:s + c] = np.array(g["dec"], np.uint64)
            out[s:s + c] = np.array(g["out"], np.uint8)
            covered += c
        assert covered == total
        assert np.array_equal(dec, od) and np.array_equal(out, oo), (world, n, m)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_instance_split_multi_matches_oracle(world, tmp_path_factory):
    """ba_run_instance_split_level_multi at levels 1 and 2, batch 1 to 130: on every
    rank, twice (the second call reuses the vote buffer), decisions, outcome bytes
    and counters equal the oracle -- so every rank's vote rows crossed the grouped
    broadcasts into the places the root pass reads."""
    res = ranks(world, tmp_path_factory)
    for k, (n, m, level, B, f, first) in enumerate(MR.SPLIT_CASES):
        od, oo, oc = oracle(n, m, B, f, first)
        for r in res:
            g = r["split"][k]
            assert g["case"] == [n, m, level, B, f, first]
            for call in g["calls"]:
                assert np.array_equal(np.array(call["dec"], np.uint64), od), (world, r["rank"], g["case"])
                assert np.array_equal(np.array(call["out"], np.uint8), oo), (world, r["rank"], g["case"])
                assert {c: call["counters"][c] for c in oc} == oc


@pytest.mark.parametrize("world", [2, 3, 8])
def test_split_graphs_multi_match_oracle(world, tmp_path_factory):
    """InstanceSplitGraphs with N ranks: graph 1 (this rank's votes), the eager
    vote all-gather, graph 2 (roots + quorum); every replay on every rank equals
    the oracle."""
    res = ranks(world, tmp_path_factory)
    for k, (n, m, level, B) in enumerate(MR.GRAPH_CASES):
        od, oo, oc = oracle(n, m, B, (n - 1) // 3, 64 * 5)
        for r in res:
            for rep in r["graphs"][k]["replays"]:
                assert np.array_equal(np.array(rep["dec"], np.uint64), od), (world, r["rank"], k)
                assert np.array_equal(np.array(rep["out"], np.uint8), oo)
                assert rep["counters"] == list(oc.values())


@pytest.mark.parametrize("world", [2, 3, 8])
def test_one_rank_vote_enomem_fails_every_rank(world, tmp_path_factory):
    """Rank 1 alone cannot allocate its vote buffer (BA_TEST_VOTE_ENOMEM on that
    process only): it returns ENOMEM, every other rank 'other rank(s) failed',
    agreed BEFORE the exchange (no rank waits in a broadcast rank 1 skipped); the
    next call on the same communicator is exact on every rank."""
    res = ranks(world, tmp_path_factory)
    od, _, oc = oracle(10, 3, 200, 3, 0, seed=3)
    for r in res:
        first = r["enomem"]["first"]
        if r["rank"] == 1:
            assert first["code"] == ENOMEM, first
        else:
            assert first["code"] == EDEVICE and "other rank(s) failed" in first["msg"], first
        after = r["enomem"]["after"]
        assert np.array_equal(np.array(after["dec"], np.uint64), od)
        assert {c: after["counters"][c] for c in oc} == oc
    assert max(r["elapsed"]["enomem"] for r in res) < 60


FAIL_SCEN = ("preagree_upload", "preagree_upload_memset", "preagree_readback", "abort_dp")


@pytest.mark.parametrize("world", [3])
def test_transport_failures_end_every_rank(world, tmp_path_factory):
    """Rank 1's own agreement transport fails (BA_TEST_PREAGREE_FAIL):
    - upload: the flag is raised by a device memset instead: every rank fails
      together and the communicator stays usable;
    - upload_memset / readback: rank 1 cannot raise or read the flag, so it aborts
      its communicator (EABORTED) -- its peers, which would wait for it in the
      all-reduce or the vote exchange, leave through their watchdog (4 s here)
      with EABORTED instead of hanging; every further call fails fast;
    - abort_dp: the last rank aborts before a trial-DP job; its peers' counter
      all-reduce ends at their watchdog (3 s).
    After each, a new communicator over the same processes is exact."""
    res = ranks(world, tmp_path_factory, FAIL_SCEN)
    n, m, B = 16, 5, 70
    _, _, oc = oracle(n, m, B, 5, 0, seed=9)
    for r in res:
        up = r["preagree_upload"]
        if r["rank"] == 1:
            assert up["first"]["code"] == EDEVICE and "upload" in up["first"]["msg"], up
        else:
            assert up["first"]["code"] == EDEVICE and "other rank(s) failed" in up["first"]["msg"], up
        assert up["again"] == {"code": 0, "trials": B}, up  # agreed failure: comm still usable
        for mode in ("upload_memset", "readback"):
            g = r["preagree_" + mode]
            assert g["first"]["code"] == EABORTED, (mode, g)
            if r["rank"] == 1:
                assert g["first"]["seconds"] < 2.0, (mode, g)  # aborts itself at once
            else:
                assert g["first"]["seconds"] < 30.0, (mode, g)  # its watchdog, not a hang
            assert g["again"]["code"] == EABORTED, (mode, g)
        for name in FAIL_SCEN[:3]:
            assert {c: r[name]["fresh"][c] for c in oc} == oc, name
        ab = r["abort_dp"]
        assert ab["first"]["code"] == EABORTED, ab
        assert ab["first"]["seconds"] < 30.0, ab
        _, _, oc_dp = oracle(10, 3, 64 * 100, 3, 0, seed=1)
        assert {c: ab["fresh"][c] for c in oc_dp} == oc_dp


def test_bench_two_ranks_through_library_collectives(tmp_path):
    """bench.py --gpus 2 with both ranks on cuda:0 (BA_BENCH_DEVICE=0) and the
    stand-in behind the library's RCCL calls: the N>1 flow the driver's 8-GPU run
    takes -- torch.distributed.run child, per-rank staging, the device-side RCCL
    barrier (ba_comm_allreduce_device of a dummy buffer) opening the timed region,
    the counter all-reduce closing it, max-over-ranks timing -- with the counters
    summed over both ranks and rank 0's cpu_baseline checked against its own
    pre-all-reduce tallies.  The rate means nothing (two ranks share one GPU)."""
    import json
    import os
    import subprocess
    import sys
    steps, B = 4, 1 << 16
    env = dict(os.environ, BA_BENCH_DEVICE="0", BA_RCCL_LIB=MR.build_fake(),
               FAKE_RCCL_TIMEOUT_S="90", MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, os.path.join(MR.ROOT, "bench.py"), "--gpus", "2",
                        "--steps", str(steps), "--warmup", "1", "--batch", str(B), "--warm-s", "0.2",
                        "--cpu-budget-s", "1", "--no-profile"],
                       env=env, capture_output=True, text=True, timeout=300, cwd=MR.ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "trial-dp2"
    assert line["collective"].startswith("rccl API of BA_RCCL_LIB=libfake_rccl.so"), line["collective"]
    assert line["counters"]["trials"] == 2 * steps * B
    assert line["counters"]["agreement"] == 2 * steps * B  # f <= 3 < n/3 at n=10: IC1 holds
    assert line["cpu_baseline"]["counters_match"] is True
    assert line["cpu_baseline"]["counters_checked"]["trials"] == steps * B
