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
