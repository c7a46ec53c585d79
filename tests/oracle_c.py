"""ctypes wrapper of the C oracle (oracle/ba_oracle.c) for the tests and bench.py's
cpu_baseline leg.  Test infrastructure only."""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "oracle", "_build", "libba_oracle.so")
COUNTER_NAMES = ["trials", "agreement", "validity_applicable", "validity", "quorum_retreat",
                 "quorum_attack", "quorum_undetermined", "undefined_decisions", "in_bound",
                 "bound_violations", "faulty_total", "attack_decisions"]
_lib = None


def load():
    global _lib
    if _lib is None:
        srcs = [os.path.join(ROOT, "oracle", f) for f in ("ba_oracle.c", "ba_sliced.c")]
        if not os.path.exists(SO) or max(map(os.path.getmtime, srcs)) > os.path.getmtime(SO):
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
        lib = ctypes.CDLL(SO)
        u32, u64, vp = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p
        lib.ba_oracle_run.argtypes = [u32, u32, u64, u32, u32, u32, u32, u32, u64, u32, u64,
                                      vp, vp, vp, vp, vp, vp, vp, ctypes.c_int]
        lib.ba_oracle_lie.argtypes = [u64, u64, u32, u64]
        lib.ba_oracle_lie.restype = u32
        lib.ba_oracle_philox.argtypes = [vp, vp, vp]
        lib.ba_oracle_gen.argtypes = [u32, u64, u32, u32, u32, u32, u64, vp, vp]
        lib.ba_oracle_votes.argtypes = [u32, u32, u64, u32, u32, u32, u32, u64, u64, vp, vp, vp,
                                        ctypes.c_int]
        lib.ba_oracle_votes2.argtypes = lib.ba_oracle_votes.argtypes
        lib.ba_sliced_run.argtypes = [u32, u32, u64, u32, u32, u32, u32, u64, u64, vp, vp, vp, vp,
                                      vp, ctypes.c_int]
        lib.ba_sliced_gen.argtypes = [u32, u64, u32, u32, u32, u32, u64, u64, vp, vp, ctypes.c_int]
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


def run(n, m, batch, seed=0, lie_mode=0, faulty_mode=0, f=0, order_mode=0, order_value=1,
        first_trial=0, faulty=None, order=None, table=None, poll=None, threads=0):
    """Returns (decisions uint64[batch], outcome uint8[batch], counters dict)."""
    lib = load()
    faulty = None if faulty is None else np.ascontiguousarray(faulty, np.uint32)
    order = None if order is None else np.ascontiguousarray(order, np.uint8)
    stride = 0
    if table is not None:
        table = np.ascontiguousarray(table, np.uint32)
        stride = table.shape[1]
    poll = None if poll is None else np.ascontiguousarray(poll, np.uint32)
    dec = np.zeros(batch, np.uint64)
    out = np.zeros(batch, np.uint8)
    cnt = np.zeros(16, np.uint64)
    rc = lib.ba_oracle_run(n, m, seed, lie_mode, faulty_mode, f, order_mode, order_value,
                           first_trial, stride, batch, _p(faulty), _p(order), _p(table), _p(poll),
                           _p(dec), _p(out), _p(cnt), threads)
    if rc != 0:
        raise RuntimeError(f"oracle rc={rc}")
    return dec, out, dict(zip(COUNTER_NAMES, [int(x) for x in cnt[:12]]))


def votes(n, m, batch, seed=0, faulty_mode=0, f=0, order_mode=0, order_value=1, first_trial=0,
          faulty=None, order=None, threads=0):
    """Level-1 child results uint8[batch, n-1, n-2] (see ba_oracle_votes)."""
    lib = load()
    faulty = None if faulty is None else np.ascontiguousarray(faulty, np.uint32)
    order = None if order is None else np.ascontiguousarray(order, np.uint8)
    out = np.zeros((batch, n - 1, n - 2), np.uint8)
    rc = lib.ba_oracle_votes(n, m, seed, faulty_mode, f, order_mode, order_value, first_trial,
                             batch, _p(faulty), _p(order), _p(out), threads)
    if rc != 0:
        raise RuntimeError(f"oracle rc={rc}")
    return out


def votes2(n, m, batch, seed=0, faulty_mode=0, f=0, order_mode=0, order_value=1, first_trial=0,
           faulty=None, order=None, threads=0):
    """Level-2 results uint8[batch, (n-1)(n-2), n-3] of every level-1 slot (second-hop
    split units; see ba_oracle_votes2)."""
    lib = load()
    faulty = None if faulty is None else np.ascontiguousarray(faulty, np.uint32)
    order = None if order is None else np.ascontiguousarray(order, np.uint8)
    out = np.zeros((batch, (n - 1) * (n - 2), n - 3), np.uint8)
    rc = lib.ba_oracle_votes2(n, m, seed, faulty_mode, f, order_mode, order_value, first_trial,
                              batch, _p(faulty), _p(order), _p(out), threads)
    if rc != 0:
        raise RuntimeError(f"oracle rc={rc}")
    return out


def pack_votes(v, jb=0, je=None):
    """uint8[batch, units, per-unit] -> the library's vote layout uint64[(je-jb)*per-unit, W]
    (first-hop units: [batch, L, L-1]; second-hop units: [batch, L(L-1), L-2])."""
    batch, L, _ = v.shape
    je = L if je is None else je
    W = (batch + 63) // 64
    flat = v[:, jb:je, :].reshape(batch, -1)
    pad = np.zeros((W * 64, flat.shape[1]), np.uint8)
    pad[:batch] = flat
    bits = pad.reshape(W, 64, -1).transpose(2, 0, 1)  # slot, word, lane
    weights = (np.uint64(1) << np.arange(64, dtype=np.uint64))
    return (bits.astype(np.uint64) * weights).sum(axis=2, dtype=np.uint64)


def sliced_run(n, m, batch, seed=0, faulty_mode=0, f=0, order_mode=0, order_value=1,
               first_trial=0, faulty=None, order=None, threads=0, want_outputs=True):
    """Word-sliced OpenMP port (oracle/ba_sliced.c), Philox lies only.
    Returns (decisions, outcome, counters) like run(); outputs None when not wanted."""
    lib = load()
    faulty = None if faulty is None else np.ascontiguousarray(faulty, np.uint32)
    order = None if order is None else np.ascontiguousarray(order, np.uint8)
    dec = np.zeros(batch, np.uint64) if want_outputs else None
    out = np.zeros(batch, np.uint8) if want_outputs else None
    cnt = np.zeros(16, np.uint64)
    rc = lib.ba_sliced_run(n, m, seed, faulty_mode, f, order_mode, order_value, first_trial, batch,
                           _p(faulty), _p(order), _p(dec), _p(out), _p(cnt), threads)
    if rc != 0:
        raise RuntimeError(f"sliced port rc={rc}")
    return dec, out, dict(zip(COUNTER_NAMES, [int(x) for x in cnt[:12]]))


def sliced_gen(n, batch, seed=0, faulty_mode=1, f=0, order_mode=1, order_value=1, first_trial=0,
               threads=0):
    """Synthetic inputs (faulty uint32[batch], order uint8[batch]) of the given stream."""
    lib = load()
    faulty = np.zeros(batch, np.uint32)
    order = np.zeros(batch, np.uint8)
    rc = lib.ba_sliced_gen(n, seed, faulty_mode, f, order_mode, order_value, first_trial, batch,
                           _p(faulty), _p(order), threads)
    if rc != 0:
        raise RuntimeError(f"sliced gen rc={rc}")
    return faulty, order
