"""ctypes binding of libba_hip.so (include/ba.h).

This is the only way the Python side reaches the hot path.  There is no CPU
fallback: if the shared library is missing, or no HIP device is visible, the
calls raise.  The oracle under /oracle is test infrastructure and is never
imported here.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BA_HIP_LIB", os.path.join(HERE, "libba_hip.so"))

# numeric contract of include/ba.h
ABI_VERSION = 1
MAX_GENERALS = 32
MAX_DEPTH = 8
NCOUNTERS = 16
OK, EINVAL, ENOMEM, EDEVICE, ENOTSUP, ETOOBIG, EABORTED = 0, -1, -2, -3, -4, -5, -6
LIE_PHILOX, LIE_TABLE = 0, 1
FAULTY_GIVEN, FAULTY_RANDOM, FAULTY_EXACT = 0, 1, 2
ORDER_GIVEN, ORDER_RANDOM, ORDER_CONST = 0, 1, 2
RETREAT, ATTACK, OTHER, UNDEFINED = 0, 1, 2, 2
Q_RETREAT, Q_ATTACK, Q_UNDETERMINED = 0, 1, 2
ENGINE_AUTO, ENGINE_FUSED, ENGINE_LEVELS = 0, 1, 2
SPLIT_FIRST_HOP, SPLIT_SECOND_HOP = 1, 2
COUNTER_NAMES = ["trials", "agreement", "validity_applicable", "validity", "quorum_retreat",
                 "quorum_attack", "quorum_undetermined", "undefined_decisions", "in_bound",
                 "bound_violations", "faulty_total", "attack_decisions"]
EXPORTS = ["ba_version", "ba_device_count", "ba_ctx_create", "ba_ctx_destroy", "ba_last_error",
           "ba_run_trials", "ba_run_trials_device", "ba_tree_slots", "ba_level_slots",
           "ba_engine_for", "ba_profile_enable", "ba_profile_read", "ba_mt_seed", "ba_mt_next32",
           "ba_om1_coin_count", "ba_mt_draw_coins", "ba_mt_table", "ba_vote_slots",
           "ba_subtree_votes_device", "ba_root_from_votes_device", "ba_gen_inputs_device",
           "ba_ctx_device", "ba_ctx_stream", "ba_comm_unique_id", "ba_comm_create", "ba_comm_destroy",
           "ba_trial_share", "ba_run_trials_multi", "ba_comm_rank", "ba_subtree_share",
           "ba_comm_allreduce_device", "ba_comm_allgather_votes_device",
           "ba_run_instance_split_multi", "ba_split_units", "ba_split_vote_slots",
           "ba_split_share", "ba_split_votes_device", "ba_root_from_split_votes_device",
           "ba_comm_allgather_split_votes_device", "ba_run_instance_split_level_multi",
           "ba_clock_probe_device", "ba_ctx_memory", "ba_comm_set_timeout", "ba_comm_abort",
           "ba_mt_table_device"]
PROBE_BLOCKS = 2048  # BA_PROBE_BLOCKS


class BAError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libba_hip error {code}: {msg}")
        self.code = code


class Params(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint32), ("m", ctypes.c_uint32), ("seed", ctypes.c_uint64),
                ("lie_mode", ctypes.c_uint32), ("faulty_mode", ctypes.c_uint32),
                ("f", ctypes.c_uint32), ("order_mode", ctypes.c_uint32),
                ("order_value", ctypes.c_uint32), ("engine", ctypes.c_uint32),
                ("first_trial", ctypes.c_uint64), ("table_stride", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32 * 5)]


class MTState(ctypes.Structure):
    """ba_mt: CPython-compatible MT19937 state (include/ba.h)."""
    _fields_ = [("state", ctypes.c_uint32 * 624), ("index", ctypes.c_uint32)]


class Counters(ctypes.Structure):
    _fields_ = [("v", ctypes.c_uint64 * NCOUNTERS)]


_lib = None


def load(path: str | None = None):
    """Load libba_hip.so (raises if it is absent: there is no fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise FileNotFoundError(f"{p} not built: run `make -C byzantine-agreement_amd` "
                                f"or __graft_entry__.build()")
    # torch's wheel bundles its own libamdhip64.so.7 (same soname as /opt/rocm's).
    # Whichever loads first serves the whole process, so let torch's load first
    # when it is installed: then torch tensors/streams and our kernels share one
    # HIP runtime (device pointers and hipStream_t handles are passed across).
    if os.environ.get("BA_NO_TORCH", "0") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    lib = ctypes.CDLL(p)
    vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    lib.ba_version.restype = i32
    lib.ba_device_count.argtypes = [ctypes.POINTER(i32)]
    lib.ba_ctx_create.argtypes = [i32, ctypes.POINTER(vp)]
    lib.ba_ctx_destroy.argtypes = [vp]
    lib.ba_ctx_destroy.restype = None
    lib.ba_last_error.restype = ctypes.c_char_p
    lib.ba_run_trials.argtypes = [vp, ctypes.POINTER(Params), u64, vp, vp, vp, vp, vp, vp,
                                  ctypes.POINTER(Counters)]
    lib.ba_run_trials_device.argtypes = [vp, ctypes.POINTER(Params), u64, vp, vp, vp, vp, vp,
                                         vp, vp, vp]
    lib.ba_gen_inputs_device.argtypes = [vp, ctypes.POINTER(Params), u64, vp, vp, vp]
    lib.ba_tree_slots.argtypes = [u32, u32]
    lib.ba_tree_slots.restype = u64
    lib.ba_level_slots.argtypes = [u32, u32, u32]
    lib.ba_level_slots.restype = u64
    lib.ba_engine_for.argtypes = [u32, u32]
    lib.ba_profile_enable.argtypes = [vp, i32]
    lib.ba_profile_read.argtypes = [vp, i32, ctypes.c_char_p, i32, ctypes.POINTER(u64),
                                    ctypes.POINTER(ctypes.c_double)]
    lib.ba_mt_seed.argtypes = [ctypes.POINTER(MTState), u64]
    lib.ba_mt_seed.restype = None
    lib.ba_mt_next32.argtypes = [ctypes.POINTER(MTState)]
    lib.ba_mt_next32.restype = u32
    lib.ba_om1_coin_count.argtypes = [u32, u32, u32, u32]
    lib.ba_om1_coin_count.restype = u32
    lib.ba_mt_draw_coins.argtypes = [ctypes.POINTER(MTState), u32, vp, u32]
    lib.ba_mt_table.argtypes = [u32, u32, u64, vp, vp, vp, u32, vp, vp, i32]
    if hasattr(lib, "ba_mt_table_device"):  # (A/B runs may load an older library)
        lib.ba_mt_table_device.argtypes = [vp, u32, u32, u64, vp, vp, vp, u32, vp, vp, vp]
    lib.ba_vote_slots.argtypes = [u32, u32, u32, u32]
    lib.ba_vote_slots.restype = u64
    lib.ba_subtree_votes_device.argtypes = [vp, ctypes.POINTER(Params), u64, u32, u32, vp, vp, vp,
                                            vp]
    lib.ba_root_from_votes_device.argtypes = [vp, ctypes.POINTER(Params), u64, vp, vp, vp, vp, vp,
                                              vp, vp]
    lib.ba_ctx_device.argtypes = [vp, ctypes.POINTER(i32)]
    lib.ba_ctx_stream.argtypes = [vp, ctypes.POINTER(vp)]
    lib.ba_clock_probe_device.argtypes = [vp, vp, vp]
    lib.ba_ctx_memory.argtypes = [vp, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(u64)]
    lib.ba_comm_unique_id.argtypes = [ctypes.c_char_p]
    lib.ba_comm_create.argtypes = [vp, i32, i32, ctypes.c_char_p, ctypes.POINTER(vp)]
    lib.ba_comm_destroy.argtypes = [vp]
    lib.ba_comm_destroy.restype = None
    lib.ba_trial_share.argtypes = [u64, i32, i32, ctypes.POINTER(u64), ctypes.POINTER(u64)]
    lib.ba_run_trials_multi.argtypes = [vp, vp, ctypes.POINTER(Params), u64, vp, vp,
                                        ctypes.POINTER(Counters), ctypes.POINTER(u64),
                                        ctypes.POINTER(u64)]
    lib.ba_comm_rank.argtypes = [vp, ctypes.POINTER(i32), ctypes.POINTER(i32)]
    if hasattr(lib, "ba_comm_abort"):
        lib.ba_comm_set_timeout.argtypes = [vp, u64]
        lib.ba_comm_abort.argtypes = [vp]
    lib.ba_subtree_share.argtypes = [u32, i32, i32, ctypes.POINTER(u32), ctypes.POINTER(u32)]
    lib.ba_comm_allreduce_device.argtypes = [vp, vp, vp]
    lib.ba_comm_allgather_votes_device.argtypes = [vp, u32, u32, u64, vp, vp]
    lib.ba_run_instance_split_multi.argtypes = [vp, vp, ctypes.POINTER(Params), u64, vp, vp, vp,
                                                vp, ctypes.POINTER(Counters)]
    lib.ba_split_units.argtypes = [u32, u32, u32]
    lib.ba_split_units.restype = u64
    lib.ba_split_vote_slots.argtypes = [u32, u32, u32, u32, u32]
    lib.ba_split_vote_slots.restype = u64
    lib.ba_split_share.argtypes = [u32, u32, u32, i32, i32, ctypes.POINTER(u32),
                                   ctypes.POINTER(u32)]
    lib.ba_split_votes_device.argtypes = [vp, ctypes.POINTER(Params), u64, u32, u32, u32, vp, vp,
                                          vp, vp]
    lib.ba_root_from_split_votes_device.argtypes = [vp, ctypes.POINTER(Params), u64, u32, vp, vp,
                                                    vp, vp, vp, vp, vp]
    lib.ba_comm_allgather_split_votes_device.argtypes = [vp, u32, u32, u32, u64, vp, vp]
    lib.ba_run_instance_split_level_multi.argtypes = [vp, vp, ctypes.POINTER(Params), u32, u64,
                                                      vp, vp, vp, vp, ctypes.POINTER(Counters)]
    if lib.ba_version() != ABI_VERSION:
        raise RuntimeError(f"libba_hip ABI {lib.ba_version()} != {ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


def _check(lib, rc: int):
    if rc != OK:
        raise BAError(rc, lib.ba_last_error().decode())


C_HANDOFF_LOST = 14  # BA_C_CHECK_MISMATCH: a cascade hand-off poll ran out of time


def check_handoff(counters):
    """Raise BAError(EDEVICE) if a device-path call's counters (16 int64: a torch
    tensor, numpy array, list or COUNTER dict with "CHECK_MISMATCH") carry a lost
    in-launch hand-off (slot 14, include/ba.h): that call's results are invalid.
    ba_run_trials and the multi-rank jobs check it themselves; callers of the
    asynchronous *_device entry points check it after their synchronize."""
    if isinstance(counters, dict):
        v = int(counters.get("CHECK_MISMATCH", 0))
    else:
        v = int(counters[C_HANDOFF_LOST])
    if v != 0:
        raise BAError(EDEVICE, f"in-launch hand-off timed out ({v} stale granule poll(s), counter "
                               f"slot {C_HANDOFF_LOST}); results invalid")


def effective_depth(n: int, m: int) -> int:
    return min(m, n - 2) if n >= 2 else 0


def default_fmax(n: int) -> int:
    """f ~ U{0..floor((n-1)/3)} for random-set configs."""
    return (n - 1) // 3


def table_stride(n: int) -> int:
    """uint32 words per trial a ba.py draw-order table needs: (n-1) + (n-1)^2 coins."""
    L = n - 1
    return max(1, (L + L * L + 31) // 32)


@dataclass
class RunResult:
    decisions: np.ndarray | None
    outcome: np.ndarray | None
    counters: dict = field(default_factory=dict)

    def decision(self, t: int, r: int) -> int:
        """Decision code of lieutenant r (1..n-1) in trial t."""
        return int((int(self.decisions[t]) >> (2 * (r - 1))) & 3)


def make_params(n, m, seed=0, lie_mode=LIE_PHILOX, faulty_mode=FAULTY_GIVEN, f=0,
                order_mode=ORDER_GIVEN, order_value=ATTACK, engine=ENGINE_AUTO,
                first_trial=0, stride=0) -> Params:
    p = Params()
    p.n, p.m, p.seed = n, m, seed & ((1 << 64) - 1)
    p.lie_mode, p.faulty_mode, p.f = lie_mode, faulty_mode, f
    p.order_mode, p.order_value, p.engine = order_mode, order_value, engine
    p.first_trial, p.table_stride = first_trial, stride
    return p


def _ptr(a):
    return None if a is None else a.ctypes.data


class Engine:
    """One libba_hip context on one HIP device (mirrors a ba.py process group)."""

    def __init__(self, device: int = 0):
        self.lib = load()
        h = ctypes.c_void_p()
        _check(self.lib, self.lib.ba_ctx_create(device, ctypes.byref(h)))
        self.handle = h
        self.device = device

    def close(self):
        if self.handle:
            self.lib.ba_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, n, m, batch, seed=0, lie_mode=LIE_PHILOX, faulty_mode=FAULTY_GIVEN, f=0,
            order_mode=ORDER_GIVEN, order_value=ATTACK, engine=ENGINE_AUTO, first_trial=0,
            faulty=None, order=None, table=None, poll=None, want_decisions=True,
            want_outcome=True) -> RunResult:
        """Resolve `batch` trials through host buffers (PCIe copies included)."""
        faulty = None if faulty is None else np.ascontiguousarray(faulty, dtype=np.uint32)
        order = None if order is None else np.ascontiguousarray(order, dtype=np.uint8)
        stride = 0
        if table is not None:
            table = np.ascontiguousarray(table, dtype=np.uint32)
            stride = table.shape[1]
        poll = None if poll is None else np.ascontiguousarray(poll, dtype=np.uint32)
        dec = np.zeros(batch, np.uint64) if want_decisions else None
        out = np.zeros(batch, np.uint8) if want_outcome else None
        p = make_params(n, m, seed, lie_mode, faulty_mode, f, order_mode, order_value, engine,
                        first_trial, stride)
        cnt = Counters()
        _check(self.lib, self.lib.ba_run_trials(self.handle, ctypes.byref(p), batch, _ptr(faulty),
                                                _ptr(order), _ptr(table), _ptr(poll), _ptr(dec),
                                                _ptr(out), ctypes.byref(cnt)))
        return RunResult(dec, out, dict(zip(COUNTER_NAMES, [int(x) for x in cnt.v])))

    def stream(self) -> int:
        """The ctx's own HIP stream (ba_ctx_stream), as an int handle."""
        h = ctypes.c_void_p()
        _check(self.lib, self.lib.ba_ctx_stream(self.handle, ctypes.byref(h)))
        return h.value or 0

    def profile(self, on: bool):
        """Enable/disable per-kernel HIP-event timing (clears the totals)."""
        _check(self.lib, self.lib.ba_profile_enable(self.handle, int(on)))

    def profile_read(self) -> dict:
        """{kernel name: (launches, total ms)} since profiling was enabled."""
        out, i = {}, 0
        name = ctypes.create_string_buffer(64)
        n = ctypes.c_uint64()
        ms = ctypes.c_double()
        while self.lib.ba_profile_read(self.handle, i, name, 64, ctypes.byref(n), ctypes.byref(ms)) == OK:
            out[name.value.decode()] = (int(n.value), float(ms.value))
            i += 1
        return out

    def run_device(self, params: Params, batch: int, d_faulty=0, d_order=0, d_table=0, d_poll=0,
                   d_decisions=0, d_outcome=0, d_counters=0, stream=0):
        """Enqueue on device pointers (ints, e.g. torch tensor .data_ptr()); asynchronous.
        After synchronizing, check the counters with check_handoff (include/ba.h)."""
        _check(self.lib, self.lib.ba_run_trials_device(
            self.handle, ctypes.byref(params), batch, d_faulty or None, d_order or None,
            d_table or None, d_poll or None, d_decisions or None, d_outcome or None,
            d_counters or None, stream or None))

    def gen_inputs_device(self, params: Params, batch: int, d_faulty=0, d_order=0, stream=0):
        """Stage the synthetic faulty sets / orders of a batch in HBM (see include/ba.h)."""
        _check(self.lib, self.lib.ba_gen_inputs_device(
            self.handle, ctypes.byref(params), batch, d_faulty or None, d_order or None,
            stream or None))

    def subtree_votes_device(self, params: Params, batch: int, j_begin: int, j_end: int,
                             d_votes: int, d_faulty=0, d_order=0, stream=0):
        """Level-1 child results of first-hop subtrees [j_begin, j_end)."""
        _check(self.lib, self.lib.ba_subtree_votes_device(
            self.handle, ctypes.byref(params), batch, j_begin, j_end, d_faulty or None,
            d_order or None, d_votes, stream or None))

    def memory(self) -> dict:
        """Device bytes the ctx holds (ba_ctx_memory): LEVELS scratch, cascade fan-in
        counters, and the budget they are chunked to."""
        sc, cn, bu = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(self.lib, self.lib.ba_ctx_memory(self.handle, ctypes.byref(sc), ctypes.byref(cn),
                                                ctypes.byref(bu)))
        return {"scratch": sc.value, "counters": cn.value, "budget": bu.value}

    def mt_table_device(self, n: int, m: int, batch: int, d_seeds: int, d_faulty: int, stride: int,
                        d_table: int, d_poll=0, d_next_word=0, stream=0):
        """ba.py's coin table on the device (ba_mt_table_device): row t = the coins of
        random.seed(seeds[t]) + one round over (faulty[t], poll[t]); asynchronous."""
        _check(self.lib, self.lib.ba_mt_table_device(self.handle, n, m, batch, d_seeds, d_faulty,
                                                     d_poll or None, stride, d_table,
                                                     d_next_word or None, stream or None))

    def clock_probe_device(self, d_out: int, stream=0):
        """Enqueue the engine-clock probe (ba_clock_probe_device): PROBE_BLOCKS rows of
        {XCC id, HW id, s_memtime, s_memrealtime} into d_out (uint64)."""
        _check(self.lib, self.lib.ba_clock_probe_device(self.handle, d_out, stream or None))

    def split_votes_device(self, params: Params, batch: int, level: int, u_begin: int, u_end: int,
                           d_votes: int, d_faulty=0, d_order=0, stream=0):
        """Level-`level` results of split units [u_begin, u_end) (ba_split_votes_device)."""
        _check(self.lib, self.lib.ba_split_votes_device(
            self.handle, ctypes.byref(params), batch, level, u_begin, u_end, d_faulty or None,
            d_order or None, d_votes, stream or None))

    def root_from_split_votes_device(self, params: Params, batch: int, level: int, d_votes: int,
                                     d_counters: int, d_faulty=0, d_order=0, d_decisions=0,
                                     d_outcome=0, stream=0):
        """Majorities above the split level, roots and quorum from every unit's votes."""
        _check(self.lib, self.lib.ba_root_from_split_votes_device(
            self.handle, ctypes.byref(params), batch, level, d_faulty or None, d_order or None,
            d_votes, d_decisions or None, d_outcome or None, d_counters, stream or None))

    def root_from_votes_device(self, params: Params, batch: int, d_votes: int, d_counters: int,
                               d_faulty=0, d_order=0, d_decisions=0, d_outcome=0, stream=0):
        """Root majorities + quorum from the gathered votes of every subtree."""
        _check(self.lib, self.lib.ba_root_from_votes_device(
            self.handle, ctypes.byref(params), batch, d_faulty or None, d_order or None, d_votes,
            d_decisions or None, d_outcome or None, d_counters, stream or None))


def comm_unique_id() -> bytes:
    """RCCL unique id (BA_COMM_ID_BYTES) for ba_comm_create; rank 0 makes it."""
    lib = load()
    buf = ctypes.create_string_buffer(128)
    _check(lib, lib.ba_comm_unique_id(buf))
    return buf.raw


def trial_share(total_trials: int, nranks: int, rank: int):
    """(first, count) of rank's word-aligned share (ba_trial_share)."""
    lib = load()
    f, c = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib, lib.ba_trial_share(total_trials, nranks, rank, ctypes.byref(f), ctypes.byref(c)))
    return f.value, c.value


def subtree_share(n: int, nranks: int, rank: int):
    """[j_begin, j_end) first-hop subtrees of rank (ba_subtree_share)."""
    lib = load()
    b, e = ctypes.c_uint32(), ctypes.c_uint32()
    _check(lib, lib.ba_subtree_share(n, nranks, rank, ctypes.byref(b), ctypes.byref(e)))
    return b.value, e.value


def split_units(n: int, m: int, level: int) -> int:
    """Units of a split level (ba_split_units): n-1 first hops, (n-1)(n-2) second hops."""
    return int(load().ba_split_units(n, m, level))


def split_vote_slots(n: int, m: int, level: int, u_begin: int, u_end: int) -> int:
    return int(load().ba_split_vote_slots(n, m, level, u_begin, u_end))


def split_share(n: int, m: int, level: int, nranks: int, rank: int):
    """[u_begin, u_end) split units of rank (ba_split_share)."""
    lib = load()
    b, e = ctypes.c_uint32(), ctypes.c_uint32()
    _check(lib, lib.ba_split_share(n, m, level, nranks, rank, ctypes.byref(b), ctypes.byref(e)))
    return b.value, e.value


class Comm:
    """An RCCL communicator owned by the C ABI (ba_comm_create) on an Engine's
    device: ba_run_trials_multi shards trials over the ranks and all-reduces
    the run counters itself, for hosts without torch.distributed."""

    def __init__(self, engine: Engine, nranks: int, rank: int, uid: bytes):
        self.engine, self.lib = engine, engine.lib
        h = ctypes.c_void_p()
        _check(self.lib, self.lib.ba_comm_create(engine.handle, nranks, rank, uid, ctypes.byref(h)))
        self.handle = h

    @property
    def rank(self):
        nr, r = ctypes.c_int(), ctypes.c_int()
        _check(self.lib, self.lib.ba_comm_rank(self.handle, ctypes.byref(nr), ctypes.byref(r)))
        return r.value

    @property
    def nranks(self):
        nr, r = ctypes.c_int(), ctypes.c_int()
        _check(self.lib, self.lib.ba_comm_rank(self.handle, ctypes.byref(nr), ctypes.byref(r)))
        return nr.value

    def run_trials(self, params: Params, total_trials: int, d_decisions=0, d_outcome=0):
        """Trial-DP job (ba_run_trials_multi) -> (whole-job counters dict, share first,
        share count)."""
        cnt = Counters()
        f, c = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self.lib, self.lib.ba_run_trials_multi(
            self.engine.handle, self.handle, ctypes.byref(params), total_trials,
            d_decisions or None, d_outcome or None, ctypes.byref(cnt), ctypes.byref(f),
            ctypes.byref(c)))
        return dict(zip(COUNTER_NAMES, [int(x) for x in cnt.v])), f.value, c.value

    def run_instance_split(self, params: Params, batch: int, d_decisions=0, d_outcome=0,
                           d_faulty=0, d_order=0, level: int = SPLIT_FIRST_HOP):
        """Subtree split job (ba_run_instance_split_level_multi; level 1 = first hop,
        2 = second hop) -> counters dict (same on every rank); decisions / outcome
        (batch entries) to the device buffers."""
        cnt = Counters()
        _check(self.lib, self.lib.ba_run_instance_split_level_multi(
            self.engine.handle, self.handle, ctypes.byref(params), level, batch, d_faulty or None,
            d_order or None, d_decisions or None, d_outcome or None, ctypes.byref(cnt)))
        return dict(zip(COUNTER_NAMES, [int(x) for x in cnt.v]))

    def allgather_split_votes_device(self, n: int, m: int, level: int, batch: int, d_votes: int,
                                     stream=0):
        """Every rank's split-vote rows (level 1 or 2) to every rank, in place."""
        _check(self.lib, self.lib.ba_comm_allgather_split_votes_device(
            self.handle, n, m, level, batch, d_votes, stream or None))

    def allreduce_device(self, d_counters: int, stream=0):
        """Sum the 16 device counters over the ranks in place (async on stream)."""
        _check(self.lib, self.lib.ba_comm_allreduce_device(self.handle, d_counters, stream or None))

    def allgather_votes_device(self, n: int, m: int, batch: int, d_votes: int, stream=0):
        """Every rank's subtree-vote rows to every rank, in place (async on stream)."""
        _check(self.lib, self.lib.ba_comm_allgather_votes_device(self.handle, n, m, batch,
                                                                 d_votes, stream or None))

    def set_timeout(self, timeout_ms: int):
        """Watchdog of the blocking jobs (ba_comm_set_timeout): past it a job aborts
        the communicator and raises BAError(EABORTED)."""
        _check(self.lib, self.lib.ba_comm_set_timeout(self.handle, timeout_ms))

    def abort(self):
        """ncclCommAbort on this rank (ba_comm_abort); every further call raises
        BAError(EABORTED); close() still frees the comm."""
        _check(self.lib, self.lib.ba_comm_abort(self.handle))

    def close(self):
        if self.handle:
            self.lib.ba_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MT:
    """ba.py's coin source (random.seed / random.randint(0, 1)), host-side C++."""

    def __init__(self, seed: int = 0):
        self.lib = load()
        self.st = MTState()
        self.seed(seed)

    def seed(self, seed: int):
        if not 0 <= seed < (1 << 64):
            raise ValueError("seed must be in [0, 2^64)")
        self.lib.ba_mt_seed(ctypes.byref(self.st), seed)

    def next32(self) -> int:
        return int(self.lib.ba_mt_next32(ctypes.byref(self.st)))

    def coins(self, count: int, words: int | None = None) -> np.ndarray:
        """Draw `count` coins (1 = attack) packed into uint32 words."""
        words = max(1, (count + 31) // 32) if words is None else words
        buf = np.zeros(words, np.uint32)
        _check(self.lib, self.lib.ba_mt_draw_coins(ctypes.byref(self.st), count, buf.ctypes.data,
                                                   words))
        return buf


def om1_coin_count(n: int, m: int, faulty_mask: int, poll: int = 0) -> int:
    return int(load().ba_om1_coin_count(n, m, faulty_mask, poll))


def mt_table(n, m, seeds, faulty, poll=None, threads=0):
    """Batched ba.py replay table: (table[batch, stride] uint32, next_word[batch] uint32)."""
    lib = load()
    seeds = np.ascontiguousarray(seeds, np.uint64)
    faulty = np.ascontiguousarray(faulty, np.uint32)
    poll = None if poll is None else np.ascontiguousarray(poll, np.uint32)
    stride = table_stride(n)
    tab = np.zeros((len(seeds), stride), np.uint32)
    nxt = np.zeros(len(seeds), np.uint32)
    _check(lib, lib.ba_mt_table(n, m, len(seeds), seeds.ctypes.data, faulty.ctypes.data,
                                _ptr(poll), stride, tab.ctypes.data, nxt.ctypes.data, threads))
    return tab, nxt


def vote_slots(n: int, m: int, j_begin: int, j_end: int) -> int:
    """Vote slots of first-hop subtrees [j_begin, j_end) per 64-trial word."""
    return int(load().ba_vote_slots(n, m, j_begin, j_end))


def pack_coins(rows, n):
    """Pack per-trial coin lists (1 = attack) into a (batch, stride) uint32 table."""
    stride = table_stride(n)
    tab = np.zeros((len(rows), stride), np.uint32)
    for i, coins in enumerate(rows):
        for c, v in enumerate(coins):
            if v:
                tab[i, c >> 5] |= np.uint32(1 << (c & 31))
    return tab
