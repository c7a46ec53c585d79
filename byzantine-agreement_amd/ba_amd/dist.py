"""Multi-GPU layer: one process per GPU, torch.distributed over
RCCL/xGMI ("nccl" on ROCm), gloo for CPU tests.

Two ways the OM(m) hot path shards:

* Trial data-parallel (configs 2-4).  Trials are independent and every random
  draw is keyed by the GLOBAL trial index, so contiguous word-aligned trial
  ranges per rank give bit-identical results to one unsharded run.  No data-path
  collective: the only exchange is one all-reduce(SUM) of the 16 uint64 run
  counters at the end.
* One huge instance split by first-hop subtree (config 5, n=16 m=5: 4M tree
  slots).  Rank r owns lieutenants [jb, je) as first hops; each subtree's relay
  levels and inner majorities need only L_0[j].  Ranks exchange their level-1
  child results (the votes every lieutenant counts about j) with ONE all-gather
  of (n-1)(n-2) x W words in total, then every rank finishes the root
  majorities + quorum (ba.py:159-255) on the gathered votes.

The "backend" object does the device work; DeviceBackend wraps a libba_hip
Engine on one GPU (torch owns the buffers and the stream).  Tests substitute a
CPU stand-in to exercise this module with gloo.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import lib as L


def _rank_world(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def word_shard(total_trials: int, rank: int, world: int):
    """(first trial, count) of rank's contiguous share, whole 64-trial words,
    words split as evenly as possible."""
    words = (total_trials + 63) // 64
    w0 = words * rank // world
    w1 = words * (rank + 1) // world
    first = w0 * 64
    return first, max(0, min(total_trials, w1 * 64) - first)


def subtree_ranges(n_lieutenants: int, world: int):
    """Contiguous first-hop ranges [jb, je) per rank (15 over 8 -> 1,2,2,2,2,2,2,2)."""
    return [(n_lieutenants * r // world, n_lieutenants * (r + 1) // world) for r in range(world)]


class DeviceBackend:
    """libba_hip on one GPU through torch tensors (device pointers + stream)."""

    def __init__(self, engine: L.Engine, device: torch.device, stream: torch.cuda.Stream | None = None):
        self.engine = engine
        self.device = device
        self.stream = stream or torch.cuda.current_stream(device)

    def counters(self):
        return torch.zeros(16, dtype=torch.int64, device=self.device)

    def run_trials(self, params: L.Params, batch: int, counters: torch.Tensor,
                   decisions: torch.Tensor | None = None, outcome: torch.Tensor | None = None):
        self.engine.run_device(params, batch,
                               d_decisions=decisions.data_ptr() if decisions is not None else 0,
                               d_outcome=outcome.data_ptr() if outcome is not None else 0,
                               d_counters=counters.data_ptr(), stream=self.stream.cuda_stream)

    def subtree_votes(self, params: L.Params, batch: int, jb: int, je: int) -> torch.Tensor:
        W = (batch + 63) // 64
        v = torch.empty((L.vote_slots(params.n, params.m, jb, je), W), dtype=torch.int64,
                        device=self.device)
        self.engine.subtree_votes_device(params, batch, jb, je, v.data_ptr(),
                                         stream=self.stream.cuda_stream)
        return v

    def root_from_votes(self, params: L.Params, batch: int, votes: torch.Tensor):
        dec = torch.empty(batch, dtype=torch.int64, device=self.device)
        out = torch.empty(batch, dtype=torch.uint8, device=self.device)
        cnt = self.counters()
        votes = votes.contiguous()
        self.engine.root_from_votes_device(params, batch, votes.data_ptr(), cnt.data_ptr(),
                                           d_decisions=dec.data_ptr(), d_outcome=out.data_ptr(),
                                           stream=self.stream.cuda_stream)
        return dec, out, cnt


def run_trials_dp(backend, n: int, m: int, total_trials: int, *, seed: int = 0xBA5EED,
                  faulty_mode: int = L.FAULTY_RANDOM, f: int | None = None,
                  order_mode: int = L.ORDER_RANDOM, order_value: int = L.ATTACK,
                  engine: int = L.ENGINE_AUTO, base_trial: int = 0, chunk: int = 1 << 22,
                  group=None) -> torch.Tensor:
    """Resolve trials [base_trial, base_trial + total_trials) across the group;
    returns the all-reduced counters (int64[16], same on every rank).  Each
    rank processes its share in chunks of at most `chunk` trials."""
    rank, world = _rank_world(group)
    f = L.default_fmax(n) if f is None else f
    first, count = word_shard(total_trials, rank, world)
    cnt = backend.counters()
    done = 0
    while done < count:
        b = min(chunk, count - done)
        p = L.make_params(n, m, seed, L.LIE_PHILOX, faulty_mode, f, order_mode, order_value,
                          engine, base_trial + first + done)
        backend.run_trials(p, b, cnt)
        done += b
    if world > 1:
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM, group=group)
    return cnt


def run_instance_split(backend, params: L.Params, batch: int, group=None):
    """First-hop subtree split of `batch` instances (normally a few huge ones).
    Returns (decisions, outcome, counters) -- identical on every rank and equal
    to an unsplit ba_run_trials on the same params."""
    rank, world = _rank_world(group)
    Lts = params.n - 1
    ranges = subtree_ranges(Lts, world)
    jb, je = ranges[rank]
    W = (batch + 63) // 64
    per = max(b - a for a, b in ranges) * (params.n - 2)
    buf = torch.zeros((per, W), dtype=torch.int64, device=backend.device)
    if je > jb:
        local = backend.subtree_votes(params, batch, jb, je)
        buf[:local.shape[0]] = local
    if world > 1:
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf, group=group)
    else:
        parts = [buf]
    full = torch.cat([parts[r][:(b - a) * (params.n - 2)] for r, (a, b) in enumerate(ranges)])
    return backend.root_from_votes(params, batch, full)


class InstanceSplitGraphs:
    """run_instance_split with the launch sequence captured in hipGraphs.

    A config-5 call (n=16, m=5) is ~17 kernels, most of them small (input
    bit-slicing, the fused top relay, three inner majority levels, the root
    epilogue, the counter reduction), so at small batches the launch gaps cost
    about as much as the work.  The local halves of the split are captured once
    per (params, batch) and replayed: graph 1 = this rank's subtree votes into a
    fixed buffer, graph 2 = root majorities + quorum over the gathered votes.
    The all-gather between them (world > 1) stays an eager RCCL call, so the
    graphs hold no collective.  Outputs are the same tensors on every replay
    (overwritten); results equal run_instance_split's bit for bit (GPU test).
    """

    def __init__(self, engine: L.Engine, device: torch.device, params: L.Params, batch: int,
                 group=None):
        self.engine, self.device, self.params, self.batch, self.group = engine, device, params, batch, group
        self.rank, self.world = _rank_world(group)
        n = params.n
        self.ranges = subtree_ranges(n - 1, self.world)
        self.jb, self.je = self.ranges[self.rank]
        W = (batch + 63) // 64
        self.rows = [L.vote_slots(n, params.m, a, b) for a, b in self.ranges]
        self.stream = torch.cuda.Stream(device)
        self.buf = torch.zeros((max(self.rows), W), dtype=torch.int64, device=device)
        self.full = (self.buf if self.world == 1 else
                     torch.zeros((sum(self.rows), W), dtype=torch.int64, device=device))
        self.gathered = (None if self.world == 1 else
                         torch.zeros((self.world, max(self.rows), W), dtype=torch.int64, device=device))
        self.dec = torch.empty(batch, dtype=torch.int64, device=device)
        self.out = torch.empty(batch, dtype=torch.uint8, device=device)
        self.cnt = torch.zeros(16, dtype=torch.int64, device=device)
        with torch.cuda.stream(self.stream):  # warm-up: geometry upload, scratch growth
            self._tree()
            self._gather()
            self._root()
        torch.cuda.synchronize(device)
        if self.world == 1:  # no collective: one graph for the whole call
            self.g_tree = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_tree, stream=self.stream):
                self._tree()
                self._root()
            self.g_root = None
        else:
            self.g_tree = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_tree, stream=self.stream):
                self._tree()
            self.g_root = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_root, stream=self.stream):
                self._root()

    def _tree(self):
        if self.je > self.jb:
            self.engine.subtree_votes_device(self.params, self.batch, self.jb, self.je,
                                             self.buf.data_ptr(),
                                             stream=self.stream.cuda_stream)

    def _gather(self):
        if self.world == 1:
            return
        dist.all_gather([self.gathered[r] for r in range(self.world)], self.buf, group=self.group)
        o = 0
        for r, k in enumerate(self.rows):
            self.full[o:o + k].copy_(self.gathered[r, :k])
            o += k

    def _root(self):
        self.cnt.zero_()
        self.engine.root_from_votes_device(self.params, self.batch, self.full.data_ptr(),
                                           self.cnt.data_ptr(), d_decisions=self.dec.data_ptr(),
                                           d_outcome=self.out.data_ptr(),
                                           stream=self.stream.cuda_stream)

    def replay(self):
        """One split call; returns (decisions, outcome, counters) (reused tensors).
        Ordered after the caller's current stream and before its later work."""
        if self.g_root is None:  # replays on the caller's current stream
            self.g_tree.replay()
            return self.dec, self.out, self.cnt
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            self.g_tree.replay()
            self._gather()
            self.g_root.replay()
        cur.wait_stream(self.stream)
        return self.dec, self.out, self.cnt
