"""Multi-GPU host layer: one process per GPU, collectives inside
the C ABI.

The data path's collectives live in libba_hip (csrc/ba_multi.cpp, include/ba.h
"multi-GPU"): the library owns the RCCL communicator (ba_comm_*), shards the
work (ba_trial_share, ba_subtree_share) and runs exactly the exchange each
sharding needs -- an all-reduce of the 16 run counters for trial-DP, one vote
all-gather for the first-hop split.  torch.distributed is only the launcher's
rendezvous here: it carries RCCL's 128-byte unique id from rank 0 to every rank
(rendezvous_uid), and bench.py uses its barrier and a max-over-ranks of the
wall time.  So a host without torch gets the same multi-GPU path through the
C ABI alone, and there is one implementation of it.

Two ways the OM(m) hot path shards:

* Trial data-parallel (configs 2-4).  Trials are independent and every random
  draw is keyed by the GLOBAL trial index, so contiguous word-aligned trial
  ranges per rank give bit-identical results to one unsharded run.
* One huge instance split by subtree (config 5, n=16 m=5: 4M tree slots).
  At level 1 rank r owns lieutenants [jb, je) as first hops; each subtree's
  relay levels and inner majorities need only L_0[j].  Ranks exchange their
  level-1 child results (the votes every lieutenant counts about j), then
  every rank finishes the root majorities + quorum (ba.py:159-255).  At level 2
  the units are the (n-1)(n-2) second-hop subtrees (210 at n=16: 26/27 per
  rank over 8 ranks instead of 1-2 of 15 first hops), the exchange is their
  level-2 results, and every rank also takes the level-1 majorities.
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
    """(first trial, count) of rank's contiguous share (ba_trial_share)."""
    return L.trial_share(total_trials, world, rank)


def subtree_ranges(n_lieutenants: int, world: int):
    """First-hop ranges [jb, je) per rank (ba_subtree_share; 15 over 8 -> 1,2,...,2)."""
    return [L.subtree_share(n_lieutenants + 1, world, r) for r in range(world)]


def rendezvous_uid(group=None, make_uid=L.comm_unique_id) -> bytes:
    """RCCL unique id made on rank 0, delivered to every rank of the group."""
    rank, world = _rank_world(group)
    box = [make_uid() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(box, src=0, group=group)
    return box[0]


def init_comm(engine: L.Engine, group=None) -> L.Comm:
    """The C-ABI communicator of this rank (one GPU per process)."""
    rank, world = _rank_world(group)
    return L.Comm(engine, world, rank, rendezvous_uid(group))


def run_trials_dp(comm: L.Comm, n: int, m: int, total_trials: int, *, seed: int = 0xBA5EED,
                  faulty_mode: int = L.FAULTY_RANDOM, f: int | None = None,
                  order_mode: int = L.ORDER_RANDOM, order_value: int = L.ATTACK,
                  engine: int = L.ENGINE_AUTO, base_trial: int = 0) -> dict:
    """Resolve trials [base_trial, base_trial + total_trials) across the comm's ranks
    (ba_run_trials_multi); returns the whole job's counters (same on every rank)."""
    f = L.default_fmax(n) if f is None else f
    p = L.make_params(n, m, seed, L.LIE_PHILOX, faulty_mode, f, order_mode, order_value, engine,
                      base_trial)
    counters, _, _ = comm.run_trials(p, total_trials)
    return counters


def split_ranges(n: int, m: int, level: int, world: int):
    """Unit ranges [u_begin, u_end) per rank of a split level (ba_split_share;
    level 2 at n=16 over 8 ranks: 26/27 of 210 second-hop subtrees each)."""
    return [L.split_share(n, m, level, world, r) for r in range(world)]


def run_instance_split(comm: L.Comm, params: L.Params, batch: int, device: torch.device,
                       level: int = L.SPLIT_FIRST_HOP):
    """Subtree split of `batch` instances at `level` (1: first hop, 2: second hop;
    ba_run_instance_split_level_multi).  Returns (decisions int64[batch], outcome
    uint8[batch], counters dict) -- identical on every rank and equal to an
    unsplit ba_run_trials."""
    dec = torch.empty(batch, dtype=torch.int64, device=device)
    out = torch.empty(batch, dtype=torch.uint8, device=device)
    torch.cuda.current_stream(device).synchronize()  # the comm's stream runs the job
    cnt = comm.run_instance_split(params, batch, d_decisions=dec.data_ptr(),
                                  d_outcome=out.data_ptr(), level=level)
    return dec, out, cnt


class InstanceSplitGraphs:
    """The first-hop split with its launch sequence captured in hipGraphs.

    A config-5 call (n=16, m=5) is 6-10 kernels, most of them small, so at small
    batches the launch gaps cost about as much as the work.  The local halves of
    the split are captured once per (params, batch) and replayed: with one rank
    (which owns every subtree) the call is the unsplit pass, one graph; with N
    ranks graph 1 = this rank's subtree votes into its rows of the full vote
    array, then the C-ABI vote all-gather (RCCL, eager), then graph 2 = root
    majorities + quorum.  The graphs run on their own
    Engine (ctx): the device buffers they captured (scratch, counter sink) can
    never be regrown under them by another caller of a shared ctx.  Outputs are
    the same tensors on every replay (overwritten); results equal the eager split
    bit for bit (GPU test).
    """

    def __init__(self, device: torch.device, params: L.Params, batch: int,
                 comm: L.Comm | None = None, level: int = L.SPLIT_FIRST_HOP):
        self.device, self.params, self.batch, self.comm = device, params, batch, comm
        self.level = level
        self.world = comm.nranks if comm is not None else 1
        self.rank = comm.rank if comm is not None else 0
        self.engine = L.Engine(device.index)  # own ctx: nothing else grows its scratch
        n, m = params.n, params.m
        units = L.split_units(n, m, level)
        if units == 0:
            raise L.BAError(L.ENOTSUP, f"no level-{level} split for n={n}, m={m}")
        self.jb, self.je = L.split_share(n, m, level, self.world, self.rank)
        W = (batch + 63) // 64
        self.row = (n - 1 - level) * W  # vote words per unit
        self.stream = torch.cuda.Stream(device)
        self.votes = torch.zeros((L.split_vote_slots(n, m, level, 0, units), W), dtype=torch.int64,
                                 device=device)
        self.dec = torch.empty(batch, dtype=torch.int64, device=device)
        self.out = torch.empty(batch, dtype=torch.uint8, device=device)
        self.cnt = torch.zeros(16, dtype=torch.int64, device=device)
        # the warm-up (geometry upload, scratch growth) runs after the tensors'
        # initialisation on the current stream
        self.stream.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(self.stream):
            if self.world == 1:
                self._whole()
            else:
                self._tree()
                self._gather()
                self._root()
        torch.cuda.synchronize(device)
        if self.world == 1:  # one rank, no collective: the unsplit pass as one graph
            self.g_tree = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_tree, stream=self.stream):
                self._whole()
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
            per = self.params.n - 1 - self.level
            self.engine.split_votes_device(self.params, self.batch, self.level, self.jb, self.je,
                                           self.votes[self.jb * per:].data_ptr(),
                                           stream=self.stream.cuda_stream)

    def _whole(self):
        self.cnt.zero_()
        self.engine.run_device(self.params, self.batch, d_decisions=self.dec.data_ptr(),
                               d_outcome=self.out.data_ptr(), d_counters=self.cnt.data_ptr(),
                               stream=self.stream.cuda_stream)

    def _gather(self):
        if self.world > 1:
            self.comm.allgather_split_votes_device(self.params.n, self.params.m, self.level,
                                                   self.batch, self.votes.data_ptr(),
                                                   stream=self.stream.cuda_stream)

    def _root(self):
        self.cnt.zero_()
        self.engine.root_from_split_votes_device(self.params, self.batch, self.level,
                                                 self.votes.data_ptr(), self.cnt.data_ptr(),
                                                 d_decisions=self.dec.data_ptr(),
                                                 d_outcome=self.out.data_ptr(),
                                                 stream=self.stream.cuda_stream)

    def replay(self):
        """One split call; returns (decisions, outcome, counters) (reused tensors).
        Ordered after the caller's current stream and before its later work.
        Asynchronous: after synchronizing, L.check_handoff(counters) (a lost
        in-launch hand-off makes the call's results invalid; a graph replays its
        launch's epoch, so after such an error the graphs must be rebuilt)."""
        if self.g_root is None:  # one graph, replayed on the caller's current stream
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

    def close(self):
        self.engine.close()
