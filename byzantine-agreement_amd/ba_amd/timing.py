"""Election and heartbeat timing of ba.py, emulated on a virtual clock
(SURVEY.md §8f row 4).

ba.py gives every general a `run` thread (ba.py:295-319) that sleeps 0.1 s,
exits if killed, and -- unless it is primary -- connects to its primary_port as
a heartbeat (ba.py:306-310); a failed connect starts an election (`elect`,
ba.py:126-157: win if no reachable general has a lower id, then broadcast
`new_leader` and become primary for life).  The same loop computes a
lieutenant's majority once an order has arrived (ba.py:318-319), and the REPL
waits for each general's majority by polling every 0.1 s (`wait_majority`,
ba.py:287-289).  So what ba.py prints depends on WHEN commands arrive relative
to those ticks: a `g-state` typed before the first tick shows every general
as secondary, an `actual-order` then fails the primary assert (ba.py:259), and
a killed primary is replaced one tick later by the lowest live id.

`TimedCluster` replays that on a virtual clock instead of threads and sleeps:

  * general g's loop wakes at start_g + k * period (k >= 1); start_g is the
    time its `start()` ran (all at t=0 for `python3 ba.py N`, the time of the
    `g-add` for later ones), plus an optional deterministic per-general phase
    (`jitter`, seeded) standing in for thread start-up skew;
  * ticks are processed in time order (ties: lower id first), each running
    ba.py:303-319 on the membership state of `generals.Cluster`, which already
    restates discover_leader / elect / kill / add exactly;
  * RPCs take zero virtual time (ba.py's localhost connects are ~ms against the
    100 ms ticks).

The emulator only decides timing and roles.  The majority VALUES of an
`actual-order` still come from one batch=1 libba_hip call (Cluster.actual_order),
so this module adds no CPU decision path.  Every event is logged as
(time, kind, general id, detail) for tests and demos.
"""
from __future__ import annotations

import heapq
import random

from .generals import Cluster, General

PERIOD = 0.1       # run-loop sleep, ba.py:301
WAIT_POLL = 0.1    # wait_majority poll, ba.py:287-289


class TimedCluster(Cluster):
    """A Cluster whose membership changes happen on ba.py's tick schedule."""

    def __init__(self, n: int, seed: int | None = None, om: int = 1, engine=None,
                 device: int = 0, period: float = PERIOD, jitter: float = 0.0,
                 jitter_seed: int = 0):
        self.now = 0.0
        self.period = period
        self.jitter = jitter
        self._rng = random.Random(jitter_seed)
        self._heap: list[tuple[float, int, int]] = []  # (time, id, port)
        self.events: list[tuple[float, str, int, str]] = []
        self.pending: dict[int, bool] = {}  # port -> order received, majority not yet taken
        self._dead: dict[int, General] = {}  # killed generals whose thread has not exited yet
        self.last_round_latency = None
        super().__init__(n, seed=seed, om=om, engine=engine, device=device)
        for g in self.processes:  # __main__ starts every process at t=0 (ba.py:362-363)
            self._schedule_first(g)

    # ---- clock ----------------------------------------------------------------
    def _schedule_first(self, g: General):
        phase = self._rng.uniform(0.0, self.jitter) if self.jitter > 0 else 0.0
        heapq.heappush(self._heap, (round(self.now + phase + self.period, 9), g.id, g.port))

    def _log(self, kind: str, g: General, detail: str = ""):
        self.events.append((round(self.now, 9), kind, g.id, detail))

    def _tick(self, g: General):
        """One iteration of Process.run after its sleep (ba.py:303-319)."""
        if g.killed:  # ba.py:303-304: the thread exits
            self._dead.pop(g.port, None)
            self._log("exit", g)
            return False
        if not g.primary:
            if self._reachable(g.primary_port) is None:  # heartbeat connect fails, ba.py:306-310
                self._log("heartbeat-fail", g, str(g.primary_port))
                self._elect(g)
                self._log("elect-win" if g.primary else "elect-lose", g)
            if self.pending.get(g.port):  # ba.py:318-319: the majority is taken now
                self.pending[g.port] = False
                self._log("majority", g)
        return True

    def advance_to(self, t: float):
        """Run every tick due at or before virtual time t, in time order."""
        while self._heap and self._heap[0][0] <= t + 1e-12:
            when, gid, port = heapq.heappop(self._heap)
            self.now = when
            g = self.live.get(port) or self._dead.get(port)
            if g is None:
                continue
            if self._tick(g):
                heapq.heappush(self._heap, (round(when + self.period, 9), gid, port))
        self.now = max(self.now, t)

    def advance(self, dt: float):
        self.advance_to(self.now + dt)

    # ---- membership with timing -------------------------------------------------
    def kill(self, gid: int) -> bool:
        i = self.index_of(gid)
        if i is None:
            return False
        g = self.processes[i]
        ok = super().kill(gid)
        self._dead[g.port] = g  # its run thread notices at its next tick
        self._log("kill", g, "primary" if g.primary else "")
        return ok

    def add(self, k: int):
        before = len(self.processes)
        super().add(k)
        for g in self.processes[before:]:
            self._log("add", g, f"primary_port={g.primary_port}")
            self._schedule_first(g)

    def tick(self):
        """The canonical schedule's tick is replaced by the clock: no-op."""

    # ---- orders ------------------------------------------------------------------
    def primary(self) -> General | None:
        for g in self.processes:
            if g.primary:
                return g
        return None

    def round_timing(self) -> float:
        """Issue an order at the current time and advance the clock through the
        REPL's wait_majority loop (ba.py:287-289, in process order); returns the
        round's virtual latency.  The primary decides at once (ba.py:285),
        a lieutenant at its next tick (ba.py:318-319)."""
        t0 = self.now
        for g in self.processes[1:]:
            self.pending[g.port] = True
        for g in self.processes[1:]:
            if g.primary:  # never takes a majority (ba.py:306): ba.py would wait forever
                raise RuntimeError(f"G{g.id} is primary but not the commander: ba.py hangs here")
            while self.pending.get(g.port):
                self.advance(WAIT_POLL)
        self.pending.clear()
        return self.now - t0

    def actual_order(self, order: str):
        """ba.py's `actual-order`: the primary assert, the majorities (one
        libba_hip call), and the clock advanced by the round's wait."""
        res = super().actual_order(order)
        self.last_round_latency = self.round_timing()
        return res

    def failover_time(self) -> float | None:
        """Virtual time from the last kill of a primary to the next election
        win, from the event log (None if not both present)."""
        kill_t = None
        for t, kind, gid, detail in self.events:
            if kind == "kill" and detail == "primary":
                kill_t = t
            elif kind == "elect-win" and kill_t is not None and t >= kill_t:
                return t - kill_t
        return None


def run_timed(cluster: TimedCluster, timed_lines, out, execute):
    """REPL over (time, line) pairs: the clock runs to each command's arrival
    time, then the command executes against whatever the ticks have done."""
    for t, line in timed_lines:
        cluster.advance_to(max(t, cluster.now))
        if not execute(cluster, line.rstrip("\n"), out):
            break
