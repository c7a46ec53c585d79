"""The Byzantine generals of ba.py as host-side bookkeeping over libba_hip.

ba.py (mathiasplans/byzantine-agreement) runs one `Process` per general, each
with an rpyc server thread and a 0.1 s polling loop (ba.py:66-319).  Here a
general is a plain record; membership (discover_leader, elect, kill, add) is
replayed exactly as ba.py's canonical single-threaded schedule runs it, and an
`actual-order` round is ONE batch=1 call into libba_hip.so (ba_run_trials):

  * the live generals sorted by id become indices 0..n-1 (0 = commander,
    the lowest live id, which ba.py's lowest-id election makes primary);
  * `faulty` flags become the trial's faulty mask (ba.py:401-407);
  * a lieutenant whose primary_port is stale also polls the commander
    (ba.py:171 skips only the port it believes is the primary's) -> poll mask;
  * ba.py's coins come from the C++ MT19937 replay (ba_mt_*) in its canonical
    draw order, fed to the kernel as a BA_LIE_TABLE row -- so a seeded round
    reproduces ba.py's output byte for byte (tests/golden/repl_transcripts.json).

With om > 1 the round is OM(om) instead (no reference code; SURVEY.md
Appendix A): lies come from Philox keyed by (seed, round).  No decision is
computed in Python: without a HIP device `actual_order` raises.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

from . import lib as L

BASE_PORT = 18812  # ba.py:355
CODE_TEXT = {L.RETREAT: "retreat", L.ATTACK: "attack", L.UNDEFINED: "undefined"}


@dataclass
class General:
    """ba.py Process state that the protocol reads (ba.py:66-77)."""
    id: int
    port: int
    primary: bool = False
    primary_port: int = -1
    faulty: bool = False
    killed: bool = False


class Cluster:
    """The generals of one ba.py program run (`python3 ba.py N`)."""

    def __init__(self, n: int, seed: int | None = None, om: int = 1, engine=None, device: int = 0):
        if seed is None:  # ba.py never seeds its RNG
            seed = int.from_bytes(os.urandom(8), "little")
        self.om = om
        self.seed = seed
        self.mt = L.MT(seed) if om <= 1 else None
        self.rounds = 0
        self._engine = engine
        self._device = device
        self.others: list[int] = []  # every port ever created (ba.py:13, never shrinks)
        self.live: dict[int, General] = {}  # port -> general with a running server
        self.processes: list[General] = []  # ba.py:357, sorted by id
        self._next_id, self._next_port = 1, BASE_PORT  # gen_processes, ba.py:344-351
        for _ in range(n):
            self._spawn()
        for p in list(self.processes):
            self._discover_leader(p)  # Process.start, ba.py:104-108

    # ---- membership (ba.py:86-157, 322-351) --------------------------------
    def _spawn(self) -> General:
        g = General(self._next_id, self._next_port)
        self._next_id += 1
        self._next_port += 1
        self.processes.append(g)
        self.others.append(g.port)
        self.live[g.port] = g
        return g

    def _reachable(self, port: int) -> General | None:
        return self.live.get(port)

    def _discover_leader(self, g: General):
        for port in self.others:  # ba.py:86-102
            if port == g.port:
                continue
            peer = self._reachable(port)
            if peer is None:
                continue
            g.primary_port = peer.primary_port
            if g.primary_port != -1:
                break

    def _elect(self, g: General):
        lowest = True  # ba.py:126-157
        for port in self.others:
            if port == g.port:
                continue
            peer = self._reachable(port)
            if peer is not None and peer.id < g.id:
                lowest = False
                break
        if lowest:
            for port in self.others:
                peer = self._reachable(port) if port != g.port else None
                if peer is not None:
                    peer.primary_port = g.port
            g.primary = True
        else:
            g.primary = False

    def tick(self):
        """One pass of every general's run loop liveness check (ba.py:300-314)."""
        for g in self.processes:
            if g.primary:
                continue
            if self._reachable(g.primary_port) is None:
                self._elect(g)

    def index_of(self, gid: int) -> int | None:
        """id_to_index (ba.py:322-342): position of id in the sorted list, or None."""
        for i, g in enumerate(self.processes):
            if g.id == gid:
                return i
        return None

    def kill(self, gid: int) -> bool:
        i = self.index_of(gid)
        if i is None:
            return False
        g = self.processes.pop(i)  # ba.py:415-425
        g.killed = True
        self.live.pop(g.port, None)
        return True

    def add(self, k: int):
        for _ in range(k):  # ba.py:427-437
            self._discover_leader(self._spawn())

    def set_faulty(self, gid: int, faulty: bool) -> bool:
        i = self.index_of(gid)
        if i is None:
            return False
        self.processes[i].faulty = faulty
        return True

    # ---- the hot path: one round through libba_hip --------------------------
    @property
    def engine(self):
        if self._engine is None:
            self._engine = L.Engine(self._device)
        return self._engine

    def round_inputs(self, order: str):
        """(n, faulty mask, poll mask, order code) of the live generals."""
        procs = self.processes
        n = len(procs)
        fm = sum(1 << i for i, g in enumerate(procs) if g.faulty)
        cport = procs[0].port
        pm = sum(1 << i for i, g in enumerate(procs) if i > 0 and g.primary_port != cport)
        oc = {"attack": L.ATTACK, "retreat": L.RETREAT}.get(order, L.OTHER)
        return n, fm, pm, oc

    def actual_order(self, order: str) -> tuple[list[str], int]:
        """Process.order + every lieutenant's get_majority (ba.py:257-285,
        159-195) as one kernel call.  Returns (majority strings in process
        order, quorum code)."""
        if not self.processes:
            raise IndexError("list index out of range")  # ba.py:381 processes[0]
        if not self.processes[0].primary:
            raise AssertionError("commander is not primary")  # ba.py:259
        n, fm, pm, oc = self.round_inputs(order)
        if self.om <= 1:
            count = L.om1_coin_count(n, self.om, fm, pm)
            table = self.mt.coins(count, L.table_stride(n))[None, :]
            res = self.engine.run(n, self.om, 1, lie_mode=L.LIE_TABLE, faulty=[fm], order=[oc],
                                  table=table, poll=[pm])
        else:
            res = self.engine.run(n, self.om, 1, seed=self.seed, faulty=[fm], order=[oc],
                                  first_trial=64 * self.rounds)
        self.rounds += 1
        majorities = [order] + [CODE_TEXT[res.decision(0, r)] for r in range(1, n)]  # ba.py:285
        return majorities, int(res.outcome[0]) & 3

    # ---- ba.py-format text ---------------------------
    @staticmethod
    def quorum_line(majorities: list[str], nr_faulty: int, q: int) -> str:
        """Process.quorum's printout (ba.py:225-255) from the round's tally.  The
        quorum decision itself (q) comes from the kernel's epilogue."""
        na = sum(m == "attack" for m in majorities)
        nr = sum(m == "retreat" for m in majorities)
        total = len(majorities)
        nu = total - na - nr
        k = (total - 1) // 3
        needed = 2 * k + 1
        if total <= 3:
            needed = total - 1
        if total == 1:
            needed = 1
        ft = f"{nr_faulty} faulty node(s) in the system" if nr_faulty > 0 else \
            "Non-faulty nodes in the system"
        if q == L.Q_RETREAT:
            d = f"retreat! {ft} - {needed} out of {total} quorum suggests retreat"
        elif q == L.Q_ATTACK:
            d = f"attack! {ft} - {needed} out of {total} quorum suggests attack"
        else:
            d = (f"cannot be determined - not enough generals in the system! {ft} - "
                 f"{nu} out of {total} quorum not consistent")
        return f"Execute order: {d}"
