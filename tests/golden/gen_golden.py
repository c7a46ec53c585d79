"""Generate golden fixtures from the reference ba.py (dev container only).

Runs /root/reference/ba.py (mathiasplans/byzantine-agreement) itself, unchanged,
over an in-process fake `rpyc` transport (rpyc is not installed and there is no
network).  Every general's Serv is registered in a port ->
service dict, `rpyc.connect` resolves `c.root.<name>` to
`service.exposed_<name>`, and closed/unknown ports raise ConnectionRefusedError,
which ba.py already swallows (ba.py:100-102, 185-186, 219-221, 281-282).

Parity is defined under ba.py's CANONICAL single-threaded schedule (the real
program interleaves an unseeded global RNG across threads, ba.py:45/269, so its
draw order is not reproducible):
  1. create/start generals (ba.py:355-363), run one election tick per general
     (ba.py:306-314) before every command;
  2. random.seed(seed);
  3. processes[0].order(o)                                     (ba.py:381)
  4. get_majority on every lieutenant in id order              (ba.py:318-319, 385-386)
  5. processes[0].quorum(nr_faulty), stdout captured           (ba.py:395)

Outputs (committed, small):
  om1_cases.json       structured OM(1) cases: live ids, faulty flags, order,
                       the coins in draw order, every general's majority, the
                       quorum line and the next MT word after the round.
  repl_transcripts.json  command scripts fed to ba.py's own __main__ loop
                       (ba.py:354-445) with the canonical schedule, and the
                       exact stdout it printed.

This script refuses to run when /root/reference is absent (the GPU box never
has it); the fixtures it wrote are what travel.
"""
from __future__ import annotations

import contextlib
import functools
import importlib.util
import io
import json
import os
import random
import sys
import types

REF = "/root/reference/ba.py"
HERE = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------
# fake rpyc transport
# --------------------------------------------------------------------------
def install_fake_rpyc():
    registry: dict[int, object] = {}

    rpyc = types.ModuleType("rpyc")
    utils = types.ModuleType("rpyc.utils")
    server = types.ModuleType("rpyc.utils.server")
    helpers = types.ModuleType("rpyc.utils.helpers")

    class Service:  # rpyc.Service stand-in: plain base class
        pass

    class _Root:
        def __init__(self, svc):
            self._svc = svc

        def __getattr__(self, name):
            return getattr(self._svc, "exposed_" + name)

    class _Conn:
        def __init__(self, svc):
            self.root = _Root(svc)

        def close(self):
            pass

    def connect(host, port):
        svc = registry.get(port)
        if svc is None:
            raise ConnectionRefusedError(f"port {port}")
        return _Conn(svc)

    class ThreadedServer:
        def __init__(self, factory, port):
            self.port = port
            registry[port] = factory()

        def start(self):
            pass

        def close(self):
            registry.pop(self.port, None)

    rpyc.Service = Service
    rpyc.connect = connect
    server.ThreadedServer = ThreadedServer
    helpers.classpartial = functools.partial
    rpyc.utils = utils
    utils.server = server
    utils.helpers = helpers
    sys.modules.update({"rpyc": rpyc, "rpyc.utils": utils,
                        "rpyc.utils.server": server, "rpyc.utils.helpers": helpers})
    return registry


class CoinRecorder:
    """Wraps random.randint to record ba.py's coins in draw order (1 = attack)."""

    def __init__(self):
        self.orig = random.randint
        self.coins: list[int] = []

    def __enter__(self):
        def rec(a, b):
            v = self.orig(a, b)
            self.coins.append(1 if v == 0 else 0)  # ba.py:45/269: 0 -> "attack"
            return v
        random.randint = rec
        return self

    def __exit__(self, *exc):
        random.randint = self.orig


def load_ba(n: int):
    """Import ba.py as a module (module-level code only, ba.py:1-351)."""
    install_fake_rpyc()
    sys.argv = ["ba.py", str(n)]  # ba.py:12
    spec = importlib.util.spec_from_file_location("ba_ref", REF)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def election_tick(mod, procs):
    """One pass of the run-loop's liveness check (ba.py:306-314) per general."""
    for p in procs:
        if p.primary:
            continue
        try:
            c = sys.modules["rpyc"].connect("localhost", p.primary_port)
            c.close()
        except Exception:
            p.elect()


# --------------------------------------------------------------------------
# structured OM(1) cases
# --------------------------------------------------------------------------
def om1_case(rng: random.Random, idx: int) -> dict:
    n0 = rng.choice([1, 2, 3, 4, 4, 4, 5, 6, 7, 8, 10, 13, 16, 20])
    mod = load_ba(n0)
    pgen = mod.gen_processes(18812)  # ba.py:355
    procs = []
    for _ in range(n0):
        port, p = next(pgen)
        procs.append(p)
        mod.others.append(port)
    for p in procs:
        p.discover_leader()  # ba.py:105
    election_tick(mod, procs)
    # optional crash injection (g-kill, ba.py:415-425) and joins (g-add, ba.py:427-437)
    kills = []
    if n0 > 1 and rng.random() < 0.35:
        for gid in rng.sample([p.id for p in procs], rng.randint(1, min(3, n0 - 1))):
            i = mod.id_to_index(procs, gid)
            procs[i].kill()
            del procs[i]
            kills.append(gid)
        election_tick(mod, procs)
    adds = 0
    if rng.random() < 0.25:
        adds = rng.randint(1, 3)
        for _ in range(adds):
            port, p = next(pgen)
            procs.append(p)
            mod.others.append(port)
            p.discover_leader()
        election_tick(mod, procs)
    pf = rng.choice([0.0, 0.2, 0.34, 0.5])
    for p in procs:
        p.faulty = rng.random() < pf  # g-state <id> faulty, ba.py:407
    if rng.random() < 0.15 and procs:
        procs[0].faulty = True
    order = rng.choice(["attack"] * 5 + ["retreat"] * 5 + ["foo"])
    seed = rng.randrange(1 << 31)
    random.seed(seed)
    out = io.StringIO()
    with CoinRecorder() as rec, contextlib.redirect_stdout(out):
        procs[0].order(order)  # ba.py:381
        for p in procs[1:]:
            p.get_majority(p.command)  # ba.py:318-319, canonical id order
        nr_faulty = sum(1 for p in procs if p.faulty)
        procs[0].quorum(nr_faulty)  # ba.py:395
    next_word = random.getrandbits(32)
    return {
        "case": idx,
        "n_started": n0,
        "kills": kills,
        "adds": adds,
        "ids": [p.id for p in procs],
        "faulty": [bool(p.faulty) for p in procs],
        "primary": [bool(p.primary) for p in procs],
        # ba.py:169-172 skips only the port it believes is the primary's; a
        # lieutenant holding a stale/-1 primary_port (after g-add / g-kill)
        # therefore also polls the commander (ba.py:86-102, 114-115).
        "polls_commander": [i > 0 and p.primary_port != procs[0].port
                            for i, p in enumerate(procs)],
        "order": order,
        "seed": seed,
        "coins": rec.coins,
        "majorities": [p.majority for p in procs],
        "quorum_line": out.getvalue().rstrip("\n"),
        "next_mt_word": next_word,
    }


# --------------------------------------------------------------------------
# REPL transcripts through ba.py's own __main__ block
# --------------------------------------------------------------------------
def run_transcript(n: int, commands: list[str], seed: int) -> str:
    registry = install_fake_rpyc()
    registry.clear()
    fake_thread = types.ModuleType("_thread")
    fake_thread.start_new_thread = lambda fn, args: None  # no threads: canonical schedule
    fake_thread.exit = lambda: None
    saved_thread = sys.modules.get("_thread")
    sys.modules["_thread"] = fake_thread
    sys.argv = ["ba.py", str(n)]
    src = open(REF).read()
    ns: dict = {"__name__": "__main__", "__file__": REF}
    feed = iter(commands)

    def canonical_wait_majority(self):
        # ba.py:287-289 waits for the run loop (ba.py:318-319) to compute the
        # majority; under the canonical schedule it is computed here, in id order.
        if self.majority is None:
            self.get_majority(self.command)

    def fake_input(prompt=""):
        ns["Process"].wait_majority = canonical_wait_majority
        election_tick(None, ns["processes"])
        try:
            return next(feed)
        except StopIteration:
            return "Exit"

    ns["input"] = fake_input
    random.seed(seed)
    out = io.StringIO()
    try:
        with contextlib.redirect_stdout(out):
            exec(compile(src, REF, "exec"), ns)
    finally:
        if saved_thread is not None:
            sys.modules["_thread"] = saved_thread
    return out.getvalue()


TRANSCRIPTS = [
    (4, ["g-state", "actual-order attack", "List"], 0),
    (4, ["g-state 2 faulty", "actual-order attack", "g-kill 1", "actual-order retreat", "g-state"], 0),
    (4, ["actual-order", "actual-order foo", "bogus", "g-state 9 faulty", "g-state 5"], 3),
    (5, ["g-state 1 faulty", "actual-order attack", "actual-order retreat", "List"], 11),
    (7, ["g-state 3 faulty", "g-state 6 faulty", "actual-order retreat", "g-add 2", "g-state",
         "actual-order attack", "g-kill 3", "actual-order attack"], 42),
    (3, ["g-state 1 faulty", "actual-order attack", "g-kill 2", "actual-order attack",
         "g-kill 1", "actual-order retreat", "List"], 7),
    (10, ["g-state 2 faulty", "g-state 5 faulty", "g-state 9 faulty", "actual-order attack",
          "g-state 2 non-faulty", "actual-order retreat", "g-add 3", "actual-order attack"], 1234),
    (1, ["actual-order attack", "g-state 1 faulty", "actual-order retreat", "List"], 5),
    (2, ["g-state 1 faulty", "actual-order attack", "actual-order attack"], 99),
    (6, ["g-kill 4", "g-state 1 faulty", "g-state 2 faulty", "actual-order attack", "g-kill 1",
         "actual-order attack", "g-add 1", "g-state 7 faulty", "actual-order retreat", "List"], 2024),
]


def main():
    if not os.path.exists(REF):
        raise SystemExit(f"{REF} not present: fixtures can only be generated in the dev container")
    rng = random.Random(0xBA5EED)
    cases = [om1_case(rng, i) for i in range(400)]
    with open(os.path.join(HERE, "om1_cases.json"), "w") as fh:
        json.dump({"generator": "tests/golden/gen_golden.py", "reference": "ba.py",
                   "schedule": "canonical", "cases": cases}, fh, separators=(",", ":"))
    trans = []
    for n, cmds, seed in TRANSCRIPTS:
        trans.append({"n": n, "seed": seed, "commands": cmds,
                      "stdout": run_transcript(n, cmds, seed)})
    with open(os.path.join(HERE, "repl_transcripts.json"), "w") as fh:
        json.dump({"generator": "tests/golden/gen_golden.py", "reference": "ba.py __main__",
                   "schedule": "canonical", "transcripts": trans}, fh, indent=1)
    print(f"wrote {len(cases)} OM(1) cases, {len(trans)} transcripts")


if __name__ == "__main__":
    main()
