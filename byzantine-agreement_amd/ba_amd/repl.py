"""ba.py's command surface over libba_hip.

    python -m ba_amd.repl N [--seed S] [--om M] [--timed [--gap SEC]]

Commands and output formats are ba.py's (ba.py:354-445):
  actual-order <o>          every general's majority, then the quorum line
  g-state [<id> faulty|non-faulty]
  g-kill <id> / g-add <k> / List / Exit
Each `actual-order` is one batch=1 ba_run_trials call; the generals run
ba.py's canonical schedule (one election tick before every command), so with
--seed S the output equals `random.seed(S)` + ba.py under that schedule.
--om M > 1 runs OM(M) rounds (Philox lies) instead of ba.py's OM(1).
--timed replaces that schedule by ba.py's own timing on a virtual clock
(ba_amd.timing: 0.1 s run-loop ticks, heartbeat, election, wait_majority):
commands arrive --gap seconds apart (the first --gap after start-up), or at
"@T <command>" (absolute seconds),
so e.g. a g-state at t=0 shows every general as secondary, as ba.py does.
Differences from ba.py: no threads, sockets or sleeps; EOF ends the loop
instead of raising EOFError (ba.py:367).
"""
from __future__ import annotations

import argparse
import sys

from .generals import Cluster
from .timing import TimedCluster, run_timed


def execute(cluster: Cluster, line: str, out) -> bool:
    """Run one REPL line (ba.py:366-445).  Returns False on Exit."""
    cmd = line.split(" ")
    command = cmd[0]
    procs = cluster.processes
    if command == "Exit":
        return False
    if command == "actual-order":
        if len(cmd) == 1:
            return True
        majorities, q = cluster.actual_order(cmd[1])
        nr_faulty = 0
        for g, maj in zip(procs, majorities):
            status = "primary" if g.primary else "secondary"
            s = "F" if g.faulty else "NF"
            print(f"G{g.id}, {status}, majority={maj}, state={s}", file=out)
            nr_faulty += g.faulty
        print(Cluster.quorum_line(majorities, nr_faulty, q), file=out)
    elif command == "g-state":
        if len(cmd) == 3:
            if not cluster.set_faulty(int(cmd[1]), cmd[2] == "faulty"):
                return True
        for g in procs:
            s = "F" if g.faulty else "NF"
            prim = "" if len(cmd) == 3 else (", primary" if g.primary else ", secondary")
            print(f"G{g.id}{prim}, state={s}", file=out)
    elif command == "g-kill":
        if len(cmd) > 1:
            cluster.kill(int(cmd[1]))
    elif command == "g-add":
        if len(cmd) > 1:
            cluster.add(int(cmd[1]))
    elif command == "List":
        for g in procs:
            print(f"P{g.id}, {g.primary}", file=out)
    return True


def run(cluster: Cluster, lines, out=sys.stdout):
    """Feed command lines under the canonical schedule (tick before each)."""
    for line in lines:
        cluster.tick()
        if not execute(cluster, line.rstrip("\n"), out):
            break


def timed_lines(lines, gap: float):
    """(arrival time, command) pairs: "@T cmd" arrives at T, others gap after
    the previous command (the first one gap after start-up)."""
    t = gap
    for line in lines:
        if line.startswith("@"):
            stamp, _, line = line[1:].partition(" ")
            t = float(stamp)
        yield t, line
        t += gap


def main(argv=None):
    ap = argparse.ArgumentParser(prog="ba_amd.repl", description=__doc__.split("\n\n")[0])
    ap.add_argument("N", type=int, help="generals at start (ba.py:12)")
    ap.add_argument("--seed", type=int, default=None, help="random.seed() of ba.py's RNG")
    ap.add_argument("--om", type=int, default=1, help="OM depth (1 = ba.py)")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--timed", action="store_true", help="ba.py's tick timing (ba_amd.timing)")
    ap.add_argument("--gap", type=float, default=1.0, help="seconds between commands (--timed)")
    a = ap.parse_args(argv)
    if a.timed:
        cluster = TimedCluster(a.N, seed=a.seed, om=a.om, device=a.device)
    else:
        cluster = Cluster(a.N, seed=a.seed, om=a.om, device=a.device)

    def lines():
        while True:
            try:
                yield input()
            except EOFError:
                return

    if a.timed:
        run_timed(cluster, timed_lines(lines(), a.gap), sys.stdout, execute)
    else:
        run(cluster, lines())


if __name__ == "__main__":
    main()
