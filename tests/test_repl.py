"""The ba.py command surface (ba_amd.repl) against transcripts of ba.py itself.

tests/golden/repl_transcripts.json holds command scripts fed to ba.py's own
__main__ loop (ba.py:354-445) under the canonical schedule with random.seed(S),
and the exact stdout it printed.  The REPL must print the same bytes.

CPU tests drive the REPL with a test double of the engine that answers from the
C oracle (test infrastructure): they pin the host logic -- membership replay,
poll masks, MT coin plumbing, formatting.  The GPU test runs the real
libba_hip engine (batch=1 ba_run_trials per round)."""
import io
import json
import os

import pytest

import oracle_c

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def transcripts():
    return json.load(open(os.path.join(GOLD, "repl_transcripts.json")))["transcripts"]


class OracleEngine:
    """Stands in for ba_amd.lib.Engine in CPU tests; computes with the oracle."""

    def __init__(self):
        self.calls = 0

    def run(self, n, m, batch, seed=0, lie_mode=0, faulty=None, order=None, table=None,
            poll=None, first_trial=0, **_):
        from ba_amd import lib as L
        self.calls += 1
        dec, out, cnt = oracle_c.run(n, m, batch, seed=seed, lie_mode=lie_mode, faulty=faulty,
                                     order=order, table=table, poll=poll, first_trial=first_trial)
        return L.RunResult(dec, out, cnt)


def replay(t, engine):
    from ba_amd.generals import Cluster
    from ba_amd.repl import run
    out = io.StringIO()
    run(Cluster(t["n"], seed=t["seed"], engine=engine), t["commands"] + ["Exit"], out)
    return out.getvalue()


@pytest.mark.parametrize("i", range(10))
def test_transcript_host_logic(i):
    t = transcripts()[i]
    eng = OracleEngine()
    assert replay(t, eng) == t["stdout"]
    assert eng.calls == sum(c.startswith("actual-order ") for c in t["commands"])


def test_bookkeeping_commands_need_no_engine():
    from ba_amd.generals import Cluster
    from ba_amd.repl import run
    out = io.StringIO()
    c = Cluster(4, seed=0, engine=object())
    run(c, ["g-state", "g-kill 1", "g-state 3 faulty", "g-add 2", "g-state 9 faulty", "List",
            "g-state"], out)
    assert out.getvalue().splitlines() == [
        "G1, primary, state=NF", "G2, secondary, state=NF", "G3, secondary, state=NF",
        "G4, secondary, state=NF",
        "G2, state=NF", "G3, state=F", "G4, state=NF",
        "P2, True", "P3, False", "P4, False", "P5, False", "P6, False",
        "G2, primary, state=NF", "G3, secondary, state=F", "G4, secondary, state=NF",
        "G5, secondary, state=NF", "G6, secondary, state=NF"]
    # g-add after a failover: the new generals learn the commander's stale port
    n, fm, pm, oc = c.round_inputs("attack")
    assert (n, fm, oc) == (5, 0b00010, 1)
    assert pm == 0b11000  # G5, G6 poll the commander too (ba.py:171)


def test_commander_must_be_primary():
    from ba_amd.generals import Cluster
    c = Cluster(3, seed=1, engine=OracleEngine())
    with pytest.raises(AssertionError):  # no election tick yet: ba.py:259
        c.actual_order("attack")


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(10))
def test_transcript_on_gpu(engine, i):
    t = transcripts()[i]
    assert replay(t, engine) == t["stdout"]


@pytest.mark.gpu
def test_om3_rounds_on_gpu(engine):
    """--om 3: OM(3) rounds through the REPL, identical to the oracle's."""
    from ba_amd.generals import Cluster
    from ba_amd.repl import run
    cmds = ["g-state 2 faulty", "g-state 7 faulty", "g-state 9 faulty", "actual-order attack",
            "actual-order retreat", "g-kill 1", "actual-order attack"]
    outs = []
    for eng in (engine, OracleEngine()):
        out = io.StringIO()
        run(Cluster(10, seed=77, om=3, engine=eng), cmds, out)
        outs.append(out.getvalue())
    assert outs[0] == outs[1]
    assert outs[0].count("Execute order") == 3
