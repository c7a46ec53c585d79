"""ba.py's election / heartbeat timing on a virtual clock (ba_amd.timing,
SURVEY.md §8f row 4): startup election at the first tick, failover one tick
after a primary is killed, g-add discovery, the REPL's wait_majority latency,
and the timed REPL reproducing ba.py's transcripts when commands are spaced
like a human typing (the canonical schedule's tick-before-command is then the
same as the clock's)."""
import io

import pytest

from test_repl import OracleEngine, transcripts


def timed(n, **kw):
    from ba_amd.timing import TimedCluster
    kw.setdefault("engine", OracleEngine())
    return TimedCluster(n, seed=kw.pop("seed", 0), **kw)


def kinds(c, kind):
    return [(t, gid) for t, k, gid, _ in c.events if k == kind]


def test_startup_before_and_after_first_tick():
    c = timed(4)
    assert [g.primary for g in c.processes] == [False] * 4  # g-state at t=0: all secondary
    with pytest.raises(AssertionError):  # actual-order before the first tick (ba.py:259)
        c.actual_order("attack")
    c.advance_to(0.1)
    # G1's heartbeat to port -1 fails first (ties by id), it wins and broadcasts;
    # G2..G4 then reach the new primary and do not elect
    assert kinds(c, "elect-win") == [(0.1, 1)]
    assert kinds(c, "heartbeat-fail") == [(0.1, 1)]
    assert [g.primary for g in c.processes] == [True, False, False, False]
    assert all(g.primary_port == c.processes[0].port for g in c.processes[1:])


def test_failover_one_tick_after_kill():
    c = timed(5)
    c.advance_to(1.05)
    c.kill(1)
    assert not c.processes[0].primary  # G2 has not noticed yet
    c.advance_to(1.1)
    assert c.failover_time() == pytest.approx(0.05)
    assert kinds(c, "elect-win")[-1] == (1.1, 2)
    assert (1.1, 1) in kinds(c, "exit")  # the killed general's thread exits at its tick
    assert [g.id for g in c.processes if g.primary] == [2]


def test_failover_with_phase_jitter_loses_then_wins():
    # with start-up skew a higher id can tick first: it sees G2 alive and loses
    # (no broadcast), keeps a stale port, and G2's own tick then wins
    for seed in range(20):
        c = timed(4, jitter=0.09, jitter_seed=seed)
        c.advance_to(1.0)
        c.kill(1)
        c.advance_to(1.2)
        assert [g.id for g in c.processes if g.primary] == [2]
        wins = [e for e in c.events if e[1] == "elect-win" and e[0] > 1.0]
        loses = [e for e in c.events if e[1] == "elect-lose" and e[0] > 1.0]
        assert len(wins) == 1 and all(t <= wins[0][0] for t, *_ in loses)
        assert 0 < c.failover_time() <= 0.1 + 1e-9
        if loses:
            return
    pytest.fail("no seed gave a higher id the first tick after the kill")


def test_g_add_discovers_leader_and_ticks():
    c = timed(3)
    c.advance_to(0.5)
    c.add(2)
    assert [g.primary_port for g in c.processes[3:]] == [c.processes[0].port] * 2
    c.advance_to(0.6)
    assert kinds(c, "heartbeat-fail") == [(0.1, 1)]  # the new generals' heartbeats succeed


def test_round_latency_is_one_wait_poll():
    c = timed(4)
    c.advance_to(0.35)
    assert c.round_timing() == pytest.approx(0.1)  # lieutenants decide at 0.4, REPL checks at 0.45
    assert [t for t, _ in kinds(c, "majority")] == [0.4, 0.4, 0.4]
    c.advance_to(0.4)
    assert c.round_timing() == pytest.approx(0.1)


def test_round_timing_hangs_where_ba_py_hangs():
    c = timed(3)
    c.advance_to(0.1)
    c.processes[1].primary = True  # a primary lieutenant never takes its majority
    with pytest.raises(RuntimeError):
        c.round_timing()


@pytest.mark.parametrize("i", range(10))
def test_timed_repl_reproduces_transcripts(i):
    """Commands one second apart: byte-identical to ba.py's transcripts."""
    from ba_amd.repl import execute, timed_lines
    from ba_amd.timing import run_timed
    t = transcripts()[i]
    out = io.StringIO()
    c = timed(t["n"], seed=t["seed"])
    run_timed(c, timed_lines(t["commands"] + ["Exit"], 1.0), out, execute)
    assert out.getvalue() == t["stdout"]


def test_timed_repl_g_state_at_t0_all_secondary():
    from ba_amd.repl import execute, timed_lines
    from ba_amd.timing import run_timed
    out = io.StringIO()
    c = timed(3)
    run_timed(c, timed_lines(["@0 g-state", "@0.2 g-state"], 0.0), out, execute)
    assert out.getvalue().splitlines() == [
        "G1, secondary, state=NF", "G2, secondary, state=NF", "G3, secondary, state=NF",
        "G1, primary, state=NF", "G2, secondary, state=NF", "G3, secondary, state=NF"]


@pytest.mark.gpu
@pytest.mark.parametrize("i", [0, 5, 9])
def test_timed_repl_transcripts_on_gpu(engine, i):
    """The timed REPL over the real libba_hip engine: same bytes as ba.py."""
    from ba_amd.repl import execute, timed_lines
    from ba_amd.timing import run_timed
    t = transcripts()[i]
    out = io.StringIO()
    c = timed(t["n"], seed=t["seed"], engine=engine)
    run_timed(c, timed_lines(t["commands"] + ["Exit"], 1.0), out, execute)
    assert out.getvalue() == t["stdout"]
