"""N ranks of the library's multi-GPU layer on ONE GPU (test infrastructure).

RCCL refuses two ranks on one GPU, so the library's N>1 paths would first run
on an 8-GPU node.  Here `launch()` starts N processes on cuda:0 (plain child
processes, started before any of them touches the GPU), each with
BA_RCCL_LIB = tests/native's shared-memory RCCL stand-in (fake_rccl.c), a gloo
group for the rendezvous (ba_amd.dist.init_comm: rank 0's unique id to every
rank, as on a real node), and one libba_hip communicator.  Each rank runs the
named scenarios through the C ABI's multi entries -- ba_run_trials_multi,
ba_run_instance_split_level_multi, the hipGraph split with its eager
all-gather, the failure paths -- and writes what it got to a JSON file; the
tests compare those with the oracle in the parent process.

    python multirank.py WORLD RANK PORT OUT SCENARIO[,SCENARIO...]
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
FAKE_RCCL = os.path.join(HERE, "native", "_build", "libfake_rccl.so")

# (n, m, total trials, f, first_trial) of the trial-DP cases: ragged totals,
# more ranks than words (70 trials = 2 words), every engine family
DP_CASES = [(10, 3, 64 * 37 + 11, 3, 0), (13, 4, 1000, 4, 64 * 3), (16, 5, 70, 5, 64 * 11),
            (9, 2, 200, 3, 64)]
# (n, m, level, batch, f, first_trial) of the split cases
SPLIT_CASES = [(16, 5, 1, 1, 5, 64 * 7), (16, 5, 1, 70, 5, 64 * 7), (16, 5, 2, 1, 5, 64 * 7),
               (16, 5, 2, 70, 5, 64 * 7), (10, 3, 1, 130, 4, 0), (10, 3, 2, 130, 4, 0),
               (9, 4, 2, 65, 3, 64)]
GRAPH_CASES = [(16, 5, 1, 70), (16, 5, 2, 1), (10, 3, 2, 300)]
SEED = 0xBA5EED


def build_fake() -> str:
    """The stand-in's .so (built here if missing; test infrastructure only)."""
    src = os.path.join(HERE, "native", "fake_rccl.c")
    if not os.path.exists(FAKE_RCCL) or os.path.getmtime(src) > os.path.getmtime(FAKE_RCCL):
        subprocess.run(["make", "-s", "-C", os.path.join(HERE, "native")], check=True)
    return FAKE_RCCL


def launch(world: int, scenarios: list, tmpdir: str, timeout: float = 240.0, env_extra=None):
    """Run `scenarios` on `world` ranks; returns [rank 0 result, ...] (JSON dicts,
    each with 'elapsed' per scenario) or raises with the ranks' output."""
    import socket
    build_fake()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, BA_RCCL_LIB=FAKE_RCCL, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               FAKE_RCCL_TIMEOUT_S="90", PYTHONUNBUFFERED="1")
    env.pop("BA_FORCE_SPLIT", None)
    env.update(env_extra or {})
    procs, outs, logs = [], [], []
    for r in range(world):
        out = os.path.join(tmpdir, f"rank{r}.json")
        log = open(os.path.join(tmpdir, f"rank{r}.log"), "w")
        outs.append(out)
        logs.append(log)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), str(world), str(r),
                                       str(port), out, ",".join(scenarios)],
                                      env=env, stdout=log, stderr=subprocess.STDOUT, cwd=ROOT))
    t0 = time.time()
    try:
        for p in procs:
            p.wait(timeout=max(1.0, timeout - (time.time() - t0)))
    except subprocess.TimeoutExpired:
        for p in procs:
            p.kill()
        for p in procs:
            p.wait()
    for log in logs:
        log.close()
    bad = [r for r, p in enumerate(procs) if p.returncode != 0]
    if bad:
        text = "".join(f"--- rank {r} (rc {procs[r].returncode}) ---\n" +
                       open(os.path.join(tmpdir, f"rank{r}.log")).read()[-4000:] for r in bad)
        raise AssertionError(f"ranks {bad} failed:\n{text}")
    return [json.load(open(o)) for o in outs]


# --- rank side -------------------------------------------------------------------
def _err(e):
    return {"code": e.code, "msg": str(e)}


def main():
    world, rank, port, out, scen = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]),
                                    sys.argv[4], sys.argv[5].split(","))
    sys.path.insert(0, os.path.join(ROOT, "byzantine-agreement_amd"))
    import numpy as np
    import torch
    import torch.distributed as dist

    from ba_amd import dist as D
    from ba_amd import lib as L

    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    eng = L.Engine(0)
    res = {"rank": rank, "world": world, "elapsed": {}}

    def u64(t):
        return [int(x) for x in t.cpu().numpy().view(np.uint64)]

    def u8(t):
        return [int(x) for x in t.cpu().numpy()]

    comm = D.init_comm(eng)
    assert comm.nranks == world and comm.rank == rank

    def fresh_comm():
        nonlocal comm
        comm.close()
        comm = D.init_comm(eng)

    for name in scen:
        t0 = time.time()
        if name == "dp":
            got = []
            for n, m, total, f, first in DP_CASES:
                p = L.make_params(n, m, SEED, L.LIE_PHILOX, L.FAULTY_RANDOM, f, L.ORDER_RANDOM,
                                  L.ATTACK, L.ENGINE_AUTO, first)
                _, count = L.trial_share(total, world, rank)
                dec = torch.zeros(max(count, 1), dtype=torch.int64, device=dev)
                outc = torch.zeros(max(count, 1), dtype=torch.uint8, device=dev)
                cnt, sf, sc = comm.run_trials(p, total, d_decisions=dec.data_ptr(),
                                              d_outcome=outc.data_ptr())
                torch.cuda.synchronize()
                got.append({"case": [n, m, total, f, first], "counters": cnt, "first": sf,
                            "count": sc, "dec": u64(dec[:sc]), "out": u8(outc[:sc])})
            res["dp"] = got
        elif name == "split":
            got = []
            for n, m, level, B, f, first in SPLIT_CASES:
                p = L.make_params(n, m, SEED, L.LIE_PHILOX, L.FAULTY_RANDOM, f, L.ORDER_RANDOM,
                                  L.ATTACK, L.ENGINE_AUTO, first)
                rows = []
                for _ in range(2):  # the second call reuses the grown vote buffer
                    dec, outc, cnt = D.run_instance_split(comm, p, B, dev, level=level)
                    rows.append({"counters": cnt, "dec": u64(dec), "out": u8(outc)})
                got.append({"case": [n, m, level, B, f, first], "calls": rows})
            res["split"] = got
        elif name == "graphs":
            got = []
            for n, m, level, B in GRAPH_CASES:
                p = L.make_params(n, m, SEED, L.LIE_PHILOX, L.FAULTY_RANDOM, (n - 1) // 3,
                                  L.ORDER_RANDOM, L.ATTACK, L.ENGINE_AUTO, 64 * 5)
                g = D.InstanceSplitGraphs(dev, p, B, comm=comm, level=level)
                try:
                    reps = []
                    for _ in range(2):
                        dec, outc, cnt = g.replay()
                        torch.cuda.synchronize()
                        reps.append({"counters": [int(x) for x in cnt.cpu().tolist()[:12]],
                                     "dec": u64(dec), "out": u8(outc)})
                finally:
                    g.close()
                got.append({"case": [n, m, level, B], "replays": reps})
            res["graphs"] = got
        elif name == "enomem":
            # rank 1 alone cannot allocate its vote buffer: every rank returns an
            # error (agreed before the exchange), and the comm stays usable
            p = L.make_params(10, 3, 3, L.LIE_PHILOX, L.FAULTY_RANDOM, 3, L.ORDER_RANDOM,
                              L.ATTACK, L.ENGINE_AUTO, 0)
            if rank == 1:
                os.environ["BA_TEST_VOTE_ENOMEM"] = "1"
            try:
                D.run_instance_split(comm, p, 200, dev, level=2)
                first = {"code": 0}
            except L.BAError as e:
                first = _err(e)
            os.environ.pop("BA_TEST_VOTE_ENOMEM", None)
            dec, outc, cnt = D.run_instance_split(comm, p, 200, dev, level=2)
            res["enomem"] = {"first": first, "after": {"counters": cnt, "dec": u64(dec)}}
        elif name.startswith("preagree_"):
            # rank 1's agreement transport fails (BA_TEST_PREAGREE_FAIL); every rank
            # must return an error within the watchdog's bound
            mode = name[len("preagree_"):]
            comm.set_timeout(4000)
            p = L.make_params(16, 5, 9, L.LIE_PHILOX, L.FAULTY_RANDOM, 5, L.ORDER_RANDOM,
                              L.ATTACK, L.ENGINE_AUTO, 0)
            if rank == 1:
                os.environ["BA_TEST_PREAGREE_FAIL"] = mode
            t1 = time.time()
            try:
                D.run_instance_split(comm, p, 70, dev, level=2)
                first = {"code": 0}
            except L.BAError as e:
                first = _err(e)
            first["seconds"] = time.time() - t1
            os.environ.pop("BA_TEST_PREAGREE_FAIL", None)
            try:  # an aborted comm fails fast; a comm that agreed on the error works on
                c2 = comm.run_instance_split(p, 70)
                again = {"code": 0, "trials": c2["trials"]}
            except L.BAError as e:
                again = _err(e)
            dist.barrier()
            fresh_comm()  # a new communicator over the same ranks is exact again
            cnt = comm.run_instance_split(p, 70, level=2)
            res[name] = {"first": first, "again": again, "fresh": cnt}
        elif name == "abort_dp":
            # a rank that stops taking part (ba_comm_abort) leaves its peers to their
            # watchdog: they raise EABORTED instead of hanging in the all-reduce
            comm.set_timeout(3000)
            p = L.make_params(10, 3, 1, L.LIE_PHILOX, L.FAULTY_RANDOM, 3, L.ORDER_RANDOM,
                              L.ATTACK, L.ENGINE_AUTO, 0)
            t1 = time.time()
            if rank == world - 1:
                comm.abort()
            try:
                comm.run_trials(p, 64 * 100)
                first = {"code": 0}
            except L.BAError as e:
                first = _err(e)
            first["seconds"] = time.time() - t1
            dist.barrier()
            fresh_comm()
            cnt, _, _ = comm.run_trials(p, 64 * 100)
            res["abort_dp"] = {"first": first, "fresh": cnt}
        else:
            raise SystemExit(f"unknown scenario {name}")
        res["elapsed"][name] = time.time() - t0
        dist.barrier()
    comm.close()
    eng.close()
    with open(out, "w") as fh:
        json.dump(res, fh)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
