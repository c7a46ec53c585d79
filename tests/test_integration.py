"""INTEGRATION.md §1 is executable: the ctypes stub a ba.py maintainer would add
is run exactly as written (only the library path is substituted)."""
import os
import random
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "byzantine-agreement_amd", "ba_amd", "libba_hip.so")


def stub_source():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = re.search(r"## 1\..*?```python\n(.*?)```", text, re.S).group(1)
    assert "/path/to/byzantine-agreement_amd/ba_amd/libba_hip.so" in block
    return block.replace("/path/to/byzantine-agreement_amd/ba_amd/libba_hip.so", SO)


def test_stub_compiles_and_params_layout_is_the_abi():
    """The stub's Params / Counters equal ba_amd.lib's (include/ba.h) field by field."""
    import ctypes
    from ba_amd import lib as L
    src = stub_source()
    compile(src, "INTEGRATION.md#1", "exec")
    # evaluate only the structure definitions (no library load, no device)
    ns = {"ctypes": ctypes}
    structs = re.search(r"(class Params.*?)\n_vp = ", src, re.S).group(1)
    exec(structs, ns)
    for mine, abi in ((ns["Params"], L.Params), (ns["Counters"], L.Counters)):
        assert ctypes.sizeof(mine) == ctypes.sizeof(abi)
        for (fa, ta), (fb, tb) in zip(mine._fields_, abi._fields_):
            assert fa == fb and ctypes.sizeof(ta) == ctypes.sizeof(tb)
            assert getattr(mine, fa).offset == getattr(abi, fb).offset


class Proc:
    """The attributes of a ba.py Process that round_on_gpu reads (ba.py:66-77)."""

    def __init__(self, port, faulty, primary_port):
        self.port, self.faulty, self.primary_port = port, faulty, primary_port


@pytest.mark.gpu
def test_stub_round_on_gpu_matches_oracle():
    """round_on_gpu draws ba.py's coins from the global `random` in canonical order
    and returns the majorities and quorum code the oracle computes from the same coins."""
    import oracle_c
    ns = {}
    exec(stub_source(), ns)
    round_on_gpu = ns["round_on_gpu"]
    rng = np.random.default_rng(5)
    checked = 0
    for trial in range(200):
        n = int(rng.integers(1, 12))
        ports = [18812 + i for i in range(n)]
        faulty = [bool(rng.random() < 0.3) for _ in range(n)]
        stale = [i > 0 and rng.random() < 0.2 for i in range(n)]
        procs = [Proc(ports[i], faulty[i], -1 if stale[i] else ports[0]) for i in range(n)]
        command = ["attack", "retreat", "foo"][int(rng.integers(0, 3))]
        seed = int(rng.integers(0, 1 << 32))
        random.seed(seed)
        majorities, q = round_on_gpu(procs, command)
        # the oracle replays the same coins (ba_oracle_run, table mode)
        random.seed(seed)
        from ba_amd import lib as L
        fm = sum(1 << i for i in range(n) if faulty[i])
        poll = sum(1 << i for i in range(1, n) if stale[i])
        coins = [1 if random.randint(0, 1) == 0 else 0
                 for _ in range(L.om1_coin_count(n, 1, fm, poll))]
        oc = {"attack": 1, "retreat": 0}.get(command, 2)
        od, oo, _ = oracle_c.run(n, 1, 1, lie_mode=1, faulty=[fm], order=[oc],
                                 table=L.pack_coins([coins], n), poll=[poll])
        text = {0: "retreat", 1: "attack", 2: "undefined"}
        assert majorities == [command] + [text[(int(od[0]) >> (2 * (r - 1))) & 3] for r in range(1, n)]
        assert q == int(oo[0]) & 3
        checked += 1
    assert checked == 200
