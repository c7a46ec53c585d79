"""Exhaustive CPU check of the bit-sliced majority threshold (Csa::ge).

Every majority of the OM tree (ba.py:159-195: inner levels, leaf blocks, roots)
is a carry-save count followed by Csa<NL>::ge<K, TH> (ba_device.hpp).  Round 3
replaced the resolve-then-compare form with ge_from (the threshold read
straight off the level bits); tests/native/csa_ge_check.cpp runs both code
paths' shared header on the host over every input pattern of K <= 16 inputs
and every threshold, for the default build and for BA_CSA_GE_RESOLVE (the
previous form, kept for A/B builds).
"""
import os
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "csa_ge_check.cpp")
INC = os.path.join(ROOT, "byzantine-agreement_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc absent")
@pytest.mark.parametrize("defs", [[], ["-DBA_CSA_GE_RESOLVE"]])
def test_csa_ge_exhaustive(defs):
    with tempfile.TemporaryDirectory() as td:
        exe = os.path.join(td, "csa")
        subprocess.run([HIPCC, "-O1", "-std=c++17", f"-I{INC}", *defs, SRC, "-o", exe],
                       check=True, capture_output=True)
        r = subprocess.run([exe], capture_output=True, text=True)
        assert r.returncode == 0 and "bad=0" in r.stdout, r.stdout + r.stderr
