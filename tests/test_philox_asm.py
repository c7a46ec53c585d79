"""CPU check of the generated Philox asm (csrc/ba_philox_asm.hpp).

The header holds rounds 2..9 of G interleaved Philox4x32-10 calls as one inline
asm statement with fixed, rotating register pairs (tools/gen_philox_asm.py).
This test interprets that asm text -- v_mad_u64_u32 and v_bitop3_b32 on a
register file, %N operands bound as the constraint lists say -- and compares
the result with a plain Philox4x32-10 (Salmon et al. 2011; the same algebra as
ba_device.hpp philox10 and oracle/ba_oracle.c), so a register-rotation slip
in the generator shows up here before any GPU run.  It also checks that the
header is what the generator produces now.
"""
import os
import random
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "byzantine-agreement_amd", "csrc", "ba_philox_asm.hpp")
GEN = os.path.join(ROOT, "tools", "gen_philox_asm.py")
M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox_rounds(c, k0, k1, r0, r1):
    x, y, z, w = c
    for i in range(r0, r1):
        p0, p1 = M0 * x, M1 * z
        ka, kb = (k0 + i * W0) & MASK, (k1 + i * W1) & MASK
        x, y, z, w = (p1 >> 32) ^ y ^ ka, p1 & MASK, (p0 >> 32) ^ w ^ kb, p0 & MASK
    return [x, y, z, w]


_LAB = []


def lab_header() -> str:
    """The generator's --lab output (all three variants; lab builds only)."""
    if not _LAB:
        _LAB.append(subprocess.run([sys.executable, GEN, "--lab"], capture_output=True, text=True,
                                   check=True).stdout)
    return _LAB[0]


def parse(G, name="philox_r29_asm_vkm"):
    src = open(HDR).read() if name == "philox_r29_asm_vkm" else lab_header()
    m = re.search(r"%s<%d>\(.*?asm volatile\((.*?)\);\n}" % (name, G), src, re.S)
    assert m, f"no G={G} specialisation"
    body = m.group(1)
    parts = body.split("\n        : ")
    code = "".join(re.findall(r'"((?:[^"\\]|\\.)*)"', parts[0])).replace("\\n\\t", "\n")
    outs = re.findall(r'"([^"]+)"\(([^)]+)\)', parts[1])
    ins = re.findall(r'"([^"]+)"\(([^)]+)\)', parts[2])
    return code.strip().splitlines(), outs, ins


def run_asm(lines, outs, ins, env):
    """env: C-level names -> values; returns the C-level outputs."""
    reg = {}
    ops = []  # operand number -> register name or scalar value
    for i, (con, name) in enumerate(outs + ins):
        fixed = re.match(r"=&\{(v\d+)\}", con)
        if fixed:
            ops.append(fixed.group(1))
        elif con.startswith("+v") or con.startswith("=&s"):
            ops.append(f"op{i}")
            reg[f"op{i}"] = env.get(name, 0)
        else:
            ops.append(f"op{i}")
            v = name
            if v.endswith("u") and v.startswith("0x"):
                reg[f"op{i}"] = int(v[:-1], 16)
            else:
                reg[f"op{i}"] = env[name]

    def rd(tok):
        tok = tok.strip()
        if tok.startswith("%"):
            return reg[ops[int(tok[1:])]]
        if tok == "0":
            return 0
        return reg[tok]

    def wr(tok, val):
        tok = tok.strip()
        name = ops[int(tok[1:])] if tok.startswith("%") else tok
        reg[name] = val & MASK

    for ln in lines:
        op, rest = ln.split(None, 1)
        if op == "v_mad_u64_u32":
            dst, _cc, a, b, c = [t.strip() for t in rest.split(",")]
            lo = int(re.match(r"v\[(\d+):(\d+)\]", dst).group(1))
            p = rd(a) * rd(b) + rd(c)
            reg[f"v{lo}"], reg[f"v{lo + 1}"] = p & MASK, (p >> 32) & MASK
        elif op == "v_bitop3_b32":
            rest, imm = rest.split(" bitop3:")
            assert imm.strip() == "0x96"
            d, a, b, c = [t.strip() for t in rest.split(",")]
            wr(d, rd(a) ^ rd(b) ^ rd(c))
        else:
            raise AssertionError(f"unexpected instruction {op}")
    out = {}
    for i, (con, name) in enumerate(outs):
        if "s" in con:
            continue
        out[name] = reg[ops[i]]
    return out


# the shipped variant (product header) and the --lab ones
@pytest.mark.parametrize("name,G", [("philox_r29_asm_vkm", g) for g in (2, 3, 4, 5)] +
                         [(nm, g) for nm in ("philox_r29_asm", "philox_r29_asm_vk") for g in (2, 3, 4)])
def test_generated_rounds_match_philox(G, name):
    lines, outs, ins = parse(G, name)
    rng = random.Random(1234 + G)
    for _ in range(50):
        k0, k1 = rng.getrandbits(32), rng.getrandbits(32)
        ctrs = [[rng.getrandbits(32) for _ in range(4)] for _ in range(G)]
        r2 = [philox_rounds(c, k0, k1, 0, 2) for c in ctrs]
        want = [philox_rounds(c, k0, k1, 0, 10) for c in ctrs]
        env = {"m0": M0, "m1": M1}  # the _vkm variant's VGPR multipliers
        for g in range(G):
            env[f"x[{g}]"], env[f"yi[{g}]"], env[f"z[{g}]"], env[f"wi[{g}]"] = r2[g]
        for i in range(8):
            env[f"k0[{i}]"] = (k0 + (2 + i) * W0) & MASK
            env[f"k1[{i}]"] = (k1 + (2 + i) * W1) & MASK
        got = run_asm(lines, outs, ins, env)
        for g in range(G):
            assert [got[f"x[{g}]"], got[f"y[{g}]"], got[f"z[{g}]"], got[f"w[{g}]"]] == want[g]


def test_header_is_generated():
    out = subprocess.run([sys.executable, GEN], capture_output=True, text=True, check=True).stdout
    assert out == open(HDR).read(), "ba_philox_asm.hpp is stale: rerun tools/gen_philox_asm.py"
    # the product header holds only the variant the kernels call
    assert "philox_r29_asm_vkm<2>" in out and "philox_r29_asm<2>" not in out
    assert "philox_r29_asm_vk<2>" not in out and "philox_r29_asm_vkm<2>" in lab_header()
