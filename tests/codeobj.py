"""Code-object inspection of the built libba_hip.so (test infrastructure, CPU only).

The HIP fat binary in the library's .hip_fatbin section is a concatenation of
clang offload bundles, one per translation unit.  code_objects() pulls out the
gfx950 ELF of each, disassemble() runs llvm-objdump on them, and
writelane_hazards() checks the one hazard the compiler cannot see: the WAVE
kernels' writelane4 (csrc/ba_wave.hpp) drops ballots -- VALU writes of SGPRs
(v_cmp_*_e64 s[..]) -- into VGPR lanes with hand-written v_writelane_b32, and
v_writelane reads its data SGPR early, so at least WRITELANE_WAIT_STATES wait
states must separate the SGPR's VALU write from the v_writelane that reads it
(a GPU run without them got wrong planes).  The asm block carries an s_nop 4
for that; this check proves it is still there in the shipped build, whatever
the compiler scheduled around it.

Why 2: the compiler's own hazard recognizer, which sees its own code, never
lets fewer than 2 wait states separate a VALU SGPR write from a v_writelane
reading it (12k compiler-made pairs in this library, e.g. SGPR spills of
ballots: minimum 2), and the writelane4 groups built without their s_nop show
0-1 (tests/test_lib.py builds that copy).  writelane4's s_nop 4 gives 5.
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "byzantine-agreement_amd", "ba_amd", "libba_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
WRITELANE_WAIT_STATES = 2  # VALU SGPR write -> v_writelane_b32 reading that SGPR (see below)


def code_objects(lib_path: str = LIB) -> list:
    """gfx950 code objects (ELF bytes) of every bundle in the library's fat binary."""
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib_path,
                        os.path.join(td, "lib.copy")], check=True, capture_output=True)
        data = open(fb, "rb").read()
    out, pos = [], 0
    while (i := data.find(MAGIC, pos)) >= 0:
        (n,) = struct.unpack_from("<Q", data, i + len(MAGIC))
        off = i + len(MAGIC) + 8
        for _ in range(n):
            o, size, tlen = struct.unpack_from("<QQQ", data, off)
            off += 24
            triple = data[off:off + tlen].decode()
            off += tlen
            if triple.endswith("gfx950"):
                out.append(data[i + o:i + o + size])
        pos = i + 1
    return out


def disassemble(co: bytes) -> str:
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", f.name], check=True,
                              capture_output=True, text=True).stdout


def functions(asm: str) -> dict:
    """{symbol: [instruction text, ...]} of a disassembly (comments stripped)."""
    funcs, cur = {}, None
    for line in asm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        if cur is not None and line.startswith("\t"):
            ins = line.split("//")[0].strip()
            if ins:
                cur.append(ins)
    return funcs


def _sgprs(op: str) -> set:
    m = re.fullmatch(r"s(\d+)", op)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def _operands(ins: str) -> tuple:
    parts = ins.split(None, 1)
    ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
    return parts[0], ops


def _wait_states(ins: str) -> int:
    m = re.fullmatch(r"s_nop (\d+|0x[0-9a-f]+)", ins)
    return int(m.group(1), 0) + 1 if m else 1


def writelane_hazards(instrs: list, need: int = WRITELANE_WAIT_STATES) -> tuple:
    """(violations, checked): every v_writelane_b32 whose data SGPR was last written
    by a VALU instruction in the same straight-line block, with fewer than `need`
    wait states between the two, is a violation; `checked` counts the writelanes
    that had such a VALU writer (writelanes fed by SALU writes -- SGPR spills --
    carry no such hazard)."""
    bad, checked = [], 0
    for k, ins in enumerate(instrs):
        op, ops = _operands(ins)
        if op != "v_writelane_b32" or len(ops) < 2:
            continue
        regs = _sgprs(ops[1])
        if not regs:
            continue
        ws = 0
        for j in range(k - 1, -1, -1):
            pop, pops = _operands(instrs[j])
            if pop.startswith("s_cbranch") or pop in ("s_branch", "s_setpc_b64", "s_endpgm"):
                break  # block boundary: the writer is not in this block
            if pops and _sgprs(pops[0]) & regs:
                if pop.startswith("v_"):
                    checked += 1
                    if ws < need:
                        bad.append((k, ins, instrs[j], ws))
                break
            ws += _wait_states(instrs[j])
    return bad, checked


def kernel_resources(lib_path: str = LIB) -> dict:
    """{kernel symbol: {vgpr, sgpr, vgpr_spill, sgpr_spill}} from the AMDGPU metadata
    notes of every gfx950 code object in the library."""
    res = {}
    for co in code_objects(lib_path):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f.name], check=True,
                                   capture_output=True, text=True).stdout
        for blk in notes.split("- .agpr_count")[1:]:
            def field(key):
                return int(re.search(rf"\.{key}:\s+(\d+)", blk).group(1))
            name = re.search(r"\.name:\s+(\S+)", blk).group(1)
            res[name] = {"vgpr": field("vgpr_count"), "sgpr": field("sgpr_count"),
                         "vgpr_spill": field("vgpr_spill_count"),
                         "sgpr_spill": field("sgpr_spill_count")}
    return res
