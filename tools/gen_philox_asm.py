#!/usr/bin/env python3
"""Generate csrc/ba_philox_asm.hpp: Philox4x32-10 rounds 2..9 of G interleaved
calls as ONE inline-asm statement (G = 2..5; the SGPR-key lab variants G = 2, 3, 4).

Why: the products of rounds 2..9 are pinned to v_mad_u64_u32 with inline asm
(ba_device.hpp, philox_mul2_n).  The compiler's hazard recognizer cannot see
inside an asm statement, so it puts a conservative `s_nop 0` between every asm
and the next instruction that touches one of its defs -- i.e. after every
round of every group (47 per k_om3w<10> round, ~4% of its instruction
stream).  One statement per group for all eight rounds leaves one.

Sub-registers of a 64-bit asm operand cannot be named in AMDGPU inline asm, so
the products live in fixed VGPR pairs (clobbers), four per call, double
buffered (a round reads the low halves of the previous round's products while
it writes the next ones); the final y, w are bound to the low halves of the
last round's pairs through physical-register output constraints.  The fixed
registers start at v[BASE]; every kernel already uses more than 8G VGPRs, so
the allocator only has to keep its other values out of them across the asm.

Round i (products p0 = M0*x, p1 = M1*z; Salmon et al. 2011, the same algebra as
ba_device.hpp philox10):
    x' = hi(p1) ^ y ^ k0_i    y' = lo(p1)    z' = hi(p0) ^ w ^ k1_i    w' = lo(p0)
Order per round: the 2G products, then the 2G xor3s, so each product is read
2G-1 instructions after it is written (the same distance as the compiler's
schedule of philox_mul2_n).

usage: python3 tools/gen_philox_asm.py > byzantine-agreement_amd/csrc/ba_philox_asm.hpp
       python3 tools/gen_philox_asm.py --lab > <lab header>   (lab builds only)

The product header holds only the variant the kernels use: round keys and
multipliers as VGPR operands (philox_r29_asm_vkm).  --lab also emits the
SGPR-key (philox_r29_asm) and SGPR-multiplier (philox_r29_asm_vk) variants
that round 3/4's A/B runs measured -- for lab harnesses.
"""

BASE = 0  # first fixed VGPR
import os
MODE = os.environ.get("PHILOX_ASM_MODE", "rot")  # "rot": 3 pairs per call; "pairs4": 4
# lab: carry-out SGPR pairs the v_mad_u64_u32s rotate through (1 = one shared pair)
NCC = int(os.environ.get("PHILOX_ASM_NCC", "1"))


def gen(G: int, kc: str = "s", mc: str = "s") -> str:
    # operand numbering: outputs first (x[g], z[g] in/out; w[g], y[g] fixed), then
    # inputs (y_in[g], w_in[g], keys k0[0..7], k1[0..7], M0, M1), cc last output
    ops_out, ops_in = [], []
    # x, z as "+v" (one operand number each)
    for g in range(G):
        ops_out.append(f'"+v"(x[{g}])')
    for g in range(G):
        ops_out.append(f'"+v"(z[{g}])')
    def A(g): return BASE + 8 * g
    def B(g): return BASE + 8 * g + 2
    def C(g): return BASE + 8 * g + 4
    def D(g): return BASE + 8 * g + 6
    for g in range(G):
        ops_out.append(f'"=&{{vW{g}}}"(w[{g}])')
    for g in range(G):
        ops_out.append(f'"=&{{vY{g}}}"(y[{g}])')
    for q in range(NCC):
        ops_out.append(f'"=&s"(cc[{q}])' if NCC > 1 else '"=&s"(cc)')
    nout = len(ops_out)
    for g in range(G):
        ops_in.append(f'"v"(yi[{g}])')
    for g in range(G):
        ops_in.append(f'"v"(wi[{g}])')
    for i in range(8):
        ops_in.append(f'"{kc}"(k0[{i}])')
    for i in range(8):
        ops_in.append(f'"{kc}"(k1[{i}])')
    if mc == "s":
        ops_in.append('"s"(0xD2511F53u)')
        ops_in.append('"s"(0xCD9E8D57u)')
    else:  # the multipliers as VGPR operands too (the caller holds them in VGPRs)
        ops_in.append('"v"(m0)')
        ops_in.append('"v"(m1)')
    X = lambda g: g
    Z = lambda g: G + g
    CC = 4 * G
    ccn = [0]

    def cc():  # the next carry-out operand
        r = CC + ccn[0] % NCC
        ccn[0] += 1
        return r
    YI = lambda g: nout + g  # noqa: E731
    WI = lambda g: nout + G + g
    K0 = lambda i: nout + 2 * G + i
    K1 = lambda i: nout + 2 * G + 8 + i
    M0 = nout + 2 * G + 16
    M1 = M0 + 1
    lines = []
    if MODE == "rot":
        # three pairs per call, rotating roles (pw: lo = w, py: lo = y, fr: free);
        # per round: fr <- x*M0, (x reg) <- z' = hi(fr)^w^k1, pw <- z*M1 (pw is
        # free once its w is read), (z reg) <- x' = hi(pw)^y^k0; the x and z
        # registers swap roles every round (8 rounds: back in place)
        pairs = [[BASE + 6 * g + 2 * j for j in range(3)] for g in range(G)]
        free = [list(pairs[g]) for g in range(G)]
        pw, py = [None] * G, [None] * G
        xr = [f"%{X(g)}" for g in range(G)]
        zr = [f"%{Z(g)}" for g in range(G)]
        for i in range(8):
            f = [free[g].pop(0) for g in range(G)]
            for g in range(G):   # p0 = M0 * x
                lines.append(f"v_mad_u64_u32 v[{f[g]}:{f[g] + 1}], %{cc()}, {xr[g]}, %{M0}, 0")
            for g in range(G):   # z' = hi(p0) ^ w ^ k1, into x's register
                wprev = f"%{WI(g)}" if pw[g] is None else f"v{pw[g]}"
                lines.append(f"v_bitop3_b32 {xr[g]}, v{f[g] + 1}, {wprev}, %{K1(i)} bitop3:0x96")
                if pw[g] is not None:
                    free[g].append(pw[g])
            q = [free[g].pop(0) for g in range(G)]
            for g in range(G):   # p1 = M1 * z
                lines.append(f"v_mad_u64_u32 v[{q[g]}:{q[g] + 1}], %{cc()}, {zr[g]}, %{M1}, 0")
            for g in range(G):   # x' = hi(p1) ^ y ^ k0, into z's register
                yprev = f"%{YI(g)}" if py[g] is None else f"v{py[g]}"
                lines.append(f"v_bitop3_b32 {zr[g]}, v{q[g] + 1}, {yprev}, %{K0(i)} bitop3:0x96")
                if py[g] is not None:
                    free[g].append(py[g])
            pw, py = f, q
            xr, zr = zr, xr
        assert xr == [f"%{X(g)}" for g in range(G)]
        outs_w, outs_y = list(pw), list(py)
        used = sorted({r for g in range(G) for r in pairs[g]})
    else:
        for i in range(8):  # round 2 + i
            if i % 2 == 0:
                P0, P1 = C, D
            else:
                P0, P1 = A, B
            for g in range(G):
                lines.append(f"v_mad_u64_u32 v[{P0(g)}:{P0(g) + 1}], %{CC}, %{X(g)}, %{M0}, 0")
                lines.append(f"v_mad_u64_u32 v[{P1(g)}:{P1(g) + 1}], %{CC}, %{Z(g)}, %{M1}, 0")
            for g in range(G):
                if i == 0:
                    yprev, wprev = f"%{YI(g)}", f"%{WI(g)}"
                elif i % 2 == 1:  # previous round wrote C (p0), D (p1)
                    yprev, wprev = f"v{D(g)}", f"v{C(g)}"
                else:             # previous round wrote A (p0), B (p1)
                    yprev, wprev = f"v{B(g)}", f"v{A(g)}"
                lines.append(f"v_bitop3_b32 %{X(g)}, v{P1(g) + 1}, {yprev}, %{K0(i)} bitop3:0x96")
                lines.append(f"v_bitop3_b32 %{Z(g)}, v{P0(g) + 1}, {wprev}, %{K1(i)} bitop3:0x96")
        outs_w = [A(g) for g in range(G)]; outs_y = [B(g) for g in range(G)]
        used = sorted({r for g in range(G) for r in (A(g), B(g), C(g), D(g))})
    outset = set(outs_w) | set(outs_y)
    clob = []
    for r in used:
        for q in (r, r + 1):
            if q not in outset:
                clob.append(f'"v{q}"')
    for g in range(G):
        ops_out = [o.replace(f"vW{g}}}", f"v{outs_w[g]}}}").replace(f"vY{g}}}", f"v{outs_y[g]}}}") for o in ops_out]
    # one source line per phase of a round (its G products or its G xor3s):
    # the asm text is the same instruction string, a quarter as many lines
    text = [l + ("\\n\\t" if k + 1 < len(lines) else "") for k, l in enumerate(lines)]
    body = "\n".join('        "' + "".join(text[k:k + G]) + '"' for k in range(0, len(text), G))
    fname = "philox_r29_asm" if kc == "s" else ("philox_r29_asm_vk" if mc == "s" else "philox_r29_asm_vkm")
    mparams = "" if mc == "s" else ",\n                                                 uint32_t m0, uint32_t m1"
    return f"""template <>
__device__ __forceinline__ void {fname}<{G}>(uint32_t (&x)[{G}], uint32_t (&y)[{G}],
                                                 uint32_t (&z)[{G}], uint32_t (&w)[{G}],
                                                 const uint32_t (&k0)[8], const uint32_t (&k1)[8]{mparams}) {{
    uint32_t yi[{G}], wi[{G}];
    uint64_t cc{"[" + str(NCC) + "]" if NCC > 1 else ""};
    for (int g = 0; g < {G}; ++g) {{ yi[g] = y[g]; wi[g] = w[g]; }}
    asm volatile(
{body}
        : {", ".join(ops_out)}
        : {", ".join(ops_in)}
        : {", ".join(clob)});
}}
"""


GS = (2, 3, 4, 5)  # call-group sizes of the shipped variant (philox10_n: G = 2..5)


def main():
    import sys
    lab = "--lab" in sys.argv[1:]
    out = ['// GENERATED by tools/gen_philox_asm.py' + (' --lab' if lab else '') + ' -- do not edit by hand.',
           '// Philox4x32-10 rounds 2..9 of G interleaved calls in one asm statement',
           '// (why and how: the generator\'s docstring).  Included by ba_device.hpp.',
           '#pragma once',
           '#include <stdint.h>',
           '',
           'namespace ba {',
           '']
    if lab:
        out += ['template <int G>',
                '__device__ __forceinline__ void philox_r29_asm(uint32_t (&x)[G], uint32_t (&y)[G],',
                '                                               uint32_t (&z)[G], uint32_t (&w)[G],',
                '                                               const uint32_t (&k0)[8], const uint32_t (&k1)[8]);',
                '// the same with the round keys as VGPR operands (VALU ops with an SGPR operand',
                '// issue slower: tools/valu_cost operands)',
                'template <int G>',
                '__device__ __forceinline__ void philox_r29_asm_vk(uint32_t (&x)[G], uint32_t (&y)[G],',
                '                                                  uint32_t (&z)[G], uint32_t (&w)[G],',
                '                                                  const uint32_t (&k0)[8], const uint32_t (&k1)[8]);']
    out += ['// round keys and multipliers as VGPR operands (VALU ops with an SGPR operand',
            '// issue slower: tools/valu_cost operands)',
            'template <int G>',
            '__device__ __forceinline__ void philox_r29_asm_vkm(uint32_t (&x)[G], uint32_t (&y)[G],',
            '                                                   uint32_t (&z)[G], uint32_t (&w)[G],',
            '                                                   const uint32_t (&k0)[8], const uint32_t (&k1)[8],',
            '                                                   uint32_t m0, uint32_t m1);',
            '']
    out.append('#ifdef __HIP_DEVICE_COMPILE__  // device code only (host passes never call it)')
    if lab:
        for G in (2, 3, 4):
            out.append(gen(G))
        for G in (2, 3, 4):
            out.append(gen(G, "v"))
    for G in GS:
        out.append(gen(G, "v", "v"))
    out.append('#endif')
    out.append('}  // namespace ba')
    print("\n".join(out))


if __name__ == "__main__":
    main()
