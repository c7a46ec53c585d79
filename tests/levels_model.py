"""NumPy model of the LEVELS engine's bit-sliced slot arithmetic (tests only).

Mirrors what the HIP kernels compute -- 64-trial words, parent(x) = x // (L-k),
children of (sigma, b) at (sigma_rank*s + a)*(s-1) + b - [b > a], the sender
table, lie words from one Philox call per slot pair -- so that the closed-form
indexing can be checked against the recursive oracle on the CPU, independent
of the GPU.
"""
from __future__ import annotations

import itertools
import sys

import numpy as np

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__file__), "..", "oracle"))
import ba_oracle as O  # noqa: E402

U64 = np.uint64


def perm_count(L, length):
    p = 1
    for i in range(length):
        p *= L - i
    return max(p, 0)


def sender_table(L, me):
    """Per level k < me: general index of the last element of every slot (lex order)."""
    out = []
    for k in range(me):
        out.append([tau[-1] + 1 for tau in itertools.permutations(range(L), k + 1)])
    return out


def lie_words(seed, k, pair, gw):
    o = O.philox4x32_10((pair, k, gw & 0xFFFFFFFF, gw >> 32), (seed & 0xFFFFFFFF, seed >> 32))
    return (o[1] << 32 | o[0]), (o[3] << 32 | o[2])


def count_ge(words, T):
    """Bit-sliced: for each bit position, [number of words with that bit set >= T]."""
    cnt = [0] * 64
    for w in words:
        for b in range(64):
            cnt[b] += (int(w) >> b) & 1
    return sum(1 << b for b in range(64) if cnt[b] >= T)


def run_word(n, m, seed, gw, fmasks, orders):
    """Resolve one 64-trial word.  fmasks/orders: 64 per-trial inputs."""
    L, me = n - 1, O.effective_depth(n, m)
    F = [sum(((fmasks[t] >> g) & 1) << t for t in range(64)) for g in range(n)]
    OB = sum((1 if orders[t] == 1 else 0) << t for t in range(64))
    snd = sender_table(L, me)
    Lv = []
    for k in range(me + 1):
        S = perm_count(L, k + 1)
        lvl = [0] * S
        for pair in range((S + 1) // 2):
            lw = lie_words(seed, k, pair, gw)
            for h in range(2):
                x = 2 * pair + h
                if x >= S:
                    break
                if k == 0:
                    parent, fw = OB, F[0]
                else:
                    y = x // (L - k)
                    parent, fw = Lv[k - 1][y], F[snd[k - 1][y]]
                lvl[x] = (fw & lw[h]) | (~fw & parent & 0xFFFFFFFFFFFFFFFF)
        Lv.append(lvl)
    R = {me: Lv[me]}
    for p in range(me - 1, 0, -1):
        s = L - p
        C = R[p + 1]
        Rp = []
        for y in range(perm_count(L, p + 1)):
            sr, b = divmod(y, s)
            ins = [Lv[p][y]] + [C[(sr * s + a) * (s - 1) + (b - (b > a))] for a in range(s) if a != b]
            Rp.append(count_ge(ins, s // 2 + 1))
        R[p] = Rp
    dec = [[0] * L for _ in range(64)]
    for b in range(L):
        ins = [Lv[0][b]]
        if me >= 1:
            ins += [R[1][a * (L - 1) + (b - (b > a))] for a in range(L) if a != b]
        att = count_ge(ins, L // 2 + 1)
        tie = 0 if L & 1 else (count_ge(ins, L // 2) & ~att)
        for t in range(64):
            dec[t][b] = 1 if (att >> t) & 1 else (2 if (tie >> t) & 1 else 0)
    return dec
