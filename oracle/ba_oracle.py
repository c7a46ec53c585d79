"""Pure-Python restatement of the reference's OM(m) hot path.

TEST INFRASTRUCTURE ONLY: the parity checker for libba_hip.so (used by tests/
and nothing else).  Pure-Python loops -- small cases only.  The faster C twin
is oracle/ba_oracle.c; tests cross-check the two.

Reference anchors (/root/reference/ba.py):
  Process.order            ba.py:257-285  commander send; faulty -> coin per recipient
  Serv.exposed_get_order   ba.py:42-57    relay; faulty -> fresh coin per query
  coin                     ba.py:45, 269  random.randint(0, 1) == 0 -> "attack"
  Process.get_majority     ba.py:159-195  own value + answers, strict majority, tie undefined
  get_majorities/quorum    ba.py:197-255  tally every live general, 2k+1 of 3k+1
OM(m>=2) follows SURVEY.md Appendix A (inner tie -> non-attack).
"""
from __future__ import annotations

import random

M32 = 0xFFFFFFFF
RETREAT, ATTACK, OTHER, UNDEFINED = 0, 1, 2, 2
Q_RETREAT, Q_ATTACK, Q_UNDET = 0, 1, 2
LIE_PHILOX, LIE_TABLE = 0, 1
FAULTY_GIVEN, FAULTY_RANDOM, FAULTY_EXACT = 0, 1, 2
ORDER_GIVEN, ORDER_RANDOM, ORDER_CONST = 0, 1, 2
COUNTERS = ["trials", "agreement", "validity_applicable", "validity", "quorum_retreat",
            "quorum_attack", "quorum_undetermined", "undefined_decisions", "in_bound",
            "bound_violations", "faulty_total", "attack_decisions"]


def philox4x32_10(ctr, key):
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    for _ in range(10):
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & M32, p1 & M32, ((p0 >> 32) ^ c3 ^ k1) & M32, p0 & M32
        k0 = (k0 + 0x9E3779B9) & M32
        k1 = (k1 + 0xBB67AE85) & M32
    return c0, c1, c2, c3


def lie(seed: int, t: int, k: int, x: int) -> int:
    """Lie bit (1 = attack) of trial t at level k, slot x (docs/SEMANTICS.md §3)."""
    w = t >> 6
    o = philox4x32_10((x >> 1, k, w & M32, w >> 32), (seed & M32, seed >> 32))
    half = (o[3] << 32 | o[2]) if (x & 1) else (o[1] << 32 | o[0])
    return (half >> (t & 63)) & 1


def gen(n, seed, faulty_mode, f, order_mode, order_value, t):
    """Synthetic (faulty_mask, order) of trial t (docs/SEMANTICS.md §4)."""
    u = []
    call = 0
    while len(u) < 2 + n:
        u.extend(philox4x32_10((call, M32, t & M32, t >> 32), (seed & M32, seed >> 32)))
        call += 1
    order = None
    if order_mode == ORDER_RANDOM:
        order = u[0] >> 31
    elif order_mode == ORDER_CONST:
        order = order_value
    mask = None
    if faulty_mode != FAULTY_GIVEN:
        if faulty_mode == FAULTY_RANDOM:
            nf = (u[1] * (min(f, n) + 1)) >> 32
        else:
            nf = min(f, n)
        mask = 0
        for i in range(nf):  # j-th (ascending) general not chosen yet
            j = (u[2 + i] * (n - i)) >> 32
            free = [g for g in range(n) if not (mask >> g) & 1]
            mask |= 1 << free[j]
    return mask, order


def path_rank(tau, L):
    """Lexicographic rank of the relay path tau among len(tau)-permutations of L lieutenants."""
    rank, used = 0, set()
    for i, x in enumerate(tau):
        rank = rank * (L - i) + sum(1 for y in range(x) if y not in used)
        used.add(x)
    return rank


def effective_depth(n, m):
    return min(m, n - 2) if n >= 2 else 0


def om_decisions(n, m, seed, t, fmask, ob):
    """Root decisions of lieutenants 1..n-1 (list index r-1), Philox lies."""
    L, me = n - 1, effective_depth(n, m)

    def faulty(g):
        return (fmask >> g) & 1

    def val(sigma, r):  # value r received through relay chain sigma
        sender = 0 if not sigma else sigma[-1] + 1
        if faulty(sender):
            return lie(seed, t, len(sigma), path_rank(sigma + (r,), L))
        if not sigma:
            return ob
        return val(sigma[:-1], sigma[-1])

    def resolve(sigma, r):
        v = val(sigma, r)
        if len(sigma) == me:
            return v
        a, c = v, 1
        for j in range(L):
            if j in sigma or j == r:
                continue
            a += resolve(sigma + (j,), r)
            c += 1
        if not sigma:
            return ATTACK if 2 * a > c else (RETREAT if 2 * a < c else UNDEFINED)
        return 1 if 2 * a > c else 0

    return [resolve((), r) for r in range(L)]


def canonical_coin_count(n, fmask, m=1, poll=0):
    """Coins ba.py draws for one actual-order round (canonical schedule)."""
    L = n - 1
    c = L if fmask & 1 else 0
    if m >= 1:
        nf = sum((fmask >> g) & 1 for g in range(1, n))
        for r in range(1, n):
            c += nf - ((fmask >> r) & 1)
            if (poll >> r) & 1 and fmask & 1:
                c += 1
    return c


def om1_table_decisions(n, m, fmask, ob, coins, poll=0):
    """ba.py's OM(1) in canonical draw order; coins[i] = 1 means attack.

    poll bit r: lieutenant r also polls the commander (stale primary_port,
    ba.py:169-172); the relay round exists iff m >= 1."""
    it = iter(coins)
    v = [0] * n
    for r in range(1, n):  # ba.py:263-277
        v[r] = next(it) if fmask & 1 else ob
    dec = []
    for r in range(1, n):  # ba.py:159-195, receiver-major, port order
        a, c = v[r], 1
        if m >= 1:
            if (poll >> r) & 1:
                a += next(it) if fmask & 1 else ob
                c += 1
            for j in range(1, n):
                if j == r:
                    continue
                a += next(it) if (fmask >> j) & 1 else v[j]
                c += 1
        dec.append(ATTACK if 2 * a > c else (RETREAT if 2 * a < c else UNDEFINED))
    return dec


def quorum(n, order_code, dec):
    """(code, na, nr, nu, needed) of ba.py:225-253 over every live general."""
    na = nr = nu = 0
    for d in [order_code] + list(dec):
        if d == ATTACK:
            na += 1
        elif d == RETREAT:
            nr += 1
        else:
            nu += 1
    total = na + nr + nu
    needed = 2 * ((total - 1) // 3) + 1
    if total <= 3:
        needed = total - 1
    if total == 1:
        needed = 1
    code = Q_RETREAT if needed <= nr else (Q_ATTACK if needed <= na else Q_UNDET)
    return code, na, nr, nu, needed


def trial_outcome(n, m, fmask, order_code, dec):
    me = effective_depth(n, m)
    q = quorum(n, order_code, dec)[0]
    loyal = [dec[r - 1] for r in range(1, n) if not (fmask >> r) & 1]
    agree = int(len(set(loyal)) <= 1)
    appl = int(not fmask & 1)
    want = ATTACK if order_code == ATTACK else RETREAT
    valid = int(appl and all(d == want for d in loyal))
    nf = bin(fmask).count("1")
    inb = int(nf <= me and n > 3 * me)
    return q | agree << 2 | appl << 3 | valid << 4 | inb << 5


def run(n, m, seed=0, lie_mode=LIE_PHILOX, faulty_mode=FAULTY_GIVEN, f=0,
        order_mode=ORDER_GIVEN, order_value=ATTACK, first_trial=0, batch=1,
        faulty=None, order=None, table=None, poll=None):
    """Python twin of ba_oracle_run: returns (decisions, outcomes, counters dict)."""
    decisions, outcomes = [], []
    cnt = dict.fromkeys(COUNTERS, 0)
    me = effective_depth(n, m)
    for i in range(batch):
        t = first_trial + i
        gm, go = gen(n, seed, faulty_mode, f, order_mode, order_value, t)
        fmask = faulty[i] if faulty_mode == FAULTY_GIVEN else gm
        fmask &= (1 << n) - 1
        oc = order[i] if order_mode == ORDER_GIVEN else go
        ob = int(oc == ATTACK)
        if lie_mode == LIE_TABLE:
            pm = (poll[i] if poll is not None else 0) & ((1 << n) - 2)
            dec = om1_table_decisions(n, m, fmask, ob, table[i], pm)
        else:
            dec = om_decisions(n, m, seed, t, fmask, ob)
        word = 0
        for r, d in enumerate(dec):
            word |= d << (2 * r)
        out = trial_outcome(n, m, fmask, oc, dec)
        decisions.append(word)
        outcomes.append(out)
        q = out & 3
        cnt["trials"] += 1
        cnt["agreement"] += (out >> 2) & 1
        cnt["validity_applicable"] += (out >> 3) & 1
        cnt["validity"] += (out >> 4) & 1
        cnt[["quorum_retreat", "quorum_attack", "quorum_undetermined"][q]] += 1
        cnt["undefined_decisions"] += sum(1 for d in dec if d == UNDEFINED)
        cnt["attack_decisions"] += sum(1 for d in dec if d == ATTACK)
        inb = (out >> 5) & 1
        cnt["in_bound"] += inb
        ok = ((out >> 2) & 1) and (not ((out >> 3) & 1) or ((out >> 4) & 1))
        cnt["bound_violations"] += int(inb and not ok)
        cnt["faulty_total"] += bin(fmask).count("1")
    return decisions, outcomes, cnt


def mt_coins(rng: random.Random, n: int, fmask: int, m: int = 1, poll: int = 0):
    """Draw one round's coins exactly as ba.py does (random.randint(0,1)), 1 = attack."""
    return [1 if rng.randint(0, 1) == 0 else 0
            for _ in range(canonical_coin_count(n, fmask, m, poll))]
