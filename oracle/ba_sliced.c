/*
 * ba_sliced.c -- word-sliced CPU restatement of the OM(m) hot path, OpenMP
 * over 64-trial words.
 *
 * TEST / BENCH INFRASTRUCTURE ONLY (see ba_oracle.h).  It is SURVEY.md §8b's
 * "CPU twin" (ba_run_trials_cpu) kept outside the product library: bench.py's
 * cpu_baseline leg times it (the fair CPU port: 64 trials per uint64 word and
 * one Philox call per two slot-words, the same minimum draw count the GPU
 * engines use), and the tests use it as a second checker at sizes the
 * textbook recursion of ba_oracle.c cannot reach (config 5: n=16, m=5, 1024
 * instances).  It is itself pinned bit-exactly against ba_oracle.c
 * (tests/test_oracle.py::test_sliced_port_equals_recursion), which is pinned
 * against ba.py's own fixtures.
 *
 * Method (level arrays, as the LEVELS engine does it, written independently):
 *   relay      L_k[x] = F[sender(x)] ? lie(k, x) : L_{k-1}[x / (L-k)]    ba.py:42-57, 263-277
 *   leaves     L_me generated block by block inside the level me-1 majority
 *   majority   R_p[s.b + b] = maj(L_p[s.b + b], R_{p+1}[(s.b + a)(s-1) + b - (b>a)] : a != b)
 *              strict; inner tie -> non-attack, root tie -> undefined      ba.py:159-195
 *   epilogue   quorum + IC1/IC2 per trial, as ba_oracle.c                   ba.py:197-255
 * Lies: bit t%64 of half x%2 of Philox4x32-10(key = seed, ctr = (x/2, k, w_lo, w_hi)),
 * w = t/64 (docs/SEMANTICS.md §3).  Philox mode only (table mode is OM(1) and
 * per trial: ba_oracle.c covers it).
 */
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "ba_oracle.h"

#define MAXN 32
#define MAXM 8
#define PB 16 /* Philox calls per vectorised batch */

enum { FAULTY_GIVEN = 0, FAULTY_RANDOM = 1, FAULTY_EXACT = 2 };
enum { ORDER_GIVEN = 0, ORDER_RANDOM = 1, ORDER_CONST = 2 };
enum { C_TRIALS, C_AGREE, C_VAPPL, C_VALID, C_QR, C_QA, C_QU, C_UNDEF, C_INB, C_VIOL, C_FTOT, C_ATT };

/* PB independent Philox4x32-10 calls in lockstep (the inner loops vectorise:
 * 32x32->64 products on every lane of a vector register). */
static void philox_batch(uint32_t* c0, uint32_t* c1, uint32_t* c2, uint32_t* c3, uint32_t k0,
                         uint32_t k1) {
    for (int r = 0; r < 10; ++r) {
        for (int i = 0; i < PB; ++i) {
            const uint64_t p0 = (uint64_t)0xD2511F53u * c0[i];
            const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2[i];
            const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1[i] ^ k0;
            const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3[i] ^ k1;
            c1[i] = (uint32_t)p1;
            c3[i] = (uint32_t)p0;
            c0[i] = n0;
            c2[i] = n2;
        }
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

/* lie words of level k, slots [x0, x0 + cnt) of global word gw -> out[0..cnt) */
static void lie_words(uint64_t seed, uint32_t k, uint64_t x0, uint64_t cnt, uint64_t gw,
                      uint64_t* out) {
    uint32_t c0[PB], c1[PB], c2[PB], c3[PB];
    const uint64_t p0 = x0 >> 1, p1 = (x0 + cnt + 1) >> 1; /* pairs covering the range */
    for (uint64_t pb = p0; pb < p1; pb += PB) {
        for (int i = 0; i < PB; ++i) {
            c0[i] = (uint32_t)(pb + (uint64_t)i);
            c1[i] = k;
            c2[i] = (uint32_t)gw;
            c3[i] = (uint32_t)(gw >> 32);
        }
        philox_batch(c0, c1, c2, c3, (uint32_t)seed, (uint32_t)(seed >> 32));
        for (int i = 0; i < PB && pb + (uint64_t)i < p1; ++i) {
            const uint64_t x = 2 * (pb + (uint64_t)i);
            const uint64_t h0 = (uint64_t)c1[i] << 32 | c0[i];
            const uint64_t h1 = (uint64_t)c3[i] << 32 | c2[i];
            if (x >= x0 && x < x0 + cnt) out[x - x0] = h0;
            if (x + 1 >= x0 && x + 1 < x0 + cnt) out[x + 1 - x0] = h1;
        }
    }
}

typedef struct {
    int L, me;
    uint64_t S[MAXM + 1];    /* S[k] = P(L, k+1) */
    uint8_t* last[MAXM + 1]; /* last[k][x]: last lieutenant (0-based) of path x, k < me */
} geo_t;

static uint64_t perm(int L, int len) {
    uint64_t p = 1;
    for (int i = 0; i < len; ++i) p *= (uint64_t)(L - i);
    return p;
}

/* last element of every path of levels 0..me-1, paths in lexicographic order */
static int geo_build(geo_t* g, int L, int me) {
    memset(g, 0, sizeof *g);
    g->L = L;
    g->me = me;
    for (int k = 0; k <= me; ++k) g->S[k] = perm(L, k + 1);
    for (int k = 0; k < me; ++k) {
        g->last[k] = (uint8_t*)malloc(g->S[k]);
        if (!g->last[k]) return -1;
    }
    if (me == 0) return 0;
    /* level k slot x = (parent slot) * (L-k) + rank of the appended lieutenant
     * among those not on the parent path */
    for (int r = 0; r < L; ++r) g->last[0][r] = (uint8_t)r;
    for (int k = 1; k < me; ++k) {
        const uint64_t fan = (uint64_t)(L - k);
        /* walk parents; rebuild each parent's path from its ancestors' last[] */
        for (uint64_t par = 0; par < g->S[k - 1]; ++par) {
            uint32_t used = 0;
            uint64_t a = par;
            for (int j = k - 1; j >= 0; --j) {
                used |= 1u << g->last[j][a];
                if (j > 0) a /= (uint64_t)(L - j);
            }
            uint64_t c = 0;
            for (int r = 0; r < L; ++r)
                if (!((used >> r) & 1u)) g->last[k][par * fan + c++] = (uint8_t)r;
        }
    }
    return 0;
}

static void geo_free(geo_t* g) {
    for (int k = 0; k <= MAXM; ++k) free(g->last[k]);
}

/* bit-sliced strict-majority test over s inputs: cnt[] planes, returns lanes
 * with 2*count > s (gt) and 2*count == s (eq) */
static void maj_planes(const uint64_t* c, int P, int s, uint64_t* gt, uint64_t* eq) {
    /* lanes with count >= T, T = floor(s/2)+1 ; tie: count == s/2 (s even) */
    const int T = s / 2 + 1;
    uint64_t g = 0, e = ~0ull;
    for (int i = P - 1; i >= 0; --i) {
        if ((T >> i) & 1) e &= c[i];
        else {
            g |= e & c[i];
            e &= ~c[i];
        }
    }
    *gt = g | e;
    *eq = 0;
    if (s % 2 == 0) {
        const int H = s / 2;
        uint64_t e2 = ~0ull;
        for (int i = P - 1; i >= 0; --i) e2 &= ((H >> i) & 1) ? c[i] : ~c[i];
        *eq = e2;
    }
}

static void planes_add(uint64_t* c, int P, uint64_t x) {
    for (int i = 0; i < P && x; ++i) {
        const uint64_t t = c[i] & x;
        c[i] ^= x;
        x = t;
    }
}

static int planes_for(int s) {
    int p = 1;
    while ((1 << p) <= s) ++p;
    return p;
}

typedef struct {
    uint64_t* Lk[MAXM + 1]; /* L_0 .. L_{me-1} */
    uint64_t* Rk[MAXM + 1]; /* R_1 .. R_{me-1} */
    uint64_t* lie;          /* lie words of one level (relay) or one leaf block */
    uint64_t A[MAXN], U[MAXN];
} scratch_t;

/* One 64-trial word: F[g] faulty planes, ob = order is attack, roots -> A/U. */
static void om_word(const geo_t* g, uint64_t seed, uint64_t gw, const uint64_t* F, uint64_t ob,
                    scratch_t* w) {
    const int L = g->L, me = g->me;
    /* level 0: commander send (ba.py:263-277) */
    lie_words(seed, 0, 0, (uint64_t)L, gw, w->lie);
    for (int r = 0; r < L; ++r) w->Lk[0][r] = (F[0] & w->lie[r]) | (~F[0] & ob);
    if (me == 0) {
        for (int r = 0; r < L; ++r) {
            w->A[r] = w->Lk[0][r];
            w->U[r] = 0;
        }
        return;
    }
    /* relay levels 1..me-1 (ba.py:42-57 generalised) */
    for (int k = 1; k < me; ++k) {
        const uint64_t fan = (uint64_t)(L - k);
        lie_words(seed, (uint32_t)k, 0, g->S[k], gw, w->lie);
        for (uint64_t x = 0; x < g->S[k]; ++x) {
            const uint64_t par = x / fan;
            const uint64_t fs = F[g->last[k - 1][par] + 1];
            w->Lk[k][x] = (fs & w->lie[x]) | (~fs & w->Lk[k - 1][par]);
        }
    }
    /* majorities, level me-1 down to 0; level me-1 reads leaves made on the fly */
    for (int p = me - 1; p >= 0; --p) {
        const int s = L - p; /* members of a prefix at level p */
        const int P = planes_for(s);
        const uint64_t nprefix = p == 0 ? 1 : g->S[p - 1];
        const uint64_t* Lp = w->Lk[p];
        for (uint64_t sr = 0; sr < nprefix; ++sr) {
            const uint64_t base = sr * (uint64_t)s;
            const uint64_t cbase = base * (uint64_t)(s - 1);
            const uint64_t* child;
            if (p == me - 1) { /* leaf block: L_me[cbase + a(s-1) + c] */
                lie_words(seed, (uint32_t)me, cbase, (uint64_t)s * (s - 1), gw, w->lie);
                for (int a = 0; a < s; ++a) {
                    const uint64_t fs = F[g->last[me - 1][base + a] + 1];
                    const uint64_t v = Lp[base + a];
                    uint64_t* row = w->lie + (uint64_t)a * (s - 1);
                    for (int c = 0; c < s - 1; ++c) row[c] = (fs & row[c]) | (~fs & v);
                }
                child = w->lie;
            } else {
                child = w->Rk[p + 1] + cbase;
            }
            for (int b = 0; b < s; ++b) {
                uint64_t c[6] = {0, 0, 0, 0, 0, 0};
                planes_add(c, P, Lp[base + b]);
                for (int a = 0; a < s; ++a)
                    if (a != b) planes_add(c, P, child[(uint64_t)a * (s - 1) + b - (b > a)]);
                uint64_t gt, eq;
                maj_planes(c, P, s, &gt, &eq);
                if (p == 0) {
                    w->A[b] = gt;
                    w->U[b] = eq;
                } else {
                    w->Rk[p][base + b] = gt; /* inner tie -> non-attack */
                }
            }
        }
    }
}

int ba_sliced_run(uint32_t n, uint32_t m, uint64_t seed, uint32_t faulty_mode, uint32_t f,
                  uint32_t order_mode, uint32_t order_value, uint64_t first_trial, uint64_t batch,
                  const uint32_t* faulty, const uint8_t* order, uint64_t* decisions,
                  uint8_t* outcome, uint64_t* counters, int threads) {
    if (n < 1 || n > MAXN || m > MAXM) return -1;
    if (faulty_mode > FAULTY_EXACT || order_mode > ORDER_CONST) return -1;
    if (faulty_mode == FAULTY_GIVEN && !faulty) return -1;
    if (order_mode == ORDER_GIVEN && !order) return -1;
    if (first_trial & 63) return -1;
    const int L = (int)n - 1;
    const int me = n >= 2 ? ((int)m < (int)n - 2 ? (int)m : (int)n - 2) : 0;
    if (L == 0) return -4; /* a lone commander: ba_oracle.c covers n = 1 */
    geo_t g;
    if (geo_build(&g, L, me) != 0) {
        geo_free(&g);
        return -2;
    }
    uint64_t total[BA_ORACLE_NCOUNTERS];
    memset(total, 0, sizeof total);
    const uint64_t words = (batch + 63) / 64;
    uint64_t maxlvl = 0; /* largest materialised level (L_me is never stored) */
    for (int k = 0; k < me || k == 0; ++k) maxlvl = g.S[k] > maxlvl ? g.S[k] : maxlvl;
    const uint64_t leafblk = (uint64_t)(L - me + 1) * (uint64_t)(L - me);
    int err = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel
    {
        scratch_t w;
        memset(&w, 0, sizeof w);
        int ok = 1;
        for (int k = 0; k < me || k == 0; ++k) {
            w.Lk[k] = (uint64_t*)malloc(g.S[k] * 8);
            ok &= w.Lk[k] != NULL;
        }
        for (int k = 1; k < me; ++k) {
            w.Rk[k] = (uint64_t*)malloc(g.S[k] * 8);
            ok &= w.Rk[k] != NULL;
        }
        w.lie = (uint64_t*)malloc((maxlvl > leafblk ? maxlvl : leafblk) * 8 + 16);
        ok &= w.lie != NULL;
        uint64_t cnt[BA_ORACLE_NCOUNTERS];
        memset(cnt, 0, sizeof cnt);
        if (!ok) {
#pragma omp atomic write
            err = 1;
        }
#pragma omp for schedule(dynamic, 1)
        for (int64_t wi = 0; wi < (int64_t)words; ++wi) {
            if (!ok) continue;
            uint32_t fm[64];
            uint8_t oc[64];
            uint64_t F[MAXN + 1], ob = 0, val = 0;
            memset(F, 0, sizeof F);
            for (int i = 0; i < 64; ++i) {
                const uint64_t li = (uint64_t)wi * 64 + (uint64_t)i;
                fm[i] = 0;
                oc[i] = 0;
                if (li >= batch) continue;
                fm[i] = faulty_mode == FAULTY_GIVEN ? faulty[li] : 0;
                oc[i] = order_mode == ORDER_GIVEN ? order[li] : 0;
                ba_oracle_gen(n, seed, faulty_mode, f, order_mode, order_value, first_trial + li,
                              faulty_mode == FAULTY_GIVEN ? NULL : &fm[i],
                              order_mode == ORDER_GIVEN ? NULL : &oc[i]);
                fm[i] &= n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u);
                val |= 1ull << i;
                ob |= (uint64_t)(oc[i] == 1) << i;
                for (uint32_t q = 0; q < n; ++q) F[q] |= (uint64_t)((fm[i] >> q) & 1u) << i;
            }
            om_word(&g, seed, (first_trial >> 6) + (uint64_t)wi, F, ob, &w);
            /* per-trial epilogue (ba.py:197-255), restated as in ba_oracle.c */
            for (int i = 0; i < 64; ++i) {
                if (!((val >> i) & 1u)) continue;
                const uint64_t li = (uint64_t)wi * 64 + (uint64_t)i;
                int na = 0, nr = 0, nu = 0, nA = 0, nU = 0;
                if (oc[i] == 1) ++na; else if (oc[i] == 0) ++nr; else ++nu;
                uint64_t dword = 0;
                int dec[MAXN];
                for (int r = 0; r < L; ++r) {
                    const int a = (int)((w.A[r] >> i) & 1u), u = (int)((w.U[r] >> i) & 1u);
                    dec[r] = a ? 1 : (u ? 2 : 0);
                    if (dec[r] == 1) { ++na; ++nA; }
                    else if (dec[r] == 0) ++nr;
                    else { ++nu; ++nU; }
                    dword |= (uint64_t)dec[r] << (2 * r);
                }
                const int tot = na + nr + nu;
                int needed = 2 * ((tot - 1) / 3) + 1;
                if (tot <= 3) needed = tot - 1;
                if (tot == 1) needed = 1;
                const int q = needed <= nr ? 0 : (needed <= na ? 1 : 2);
                const int appl = !(fm[i] & 1u);
                const int want = oc[i] == 1 ? 1 : 0;
                int agree = 1, first = -1, valid = appl;
                for (int r = 0; r < L; ++r) {
                    if ((fm[i] >> (r + 1)) & 1u) continue;
                    if (first < 0) first = dec[r]; else if (dec[r] != first) agree = 0;
                    if (dec[r] != want) valid = 0;
                }
                const int nf = __builtin_popcount(fm[i]);
                const int inb = nf <= me && (int)n > 3 * me;
                if (decisions) decisions[li] = dword;
                if (outcome) outcome[li] = (uint8_t)(q | agree << 2 | appl << 3 | valid << 4 | inb << 5);
                cnt[C_TRIALS] += 1;
                cnt[C_AGREE] += (uint64_t)agree;
                cnt[C_VAPPL] += (uint64_t)appl;
                cnt[C_VALID] += (uint64_t)valid;
                cnt[C_QR + q] += 1;
                cnt[C_UNDEF] += (uint64_t)nU;
                cnt[C_ATT] += (uint64_t)nA;
                cnt[C_INB] += (uint64_t)inb;
                cnt[C_VIOL] += (uint64_t)(inb && (!agree || (appl && !valid)));
                cnt[C_FTOT] += (uint64_t)nf;
            }
        }
#pragma omp critical
        for (int j = 0; j < BA_ORACLE_NCOUNTERS; ++j) total[j] += cnt[j];
        for (int k = 0; k <= MAXM; ++k) {
            free(w.Lk[k]);
            free(w.Rk[k]);
        }
        free(w.lie);
    }
    geo_free(&g);
    if (err) return -2;
    if (counters) memcpy(counters, total, sizeof total);
    return 0;
}

/* Synthetic inputs of trials [first_trial, first_trial + batch) (ba_oracle_gen,
 * OpenMP): stages a bench sample's inputs outside the timed CPU region, as
 * bench.py stages the GPU's. */
int ba_sliced_gen(uint32_t n, uint64_t seed, uint32_t faulty_mode, uint32_t f, uint32_t order_mode,
                  uint32_t order_value, uint64_t first_trial, uint64_t batch, uint32_t* faulty,
                  uint8_t* order, int threads) {
    if (n < 1 || n > MAXN || faulty_mode == FAULTY_GIVEN || order_mode == ORDER_GIVEN) return -1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < (int64_t)batch; ++i) {
        uint32_t fm = 0;
        uint8_t oc = 0;
        ba_oracle_gen(n, seed, faulty_mode, f, order_mode, order_value, first_trial + (uint64_t)i,
                      &fm, &oc);
        faulty[i] = fm & (n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u));
        order[i] = oc;
    }
    return 0;
}
