/*
 * ba_oracle.c -- CPU restatement of the reference's OM(m) hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see ba_oracle.h).  It is the checker for
 * libba_hip.so and the "port" CPU baseline of bench.py; the product never
 * links or loads it.
 *
 * The restatement is deliberately written the "textbook" way -- an explicit
 * recursion over relay paths with lexicographic path ranks computed from
 * scratch -- so that it shares no indexing arithmetic with the GPU engines
 * (which work on bit-sliced 64-trial words with closed-form slot arithmetic).
 *
 * Parity anchors (file:line in /root/reference/ba.py):
 *   commander send, faulty commander flips a coin per recipient   ba.py:263-277
 *   commander's own majority is its order                         ba.py:285
 *   faulty relay answers a fresh coin per query                   ba.py:44-49
 *   loyal relay answers what it received                          ba.py:53-57
 *   coin: random.randint(0,1) == 0 -> "attack"                    ba.py:45, 269
 *   lieutenant counts own value + answers; non-attack = retreat   ba.py:160-186
 *   strict majority, tie -> "undefined"                           ba.py:188-195
 *   quorum tally over every live general, thresholds              ba.py:197-235
 *   retreat checked before attack                                 ba.py:246-253
 * OM(m>=2): SURVEY.md Appendix A (inner tie -> non-attack, root tie -> undefined).
 */
#include "ba_oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* numeric contract shared with include/ba.h (checked by tests/test_oracle.py) */
enum { LIE_PHILOX = 0, LIE_TABLE = 1 };
enum { FAULTY_GIVEN = 0, FAULTY_RANDOM = 1, FAULTY_EXACT = 2 };
enum { ORDER_GIVEN = 0, ORDER_RANDOM = 1, ORDER_CONST = 2 };
enum { V_RETREAT = 0, V_ATTACK = 1, V_OTHER = 2, V_UNDEF = 2 };
enum { Q_RETREAT = 0, Q_ATTACK = 1, Q_UNDET = 2 };
enum {
    C_TRIALS, C_AGREE, C_VAPPL, C_VALID, C_QR, C_QA, C_QU, C_UNDEF,
    C_INB, C_VIOL, C_FTOT, C_ATT
};
#define E_INVAL (-1)
#define E_NOTSUP (-4)
#define E_TOOBIG (-5)
#define MAXN 32
#define MAXM 8

/* ------------------------------------------------------------------------- */
/* Philox4x32-10                                                             */
/* ------------------------------------------------------------------------- */
void ba_oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int round = 0; round < 10; ++round) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* lie(t, k, x): bit (t mod 64) of the 64-bit half (x mod 2) of
 * Philox4x32-10(key = seed, ctr = (x/2, k, w_lo, w_hi)), w = t / 64.
 * One Philox call therefore covers two slots of one 64-trial word. */
uint32_t ba_oracle_lie(uint64_t seed, uint64_t t, uint32_t k, uint64_t x) {
    uint64_t w = t >> 6;
    uint32_t ctr[4] = {(uint32_t)(x >> 1), k, (uint32_t)w, (uint32_t)(w >> 32)};
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t o[4];
    ba_oracle_philox(ctr, key, o);
    uint64_t half = (x & 1) ? ((uint64_t)o[3] << 32 | o[2]) : ((uint64_t)o[1] << 32 | o[0]);
    return (uint32_t)(half >> (t & 63)) & 1u;
}

static uint32_t mulhi_range(uint32_t u, uint32_t range) {
    return (uint32_t)(((uint64_t)u * range) >> 32);
}

/* Synthetic inputs, SURVEY.md §8d: order ~ Bernoulli(1/2); f ~ U{0..fmax} (or
 * exactly f); faulty set = uniform f-subset of the n generals (the commander
 * may be faulty) by sequential selection without replacement (the index form
 * of a partial Fisher-Yates draw).  Random words u[i] are word i%4 of
 * Philox4x32-10(key = seed, ctr = (i/4, 0xFFFFFFFF, t_lo, t_hi)). */
void ba_oracle_gen(uint32_t n, uint64_t seed, uint32_t faulty_mode, uint32_t f,
                   uint32_t order_mode, uint32_t order_value, uint64_t t,
                   uint32_t* faulty_mask, uint8_t* order) {
    uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    uint32_t u[4 * ((MAXN + 2 + 3) / 4)];
    uint32_t need = 2 + (n < MAXN ? n : MAXN);
    for (uint32_t call = 0; call * 4 < need; ++call) {
        uint32_t ctr[4] = {call, 0xFFFFFFFFu, (uint32_t)t, (uint32_t)(t >> 32)};
        ba_oracle_philox(ctr, key, u + 4 * call);
    }
    if (order) {
        if (order_mode == ORDER_RANDOM) *order = (uint8_t)(u[0] >> 31);
        else if (order_mode == ORDER_CONST) *order = (uint8_t)order_value;
    }
    if (faulty_mask && faulty_mode != FAULTY_GIVEN) {
        uint32_t nf;
        if (faulty_mode == FAULTY_RANDOM) {
            uint32_t fmax = f < n ? f : n;
            nf = mulhi_range(u[1], fmax + 1);
        } else {
            nf = f < n ? f : n;
        }
        /* sequential selection without replacement: step i takes the j-th
         * (ascending) general not yet chosen, j = floor(u[2+i] * (n-i) / 2^32) */
        uint32_t mask = 0;
        for (uint32_t i = 0; i < nf; ++i) {
            uint32_t j = mulhi_range(u[2 + i], n - i);
            for (uint32_t g = 0; g < n; ++g) {
                if ((mask >> g) & 1u) continue;
                if (j == 0) { mask |= 1u << g; break; }
                --j;
            }
        }
        *faulty_mask = mask;
    }
}

/* ------------------------------------------------------------------------- */
/* OM(m) restatement over explicit relay paths                               */
/* ------------------------------------------------------------------------- */
typedef struct {
    uint64_t seed, t;
    int L;          /* lieutenants: ranks 0..L-1 = generals 1..L */
    int me;         /* effective depth */
    uint32_t fmask; /* bit i = general i faulty */
    int ob;         /* relayed order bit: 1 iff order == attack */
} tctx;

/* Lexicographic rank of the path tau[0..len-1] among all len-permutations of
 * the L lieutenants (the slot index of the path in its level). */
static uint64_t path_rank(const int* tau, int len, int L) {
    uint64_t rank = 0;
    uint32_t used = 0;
    for (int i = 0; i < len; ++i) {
        uint32_t below = ((1u << tau[i]) - 1u) & ~used;
        rank = rank * (uint64_t)(L - i) + (uint64_t)__builtin_popcount(below);
        used |= 1u << tau[i];
    }
    return rank;
}

static int is_faulty(const tctx* c, int general) { return (int)((c->fmask >> general) & 1u); }

/* val_r(sigma): the value lieutenant r received through relay chain sigma
 * (path[0..len-1]); path[len] is overwritten with r. */
static int om_val(const tctx* c, int* path, int len, int r) {
    path[len] = r;
    int sender = (len == 0) ? 0 : path[len - 1] + 1;
    if (is_faulty(c, sender))  /* ba.py:44-49 / 268-273: fresh coin */
        return (int)ba_oracle_lie(c->seed, c->t, (uint32_t)len, path_rank(path, len + 1, c->L));
    if (len == 0) return c->ob; /* ba.py:276-277 loyal commander */
    return om_val(c, path, len - 1, path[len - 1]); /* ba.py:53-57 loyal relay */
}

/* resolve_r(sigma): leaf value at depth me, else majority of val_r(sigma) and
 * resolve_r(sigma.j) for every j not in sigma, j != r (ba.py:159-195). */
static int om_resolve(const tctx* c, int* path, int len, int r, uint32_t used) {
    int v = om_val(c, path, len, r);
    if (len == c->me) return v; /* at len==0 (me==0): 1 input, codes coincide */
    int a = v, cnt = 1;
    for (int j = 0; j < c->L; ++j) {
        if (((used >> j) & 1u) || j == r) continue;
        path[len] = j;
        a += om_resolve(c, path, len + 1, r, used | (1u << j));
        ++cnt;
    }
    if (len == 0) return 2 * a > cnt ? V_ATTACK : (2 * a < cnt ? V_RETREAT : V_UNDEF);
    return 2 * a > cnt; /* inner tie -> non-attack */
}

/* ba.py's canonical draw order at m=1 (SURVEY.md §8a lie row): the commander's
 * coins per recipient (ba.py:263-273), then each lieutenant r in id order asks
 * the live generals in port order (ba.py:169-176) -- every other lieutenant j,
 * and the commander too when r's primary_port is stale (poll bit r; ba.py:171
 * skips only the port r believes is the primary's).  Faulty answerers draw.
 * The relay round exists iff m >= 1 (ba.py is OM(1)). */
static void om1_table(int n, int relay, uint32_t fmask, uint32_t poll, int ob,
                      const uint32_t* row, int* dec) {
    int v[MAXN];
    uint32_t c = 0;
#define COIN() ((int)((row[c >> 5] >> (c & 31)) & 1u)); ++c
    for (int r = 1; r < n; ++r) {
        if (fmask & 1u) { v[r] = COIN(); } else { v[r] = ob; }
    }
    for (int r = 1; r < n; ++r) {
        int a = v[r], cnt = 1;
        if (relay) {
            if ((poll >> r) & 1u) { /* the commander answers get_order (ba.py:42-57) */
                int x;
                if (fmask & 1u) { x = COIN(); } else { x = ob; }
                a += x;
                ++cnt;
            }
            for (int j = 1; j < n; ++j) {
                if (j == r) continue;
                int x;
                if ((fmask >> j) & 1u) { x = COIN(); } else { x = v[j]; }
                a += x;
                ++cnt;
            }
        }
        dec[r] = 2 * a > cnt ? V_ATTACK : (2 * a < cnt ? V_RETREAT : V_UNDEF);
    }
#undef COIN
}

static uint64_t perm_count(int L, int len) {
    uint64_t p = 1;
    for (int i = 0; i < len; ++i) p *= (uint64_t)(L - i);
    return p;
}

int ba_oracle_run(uint32_t n, uint32_t m, uint64_t seed, uint32_t lie_mode,
                  uint32_t faulty_mode, uint32_t f, uint32_t order_mode,
                  uint32_t order_value, uint64_t first_trial, uint32_t table_stride,
                  uint64_t batch, const uint32_t* faulty, const uint8_t* order,
                  const uint32_t* table, const uint32_t* poll, uint64_t* decisions,
                  uint8_t* outcome, uint64_t* counters, int threads) {
    if (n < 1 || n > MAXN || m > MAXM) return E_INVAL;
    if (lie_mode > LIE_TABLE || faulty_mode > FAULTY_EXACT || order_mode > ORDER_CONST) return E_INVAL;
    if (faulty_mode == FAULTY_GIVEN && !faulty) return E_INVAL;
    if (order_mode == ORDER_GIVEN && !order) return E_INVAL;
    if (order_mode == ORDER_CONST && order_value > V_OTHER) return E_INVAL;
    if (faulty_mode == FAULTY_EXACT && f > n) return E_INVAL;
    if (first_trial & 63) return E_INVAL;
    const int L = (int)n - 1;
    const int me = n >= 2 ? ((int)m < (int)n - 2 ? (int)m : (int)n - 2) : 0;
    if (lie_mode == LIE_TABLE) {
        if (me > 1) return E_NOTSUP;
        uint64_t coins = (uint64_t)L + (uint64_t)L * (uint64_t)L; /* incl. commander polls */
        if (!table || (uint64_t)table_stride * 32u < coins) return E_INVAL;
    }
    for (int k = 0; k <= me; ++k)
        if (perm_count(L, k + 1) > (1ull << 32)) return E_TOOBIG;

    uint64_t total[BA_ORACLE_NCOUNTERS];
    memset(total, 0, sizeof total);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif

#pragma omp parallel
    {
        uint64_t cnt[BA_ORACLE_NCOUNTERS];
        memset(cnt, 0, sizeof cnt);
#pragma omp for schedule(dynamic, 64)
        for (int64_t i = 0; i < (int64_t)batch; ++i) {
            uint64_t t = first_trial + (uint64_t)i;
            uint32_t fmask = faulty_mode == FAULTY_GIVEN ? faulty[i] : 0;
            uint8_t oc = order_mode == ORDER_GIVEN ? order[i] : 0;
            ba_oracle_gen(n, seed, faulty_mode, f, order_mode, order_value, t,
                          faulty_mode == FAULTY_GIVEN ? NULL : &fmask,
                          order_mode == ORDER_GIVEN ? NULL : &oc);
            fmask &= (n >= 32) ? 0xFFFFFFFFu : ((1u << n) - 1u);
            int ob = oc == V_ATTACK;
            int dec[MAXN];
            if (lie_mode == LIE_TABLE) {
                uint32_t pm = poll ? poll[i] & ((n >= 32) ? 0xFFFFFFFEu : ((1u << n) - 2u)) : 0u;
                om1_table((int)n, m >= 1, fmask, pm, ob, table + (uint64_t)i * table_stride, dec);
            } else {
                tctx c = {seed, t, L, me, fmask, ob};
                int path[MAXM + 2];
                for (int r = 0; r < L; ++r) dec[r + 1] = om_resolve(&c, path, 0, r, 0);
            }
            /* quorum epilogue, ba.py:197-253: tally every live general. */
            int na = 0, nr = 0, nu = 0;
            if (oc == V_ATTACK) ++na; else if (oc == V_RETREAT) ++nr; else ++nu; /* ba.py:285 */
            uint64_t dword = 0;
            for (int r = 1; r < (int)n; ++r) {
                if (dec[r] == V_ATTACK) ++na; else if (dec[r] == V_RETREAT) ++nr; else ++nu;
                dword |= (uint64_t)dec[r] << (2 * (r - 1));
            }
            int total_g = na + nr + nu;
            int k = (total_g - 1) / 3;
            int needed = 2 * k + 1;
            if (total_g <= 3) needed = total_g - 1;
            if (total_g == 1) needed = 1;
            int q = needed <= nr ? Q_RETREAT : (needed <= na ? Q_ATTACK : Q_UNDET);
            /* interactive-consistency flags over loyal lieutenants */
            int agree = 1, first = -1, appl = !(fmask & 1u), valid = 1;
            int want = ob ? V_ATTACK : V_RETREAT;
            for (int r = 1; r < (int)n; ++r) {
                if ((fmask >> r) & 1u) continue;
                if (first < 0) first = dec[r]; else if (dec[r] != first) agree = 0;
                if (dec[r] != want) valid = 0;
            }
            if (!appl) valid = 0;
            int nf = __builtin_popcount(fmask);
            int inb = nf <= me && (int)n > 3 * me;
            if (decisions) decisions[i] = dword;
            if (outcome)
                outcome[i] = (uint8_t)(q | agree << 2 | appl << 3 | valid << 4 | inb << 5);
            cnt[C_TRIALS] += 1;
            cnt[C_AGREE] += (uint64_t)agree;
            cnt[C_VAPPL] += (uint64_t)appl;
            cnt[C_VALID] += (uint64_t)valid;
            cnt[C_QR + q] += 1;
            for (int r = 1; r < (int)n; ++r) {
                cnt[C_UNDEF] += dec[r] == V_UNDEF;
                cnt[C_ATT] += dec[r] == V_ATTACK;
            }
            cnt[C_INB] += (uint64_t)inb;
            cnt[C_VIOL] += (uint64_t)(inb && (!agree || (appl && !valid)));
            cnt[C_FTOT] += (uint64_t)nf;
        }
#pragma omp critical
        for (int j = 0; j < BA_ORACLE_NCOUNTERS; ++j) total[j] += cnt[j];
    }
    if (counters) memcpy(counters, total, sizeof total);
    return 0;
}

/* Level-1 child results of the first-hop split (include/ba.h ba_subtree_votes_device):
 * votes[(i * L + j) * (L - 1) + c] = resolve_r(j) for trial i, first-hop
 * lieutenant rank j, and receiver rank r = c + (c >= j): R_1[j.r] (me >= 2) or
 * L_1[j.r] (me == 1) -- what r concludes about j's relay (ba.py:169-186
 * generalised).  Returns 0 or a negative error code (E_NOTSUP for me == 0). */
int ba_oracle_votes(uint32_t n, uint32_t m, uint64_t seed, uint32_t faulty_mode, uint32_t f,
                    uint32_t order_mode, uint32_t order_value, uint64_t first_trial,
                    uint64_t batch, const uint32_t* faulty, const uint8_t* order, uint8_t* votes,
                    int threads) {
    if (n < 3 || n > MAXN || m > MAXM) return E_INVAL;
    if (faulty_mode == FAULTY_GIVEN && !faulty) return E_INVAL;
    if (order_mode == ORDER_GIVEN && !order) return E_INVAL;
    if (first_trial & 63) return E_INVAL;
    const int L = (int)n - 1;
    const int me = (int)m < (int)n - 2 ? (int)m : (int)n - 2;
    if (me < 1) return E_NOTSUP;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t i = 0; i < (int64_t)batch; ++i) {
        uint64_t t = first_trial + (uint64_t)i;
        uint32_t fmask = faulty_mode == FAULTY_GIVEN ? faulty[i] : 0;
        uint8_t oc = order_mode == ORDER_GIVEN ? order[i] : 0;
        ba_oracle_gen(n, seed, faulty_mode, f, order_mode, order_value, t,
                      faulty_mode == FAULTY_GIVEN ? NULL : &fmask,
                      order_mode == ORDER_GIVEN ? NULL : &oc);
        fmask &= (n >= 32) ? 0xFFFFFFFFu : ((1u << n) - 1u);
        tctx c = {seed, t, L, me, fmask, oc == V_ATTACK};
        int path[MAXM + 2];
        for (int j = 0; j < L; ++j)
            for (int k = 0; k < L - 1; ++k) {
                int r = k + (k >= j);
                path[0] = j;
                votes[((uint64_t)i * L + j) * (L - 1) + k] = (uint8_t)om_resolve(&c, path, 1, r, 1u << j);
            }
    }
    return 0;
}

/* Level-2 results of the second-hop split: for every level-1
 * slot (j, a) -- unit u = j*(L-1) + k with a = k + (k >= j) -- and every
 * receiver r not in {j, a}, child c in rank order, R_2[j.a.r] = the value r
 * attributes to path j.a after the recursive majority below it (ba.py:159-195
 * generalised).  votes[((i*L*(L-1) + u)*(L-2) + c].  Needs m_eff >= 3 (R_2 is
 * a majority level) and n >= 4. */
int ba_oracle_votes2(uint32_t n, uint32_t m, uint64_t seed, uint32_t faulty_mode, uint32_t f,
                     uint32_t order_mode, uint32_t order_value, uint64_t first_trial,
                     uint64_t batch, const uint32_t* faulty, const uint8_t* order, uint8_t* votes,
                     int threads) {
    if (n < 4 || n > MAXN || m > MAXM) return E_INVAL;
    if (faulty_mode == FAULTY_GIVEN && !faulty) return E_INVAL;
    if (order_mode == ORDER_GIVEN && !order) return E_INVAL;
    if (first_trial & 63) return E_INVAL;
    const int L = (int)n - 1;
    const int me = (int)m < (int)n - 2 ? (int)m : (int)n - 2;
    if (me < 3) return E_NOTSUP;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#else
    (void)threads;
#endif
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t i = 0; i < (int64_t)batch; ++i) {
        uint64_t t = first_trial + (uint64_t)i;
        uint32_t fmask = faulty_mode == FAULTY_GIVEN ? faulty[i] : 0;
        uint8_t oc = order_mode == ORDER_GIVEN ? order[i] : 0;
        ba_oracle_gen(n, seed, faulty_mode, f, order_mode, order_value, t,
                      faulty_mode == FAULTY_GIVEN ? NULL : &fmask,
                      order_mode == ORDER_GIVEN ? NULL : &oc);
        fmask &= (n >= 32) ? 0xFFFFFFFFu : ((1u << n) - 1u);
        tctx c = {seed, t, L, me, fmask, oc == V_ATTACK};
        int path[MAXM + 2];
        for (int j = 0; j < L; ++j)
            for (int k = 0; k < L - 1; ++k) {
                const int a = k + (k >= j);
                const uint64_t u = (uint64_t)j * (L - 1) + k;
                int ch = 0;
                for (int r = 0; r < L; ++r) {
                    if (r == j || r == a) continue;
                    path[0] = j;
                    path[1] = a;
                    votes[((uint64_t)i * L * (L - 1) + u) * (L - 2) + ch] =
                        (uint8_t)om_resolve(&c, path, 2, r, (1u << j) | (1u << a));
                    ++ch;
                }
            }
    }
    return 0;
}
