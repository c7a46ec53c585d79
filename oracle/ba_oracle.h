/*
 * ba_oracle.h -- CPU restatement of the reference's OM(m) hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker for libba_hip.so; it
 * is never linked into, loaded by, or called from the product path.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it.
 *
 * Reference: /root/reference/ba.py (mathiasplans/byzantine-agreement), which
 * implements OM(1) only.  Semantics restated here (docs/SEMANTICS.md):
 *   - level 0 (commander send)          ba.py:257-285
 *   - relay + lie rule                   ba.py:42-57 (get_order), ba.py:45/269 (coin)
 *   - lieutenant majority, tie rules     ba.py:159-195
 *   - quorum epilogue                    ba.py:197-255
 * OM(m>=2) is the build's own generalisation pinned
 * by its m=1 reduction and OM theory properties; m=1 table mode is pinned
 * bit-exactly against fixtures generated from ba.py itself (tests/golden/).
 */
#ifndef BA_ORACLE_H
#define BA_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BA_ORACLE_NCOUNTERS 16

/* Philox4x32-10 (Salmon et al., SC'11), independent host implementation. */
void ba_oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* Lie bit (1 = attack) for global trial t, tree level k, slot rank x. */
uint32_t ba_oracle_lie(uint64_t seed, uint64_t t, uint32_t k, uint64_t x);

/* Synthetic trial generation (faulty set by partial Fisher-Yates, order). */
void ba_oracle_gen(uint32_t n, uint64_t seed, uint32_t faulty_mode, uint32_t f,
                   uint32_t order_mode, uint32_t order_value, uint64_t t,
                   uint32_t* faulty_mask, uint8_t* order);

/* Run `batch` trials.  Argument meaning mirrors ba_run_trials in include/ba.h.
 * Returns 0 or a negative error code.  `threads` <= 0 means all cores. */
int ba_oracle_run(uint32_t n, uint32_t m, uint64_t seed, uint32_t lie_mode,
                  uint32_t faulty_mode, uint32_t f, uint32_t order_mode,
                  uint32_t order_value, uint64_t first_trial, uint32_t table_stride,
                  uint64_t batch, const uint32_t* faulty, const uint8_t* order,
                  const uint32_t* table, const uint32_t* poll, uint64_t* decisions,
                  uint8_t* outcome, uint64_t* counters, int threads);

/* Level-1 child results per (trial, first-hop j, receiver) for the first-hop
 * split (see ba_oracle.c).  votes: batch * (n-1) * (n-2) bytes, 0/1. */
int ba_oracle_votes(uint32_t n, uint32_t m, uint64_t seed, uint32_t faulty_mode, uint32_t f,
                    uint32_t order_mode, uint32_t order_value, uint64_t first_trial,
                    uint64_t batch, const uint32_t* faulty, const uint8_t* order, uint8_t* votes,
                    int threads);
/* Level-2 results R_2 of every level-1 slot (second-hop split), uint8[batch][L(L-1)][L-2]. */
int ba_oracle_votes2(uint32_t n, uint32_t m, uint64_t seed, uint32_t faulty_mode, uint32_t f,
                    uint32_t order_mode, uint32_t order_value, uint64_t first_trial,
                    uint64_t batch, const uint32_t* faulty, const uint8_t* order, uint8_t* votes,
                    int threads);

#ifdef __cplusplus
}
#endif
#endif
