/*
 * commit_kats.c — a plain C host of libhipquorum.so (what the cgo package of INTEGRATION.md
 * does, without Go): the 14 rows of the reference's TestCommit table
 * (internal/raft/raft_etcd_test.go:1111-1160) decided in one hq_commit call over pinned host
 * buffers, ring term form (entryLog.term, logentry.go:143-160), per-group voter counts.
 * Exit status 0 iff every committed index equals the reference's expectation.
 *
 *   gcc -std=c99 -Iinclude examples/commit_kats.c -Ldragonboat_amd/lib -lhipquorum \
 *       -Wl,-rpath,dragonboat_amd/lib -o commit_kats && ./commit_kats
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "hipquorum.h"

#define NG 14
#define NMAX 4
#define R 16

struct row {
    int n;                 /* voting members (remotes; no witnesses in this table) */
    uint64_t match[NMAX];  /* remote.match of every member, the leader included */
    uint64_t log_term[3];  /* term of entries 0..2 (entry 0 is the dummy, term 0) */
    uint64_t last, term, want;
};

/* raft_etcd_test.go:1118-1136, rows #0..#13 in order */
static const struct row rows[NG] = {
    {1, {1}, {0, 1, 0}, 1, 1, 1},          {1, {1}, {0, 1, 0}, 1, 2, 0},
    {1, {2}, {0, 1, 2}, 2, 2, 2},          {1, {1}, {0, 2, 0}, 1, 2, 1},
    {3, {2, 1, 1}, {0, 1, 2}, 2, 1, 1},    {3, {2, 1, 1}, {0, 1, 1}, 2, 2, 0},
    {3, {2, 1, 2}, {0, 1, 2}, 2, 2, 2},    {3, {2, 1, 2}, {0, 1, 1}, 2, 2, 0},
    {4, {2, 1, 1, 1}, {0, 1, 2}, 2, 1, 1}, {4, {2, 1, 1, 1}, {0, 1, 1}, 2, 2, 0},
    {4, {2, 1, 1, 2}, {0, 1, 2}, 2, 1, 1}, {4, {2, 1, 1, 2}, {0, 1, 1}, 2, 2, 0},
    {4, {2, 1, 2, 2}, {0, 1, 2}, 2, 2, 2}, {4, {2, 1, 2, 2}, {0, 1, 1}, 2, 2, 0},
};

#define CHECK(call)                                                                    \
    do {                                                                               \
        int rc_ = (call);                                                              \
        if (rc_ != HQ_OK) {                                                            \
            fprintf(stderr, "%s failed: %d %s\n", #call, rc_, hq_last_error(ctx));     \
            return 2;                                                                  \
        }                                                                              \
    } while (0)

int main(void) {
    hq_ctx *ctx = NULL;
    if (hq_open(0, 0, &ctx) != HQ_OK) {
        fprintf(stderr, "hq_open: %s\n", hq_last_error(NULL));
        return 2;
    }
    void *p;
    CHECK(hq_alloc_pinned(ctx, 8 * (size_t)(NMAX * NG + 4 * NG + R * NG) + NG + 16, &p));
    uint64_t *match = (uint64_t *)p, *cin = match + NMAX * NG, *cout = cin + NG, *last = cout + NG;
    uint64_t *term = last + NG, *ring = term + NG, *changed = ring + R * NG, *fallback = changed + 1;
    uint8_t *nv = (uint8_t *)(fallback + 1);
    memset(p, 0, 8 * (size_t)(NMAX * NG + 4 * NG + R * NG) + NG + 16);
    for (int g = 0; g < NG; ++g) {
        for (int s = 0; s < rows[g].n; ++s) match[s * NG + g] = rows[g].match[s];
        nv[g] = (uint8_t)rows[g].n;
        cin[g] = 0; /* committed starts at firstIndex - 1 = 0 (logentry.go:91) */
        last[g] = rows[g].last;
        term[g] = rows[g].term;
        for (uint64_t i = 0; i <= rows[g].last; ++i) ring[g * R + (i % R)] = rows[g].log_term[i];
    }
    hq_commit_args a;
    memset(&a, 0, sizeof a);
    a.G = NG;
    a.n_max = NMAX;
    a.form = HQ_FORM_TERM_RING;
    a.ring_len = R;
    a.layout = HQ_LAYOUT_COLUMNS;
    a.match_stride = NG;
    a.match = match;
    a.n_voting = nv;
    a.committed_in = cin;
    a.committed_out = cout;
    a.last_index = last;
    a.term = term;
    a.ring = ring;
    a.changed = changed;
    a.fallback = fallback;
    CHECK(hq_commit(ctx, &a));
    int bad = 0;
    for (int g = 0; g < NG; ++g) {
        const int chg = (int)((*changed >> g) & 1), fb = (int)((*fallback >> g) & 1);
        const int ok = cout[g] == rows[g].want && chg == (rows[g].want > 0) && !fb;
        printf("TestCommit #%-2d n=%d term=%llu committed=%llu want=%llu %s\n", g, rows[g].n,
               (unsigned long long)rows[g].term, (unsigned long long)cout[g],
               (unsigned long long)rows[g].want, ok ? "ok" : "MISMATCH");
        bad += !ok;
    }
    CHECK(hq_free_pinned(ctx, p));
    hq_close(ctx);
    return bad ? 1 : 0;
}
