/*
 * qref.c — CPU oracle: plain-C restatement of dragonboat's leader quorum arithmetic.
 * TEST INFRASTRUCTURE ONLY (see qref.h). Citations are to /root/reference (dragonboat v3.3-dev).
 */
#include "qref.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ================================================================ quorum arithmetic ======== */

/* raft.numVotingMembers: len(r.remotes) + len(r.witnesses) — raft.go:368-370 */
int qref_num_voting_members(int n_remotes, int n_witnesses) { return n_remotes + n_witnesses; }

/* raft.quorum: numVotingMembers()/2 + 1 — raft.go:372-374 */
int qref_quorum(int n_voting) { return n_voting / 2 + 1; }

/* raft.isSingleNodeQuorum — raft.go:376-378 */
int qref_is_single_node_quorum(int n_voting) { return qref_quorum(n_voting) == 1; }

/* raft.sortMatchValues — raft.go:861-886: unrolled 3-element bubble sort, no-op for one element,
 * sort.Slice ascending otherwise (any correct ascending sort gives the same slice). */
void qref_sort_match_values(uint64_t *m, int n) {
    if (n == 3) {
        uint64_t v;
        if (m[0] > m[1]) { v = m[0]; m[0] = m[1]; m[1] = v; }
        if (m[1] > m[2]) { v = m[1]; m[1] = m[2]; m[2] = v; }
        if (m[0] > m[1]) { v = m[0]; m[0] = m[1]; m[1] = v; }
    } else if (n == 1) {
        return;
    } else {
        for (int i = 1; i < n; i++) {
            uint64_t v = m[i];
            int j = i - 1;
            while (j >= 0 && m[j] > v) { m[j + 1] = m[j]; j--; }
            m[j + 1] = v;
        }
    }
}

/* ================================================================ entry log ================ */

/* entryLog.term — logentry.go:143-160: 0 outside [first-1, last] (termEntryRange :117-126),
 * else inMemory.getTerm / logdb.Term (inmemory.go:87-105, logentry.go:152-159). */
uint64_t qref_log_term(const qref_log *l, uint64_t index) {
    if (index < l->first_minus_1 || index > l->last) return 0;
    return l->term_at(l->ud, index);
}

/* entryLog.tryCommit — logentry.go:378-393, commitTo — logentry.go:323-332 */
int qref_log_try_commit(qref_log *l, uint64_t index, uint64_t term) {
    if (index <= l->committed) return 0;
    uint64_t lterm = qref_log_term(l, index);   /* ErrCompacted -> 0 (:383-384) */
    if (index > l->committed && lterm == term) {
        /* commitTo(index) */
        if (index <= l->committed) return 0;
        if (index > l->last) return QREF_PANIC;  /* "invalid commitTo index" (:327-330) */
        l->committed = index;
        return 1;
    }
    return 0;
}

/* raft.tryCommit — raft.go:888-909 */
int qref_try_commit(const uint64_t *remote_match, int n_remotes, const uint64_t *witness_match,
                    int n_witnesses, qref_log *log, uint64_t term, uint64_t *q_out) {
    uint64_t matched[QREF_MAX_NODES];
    int n = qref_num_voting_members(n_remotes, n_witnesses);
    if (n <= 0 || n > QREF_MAX_NODES) return QREF_PANIC;   /* matched[n-quorum] out of range */
    int idx = 0;
    for (int i = 0; i < n_remotes; i++) matched[idx++] = remote_match[i];    /* :894-897 */
    for (int i = 0; i < n_witnesses; i++) matched[idx++] = witness_match[i]; /* :898-901 */
    qref_sort_match_values(matched, n);                                       /* :902 */
    uint64_t q = matched[n - qref_quorum(n)];                                 /* :903 */
    if (q_out) *q_out = q;
    return qref_log_try_commit(log, q, term);                                 /* :908 */
}

uint64_t qref_quorum_match_by_count(const uint64_t *match, int n) {
    int quorum = qref_quorum(n);
    uint64_t best = 0;
    int found = 0;
    for (int i = 0; i < n; i++) {
        int c = 0;
        for (int j = 0; j < n; j++) c += match[j] >= match[i];
        if (c >= quorum && (!found || match[i] > best)) { best = match[i]; found = 1; }
    }
    return best;
}

/* ================================================================ ReadIndex ================ */

static int ctx_eq(qref_sysctx a, qref_sysctx b) { return a.low == b.low && a.high == b.high; }

static int ri_find(const qref_read_index *r, qref_sysctx ctx) {
    for (int i = 0; i < r->n_pending; i++)
        if (ctx_eq(r->pending[i].ctx, ctx)) return i;
    return -1;
}

void qref_ri_init(qref_read_index *r) { r->n_pending = 0; r->n_queue = 0; }   /* :36-41 */

int qref_ri_has_pending(const qref_read_index *r) { return r->n_queue > 0; }

/* readIndex.addRequest — readindex.go:43-67 */
int qref_ri_add_request(qref_read_index *r, uint64_t index, qref_sysctx ctx, uint64_t from) {
    if (ri_find(r, ctx) >= 0) return QREF_OK;                       /* :45-47 */
    if (r->n_queue > 0) {                                            /* :50-59 */
        int p = ri_find(r, r->queue[r->n_queue - 1]);
        if (p < 0) return QREF_PANIC;                                /* inconsistent */
        if (index < r->pending[p].index) return QREF_PANIC;          /* index moved backward */
    }
    if (r->n_queue >= QREF_MAX_PENDING || r->n_pending >= QREF_MAX_PENDING) return QREF_PANIC;
    r->queue[r->n_queue++] = ctx;                                    /* :60 */
    qref_read_status *s = &r->pending[r->n_pending++];               /* :61-66 */
    s->index = index;
    s->from = from;
    s->ctx = ctx;
    s->n_confirmed = 0;
    return QREF_OK;
}

/* readIndex.confirm — readindex.go:77-116 */
int qref_ri_confirm(qref_read_index *r, qref_sysctx ctx, uint64_t from, int quorum,
                    qref_read_status *out) {
    int pi = ri_find(r, ctx);
    if (pi < 0) return 0;                                            /* :79-82 */
    qref_read_status *p = &r->pending[pi];
    int seen = 0;                                                    /* :83 set insert */
    for (int i = 0; i < p->n_confirmed; i++) seen |= p->confirmed[i] == from;
    if (!seen) {
        if (p->n_confirmed >= QREF_MAX_NODES) return QREF_PANIC;
        p->confirmed[p->n_confirmed++] = from;
    }
    if (p->n_confirmed + 1 < quorum) return 0;                       /* :84-86 */
    int done = 0;
    int cs[QREF_MAX_PENDING];
    int ncs = 0;
    for (int qi = 0; qi < r->n_queue; qi++) {                        /* :89 */
        qref_sysctx pctx = r->queue[qi];
        done++;
        int si = ri_find(r, pctx);
        if (si < 0) return QREF_PANIC;                               /* :91-94 */
        cs[ncs++] = si;
        if (ctx_eq(pctx, ctx)) {                                     /* :96 */
            const qref_read_status *s = &r->pending[si];
            for (int k = 0; k < ncs; k++) {                          /* :97-105 */
                if (r->pending[cs[k]].index > s->index) return QREF_PANIC;
            }
            uint64_t idx = s->index;
            for (int k = 0; k < ncs; k++) {
                out[k] = r->pending[cs[k]];
                out[k].index = idx;                                  /* rewrite (:104) */
            }
            /* r.queue = r.queue[done:] (:106) */
            memmove(r->queue, r->queue + done, (size_t)(r->n_queue - done) * sizeof(qref_sysctx));
            r->n_queue -= done;
            /* delete(r.pending, v.ctx) (:107-109) */
            for (int k = 0; k < ncs; k++) {
                int di = ri_find(r, out[k].ctx);
                if (di >= 0) r->pending[di] = r->pending[--r->n_pending];
            }
            if (r->n_queue != r->n_pending) return QREF_PANIC;       /* :110-112 */
            return ncs;
        }
    }
    return 0;                                                        /* :115 */
}

/* ================================================================ votes ==================== */

void qref_votes_reset(qref_votes *v) { v->n = 0; }

/* raft.handleVoteResp — raft.go:1062-1080 */
int qref_handle_vote_resp(qref_votes *v, uint64_t from, int rejected) {
    int found = 0;
    for (int i = 0; i < v->n; i++) found |= v->from[i] == from;
    if (!found && v->n < QREF_MAX_NODES) {                           /* :1071-1073 first wins */
        v->from[v->n] = from;
        v->granted[v->n] = !rejected;
        v->n++;
    }
    int voted_for = 0;
    for (int i = 0; i < v->n; i++) voted_for += v->granted[i] != 0;  /* :1074-1078 */
    return voted_for;
}

/* raft.handleCandidateRequestVoteResp — raft.go:1968-1985 */
int qref_candidate_vote_resp(qref_votes *v, uint64_t from, int rejected, int from_is_observer,
                             int quorum) {
    if (from_is_observer) return QREF_CANDIDATE;                     /* :1969-1972 */
    int count = qref_handle_vote_resp(v, from, rejected);
    if (count == quorum) return QREF_LEADER;                         /* :1977-1980 */
    if (v->n - count == quorum) return QREF_FOLLOWER;                /* :1981-1984 */
    return QREF_CANDIDATE;
}

/* raft.leaderHasQuorum — raft.go:380-390 */
int qref_leader_has_quorum(const uint64_t *ids, int *active, int n_voting, uint64_t self_id) {
    int c = 0;
    for (int i = 0; i < n_voting; i++) {
        if (ids[i] == self_id || active[i]) {
            c++;
            active[i] = 0;                                           /* setNotActive */
        }
    }
    return c >= qref_quorum(n_voting);
}

/* ================================================================ batched SoA forms ======== */

static inline void bit_set(uint64_t *bm, uint64_t g) { bm[g >> 6] |= 1ull << (g & 63); }

typedef struct { const uint64_t *ring; uint64_t mask; } ring_ud;
static uint64_t ring_term_at(const void *ud, uint64_t i) {
    const ring_ud *r = (const ring_ud *)ud;
    return r->ring[i & r->mask];
}

typedef struct { uint32_t mask; uint64_t rmask; } mask_ud;
/* Form 2: bit (i mod R) says whether entry i carries the leader's term (2) or not (1). */
static uint64_t mask_term_at(const void *ud, uint64_t i) {
    const mask_ud *m = (const mask_ud *)ud;
    return ((m->mask >> (i & m->rmask)) & 1) ? 2 : 1;
}

typedef struct { uint64_t term_start; } tstart_ud;
/* The leader's log under the monotone-term invariant (entryutils.go:44-47): entries at or after
 * the leader's first current-term entry carry the current term (2 here), older ones a lower
 * term (1). */
static uint64_t tstart_term_at(const void *ud, uint64_t i) {
    return i >= ((const tstart_ud *)ud)->term_start ? 2 : 1;
}

static void commit_range(const qref_commit_args *a, uint64_t g0, uint64_t g1, int *status) {
    const uint64_t R = a->ring_len;
    for (uint64_t g = g0; g < g1; g++) {
        int n = a->n_voting ? a->n_voting[g] : (int)a->n_max;
        uint64_t cin = a->committed_in[g];
        uint64_t last = a->last_index[g];
        a->committed_out[g] = cin;
        if (n <= 0 || n > (int)a->n_max) {
            if (a->fallback) bit_set(a->fallback, g);
            continue;
        }
        uint64_t m[QREF_MAX_NODES];
        for (int s = 0; s < n; s++) m[s] = a->match[(uint64_t)s * a->match_stride + g];
        qref_log log;
        uint64_t term;
        ring_ud rud;
        tstart_ud tud;
        mask_ud mud;
        if (a->form == 2) {
            term = 2;
            if (cin > last || last - cin > R) {
                if (a->fallback) bit_set(a->fallback, g);
                continue;
            }
            mud.mask = a->term_mask[g];
            mud.rmask = R - 1;
            log.first_minus_1 = last >= R - 1 ? last - (R - 1) : 0;
            log.term_at = mask_term_at;
            log.ud = &mud;
        } else if (a->form == 1 || a->form == 3) {
            /* form 3 (the u32-ring packing of the same ring) decides from the u64 terms here:
             * the product's narrowing is checked against the full-width restatement; its
             * contract adds term >= 0xFFFFFFFF to the fallback set */
            term = a->term[g];
            if (term == 0 || cin > last || last - cin > R ||
                (a->form == 3 && term >= 0xFFFFFFFFull)) {
                if (a->fallback) bit_set(a->fallback, g);
                continue;
            }
            rud.ring = a->ring + g * R;
            rud.mask = R - 1;
            log.first_minus_1 = last >= R - 1 ? last - (R - 1) : 0;
            log.term_at = ring_term_at;
            log.ud = &rud;
        } else {
            term = 2;
            tud.term_start = a->term_start[g];
            log.first_minus_1 = cin;
            log.term_at = tstart_term_at;
            log.ud = &tud;
        }
        log.last = last;
        log.committed = cin;
        int rc = qref_try_commit(m, n, NULL, 0, &log, term, NULL);
        if (rc == QREF_PANIC) { *status = QREF_PANIC; continue; }
        a->committed_out[g] = log.committed;
        if (rc == 1 && a->changed) bit_set(a->changed, g);
    }
}

static void readindex_range(uint64_t g0, uint64_t g1, const uint8_t *ack, const uint8_t *nv,
                            uint32_t nu, uint64_t *confirmed, uint64_t *fallback, int *status) {
    static const qref_sysctx ctx = {1, 1};
    qref_read_index ri;
    qref_read_status out[QREF_MAX_PENDING];
    for (uint64_t g = g0; g < g1; g++) {
        int n = nv ? nv[g] : (int)nu;
        if (n <= 0 || n > 8) {
            if (fallback) bit_set(fallback, g);
            continue;
        }
        int quorum = qref_quorum(n);
        if (qref_is_single_node_quorum(n)) {
            /* handleLeaderReadIndex single-node short-cut: addReadyToRead (raft.go:1664) */
            bit_set(confirmed, g);
            continue;
        }
        qref_ri_init(&ri);
        /* handleLeaderReadIndex -> addRequest(committed, ctx, from) (raft.go:1656) */
        if (qref_ri_add_request(&ri, 0, ctx, 1) != QREF_OK) { *status = QREF_PANIC; continue; }
        int ok = 0;
        for (int s = 0; s < n; s++) {
            if (!((ack[g] >> s) & 1)) continue;
            /* HeartbeatResp from slot s -> handleReadIndexLeaderConfirmation (raft.go:1740) */
            int rc = qref_ri_confirm(&ri, ctx, (uint64_t)s + 1, quorum, out);
            if (rc == QREF_PANIC) { *status = QREF_PANIC; break; }
            if (rc > 0) ok = 1;
        }
        if (ok) bit_set(confirmed, g);
    }
}

static void vote_range(uint64_t g0, uint64_t g1, const uint8_t *gr, const uint8_t *rj,
                       const uint8_t *nv, uint32_t nu, uint64_t *outcome, uint64_t *fallback) {
    qref_votes v;
    for (uint64_t g = g0; g < g1; g++) {
        int n = nv ? nv[g] : (int)nu;
        int state = QREF_CANDIDATE;
        if (n <= 0 || n > 8) {
            if (fallback) bit_set(fallback, g);
        } else {
            int quorum = qref_quorum(n);
            qref_votes_reset(&v);
            for (int s = 0; s < n && state == QREF_CANDIDATE; s++) {
                int gbit = (gr[g] >> s) & 1;
                int rbit = (rj[g] >> s) & 1;
                if (!gbit && !rbit) continue;
                state = qref_candidate_vote_resp(&v, (uint64_t)s + 1, !gbit, 0, quorum);
            }
        }
        outcome[g >> 5] |= (uint64_t)state << (2 * (g & 31));
    }
}

static void checkq_range(uint64_t g0, uint64_t g1, uint8_t *active, const uint8_t *nv,
                         uint32_t nu, uint32_t self_slot, uint64_t *hq, uint64_t *fallback) {
    uint64_t ids[8];
    int act[8];
    for (uint64_t g = g0; g < g1; g++) {
        int n = nv ? nv[g] : (int)nu;
        if (n <= 0 || n > 8 || (int)self_slot >= n) {
            if (fallback) bit_set(fallback, g);
            continue;
        }
        for (int s = 0; s < n; s++) { ids[s] = (uint64_t)s + 1; act[s] = (active[g] >> s) & 1; }
        if (qref_leader_has_quorum(ids, act, n, (uint64_t)self_slot + 1)) bit_set(hq, g);
        active[g] = 0;
    }
}

/* ---- thread fan-out over contiguous 64-aligned blocks ---- */
enum { JOB_COMMIT, JOB_RI, JOB_VOTE, JOB_CHECKQ };
typedef struct {
    int kind;
    uint64_t g0, g1;
    int status;
    const qref_commit_args *ca;
    const uint8_t *b0, *b1, *nv;
    uint8_t *bw;
    uint32_t nu, self_slot;
    uint64_t *o0, *o1;
} job_t;

static void *run_job(void *p) {
    job_t *j = (job_t *)p;
    switch (j->kind) {
    case JOB_COMMIT: commit_range(j->ca, j->g0, j->g1, &j->status); break;
    case JOB_RI: readindex_range(j->g0, j->g1, j->b0, j->nv, j->nu, j->o0, j->o1, &j->status); break;
    case JOB_VOTE: vote_range(j->g0, j->g1, j->b0, j->b1, j->nv, j->nu, j->o0, j->o1); break;
    case JOB_CHECKQ: checkq_range(j->g0, j->g1, j->bw, j->nv, j->nu, j->self_slot, j->o0, j->o1); break;
    }
    return NULL;
}

static int fan_out(job_t proto, uint64_t G, int nthreads, uint64_t align) {
    if (nthreads <= 1 || G < 2 * align) {
        proto.g0 = 0; proto.g1 = G; proto.status = QREF_OK;
        run_job(&proto);
        return proto.status;
    }
    if (nthreads > 256) nthreads = 256;
    job_t jobs[256];
    pthread_t th[256];
    uint64_t blocks = (G + align - 1) / align;
    uint64_t per = (blocks + nthreads - 1) / nthreads;
    int started = 0;
    for (int t = 0; t < nthreads; t++) {
        uint64_t b0 = per * t, b1 = per * (t + 1);
        if (b0 >= blocks) break;
        if (b1 > blocks) b1 = blocks;
        jobs[t] = proto;
        jobs[t].g0 = b0 * align;
        jobs[t].g1 = b1 * align < G ? b1 * align : G;
        jobs[t].status = QREF_OK;
        if (pthread_create(&th[t], NULL, run_job, &jobs[t]) != 0) { run_job(&jobs[t]); th[t] = 0; }
        started++;
    }
    int status = QREF_OK;
    for (int t = 0; t < started; t++) {
        if (th[t]) pthread_join(th[t], NULL);
        if (jobs[t].status != QREF_OK) status = jobs[t].status;
    }
    return status;
}

static uint64_t words64(uint64_t G, uint64_t per_word) { return (G + per_word - 1) / per_word; }

int qref_commit_batch(const qref_commit_args *a, int nthreads) {
    if (!a || !a->match || !a->committed_in || !a->committed_out || !a->last_index) return -1;
    if (a->n_max < 1 || a->n_max > QREF_MAX_NODES || a->match_stride < a->G) return -1;
    if (a->form == 1 || a->form == 3) {
        if (!a->term || !a->ring || a->ring_len < 1 || (a->ring_len & (a->ring_len - 1))) return -1;
    } else if (a->form == 0) {
        if (!a->term_start) return -1;
    } else if (a->form == 2) {
        if (!a->term_mask || a->ring_len < 1 || a->ring_len > 16 ||
            (a->ring_len & (a->ring_len - 1))) return -1;
    } else {
        return -1;
    }
    if (a->changed) memset(a->changed, 0, words64(a->G, 64) * 8);
    if (a->fallback) memset(a->fallback, 0, words64(a->G, 64) * 8);
    job_t j; memset(&j, 0, sizeof j);
    j.kind = JOB_COMMIT; j.ca = a;
    return fan_out(j, a->G, nthreads, 64);
}

int qref_readindex_batch(uint64_t G, const uint8_t *ack, const uint8_t *n_voting,
                         uint32_t n_uniform, uint64_t *confirmed, uint64_t *fallback,
                         int nthreads) {
    if (!ack || !confirmed) return -1;
    memset(confirmed, 0, words64(G, 64) * 8);
    if (fallback) memset(fallback, 0, words64(G, 64) * 8);
    job_t j; memset(&j, 0, sizeof j);
    j.kind = JOB_RI; j.b0 = ack; j.nv = n_voting; j.nu = n_uniform; j.o0 = confirmed; j.o1 = fallback;
    return fan_out(j, G, nthreads, 64);
}

int qref_vote_batch(uint64_t G, const uint8_t *granted, const uint8_t *rejected,
                    const uint8_t *n_voting, uint32_t n_uniform, uint64_t *outcome,
                    uint64_t *fallback, int nthreads) {
    if (!granted || !rejected || !outcome) return -1;
    memset(outcome, 0, words64(G, 32) * 8);
    if (fallback) memset(fallback, 0, words64(G, 64) * 8);
    job_t j; memset(&j, 0, sizeof j);
    j.kind = JOB_VOTE; j.b0 = granted; j.b1 = rejected; j.nv = n_voting; j.nu = n_uniform;
    j.o0 = outcome; j.o1 = fallback;
    return fan_out(j, G, nthreads, 64);
}

int qref_check_quorum_batch(uint64_t G, uint8_t *active, const uint8_t *n_voting,
                            uint32_t n_uniform, uint32_t self_slot, uint64_t *has_quorum,
                            uint64_t *fallback, int nthreads) {
    if (!active || !has_quorum) return -1;
    memset(has_quorum, 0, words64(G, 64) * 8);
    if (fallback) memset(fallback, 0, words64(G, 64) * 8);
    job_t j; memset(&j, 0, sizeof j);
    j.kind = JOB_CHECKQ; j.bw = active; j.nv = n_voting; j.nu = n_uniform; j.self_slot = self_slot;
    j.o0 = has_quorum; j.o1 = fallback;
    return fan_out(j, G, nthreads, 64);
}

/* ================================================================ multi-ctx ReadIndex ====== */

typedef struct { uint32_t o, k, s; } ri_msg;

static void ri_multi_range(uint64_t g0, uint64_t g1, uint32_t K_max, uint32_t n_max,
                           const uint16_t *ord, const uint64_t *idx, const uint8_t *np,
                           const uint8_t *nv, uint32_t nu, uint64_t *rel, uint8_t *cnt,
                           uint8_t *bend, uint64_t *fallback, uint64_t G) {
    qref_read_index *ri = (qref_read_index *)malloc(sizeof *ri);
    qref_read_status *out = (qref_read_status *)malloc(QREF_MAX_PENDING * sizeof *out);
    ri_msg msgs[64 * 8];
    for (uint64_t g = g0; g < g1; g++) {
        uint32_t K = np ? np[g] : K_max;
        int n = nv ? nv[g] : (int)nu;
        for (uint32_t k = 0; k < K_max; k++) rel[(uint64_t)k * G + g] = UINT64_MAX;
        cnt[g] = 0;
        if (bend) bend[g] = 0;
        if (n < 1 || n > (int)n_max || K > K_max) {
            if (fallback) bit_set(fallback, g);
            continue;
        }
        int quorum = qref_quorum(n);
        qref_ri_init(ri);
        int bad = 0;
        for (uint32_t k = 0; k < K && !bad; k++) {   /* handleLeaderReadIndex -> addRequest */
            qref_sysctx c = {k + 1, k + 1};
            bad = qref_ri_add_request(ri, idx[(uint64_t)k * G + g], c, 1) != QREF_OK;
        }
        if (bad) {                                     /* index moved backward: contract */
            if (fallback) bit_set(fallback, g);
            continue;
        }
        int nm = 0;
        for (uint32_t k = 0; k < K; k++)
            for (int s = 0; s < n; s++) {
                uint16_t o = ord[((uint64_t)k * n_max + s) * G + g];
                if (o != 0xFFFF) { msgs[nm].o = o; msgs[nm].k = k; msgs[nm].s = (uint32_t)s; nm++; }
            }
        /* arrival order: ordinal, then queue position (stable for equal ordinals) */
        for (int i = 1; i < nm; i++) {
            ri_msg v = msgs[i];
            int j = i - 1;
            while (j >= 0 && (msgs[j].o > v.o || (msgs[j].o == v.o && msgs[j].k > v.k))) {
                msgs[j + 1] = msgs[j];
                j--;
            }
            msgs[j + 1] = v;
        }
        uint8_t released = 0;
        for (int i = 0; i < nm; i++) {                 /* HeartbeatResp -> confirm */
            qref_sysctx c = {msgs[i].k + 1, msgs[i].k + 1};
            int r = qref_ri_confirm(ri, c, (uint64_t)msgs[i].s + 1, quorum, out);
            for (int j = 0; j < r; j++) {
                rel[(out[j].ctx.low - 1) * G + g] = out[j].index;
                released++;
            }
            /* the confirming ctx is the last of the released batch (readindex.go:96) */
            if (r > 0 && bend) bend[g] |= (uint8_t)(1u << (out[r - 1].ctx.low - 1));
        }
        cnt[g] = released;
    }
    free(ri);
    free(out);
}

typedef struct {
    uint64_t g0, g1, G;
    uint32_t K_max, n_max, nu;
    const uint16_t *ord;
    const uint64_t *idx;
    const uint8_t *np, *nv;
    uint64_t *rel, *fb;
    uint8_t *cnt, *bend;
} ri_multi_job;

static void *ri_multi_run(void *p) {
    ri_multi_job *j = (ri_multi_job *)p;
    ri_multi_range(j->g0, j->g1, j->K_max, j->n_max, j->ord, j->idx, j->np, j->nv, j->nu, j->rel,
                   j->cnt, j->bend, j->fb, j->G);
    return NULL;
}

int qref_readindex_multi_batch(uint64_t G, uint32_t K_max, uint32_t n_max,
                               const uint16_t *ack_ordinal, const uint64_t *ctx_index,
                               const uint8_t *n_pending, const uint8_t *n_voting,
                               uint32_t n_uniform, uint64_t *released_index,
                               uint8_t *released_count, uint8_t *batch_end, uint64_t *fallback,
                               int nthreads) {
    if (!ack_ordinal || !ctx_index || !released_index || !released_count || K_max < 1 ||
        K_max > 64 || n_max < 1 || n_max > 8)
        return -1;
    if (fallback) memset(fallback, 0, words64(G, 64) * 8);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 64) nthreads = 64;
    ri_multi_job jobs[64];
    pthread_t th[64];
    uint64_t blocks = (G + 63) / 64, per = (blocks + nthreads - 1) / nthreads;
    int started = 0;
    for (int t = 0; t < nthreads; t++) {
        uint64_t b0 = per * t, b1 = per * (t + 1);
        if (b0 >= blocks) break;
        if (b1 > blocks) b1 = blocks;
        ri_multi_job j = {b0 * 64, b1 * 64 < G ? b1 * 64 : G, G, K_max, n_max, n_uniform,
                          ack_ordinal, ctx_index, n_pending, n_voting, released_index, fallback,
                          released_count, batch_end};
        jobs[t] = j;
        if (nthreads == 1 || pthread_create(&th[t], NULL, ri_multi_run, &jobs[t]) != 0) {
            ri_multi_run(&jobs[t]);
            th[t] = 0;
        }
        started++;
    }
    for (int t = 0; t < started; t++)
        if (th[t]) pthread_join(th[t], NULL);
    return 0;
}

/* ================================================================ config C1 stream ========= */

int qref_c1_run(uint64_t T, const uint64_t *match, const uint64_t *last, uint64_t term_start,
                uint64_t committed0, uint64_t *committed) {
    tstart_ud tud = {term_start};
    qref_log log;
    log.first_minus_1 = committed0;
    log.committed = committed0;
    log.term_at = tstart_term_at;
    log.ud = &tud;
    uint64_t m[3];
    for (uint64_t t = 0; t < T; t++) {
        log.last = last[t];
        for (int s = 0; s < 3; s++) m[s] = match[(uint64_t)s * T + t];
        /* handleLeaderReplicateResp -> tryCommit once per message (raft.go:1678) */
        if (qref_try_commit(m, 3, NULL, 0, &log, 2, NULL) == QREF_PANIC) return QREF_PANIC;
        committed[t] = log.committed;
    }
    return 0;
}

/* ================================================================ delta ingest ============= */

/* remote.tryUpdate — remote.go:123-133: if r.match < index { r.match = index } */
uint64_t qref_ingest_match(const uint64_t *u, uint64_t count, uint64_t *match, uint64_t stride,
                           uint64_t G, uint32_t n_max) {
    uint64_t skipped = 0;
    for (uint64_t i = 0; i < count; i++) {
        uint64_t g = u[2 * i] >> 8, s = u[2 * i] & 0xFF, index = u[2 * i + 1];
        if (g >= G || s >= n_max) { skipped++; continue; }
        uint64_t *m = &match[s * stride + g];
        if (*m < index) *m = index;
    }
    return skipped;
}

/* readIndex.confirm — readindex.go:83: p.confirmed[from] = struct{}{} */
uint64_t qref_ingest_ack(const uint64_t *gs, uint64_t count, uint8_t *ack, uint64_t G,
                         uint32_t n_max) {
    uint64_t skipped = 0;
    for (uint64_t i = 0; i < count; i++) {
        uint64_t g = gs[i] >> 8, s = gs[i] & 0xFF;
        if (g >= G || s >= n_max || s >= 8) { skipped++; continue; }
        ack[g] |= (uint8_t)(1u << s);
    }
    return skipped;
}

/* raft.appendEntries — raft.go:911-922: entries get r.term and indexes lastIndex+1.., then
 * remotes[self].tryUpdate(lastIndex) */
uint64_t qref_append(const uint64_t *u, uint64_t count, uint64_t *last_index,
                     uint64_t *match_slot0, uint16_t *term_mask, uint32_t R, uint64_t G) {
    uint64_t skipped = 0;
    for (uint64_t i = 0; i < count; i++) {
        uint64_t g = u[2 * i], new_last = u[2 * i + 1];
        if (g >= G) { skipped++; continue; }
        for (uint64_t idx = last_index[g] + 1; idx <= new_last; idx++) {
            if (term_mask) term_mask[g] |= (uint16_t)(1u << (idx & (R - 1)));
            if (new_last - idx >= R) idx = new_last - R;  /* older bits are overwritten anyway */
        }
        if (new_last > last_index[g]) last_index[g] = new_last;
        if (match_slot0[g] < last_index[g]) match_slot0[g] = last_index[g];
    }
    return skipped;
}

uint64_t qref_fnv1a64(const void *p, size_t bytes) {
    const uint8_t *b = (const uint8_t *)p;
    uint64_t h = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < bytes; i++) { h ^= b[i]; h *= 0x100000001b3ull; }
    return h;
}
