/*
 * qref.h — CPU oracle for the hipquorum parity tests. TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of dragonboat's leader quorum arithmetic (reference tree
 * /root/reference, Go module github.com/lni/dragonboat/v3, v3.3-dev). Each function cites the
 * reference file:line it restates. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / the CPU baseline — the
 * product (libhipquorum.so) never links or calls it.
 *
 * Pinning: the reference is Go and no Go toolchain exists in this image, so the reference itself
 * cannot be run. This restatement is pinned by the known-answer tables of the reference's own
 * tests, transcribed as fixtures under tests/golden/ (see tests/golden/make_golden.py for the
 * file:line of every table), plus an independent count-based definition of the commit quorum.
 */
#ifndef QREF_H
#define QREF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QREF_MAX_NODES   16
#define QREF_MAX_PENDING 64

/* reference State enum values (internal/raft/raft.go:62-71) */
#define QREF_FOLLOWER  0
#define QREF_CANDIDATE 1
#define QREF_LEADER    2

/* status codes for reference panics (the Go code panics; the oracle reports) */
#define QREF_OK            0
#define QREF_PANIC        -100

/* ---------------------------------------------------------------- quorum arithmetic ------- */
int qref_num_voting_members(int n_remotes, int n_witnesses);   /* raft.go:368-370 */
int qref_quorum(int n_voting);                                  /* raft.go:372-374 */
int qref_is_single_node_quorum(int n_voting);                   /* raft.go:376-378 */
void qref_sort_match_values(uint64_t *matched, int n);          /* raft.go:861-886 */

/* ---------------------------------------------------------------- entry log term ---------- */
/* Term source for indexes inside [first-1, last]: stands for inMemory.getTerm
 * (inmemory.go:87-105) followed by ILogDB.Term (logentry.go:152-159). Returns the term. */
typedef uint64_t (*qref_term_fn)(const void *ud, uint64_t index);

typedef struct qref_log {
    uint64_t first_minus_1;   /* termEntryRange() first (logentry.go:117-126) */
    uint64_t last;            /* lastIndex() (logentry.go:107-115) */
    uint64_t committed;       /* entryLog.committed */
    qref_term_fn term_at;
    const void *ud;
} qref_log;

uint64_t qref_log_term(const qref_log *l, uint64_t index);       /* logentry.go:143-160 */
/* entryLog.tryCommit (logentry.go:378-393) incl. commitTo (:323-332). Returns 1 if committed
 * advanced, 0 if not, QREF_PANIC where the reference panics (commitTo beyond lastIndex). */
int qref_log_try_commit(qref_log *l, uint64_t index, uint64_t term);

/* raft.tryCommit (raft.go:888-909): matched = remotes' match then witnesses' match; sort; q =
 * matched[n - quorum]; log.tryCommit(q, term). *q_out (may be NULL) receives q. */
int qref_try_commit(const uint64_t *remote_match, int n_remotes,
                    const uint64_t *witness_match, int n_witnesses,
                    qref_log *log, uint64_t term, uint64_t *q_out);

/* Independent definition used to cross-check sort + index: q = max{x in match :
 * |{i : match_i >= x}| >= quorum}. */
uint64_t qref_quorum_match_by_count(const uint64_t *match, int n);

/* ---------------------------------------------------------------- ReadIndex --------------- */
typedef struct qref_sysctx { uint64_t low, high; } qref_sysctx;   /* raftpb/raft.go:46-49 */

typedef struct qref_read_status {                                  /* readindex.go:21-26 */
    uint64_t index;
    uint64_t from;
    qref_sysctx ctx;
    int n_confirmed;
    uint64_t confirmed[QREF_MAX_NODES];
} qref_read_status;

typedef struct qref_read_index {                                   /* readindex.go:31-34 */
    qref_read_status pending[QREF_MAX_PENDING];  /* map keyed by ctx */
    int n_pending;
    qref_sysctx queue[QREF_MAX_PENDING];
    int n_queue;
} qref_read_index;

void qref_ri_init(qref_read_index *r);
/* readindex.go:43-67. Returns QREF_OK (also when the ctx was already pending: ignored) or
 * QREF_PANIC ("index moved backward", "inconsistent pending and queue"). */
int qref_ri_add_request(qref_read_index *r, uint64_t index, qref_sysctx ctx, uint64_t from);
int qref_ri_has_pending(const qref_read_index *r);                 /* readindex.go:69-71 */
/* readindex.go:77-116. Returns the number of released statuses (0 = nil) and copies them, in
 * queue order with the rewritten index, into out[0..] (capacity QREF_MAX_PENDING); QREF_PANIC
 * where the reference panics. */
int qref_ri_confirm(qref_read_index *r, qref_sysctx ctx, uint64_t from, int quorum,
                    qref_read_status *out);

/* ---------------------------------------------------------------- votes ------------------- */
typedef struct qref_votes {                                        /* raft.go:210 votes map */
    int n;
    uint64_t from[QREF_MAX_NODES];
    int granted[QREF_MAX_NODES];
} qref_votes;

void qref_votes_reset(qref_votes *v);                              /* raft.go:999 */
int qref_handle_vote_resp(qref_votes *v, uint64_t from, int rejected);   /* raft.go:1062-1080 */
/* handleCandidateRequestVoteResp (raft.go:1968-1985) for a candidate; returns the state after
 * the message (QREF_LEADER / QREF_FOLLOWER / QREF_CANDIDATE). Observer responses are dropped. */
int qref_candidate_vote_resp(qref_votes *v, uint64_t from, int rejected, int from_is_observer,
                             int quorum);

/* leaderHasQuorum (raft.go:380-390): voting members with id == self or active count; every
 * member's active flag is reset (remote.go:196-198). */
int qref_leader_has_quorum(const uint64_t *ids, int *active, int n_voting, uint64_t self_id);

/* ---------------------------------------------------------------- batched SoA forms ------- */
/* Same memory layout and semantics as hq_commit_args in include/hipquorum.h (duplicated here so
 * that the oracle does not depend on the product headers). */
typedef struct qref_commit_args {
    uint64_t G;
    uint32_t n_max;
    uint32_t form;            /* 0 = term-start, 1 = ring, 2 = current-term mask, 3 = ring
                                 (u32-packed in the product; decided here from the u64 ring) */
    uint32_t ring_len;
    uint32_t reserved;
    uint64_t match_stride;
    const uint64_t *match;
    const uint8_t *n_voting;
    const uint64_t *committed_in;
    uint64_t *committed_out;
    const uint64_t *last_index;
    const uint64_t *term_start;
    const uint64_t *term;
    const uint64_t *ring;
    uint64_t *changed;
    uint64_t *fallback;
    const uint16_t *term_mask;   /* form 2 */
} qref_commit_args;

/* Batched commit: every group goes through qref_try_commit over a log view. Returns QREF_OK,
 * -1 on bad arguments, QREF_PANIC if some group reached a reference panic. nthreads <= 1 runs
 * single-threaded; otherwise groups are split over nthreads pthreads in contiguous 64-aligned
 * blocks (bitmap words are never shared between threads). */
int qref_commit_batch(const qref_commit_args *a, int nthreads);

/* One pending ctx per group: addRequest + one confirm per acked slot in slot order
 * (readindex.go:43-116); confirmed bit = some confirm released the ctx. */
int qref_readindex_batch(uint64_t G, const uint8_t *ack, const uint8_t *n_voting,
                         uint32_t n_uniform, uint64_t *confirmed, uint64_t *fallback,
                         int nthreads);
/* campaign self-vote (raft.go:1093) then one RequestVoteResp per responding slot in slot order
 * through handleCandidateRequestVoteResp; outcome packed 2 bits per group. */
int qref_vote_batch(uint64_t G, const uint8_t *granted, const uint8_t *rejected,
                    const uint8_t *n_voting, uint32_t n_uniform, uint64_t *outcome,
                    uint64_t *fallback, int nthreads);
int qref_check_quorum_batch(uint64_t G, uint8_t *active, const uint8_t *n_voting,
                            uint32_t n_uniform, uint32_t self_slot, uint64_t *has_quorum,
                            uint64_t *fallback, int nthreads);

/* General multi-ctx ReadIndex. Per group: K pending ctxs in queue order with
 * indexes ctx_index[k*G + g] (addRequest, readindex.go:43-67); ack_ordinal[(k*n_max + s)*G + g]
 * = arrival ordinal of voting slot s's first HeartbeatResp for ctx k (0xFFFF = none). The
 * messages are replayed in ordinal order through readIndex.confirm (readindex.go:77-116);
 * released_index[k*G + g] = the rewritten index of entry k if it was released, else UINT64_MAX;
 * released_count[g] = released prefix length; batch_end[g] (may be NULL) bit k = entry k was the
 * ctx of the confirm() call that released its batch. Groups with n outside [1, n_max] or
 * K > K_max are fallback (nothing released). */
int qref_readindex_multi_batch(uint64_t G, uint32_t K_max, uint32_t n_max,
                               const uint16_t *ack_ordinal, const uint64_t *ctx_index,
                               const uint8_t *n_pending, const uint8_t *n_voting,
                               uint32_t n_uniform, uint64_t *released_index,
                               uint8_t *released_count, uint8_t *batch_end, uint64_t *fallback,
                               int nthreads);

/* ---------------------------------------------------------------- delta ingest (§8f-1) ----- */
/* Sequential restatements, applied in array order: remote.tryUpdate (remote.go:123-133) on
 * match[slot*stride + group]; the confirmed-set insert (readindex.go:83) on ack[group]; and the
 * leader's appendEntries (raft.go:911-922) on last_index / its own match / the term mask.
 * Entries with group >= G or slot >= n_max are skipped; the return value is the skip count. */
uint64_t qref_ingest_match(const uint64_t *group_slot_index, uint64_t count, uint64_t *match,
                           uint64_t stride, uint64_t G, uint32_t n_max);
uint64_t qref_ingest_ack(const uint64_t *group_slot, uint64_t count, uint8_t *ack, uint64_t G,
                         uint32_t n_max);
uint64_t qref_append(const uint64_t *group_newlast, uint64_t count, uint64_t *last_index,
                     uint64_t *match_slot0, uint16_t *term_mask, uint32_t ring_len, uint64_t G);

/* ---------------------------------------------------------------- synthetic inputs -------- */
/* Same layout as hq_synth_spec; CPU twin of the device generator. */
typedef struct qgen_spec {
    uint64_t seed;
    uint64_t G;
    uint64_t cid_base;
    uint64_t cid_stride;
    uint32_t n_max;
    uint32_t mixed_n;
    uint32_t ring_len;
    uint32_t parity_extras;
} qgen_spec;

uint64_t qgen_splitmix64(uint64_t *state);
int qgen_commit(const qgen_spec *s, const qref_commit_args *out);
int qgen_bitmaps(const qgen_spec *s, uint8_t *ack, uint8_t *granted, uint8_t *rejected,
                 uint8_t *n_voting);

/* BASELINE config C1: one group x 3 voters, a stream of T ReplicateResp steps.
 * qgen_c1_stream fills match (slot-major [3][T], the group's match vector after each step) and
 * last (lastIndex after each step): each step raises one follower's match by 0..3 (clamped to
 * last); every 8th step the leader appends 1..4 entries (its own match follows, raft.go:918).
 * qref_c1_run replays the stream through raft.tryCommit one step at a time (term-start log
 * view: entries >= term_start carry the leader's term) and writes committed after each step. */
int qgen_c1_stream(uint64_t seed, uint64_t T, uint64_t committed0, uint64_t last0,
                   uint64_t *match, uint64_t *last);
int qref_c1_run(uint64_t T, const uint64_t *match, const uint64_t *last, uint64_t term_start,
                uint64_t committed0, uint64_t *committed);

/* ---------------------------------------------------------------- one step, event by event - */
/* Sequential replay of one group's step (oracle/qref_step.c): the checker of the GPU step worker
 * (hq_worker_step). Roles and members mirror hq_member of include/hipquorum.h. */
#define QREF_ROLE_REMOTE   0
#define QREF_ROLE_OBSERVER 1
#define QREF_ROLE_WITNESS  2
#define QREF_STEP_MAX_MEMBERS 16
#define QREF_STEP_MAX_OUT     64

#define QREF_EV_READ         1   /* local ReadIndex (node.handleReadIndex): hint/hint_high = ctx */
#define QREF_EV_MSG          2   /* received message (type, from, term, log_index, hint, reject) */
#define QREF_EV_CHECK_QUORUM 3   /* the leader tick's CheckQuorum message */
#define QREF_EV_CAMPAIGN     4   /* the election tick's Election message */
#define QREF_EV_PROPOSE      5   /* proposal of log_index entries */

/* state-change reasons */
#define QREF_REASON_VOTE         1
#define QREF_REASON_CHECK_QUORUM 2
#define QREF_REASON_HIGHER_TERM  3
#define QREF_REASON_CAMPAIGN     4
/* dropped-ReadIndex reasons (reportDroppedReadIndex) */
#define QREF_DROP_WITNESS   1
#define QREF_DROP_NOT_READY 2

typedef struct qref_member {
    uint64_t node_id;
    uint64_t match;
    uint32_t role;
    uint32_t active;
} qref_member;

typedef struct qref_event {
    uint32_t kind;
    uint32_t type;
    uint64_t from, term, log_index, hint, hint_high;
    uint32_t reject;
    uint32_t reserved;
} qref_event;

#define QREF_LOG_MAX_RUNS 64

typedef struct qref_group {
    uint64_t cluster_id, node_id, term;
    int state;
    int n_members;
    uint64_t committed, last, term_start;
    qref_member members[QREF_STEP_MAX_MEMBERS];
    qref_read_index *ri;      /* allocated on the first ReadIndex; qref_group_free releases it */
    qref_votes votes;
    /* The node's log as terms by index, the way inMemory.getTerm / logdb answer it
     * (inmemory.go:87-105, logentry.go:143-160): runs of equal terms, run k covering
     * [run_start[k], run_start[k + 1]) with term run_term[k] (starts and terms increasing,
     * entryutils.go:44-47); indexes below first_minus_1 are compacted (term 0, ErrCompacted) and
     * above last do not exist (term 0). The leader's no-op and proposals extend it at r.term
     * (raft.go:911-922, 977-989). qref_group_init sets the two-run history {(0, term - 1),
     * (term_start, term)}; qref_group_set_log replaces it with any history. term_start (the
     * first current-term index) is only reported, never read by the oracle's term check. */
    uint64_t first_minus_1;
    int n_runs;
    uint64_t run_start[QREF_LOG_MAX_RUNS], run_term[QREF_LOG_MAX_RUNS];
} qref_group;

typedef struct qref_step_out {
    uint64_t committed;
    int commit_changed;
    int n_ready, n_resps, n_states, n_dropped, n_deferred;
    struct { uint64_t index, low, high; } ready[QREF_STEP_MAX_OUT];
    struct { uint64_t to, index, hint, hint_high; } resps[QREF_STEP_MAX_OUT];
    struct { uint64_t term; uint32_t state, reason; } states[QREF_STEP_MAX_OUT];
    struct { uint64_t low, high, from; uint32_t reason, reserved; } dropped[QREF_STEP_MAX_OUT];
    uint32_t deferred[QREF_STEP_MAX_OUT];   /* event indexes handed to the non-quorum CPU path */
} qref_step_out;

int qref_group_init(qref_group *g, uint64_t cluster_id, uint64_t node_id, uint64_t term,
                    int state, uint64_t committed, uint64_t last, uint64_t term_start,
                    const qref_member *members, int n_members);
void qref_group_free(qref_group *g);
/* Replace the group's log history (see qref_group): starts strictly increasing with
 * starts[0] <= first_minus_1, terms strictly increasing and <= the group's term. Returns 0 or -1. */
int qref_group_set_log(qref_group *g, uint64_t first_minus_1, int n_runs, const uint64_t *starts,
                       const uint64_t *terms);

/* Many groups, one step (the CPU baseline of the step worker): list[i] is an index into
 * `groups` whose events are events[offsets[i] .. offsets[i + 1]) — the layout of hq_step_input
 * (qref_event has hq_event's layout and kind values). Each listed group is replayed with
 * qref_group_step; the list is split over nthreads threads. Totals of the outputs go to *tot. */
typedef struct qref_step_totals {
    uint64_t commits, ready, resps, states, dropped, deferred, committed_sum;
    /* order-free content digests (sums of qref_digest_* over the step's outputs, so any split
     * of the list over threads, workers or GPUs adds up to the same value): every ReadyToRead
     * record (cluster, index, ctx) and every group whose committed index moved (cluster,
     * advance) */
    uint64_t ready_digest, commit_digest;
    /* order-sensitive: the sum over the step's ReadyToRead records, in output order (the list's
     * groups in order, each group's records in order), of (position + 1) * qref_digest_ready —
     * a reordered list changes it. Threads combine their sums by their records' offsets. */
    uint64_t ready_order_digest;
} qref_step_totals;

/* splitmix64's finalizer; the digest terms bench.py recomputes from the device results */
static inline uint64_t qref_mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
static inline uint64_t qref_digest_ready(uint64_t cluster_id, uint64_t index, uint64_t low,
                                         uint64_t high) {
    return qref_mix64(qref_mix64(cluster_id) ^ (index * 0x9e3779b97f4a7c15ULL +
                                                low * 0xc2b2ae3d27d4eb4fULL +
                                                high * 0x165667b19e3779f9ULL));
}
/* linear in the advance: a random odd coefficient per cluster (mod 2^64), cheap to recompute
 * over a whole column of advances */
static inline uint64_t qref_digest_commit(uint64_t cluster_id, uint64_t advance) {
    return (qref_mix64(cluster_id) | 1ULL) * advance;
}

/* hq_worker_group layout: a group's initial state; members of consecutive groups back to back */
typedef struct qref_group_rec {
    uint64_t cluster_id, node_id, term, committed, last_index, term_start;
    uint32_t state, n_members, n_pending_reads, suspended;
} qref_group_rec;

uint64_t qref_digest_ready_term(uint64_t cluster_id, uint64_t index, uint64_t low, uint64_t high);
uint64_t qref_digest_commit_term(uint64_t cluster_id, uint64_t advance);
qref_group *qref_groups_new(uint64_t G);
int qref_groups_init(qref_group *groups, uint64_t G, const qref_group_rec *recs,
                     const qref_member *members);
void qref_groups_free(qref_group *groups, uint64_t G);
int qref_step_batch(qref_group *groups, uint64_t G, uint64_t n_list, const uint32_t *list,
                    const uint64_t *offsets, const qref_event *events, int nthreads,
                    qref_step_totals *tot);
/* Replays the events in order; returns 0, -1 on bad arguments or QREF_PANIC where the reference
 * panics (or an output list overflows). */
int qref_group_step(qref_group *g, const qref_event *ev, int n_events, qref_step_out *out);

/* FNV-1a 64 over a byte range (fixture checksums). */
uint64_t qref_fnv1a64(const void *p, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif
