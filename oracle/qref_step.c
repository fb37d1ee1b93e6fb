/*
 * qref_step.c — CPU oracle of one step of a Raft node's quorum-relevant event stream, replayed
 * one event at a time exactly as the reference processes it. TEST INFRASTRUCTURE ONLY: it is the
 * sequential checker of the step worker (hq_worker_step in include/hipquorum.h), which batches
 * the same events and decides them on the GPU.
 *
 * Event order inside a step follows node.handleEvents (node.go:1113-1157): the local ReadIndex
 * (handleReadIndex :1197-1206 -> Peer.ReadIndex, peer.go:297-303), the received messages
 * (handleReceivedMessages :1257-1289 -> Peer.Handle, peer.go:186-198), the local tick's
 * CheckQuorum / Election messages (handleLocalTick), then proposals (handleProposals
 * :1184-1195). The caller lists the events of one group in that order.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "qref.h"

/* raftpb message types (raftpb/raft.proto:26-52) */
enum { MT_REPLICATE_RESP = 13, MT_REQUEST_VOTE_RESP = 15, MT_HEARTBEAT_RESP = 18, MT_READ_INDEX = 19 };

static int is_response_type(uint32_t t) {   /* isResponseMessageType (raft/utils.go) */
    return t == MT_REPLICATE_RESP || t == MT_REQUEST_VOTE_RESP || t == MT_HEARTBEAT_RESP ||
           t == 20 /* ReadIndexResp */ || t == 8 /* SnapshotStatus */ || t == 9 /* Unreachable */;
}

static int find_member(const qref_group *g, uint64_t id) {
    for (int i = 0; i < g->n_members; i++)
        if (g->members[i].node_id == id) return i;
    return -1;
}

static int role_of(const qref_group *g, uint64_t id) {
    int i = find_member(g, id);
    return i < 0 ? -1 : (int)g->members[i].role;
}

static int n_voting(const qref_group *g) {      /* numVotingMembers, raft.go:368-370 */
    int n = 0;
    for (int i = 0; i < g->n_members; i++) n += g->members[i].role != QREF_ROLE_OBSERVER;
    return n;
}

static int quorum(const qref_group *g) { return qref_quorum(n_voting(g)); }

/* the term of index i in the group's log history (the run that holds it; inMemory.getTerm,
 * inmemory.go:87-105, and logdb below it); qref_log_term applies the compacted / beyond-last
 * bounds first (logentry.go:143-160) */
static uint64_t history_term_at(const void *ud, uint64_t i) {
    const qref_group *g = (const qref_group *)ud;
    uint64_t t = 0;
    for (int k = 0; k < g->n_runs && g->run_start[k] <= i; k++) t = g->run_term[k];
    return t;
}

static qref_log log_view(qref_group *g) {
    qref_log l;
    l.first_minus_1 = g->first_minus_1;
    l.last = g->last;
    l.committed = g->committed;
    l.term_at = history_term_at;
    l.ud = g;
    return l;
}

/* entries appended at the group's term from index `from` on (the leader's no-op and proposals,
 * raft.go:911-922): a new run unless the last run already has this term */
static int log_extend(qref_group *g, uint64_t from) {
    if (g->n_runs && g->run_term[g->n_runs - 1] == g->term) return QREF_OK;
    if (g->n_runs && g->run_start[g->n_runs - 1] >= from) {   /* a run of no entries yet */
        g->run_start[g->n_runs - 1] = from;
        g->run_term[g->n_runs - 1] = g->term;
        return QREF_OK;
    }
    if (g->n_runs >= QREF_LOG_MAX_RUNS) return QREF_PANIC;
    g->run_start[g->n_runs] = from;
    g->run_term[g->n_runs] = g->term;
    g->n_runs++;
    return QREF_OK;
}

/* raft.tryCommit (raft.go:888-909) over the group's remotes then witnesses */
static int try_commit(qref_group *g) {
    uint64_t rm[QREF_STEP_MAX_MEMBERS], wm[QREF_STEP_MAX_MEMBERS];
    int nr = 0, nw = 0;
    for (int i = 0; i < g->n_members; i++) {
        if (g->members[i].role == QREF_ROLE_REMOTE) rm[nr++] = g->members[i].match;
        else if (g->members[i].role == QREF_ROLE_WITNESS) wm[nw++] = g->members[i].match;
    }
    qref_log l = log_view(g);
    int rc = qref_try_commit(rm, nr, wm, nw, &l, g->term, NULL);
    if (rc == QREF_PANIC) return rc;
    g->committed = l.committed;
    return rc;
}

static int push_state(qref_group *g, qref_step_out *o, int reason) {
    if (o->n_states >= QREF_STEP_MAX_OUT) return QREF_PANIC;
    o->states[o->n_states].term = g->term;
    o->states[o->n_states].state = (uint32_t)g->state;
    o->states[o->n_states].reason = (uint32_t)reason;
    o->n_states++;
    return QREF_OK;
}

/* raft.reset (raft.go:991-1010): votes, readIndex and every remote (resetRemotes/Observers/
 * Witnesses :1025-1059: match 0 except the node itself at lastIndex, active false) */
static void reset(qref_group *g, uint64_t term) {
    if (g->term != term) g->term = term;   /* vote = NoLeader: not modelled */
    qref_votes_reset(&g->votes);
    if (g->ri) qref_ri_init(g->ri);
    for (int i = 0; i < g->n_members; i++) {
        g->members[i].match = g->members[i].node_id == g->node_id ? g->last : 0;
        g->members[i].active = 0;
    }
}

static int become_follower(qref_group *g, uint64_t term, qref_step_out *o, int reason) {
    g->state = QREF_FOLLOWER;                                        /* raft.go:949-957 */
    reset(g, term);
    return push_state(g, o, reason);
}

/* raft.appendEntries (raft.go:911-922): entries get r.term and follow lastIndex; the node's own
 * remote follows the log; a single-node quorum commits at once */
static int append_entries(qref_group *g, uint64_t n) {
    if (n) {
        int rc = log_extend(g, g->last + 1);
        if (rc) return rc;
    }
    g->last += n;
    int self = find_member(g, g->node_id);
    if (self >= 0 && g->members[self].match < g->last) g->members[self].match = g->last;
    if (qref_is_single_node_quorum(n_voting(g))) {
        int rc = try_commit(g);
        if (rc == QREF_PANIC) return rc;
    }
    return QREF_OK;
}

static int become_leader(qref_group *g, qref_step_out *o) {
    g->state = QREF_LEADER;                                          /* raft.go:977-989 */
    reset(g, g->term);
    int rc = push_state(g, o, QREF_REASON_VOTE);
    if (rc) return rc;
    g->term_start = g->last + 1;   /* the no-op of p72 is the first entry of the new term */
    return append_entries(g, 1);
}

static int add_ready(qref_step_out *o, uint64_t index, uint64_t low, uint64_t high) {
    if (o->n_ready >= QREF_STEP_MAX_OUT) return QREF_PANIC;
    o->ready[o->n_ready].index = index;
    o->ready[o->n_ready].low = low;
    o->ready[o->n_ready].high = high;
    o->n_ready++;
    return QREF_OK;
}

static int add_resp(qref_step_out *o, uint64_t to, uint64_t index, uint64_t hint, uint64_t high) {
    if (o->n_resps >= QREF_STEP_MAX_OUT) return QREF_PANIC;
    o->resps[o->n_resps].to = to;
    o->resps[o->n_resps].index = index;
    o->resps[o->n_resps].hint = hint;
    o->resps[o->n_resps].hint_high = high;
    o->n_resps++;
    return QREF_OK;
}

static int add_dropped(qref_step_out *o, const qref_event *e, int reason) {
    if (o->n_dropped >= QREF_STEP_MAX_OUT) return QREF_PANIC;
    o->dropped[o->n_dropped].low = e->hint;
    o->dropped[o->n_dropped].high = e->hint_high;
    o->dropped[o->n_dropped].from = e->from;
    o->dropped[o->n_dropped].reason = (uint32_t)reason;
    o->n_dropped++;
    return QREF_OK;
}

static int defer_event(qref_step_out *o, int i) {
    if (o->n_deferred >= QREF_STEP_MAX_OUT) return QREF_PANIC;
    o->deferred[o->n_deferred++] = (uint32_t)i;
    return QREF_OK;
}

/* raft.hasCommittedEntryAtCurrentTerm (raft.go:1612-1621) */
static int has_committed_entry_at_current_term(qref_group *g) {
    qref_log l = log_view(g);
    return qref_log_term(&l, g->committed) == g->term;
}

/* raft.handleLeaderReadIndex (raft.go:1636-1669) */
static int leader_read_index(qref_group *g, const qref_event *e, qref_step_out *o) {
    qref_sysctx ctx = {e->hint, e->hint_high};
    if (role_of(g, e->from) == QREF_ROLE_WITNESS) return add_dropped(o, e, QREF_DROP_WITNESS);
    if (!qref_is_single_node_quorum(n_voting(g))) {
        if (!has_committed_entry_at_current_term(g)) return add_dropped(o, e, QREF_DROP_NOT_READY);
        if (!g->ri) {                      /* the queue is allocated on first use */
            g->ri = (qref_read_index *)malloc(sizeof *g->ri);
            if (!g->ri) return QREF_PANIC;
            qref_ri_init(g->ri);
        }
        return qref_ri_add_request(g->ri, g->committed, ctx, e->from);
    }
    int rc = add_ready(o, g->committed, ctx.low, ctx.high);
    if (rc) return rc;
    if (e->from != g->node_id && role_of(g, e->from) == QREF_ROLE_OBSERVER)
        return add_resp(o, e->from, g->committed, e->hint, e->hint_high);
    return QREF_OK;
}

/* raft.handleReadIndexLeaderConfirmation (raft.go:1740-1760) */
static int read_index_confirmation(qref_group *g, const qref_event *e, qref_step_out *o) {
    qref_read_status out[QREF_MAX_PENDING];   /* 10.7 KB on the stack; thread-safe */
    qref_sysctx ctx = {e->hint, e->hint_high};
    if (!g->ri) return QREF_OK;            /* nothing pending: confirm() returns nil */
    int r = qref_ri_confirm(g->ri, ctx, e->from, quorum(g), out);
    if (r < 0) return r;
    for (int i = 0; i < r; i++) {
        int rc = (out[i].from == 0 || out[i].from == g->node_id)
                     ? add_ready(o, out[i].index, out[i].ctx.low, out[i].ctx.high)
                     : add_resp(o, out[i].from, out[i].index, e->hint, e->hint_high);
        if (rc) return rc;
    }
    return QREF_OK;
}

/* raft.campaign (raft.go:1082-1117) after becomeCandidate (:959-975) */
static int campaign(qref_group *g, qref_step_out *o) {
    g->state = QREF_CANDIDATE;
    reset(g, g->term + 1);
    int rc = push_state(g, o, QREF_REASON_CAMPAIGN);
    if (rc) return rc;
    qref_handle_vote_resp(&g->votes, g->node_id, 0);
    if (qref_is_single_node_quorum(n_voting(g))) return become_leader(g, o);
    return QREF_OK;
}

static int handle_message(qref_group *g, const qref_event *e, int i, qref_step_out *o) {
    /* Peer.Handle (peer.go:186-198): responses from non-members are dropped */
    if (is_response_type(e->type) && find_member(g, e->from) < 0) return QREF_OK;
    /* raft.onMessageTermNotMatched (raft.go:1416-1452); none of the types here is a leader
     * message, so a higher term makes the node a follower with no known leader */
    if (e->term != 0 && e->term != g->term) {
        if (e->term < g->term) return QREF_OK;                       /* ignored */
        int rc = become_follower(g, e->term, o, QREF_REASON_HIGHER_TERM);
        if (rc) return rc;
    }
    const int self_state = g->state;
    int m = find_member(g, e->from);
    if (self_state == QREF_LEADER) {
        switch (e->type) {
        case MT_REPLICATE_RESP: {                                    /* lw + :1671-1700 */
            qref_member *rp = &g->members[m];
            rp->active = 1;
            if (!e->reject && rp->match < e->log_index) {            /* remote.tryUpdate */
                rp->match = e->log_index;
                int rc = try_commit(g);
                if (rc == QREF_PANIC) return rc;
            }
            return QREF_OK;
        }
        case MT_HEARTBEAT_RESP:                                      /* lw + :1702-1714 */
            g->members[m].active = 1;
            if (e->hint != 0) return read_index_confirmation(g, e, o);
            return QREF_OK;
        case MT_READ_INDEX:
            return leader_read_index(g, e, o);
        default:
            return QREF_OK;   /* no leader handler (RequestVoteResp) */
        }
    }
    if (self_state == QREF_CANDIDATE && e->type == MT_REQUEST_VOTE_RESP) {
        int st = qref_candidate_vote_resp(&g->votes, e->from, e->reject != 0,
                                          role_of(g, e->from) == QREF_ROLE_OBSERVER, quorum(g));
        if (st == QREF_LEADER) return become_leader(g, o);
        if (st == QREF_FOLLOWER) return become_follower(g, g->term, o, QREF_REASON_VOTE);
        return QREF_OK;
    }
    /* follower / candidate ReadIndex: forwarded to the leader or dropped outside the quorum
     * path (raft.go:1875-1883, 1937-1945) */
    if (e->type == MT_READ_INDEX) return defer_event(o, i);
    return QREF_OK;
}

void qref_group_free(qref_group *g) {
    if (g && g->ri) {
        free(g->ri);
        g->ri = NULL;
    }
}

int qref_group_init(qref_group *g, uint64_t cluster_id, uint64_t node_id, uint64_t term,
                    int state, uint64_t committed, uint64_t last, uint64_t term_start,
                    const qref_member *members, int n_members) {
    if (!g || n_members < 1 || n_members > QREF_STEP_MAX_MEMBERS || (n_members && !members))
        return -1;
    memset(g, 0, sizeof *g);
    g->cluster_id = cluster_id;
    g->node_id = node_id;
    g->term = term;
    g->state = state;
    g->committed = committed;
    g->last = last;
    g->term_start = term_start;
    g->n_members = n_members;
    memcpy(g->members, members, (size_t)n_members * sizeof *members);
    g->ri = NULL;
    /* the default history: term_start's run at the group's term, one older term below it */
    g->first_minus_1 = 0;
    g->n_runs = 0;
    if (term > 0 && term_start > 0) {
        g->run_start[g->n_runs] = 0;
        g->run_term[g->n_runs++] = term - 1;
    }
    g->run_start[g->n_runs] = term_start;
    g->run_term[g->n_runs++] = term;
    qref_votes_reset(&g->votes);
    /* a candidate holds its own vote (campaign, raft.go:1093) */
    if (state == QREF_CANDIDATE) qref_handle_vote_resp(&g->votes, node_id, 0);
    return 0;
}

int qref_group_set_log(qref_group *g, uint64_t first_minus_1, int n_runs, const uint64_t *starts,
                       const uint64_t *terms) {
    if (!g || n_runs < 1 || n_runs > QREF_LOG_MAX_RUNS || !starts || !terms) return -1;
    if (starts[0] > first_minus_1 || first_minus_1 > g->committed) return -1;
    for (int k = 0; k < n_runs; k++) {
        if (k && (starts[k] <= starts[k - 1] || terms[k] <= terms[k - 1])) return -1;
        if (terms[k] > g->term) return -1;
        g->run_start[k] = starts[k];
        g->run_term[k] = terms[k];
    }
    g->n_runs = n_runs;
    g->first_minus_1 = first_minus_1;
    return 0;
}

int qref_group_step(qref_group *g, const qref_event *ev, int n_events, qref_step_out *o) {
    if (!g || !o || (n_events && !ev)) return -1;
    /* only the counts: the lists are read up to them (the struct is ~7 KB) */
    o->committed = 0;
    o->commit_changed = 0;
    o->n_ready = o->n_resps = o->n_states = o->n_dropped = o->n_deferred = 0;
    const uint64_t committed0 = g->committed;
    for (int i = 0; i < n_events; i++) {
        const qref_event *e = &ev[i];
        int rc = QREF_OK;
        switch (e->kind) {
        case QREF_EV_READ: {       /* Peer.ReadIndex: a ReadIndex message with From = NoNode */
            qref_event m = *e;
            m.type = MT_READ_INDEX;
            m.from = 0;
            m.term = 0;
            rc = handle_message(g, &m, i, o);
            break;
        }
        case QREF_EV_MSG:
            rc = handle_message(g, e, i, o);
            break;
        case QREF_EV_CHECK_QUORUM:                                   /* raft.go:1582-1588 */
            if (g->state == QREF_LEADER) {
                uint64_t ids[QREF_STEP_MAX_MEMBERS];
                int act[QREF_STEP_MAX_MEMBERS], idx[QREF_STEP_MAX_MEMBERS], n = 0;
                for (int k = 0; k < g->n_members; k++) {
                    if (g->members[k].role == QREF_ROLE_OBSERVER) continue;
                    ids[n] = g->members[k].node_id;
                    act[n] = g->members[k].active;
                    idx[n++] = k;
                }
                int ok = qref_leader_has_quorum(ids, act, n, g->node_id);
                for (int k = 0; k < n; k++) g->members[idx[k]].active = act[k];
                if (!ok) rc = become_follower(g, g->term, o, QREF_REASON_CHECK_QUORUM);
            }
            break;
        case QREF_EV_CAMPAIGN:                                       /* raft.go:1485-1515 */
            if (g->state != QREF_LEADER) rc = campaign(g, o);
            break;
        case QREF_EV_PROPOSE:                                        /* raft.go:1590-1610 */
            if (g->state == QREF_LEADER) rc = append_entries(g, e->log_index);
            else rc = defer_event(o, i);   /* forwarded / dropped (raft.go:1845-1857, 1932) */
            break;
        default:
            return -1;
        }
        if (rc < 0) return rc;
    }
    o->committed = g->committed;
    o->commit_changed = g->committed != committed0;
    return 0;
}

/* ================================================================ many groups, one step ==== */

typedef struct {
    qref_group *groups;
    const uint32_t *list;
    const uint64_t *offsets;
    const qref_event *ev;
    uint64_t i0, i1;
    qref_step_totals tot;
    int rc;
} step_job;

static void *step_run(void *p) {
    step_job *j = (step_job *)p;
    qref_step_out *o = (qref_step_out *)malloc(sizeof *o);
    if (!o) { j->rc = QREF_PANIC; return NULL; }
    for (uint64_t i = j->i0; i < j->i1; i++) {
        uint64_t b = j->offsets[i], e = j->offsets[i + 1];
        qref_group *g = &j->groups[j->list[i]];
        const uint64_t committed0 = g->committed;
        int rc = qref_group_step(g, j->ev + b, (int)(e - b), o);
        if (rc) { j->rc = rc; break; }
        for (int r = 0; r < o->n_ready; r++) {
            const uint64_t d = qref_digest_ready(g->cluster_id, o->ready[r].index,
                                                 o->ready[r].low, o->ready[r].high);
            j->tot.ready_digest += d;
            /* (the thread's own positions from 0; qref_step_batch adds its offset) */
            j->tot.ready_order_digest += j->tot.ready * d + (uint64_t)r * d;
        }
        if (o->commit_changed)
            j->tot.commit_digest += qref_digest_commit(g->cluster_id, o->committed - committed0);
        j->tot.commits += (uint64_t)o->commit_changed;
        j->tot.ready += (uint64_t)o->n_ready;
        j->tot.resps += (uint64_t)o->n_resps;
        j->tot.states += (uint64_t)o->n_states;
        j->tot.dropped += (uint64_t)o->n_dropped;
        j->tot.deferred += (uint64_t)o->n_deferred;
        j->tot.committed_sum += o->committed;
    }
    free(o);
    return NULL;
}

int qref_step_batch(qref_group *groups, uint64_t G, uint64_t n_list, const uint32_t *list,
                    const uint64_t *offsets, const qref_event *events, int nthreads,
                    qref_step_totals *tot) {
    if (!groups || !tot || nthreads < 1 || (n_list && (!list || !offsets))) return -1;
    memset(tot, 0, sizeof *tot);
    for (uint64_t i = 0; i < n_list; i++)
        if (list[i] >= G || offsets[i + 1] < offsets[i]) return -1;
    if (nthreads > 64) nthreads = 64;
    step_job jobs[64];
    pthread_t th[64];
    uint64_t per = (n_list + (uint64_t)nthreads - 1) / (uint64_t)nthreads;
    int started = 0, rc = 0;
    for (int t = 0; t < nthreads; t++) {
        uint64_t i0 = per * (uint64_t)t, i1 = i0 + per;
        if (i0 >= n_list) break;
        if (i1 > n_list) i1 = n_list;
        memset(&jobs[t], 0, sizeof jobs[t]);
        jobs[t].groups = groups;
        jobs[t].list = list;
        jobs[t].offsets = offsets;
        jobs[t].ev = events;
        jobs[t].i0 = i0;
        jobs[t].i1 = i1;
        if (nthreads == 1 || pthread_create(&th[t], NULL, step_run, &jobs[t]) != 0) {
            step_run(&jobs[t]);
            th[t] = 0;
        }
        started++;
    }
    for (int t = 0; t < started; t++) {
        if (th[t]) pthread_join(th[t], NULL);
        if (jobs[t].rc) rc = jobs[t].rc;
        tot->commits += jobs[t].tot.commits;
        tot->ready += jobs[t].tot.ready;
        tot->resps += jobs[t].tot.resps;
        tot->states += jobs[t].tot.states;
        tot->dropped += jobs[t].tot.dropped;
        tot->deferred += jobs[t].tot.deferred;
        tot->committed_sum += jobs[t].tot.committed_sum;
        /* position p of the thread's records is offset + its own position: (p + 1) d summed =
         * own-position sum + (offset + 1) * the thread's digest (tot->ready so far = offset) */
        tot->ready_order_digest += jobs[t].tot.ready_order_digest +
                                   (tot->ready - jobs[t].tot.ready + 1) * jobs[t].tot.ready_digest;
        tot->ready_digest += jobs[t].tot.ready_digest;
        tot->commit_digest += jobs[t].tot.commit_digest;
    }
    return rc;
}

/* the digest terms, exported for tests/test_step_digest.py (bench.py restates them in numpy) */
uint64_t qref_digest_ready_term(uint64_t cluster_id, uint64_t index, uint64_t low, uint64_t high) {
    return qref_digest_ready(cluster_id, index, low, high);
}
uint64_t qref_digest_commit_term(uint64_t cluster_id, uint64_t advance) {
    return qref_digest_commit(cluster_id, advance);
}

qref_group *qref_groups_new(uint64_t G) {
    return (qref_group *)calloc(G ? G : 1, sizeof(qref_group));
}

void qref_groups_free(qref_group *groups, uint64_t G) {
    if (!groups) return;
    for (uint64_t g = 0; g < G; g++) qref_group_free(&groups[g]);
    free(groups);
}

int qref_groups_init(qref_group *groups, uint64_t G, const qref_group_rec *recs,
                     const qref_member *members) {
    if (!groups || (G && (!recs || !members))) return -1;
    uint64_t off = 0;
    for (uint64_t g = 0; g < G; g++) {
        const qref_group_rec *r = &recs[g];
        int rc = qref_group_init(&groups[g], r->cluster_id, r->node_id, r->term, (int)r->state,
                                 r->committed, r->last_index, r->term_start, members + off,
                                 (int)r->n_members);
        if (rc) return rc;
        off += r->n_members;
    }
    return 0;
}
