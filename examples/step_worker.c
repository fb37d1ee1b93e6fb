/*
 * step_worker.c — a plain C host of the step worker (what a cgo execEngine.processSteps would
 * do, INTEGRATION.md §4, without Go): three Raft groups on one device worker
 * (HQ_WORKER_ON_DEVICE | HQ_WORKER_COMMIT_ADVANCE: commits as one 4-byte advance per listed
 * group when more than a quarter of them commit), two steps of events encoded as a sized event stream
 * (hq_events_encode_sized), stepped with hq_worker_step_stream. The expected results follow the
 * reference by hand:
 *   cluster 100, leader of 3 remotes + 1 witness + 1 observer (4 voting, quorum 3), committed 5,
 *     last 7, its term's first entry 6: ReplicateResp(7) from remote 2 leaves the 3rd largest
 *     voting match at 5 (no commit, raft.go:888-909); the witness's ReplicateResp(7) makes it 7
 *     = last, term(7) = 3 → commit 7 (logentry.go:378-393); the observer's ack does not count;
 *   cluster 200, leader of 3 remotes, committed 10 at its term: a local ReadIndex (ctx 77/1) is
 *     queued at index 10 (raft.go:1636-1669) and released by one HeartbeatResp carrying the ctx
 *     (1 + 1 >= quorum 2, readindex.go:77-116) → ReadyToRead{10, 77/1};
 *   cluster 300, follower of 5 remotes at term 3: the Election tick campaigns (term 4, candidate,
 *     self vote, raft.go:1082-1117); next step two grants and a rejection at term 4 reach the
 *     quorum of 3 grants → leader (raft.go:1968-1985).
 * Exit status 0 iff every list equals that.
 *
 *   gcc -std=c99 -Iinclude examples/step_worker.c -Ldragonboat_amd/lib -lhipquorum \
 *       -Wl,-rpath,dragonboat_amd/lib -o step_worker && ./step_worker
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "hipquorum.h"

#define CHECK(call)                                                                    \
    do {                                                                               \
        int rc_ = (call);                                                              \
        if (rc_ != HQ_OK) {                                                            \
            fprintf(stderr, "%s failed: %d %s\n", #call, rc_, hq_worker_last_error(w)); \
            return 2;                                                                  \
        }                                                                              \
    } while (0)
#define EXPECT(cond, what)                                                             \
    do {                                                                               \
        if (!(cond)) {                                                                 \
            printf("%s FAILED\n", what);                                               \
            return 1;                                                                  \
        }                                                                              \
        printf("%s ok\n", what);                                                       \
    } while (0)

static hq_event msg(uint32_t type, uint64_t from, uint64_t term, uint64_t index, uint64_t hint,
                    uint64_t high, uint32_t reject) {
    hq_event e;
    memset(&e, 0, sizeof e);
    e.kind = HQ_EV_MESSAGE;
    e.type = type;
    e.from = from;
    e.term = term;
    e.log_index = index;
    e.hint = hint;
    e.hint_high = high;
    e.reject = reject;
    return e;
}

static hq_event local(uint32_t kind, uint64_t hint, uint64_t high) {
    hq_event e;
    memset(&e, 0, sizeof e);
    e.kind = kind;
    e.hint = hint;
    e.hint_high = high;
    return e;
}

/* one step: rows per group (in the order node.handleEvents takes them) -> sized stream -> step */
static int step(hq_worker *w, uint32_t n, const uint32_t *handles, const uint64_t *offsets,
                const hq_event *events, hq_step_output *out) {
    static uint8_t bytes[64 * 64];
    uint32_t sizes[8];
    uint64_t nb = 0;
    int rc = hq_events_encode_sized(n, offsets, events, bytes, sizeof bytes, sizes, &nb);
    if (rc != HQ_OK) return rc;
    hq_step_stream in;
    memset(&in, 0, sizeof in);
    in.n_groups = n;
    in.groups = handles;
    in.bytes = bytes;
    in.sizes = sizes;
    in.n_events = offsets[n];
    in.n_bytes = nb;
    return hq_worker_step_stream(w, &in, out);
}

int main(void) {
    hq_worker *w = NULL;
    if (hq_worker_open_ex(0, 8, HQ_WORKER_ON_DEVICE | HQ_WORKER_COMMIT_ADVANCE, &w) != HQ_OK) {
        fprintf(stderr, "hq_worker_open_ex: %s\n", hq_worker_last_error(NULL));
        return 2;
    }
    const hq_member ma[5] = {{1, 7, HQ_ROLE_REMOTE, 0}, {2, 5, HQ_ROLE_REMOTE, 0},
                             {3, 5, HQ_ROLE_REMOTE, 0}, {4, 5, HQ_ROLE_WITNESS, 0},
                             {5, 5, HQ_ROLE_OBSERVER, 0}};
    const hq_member mb[3] = {{1, 10, HQ_ROLE_REMOTE, 0}, {2, 10, HQ_ROLE_REMOTE, 0},
                             {3, 10, HQ_ROLE_REMOTE, 0}};
    const hq_member mc[5] = {{1, 0, HQ_ROLE_REMOTE, 0}, {2, 0, HQ_ROLE_REMOTE, 0},
                             {3, 0, HQ_ROLE_REMOTE, 0}, {4, 0, HQ_ROLE_REMOTE, 0},
                             {5, 0, HQ_ROLE_REMOTE, 0}};
    const hq_worker_group ga = {100, 1, 3, 5, 7, 6, HQ_STATE_LEADER, 5, 0, 0};
    const hq_worker_group gb = {200, 1, 2, 10, 10, 9, HQ_STATE_LEADER, 3, 0, 0};
    const hq_worker_group gc = {300, 1, 3, 9, 9, 0, HQ_STATE_FOLLOWER, 5, 0, 0};
    uint32_t h[3];
    CHECK(hq_worker_add_group(w, &ga, ma, &h[0]));
    CHECK(hq_worker_add_group(w, &gb, mb, &h[1]));
    CHECK(hq_worker_add_group(w, &gc, mc, &h[2]));

    /* step 1 */
    const hq_event ev1[] = {
        msg(HQ_MSG_REPLICATE_RESP, 2, 3, 7, 0, 0, 0),   /* cluster 100 */
        msg(HQ_MSG_REPLICATE_RESP, 4, 3, 7, 0, 0, 0),
        msg(HQ_MSG_REPLICATE_RESP, 5, 3, 7, 0, 0, 0),
        local(HQ_EV_READ, 77, 1),                       /* cluster 200 */
        msg(HQ_MSG_HEARTBEAT_RESP, 2, 2, 0, 77, 1, 0),
        local(HQ_EV_ELECTION, 0, 0),                    /* cluster 300 */
    };
    const uint64_t off1[4] = {0, 3, 5, 6};
    hq_step_output out;
    CHECK(step(w, 3, h, off1, ev1, &out));
    /* one of the three listed groups commits (> 1/4): the advance column, in listing order */
    EXPECT(out.n_commits == 1 && out.commits == NULL && out.committed_advance != NULL &&
               out.committed_advance[0] == 2 && out.committed_advance[1] == 0 &&
               out.committed_advance[2] == 0,
           "commit 100 -> 7 as advance 2 (witness ack, observer ack ignored)");
    EXPECT(out.n_ready == 1 && out.ready[0].cluster_id == 200 && out.ready[0].index == 10 &&
               out.ready[0].ctx_low == 77 && out.ready[0].ctx_high == 1,
           "ReadyToRead 200 at 10");
    EXPECT(out.n_state_changes == 1 && out.state_changes[0].cluster_id == 300 &&
               out.state_changes[0].term == 4 && out.state_changes[0].state == HQ_STATE_CANDIDATE &&
               out.state_changes[0].reason == HQ_REASON_CAMPAIGN,
           "300 campaigns at term 4");
    EXPECT(out.n_fallback_groups == 0 && out.n_deferred == 0 && out.n_dropped_reads == 0,
           "no fallback, deferred or dropped");

    /* step 2 */
    const hq_event ev2[] = {
        msg(HQ_MSG_REQUEST_VOTE_RESP, 2, 4, 0, 0, 0, 0),
        msg(HQ_MSG_REQUEST_VOTE_RESP, 3, 4, 0, 0, 0, 1),
        msg(HQ_MSG_REQUEST_VOTE_RESP, 4, 4, 0, 0, 0, 0),
    };
    const uint64_t off2[2] = {0, 3};
    CHECK(step(w, 1, &h[2], off2, ev2, &out));
    EXPECT(out.n_state_changes == 1 && out.state_changes[0].cluster_id == 300 &&
               out.state_changes[0].term == 4 && out.state_changes[0].state == HQ_STATE_LEADER &&
               out.state_changes[0].reason == HQ_REASON_VOTE,
           "300 leader at term 4 (3 of 5 grants)");
    hq_worker_group g;
    CHECK(hq_worker_get_group(w, 100, &g, NULL, 0, NULL, 0));
    EXPECT(g.committed == 7 && g.state == HQ_STATE_LEADER, "state of 100 read back");
    CHECK(hq_worker_get_group(w, 300, &g, NULL, 0, NULL, 0));
    EXPECT(g.term == 4 && g.state == HQ_STATE_LEADER && g.last_index == 10 && g.term_start == 10,
           "state of 300 read back (its no-op at 10)");
    hq_worker_close(w);
    return 0;
}
