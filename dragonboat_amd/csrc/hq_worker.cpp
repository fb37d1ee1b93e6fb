// hq_worker.cpp — the step worker of libhipquorum.so (include/hipquorum.h "step worker"): the
// caller side of the quorum kernels, in the shape of dragonboat's execEngine.processSteps
// (execengine.go:923-1000) driving node.handleEvents (node.go:1113-1157) for many groups.
//
// Host work per event is the reference's bookkeeping only — Peer.Handle's membership filter
// (peer.go:186-198), onMessageTermNotMatched (raft.go:1416-1452), remote.tryUpdate
// (remote.go:123-133), the ReadIndex confirmed-set insert (readindex.go:83) and the first-wins
// vote insert (raft.go:1071-1073). Every quorum decision is a kernel launch through the C-ABI:
// tryCommit (hq_commit_dev, term-start form), the ReadIndex release with its index rewrite
// (hq_readindex_multi_dev), the vote outcome (hq_vote_dev) and leaderHasQuorum
// (hq_check_quorum_dev). A group's events are taken in order until one needs a decision not
// yet taken (a "run"); all runs of a pass are decided in one GPU batch, applied, and the next
// pass continues where they stopped. Plain C++ (no HIP headers): the worker is a client of the
// same ABI a cgo binding would use.
//
// Storage is flat: one fixed-size record per group, its members in one pool (voting slots
// first, in slot order, so packing a group's match row is a contiguous copy) and pending
// ReadIndex queues in a pool of fixed 8-entry blocks.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/hipquorum.h"
#include "hq_dstep.h"

namespace {

constexpr uint32_t kMaxReads = 8;         // pending ReadIndex ctxs per group (k_ri_multi K_max)
constexpr uint16_t kNoAck = 0xFFFF;
constexpr uint16_t kMaxOrdinal = 0xFFF0;  // acks per run before a run is cut
constexpr uint32_t kNone = 0xFFFFFFFFu;

struct Member {                           // a remote, witness or observer of one group
    uint64_t node_id, match;
    uint8_t role, active;
    uint8_t order;                        // position in the caller's member list
    uint8_t pad[5];
};

struct ReadStatus {                       // readStatus (readindex.go:21-26)
    uint64_t index, from, low, high;
    uint16_t ord[HQ_MAX_VOTERS];          // first-ack ordinal in the current run
    uint8_t confirmed;                    // slots confirmed in earlier runs (ordinal 0)
};

struct ReadQueue {                        // readIndex.queue with its pending statuses
    uint32_t n;
    ReadStatus r[kMaxReads];
};

enum : uint8_t {
    kSuspended = 1, kTouched = 2, kInWork = 4,
    kCommitDue = 8, kRiDue = 16, kVoteDue = 32, kCqDue = 64,
    kDue = kCommitDue | kRiDue | kVoteDue | kCqDue,
};

struct Group {
    uint64_t cluster_id, node_id, term, committed, last, term_start;
    uint64_t committed0, cursor, ev_end;  // current step
    uint32_t mem;                         // first member in the pool; [0] is the node itself
    uint32_t rq;                          // read queue block, kNone when empty
    uint16_t ord;                         // acks recorded in the current run
    uint8_t n_members, mem_cap, n_voting, state, granted, rejected, flags;
    bool has(uint8_t f) const { return flags & f; }
    void set(uint8_t f) { flags |= f; }
    void clear(uint8_t f) { flags &= (uint8_t)~f; }
    bool pending() const { return flags & kDue; }
};

enum Verdict { CONSUMED, BARRIER, FALLBACK };

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

bool is_response_type(uint32_t t) {       // isResponseMessageType (internal/raft/utils.go)
    return t == HQ_MSG_REPLICATE_RESP || t == HQ_MSG_REQUEST_VOTE_RESP ||
           t == HQ_MSG_HEARTBEAT_RESP || t == 20 /* ReadIndexResp */ ||
           t == 8 /* SnapshotStatus */ || t == 9 /* Unreachable */;
}

}  // namespace

struct hq_worker {
    hq_ctx *ctx = nullptr;
    int device = -1;
    uint32_t n_max = 0;
    // HQ_WORKER_ON_DEVICE: the group state lives on the GPU (hq_dstep.hip) and a step is one
    // launch pair; the host records below are a mirror, refreshed from the device on demand
    hq_dstep *dstep = nullptr;
    bool host_stale = false;              // the device holds newer state than the mirror
    uint64_t dev_groups = 0, dev_members = 0;   // records already on the device
    std::vector<uint32_t> dirty;          // handles changed on the host since the last upload
    hq_dstep_out dout{};
    std::vector<hq_event> decoded;        // host worker: a stream step's rows
    std::vector<uint64_t> sized_off, sized_boff;   // host worker: a sized stream's prefixes
    std::vector<uint32_t> sized_groups;            // and its implicit handles
    std::string err;
    std::vector<Group> groups;
    std::vector<Member> pool;
    std::vector<ReadQueue> rqs;
    std::vector<uint32_t> rq_free;
    std::unordered_map<uint64_t, uint32_t> index;   // cluster_id -> handle
    // step scratch
    const hq_step_input *in = nullptr;
    std::vector<uint32_t> work, next_work, touched;
    std::vector<uint32_t> l_commit, l_ri, l_vote, l_cq;
    // outputs
    std::vector<hq_commit_event> commits;
    std::vector<hq_ready_to_read> ready;
    std::vector<hq_read_index_resp> resps;
    std::vector<hq_state_change> states;
    std::vector<hq_dropped_read> dropped;
    std::vector<uint64_t> deferred;
    std::vector<uint64_t> fallback;
    uint64_t decisions = 0;
    uint64_t t_pack = 0, t_device = 0, t_apply = 0;
    // staging: one pinned host buffer mirrored by one device buffer per pass
    void *host = nullptr, *dev = nullptr;
    size_t cap = 0;

    int fail(int code, const std::string &m) {
        err = m;
        return code;
    }
    int hq(int rc, const char *what) {
        if (rc) err = std::string(what) + ": " + hq_last_error(ctx);
        return rc;
    }
    Member *members(Group &g) { return pool.data() + g.mem; }
    int member_of(const Group &g, uint64_t id) const {
        const Member *m = pool.data() + g.mem;
        for (int i = 0; i < g.n_members; ++i)
            if (m[i].node_id == id) return i;
        return -1;
    }
    ReadQueue *reads(const Group &g) { return g.rq == kNone ? nullptr : &rqs[g.rq]; }
    uint32_t rq_alloc() {
        if (!rq_free.empty()) {
            const uint32_t i = rq_free.back();
            rq_free.pop_back();
            rqs[i].n = 0;
            return i;
        }
        rqs.emplace_back();
        rqs.back().n = 0;
        return (uint32_t)rqs.size() - 1;
    }
    void rq_release(Group &g) {
        if (g.rq != kNone) rq_free.push_back(g.rq);
        g.rq = kNone;
    }
    int reserve(size_t bytes);
    // device mode
    void to_device_record(const Group &g, hq_dgroup &d, hq_dread *r) const;
    int sync_to_device();
    int sync_from_device();
    int step_on_device(const hq_dstep_in &in, hq_step_output *out);
    int device_step_done(int rc, const hq_dstep_in &in, hq_step_output *out, uint64_t t0,
                         uint64_t t1);
    int load_group(Group &g, const hq_worker_group *src, const hq_member *m, bool fresh);
    int step(const hq_step_input *in, hq_step_output *out);
    Verdict handle(Group &g, const hq_event &e, uint64_t ei);
    Verdict read_index(Group &g, uint64_t from, uint64_t low, uint64_t high, uint64_t ei);
    void advance(Group &g);
    int run_pass();
    // reference state transitions (host bookkeeping of raft.go:949-1010)
    void reset(Group &g, uint64_t term);
    void become_follower(Group &g, uint64_t term, uint32_t reason);
    void become_leader(Group &g);
    void push_state(const Group &g, uint32_t reason) {
        states.push_back({g.cluster_id, g.term, g.state, reason});
    }
    void defer(uint64_t ei) { deferred.push_back(ei); }
};

// ------------------------------------------------------------------------------ state ------
// Validates and loads a group; `fresh` groups get a new member range, others reuse theirs when
// it is large enough.
int hq_worker::load_group(Group &g, const hq_worker_group *src, const hq_member *m, bool fresh) {
    const uint32_t n = src->n_members;
    if (n < 1 || !m) return fail(HQ_E_INVAL, "group has no members");
    if (n > 64) return fail(HQ_E_INVAL, "more than 64 members");
    if (src->state > HQ_STATE_LEADER) return fail(HQ_E_INVAL, "state must be follower, candidate or leader");
    int self = -1, n_voting = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (m[i].role > HQ_ROLE_WITNESS) return fail(HQ_E_INVAL, "unknown member role");
        for (uint32_t j = 0; j < i; ++j)
            if (m[j].node_id == m[i].node_id) return fail(HQ_E_INVAL, "duplicate member");
        if (m[i].role == HQ_ROLE_REMOTE && m[i].node_id == src->node_id) self = (int)i;
        n_voting += m[i].role != HQ_ROLE_OBSERVER;
    }
    if (self < 0) return fail(HQ_E_INVAL, "the node is not one of the group's remotes");
    if (n_voting > (int)n_max) return fail(HQ_E_INVAL, "more voting members than n_max");
    if (dstep && n > kDMembers)
        return fail(HQ_E_INVAL, "more than 16 members on the device path (HQ_WORKER_ON_DEVICE)");
    if (fresh || g.mem_cap < n) {
        g.mem = (uint32_t)pool.size();
        g.mem_cap = (uint8_t)n;
        pool.resize(pool.size() + n);
    }
    // pool order: the node itself, the other remotes, the witnesses (the voting slots of
    // hq_pack_commit), then the observers
    Member *dst = pool.data() + g.mem;
    int k = 0;
    auto put = [&](uint32_t i) {
        dst[k] = Member{m[i].node_id, m[i].match, (uint8_t)m[i].role, (uint8_t)(m[i].active != 0),
                        (uint8_t)i, {0, 0, 0, 0, 0}};
        ++k;
    };
    put((uint32_t)self);
    for (uint32_t role : {HQ_ROLE_REMOTE, HQ_ROLE_WITNESS, HQ_ROLE_OBSERVER})
        for (uint32_t i = 0; i < n; ++i)
            if (m[i].role == role && (int)i != self) put(i);
    g.cluster_id = src->cluster_id;
    g.node_id = src->node_id;
    g.term = src->term;
    g.committed = src->committed;
    g.last = src->last_index;
    g.term_start = src->term_start;
    g.state = (uint8_t)src->state;
    g.n_members = (uint8_t)n;
    g.n_voting = (uint8_t)n_voting;
    g.ord = 0;
    g.flags = 0;
    rq_release(g);
    // a candidate holds its own vote (campaign, raft.go:1093)
    g.granted = g.state == HQ_STATE_CANDIDATE ? 1 : 0;
    g.rejected = 0;
    return HQ_OK;
}

void hq_worker::reset(Group &g, uint64_t term) {   // raft.reset, raft.go:991-1010
    g.term = term;
    g.granted = g.rejected = 0;
    rq_release(g);
    Member *m = members(g);
    for (int i = 0; i < g.n_members; ++i) {          // resetRemotes/Observers/Witnesses
        m[i].match = m[i].node_id == g.node_id ? g.last : 0;
        m[i].active = 0;
    }
}

void hq_worker::become_follower(Group &g, uint64_t term, uint32_t reason) {
    g.state = HQ_STATE_FOLLOWER;                    // raft.go:949-957
    reset(g, term);
    push_state(g, reason);
}

void hq_worker::become_leader(Group &g) {
    g.state = HQ_STATE_LEADER;                      // raft.go:977-989
    reset(g, g.term);
    push_state(g, HQ_REASON_VOTE);
    // the no-op of p72: first entry of the new term; the node's own remote follows the log
    g.term_start = g.last + 1;
    g.last += 1;
    members(g)[0].match = g.last;
    if (g.n_voting == 1) g.set(kCommitDue);         // appendEntries: single-node tryCommit
}

// ------------------------------------------------------------------------------ events -----
Verdict hq_worker::read_index(Group &g, uint64_t from, uint64_t low, uint64_t high,
                              uint64_t ei) {
    if (g.state != HQ_STATE_LEADER) {
        if (g.has(kVoteDue)) return BARRIER;        // the vote may have made it leader
        defer(ei);                                  // forwarded / dropped (raft.go:1875, 1937)
        return CONSUMED;
    }
    // handleLeaderReadIndex (raft.go:1636-1669)
    const int fm = member_of(g, from);
    const uint8_t role = fm >= 0 ? members(g)[fm].role : 0xFF;
    if (role == HQ_ROLE_WITNESS) {
        dropped.push_back({g.cluster_id, low, high, from, HQ_DROP_WITNESS, 0});
        return CONSUMED;
    }
    if (g.has(kCommitDue)) return BARRIER;          // needs the committed index
    if (g.n_voting == 1) {                          // isSingleNodeQuorum: quorum() == 1
        ready.push_back({g.cluster_id, g.committed, low, high});
        if (from != g.node_id && role == HQ_ROLE_OBSERVER)
            resps.push_back({g.cluster_id, from, g.committed, low, high});
        return CONSUMED;
    }
    // hasCommittedEntryAtCurrentTerm (raft.go:1612-1621): term(committed) == r.term
    if (!(g.committed >= g.term_start && g.committed <= g.last)) {
        dropped.push_back({g.cluster_id, low, high, from, HQ_DROP_NOT_READY, 0});
        return CONSUMED;
    }
    // readIndex.addRequest (readindex.go:43-67)
    ReadQueue *q = reads(g);
    if (q) {
        for (uint32_t i = 0; i < q->n; ++i)
            if (q->r[i].low == low && q->r[i].high == high)
                return g.has(kRiDue) ? BARRIER : CONSUMED;   // already pending (or released)
        if (q->n && g.committed < q->r[q->n - 1].index) return FALLBACK;  // reference panics
        if (q->n >= kMaxReads) return g.has(kRiDue) ? BARRIER : FALLBACK;
    } else {
        g.rq = rq_alloc();
        q = &rqs[g.rq];
    }
    ReadStatus &s = q->r[q->n++];
    s.index = g.committed;
    s.from = from;
    s.low = low;
    s.high = high;
    s.confirmed = 0;
    std::fill(std::begin(s.ord), std::end(s.ord), kNoAck);
    return CONSUMED;
}

Verdict hq_worker::handle(Group &g, const hq_event &e, uint64_t ei) {
    switch (e.kind) {
    case HQ_EV_READ:
        return read_index(g, 0, e.hint, e.hint_high, ei);
    case HQ_EV_CHECK_QUORUM:
        if (g.state != HQ_STATE_LEADER) return g.has(kVoteDue) ? BARRIER : CONSUMED;
        if (g.has(kCqDue)) return BARRIER;
        g.set(kCqDue);
        return CONSUMED;
    case HQ_EV_ELECTION:
        if (g.pending()) return BARRIER;
        if (g.state == HQ_STATE_LEADER) return CONSUMED;   // leader ignores Election
        // campaign: becomeCandidate + the self vote (raft.go:959-975, 1082-1095)
        g.state = HQ_STATE_CANDIDATE;
        reset(g, g.term + 1);
        push_state(g, HQ_REASON_CAMPAIGN);
        g.granted = 1;
        g.set(kVoteDue);                            // isSingleNodeQuorum -> the vote kernel
        return CONSUMED;
    case HQ_EV_PROPOSE:
        if (g.pending() && (g.state != HQ_STATE_LEADER || g.has(kCqDue))) return BARRIER;
        if (g.state != HQ_STATE_LEADER) {
            defer(ei);                              // forwarded / dropped (raft.go:1845, 1932)
            return CONSUMED;
        }
        // appendEntries (raft.go:911-922)
        g.last += e.log_index;
        if (members(g)[0].match < g.last) members(g)[0].match = g.last;
        if (g.n_voting == 1) g.set(kCommitDue);
        return CONSUMED;
    case HQ_EV_MESSAGE:
        break;
    default:
        return FALLBACK;
    }
    const uint32_t type = e.type;
    if (type != HQ_MSG_REPLICATE_RESP && type != HQ_MSG_HEARTBEAT_RESP &&
        type != HQ_MSG_REQUEST_VOTE_RESP && type != HQ_MSG_READ_INDEX)
        return FALLBACK;
    const int mi = member_of(g, e.from);
    if (mi < 0 && is_response_type(type)) return CONSUMED;      // Peer.Handle drop
    if (e.term != 0 && e.term != g.term) {                      // onMessageTermNotMatched
        if (e.term < g.term) return CONSUMED;
        if (g.pending()) return BARRIER;            // decisions of the run come first
        become_follower(g, e.term, HQ_REASON_HIGHER_TERM);
    }
    if (g.state == HQ_STATE_LEADER) {
        switch (type) {
        case HQ_MSG_REPLICATE_RESP: {               // handleLeaderReplicateResp (:1671-1700)
            Member &rp = members(g)[mi];
            if (!e.reject && rp.match < e.log_index) {
                if (e.log_index > g.last) return FALLBACK;  // a follower can only ack what it got
                rp.match = e.log_index;             // remote.tryUpdate
                g.set(kCommitDue);                  // -> tryCommit
            }
            rp.active = 1;
            return CONSUMED;
        }
        case HQ_MSG_HEARTBEAT_RESP: {               // handleLeaderHeartbeatResp (:1702-1714)
            ReadQueue *q = e.hint != 0 ? reads(g) : nullptr;
            if (q) {                                // handleReadIndexLeaderConfirmation
                for (uint32_t i = 0; i < q->n; ++i) {
                    ReadStatus &r = q->r[i];
                    if (r.low != e.hint || r.high != e.hint_high) continue;
                    if (mi >= g.n_voting) return FALLBACK;   // an observer acking a ctx
                    if (g.ord >= kMaxOrdinal) return BARRIER;
                    if (!((r.confirmed >> mi) & 1) && r.ord[mi] == kNoAck) {
                        r.ord[mi] = ++g.ord;        // p.confirmed[from] = struct{}{}
                        g.set(kRiDue);
                    }
                    break;
                }
            }
            members(g)[mi].active = 1;
            return CONSUMED;
        }
        case HQ_MSG_READ_INDEX:
            return read_index(g, e.from, e.hint, e.hint_high, ei);
        default:
            return CONSUMED;                        // RequestVoteResp: no leader handler
        }
    }
    if (g.state == HQ_STATE_CANDIDATE) {
        if (type == HQ_MSG_REQUEST_VOTE_RESP) {     // handleCandidateRequestVoteResp
            if (mi >= g.n_voting) return CONSUMED;  // observer vote dropped (:1969-1972)
            if (!(((g.granted | g.rejected) >> mi) & 1)) {   // first response wins
                if (e.reject) g.rejected |= (uint8_t)(1u << mi);
                else g.granted |= (uint8_t)(1u << mi);
            }
            g.set(kVoteDue);
            return CONSUMED;
        }
        if (g.has(kVoteDue)) return BARRIER;        // may be leader by now
    }
    if (type == HQ_MSG_READ_INDEX) return read_index(g, e.from, e.hint, e.hint_high, ei);
    return CONSUMED;                                // no handler in this state
}

void hq_worker::advance(Group &g) {
    while (g.cursor < g.ev_end) {
        const uint64_t ei = g.cursor;
        if (g.has(kSuspended)) {
            defer(ei);
            ++g.cursor;
            continue;
        }
        const Verdict v = handle(g, in->events[ei], ei);
        if (v == BARRIER) return;
        if (v == FALLBACK) {
            g.set(kSuspended);
            fallback.push_back(g.cluster_id);
            continue;                               // this event and the rest are deferred
        }
        ++g.cursor;
    }
}

// ------------------------------------------------------------------------------ GPU pass ---
int hq_worker::reserve(size_t bytes) {
    if (bytes <= cap) return HQ_OK;
    size_t want = std::max(bytes, cap * 2);
    want = std::max<size_t>(want, 1 << 20);
    if (host) hq_free_pinned(ctx, host);
    if (dev) hq_free_dev(ctx, dev);
    host = dev = nullptr;
    cap = 0;
    int rc = hq(hq_alloc_pinned(ctx, want, &host), "hq_alloc_pinned");
    if (!rc) rc = hq(hq_malloc_dev(ctx, want, &dev), "hq_malloc_dev");
    if (rc) return rc;
    cap = want;
    return HQ_OK;
}

namespace {
// Carves one staging region into aligned arrays; host and device share the offsets.
struct Layout {
    size_t off = 0;
    size_t take(size_t bytes) {
        const size_t o = off;
        off = align_up(off + std::max<size_t>(bytes, 1), 256);
        return o;
    }
};
}  // namespace

int hq_worker::run_pass() {
    const uint64_t Gc = l_commit.size(), Gr = l_ri.size(), Gv = l_vote.size(), Gq = l_cq.size();
    const uint32_t N = n_max;
    uint32_t K = 1;
    for (uint32_t gi : l_ri) K = std::max<uint32_t>(K, rqs[groups[gi].rq].n);
    const uint64_t sc = align_up(std::max<uint64_t>(Gc, 1), 2);   // even stride: 16-B loads
    // inputs
    Layout L;
    const size_t c_match = L.take(8 * N * sc), c_nv = L.take(Gc), c_cin = L.take(8 * Gc),
                 c_last = L.take(8 * Gc), c_ts = L.take(8 * Gc);
    const size_t r_ord = L.take(2 * (size_t)K * N * Gr), r_idx = L.take(8 * (size_t)K * Gr),
                 r_np = L.take(Gr), r_nv = L.take(Gr);
    const size_t v_gr = L.take(Gv), v_rj = L.take(Gv), v_nv = L.take(Gv);
    const size_t q_act = L.take(Gq), q_nv = L.take(Gq);
    const size_t in_bytes = L.off;
    // outputs
    const size_t c_out = L.take(8 * Gc), c_chg = L.take(8 * ((Gc + 63) / 64)),
                 c_fb = L.take(8 * ((Gc + 63) / 64));
    // (the released indexes are not read back: the compact release, each released entry's index
    // taken from its closing ctx below)
    const size_t r_cnt = L.take(Gr), r_be = L.take(Gr), r_fb = L.take(8 * ((Gr + 63) / 64));
    const size_t v_out = L.take(8 * ((Gv + 31) / 32)), v_fb = L.take(8 * ((Gv + 63) / 64));
    const size_t q_hq = L.take(8 * ((Gq + 63) / 64)), q_fb = L.take(8 * ((Gq + 63) / 64));
    const size_t total = L.off;
    int rc = reserve(total);
    if (rc) return rc;
    auto H = [&](size_t o) { return static_cast<uint8_t *>(host) + o; };
    auto D = [&](size_t o) { return static_cast<uint8_t *>(dev) + o; };

    // pack (the SoA layout of DESIGN.md §2): voting slot s of a group is pool entry s
    const uint64_t t0 = now_ns();
    {
        uint64_t *match = reinterpret_cast<uint64_t *>(H(c_match));
        uint8_t *nv = H(c_nv);
        uint64_t *cin = reinterpret_cast<uint64_t *>(H(c_cin));
        uint64_t *last = reinterpret_cast<uint64_t *>(H(c_last));
        uint64_t *ts = reinterpret_cast<uint64_t *>(H(c_ts));
        for (uint64_t j = 0; j < Gc; ++j) {
            const Group &g = groups[l_commit[j]];
            const Member *m = pool.data() + g.mem;
            uint32_t s = 0;
            for (; s < g.n_voting; ++s) match[s * sc + j] = m[s].match;
            for (; s < N; ++s) match[s * sc + j] = 0;
            nv[j] = g.n_voting;
            cin[j] = g.committed;
            last[j] = g.last;
            ts[j] = g.term_start;
        }
        uint16_t *ord = reinterpret_cast<uint16_t *>(H(r_ord));
        uint64_t *idx = reinterpret_cast<uint64_t *>(H(r_idx));
        uint8_t *np = H(r_np), *rnv = H(r_nv);
        for (uint64_t j = 0; j < Gr; ++j) {
            const Group &g = groups[l_ri[j]];
            const ReadQueue &q = rqs[g.rq];
            np[j] = (uint8_t)q.n;
            rnv[j] = g.n_voting;
            for (uint32_t k = 0; k < K; ++k) {
                const ReadStatus *r = k < q.n ? &q.r[k] : nullptr;
                idx[(uint64_t)k * Gr + j] = r ? r->index : 0;
                for (uint32_t s = 0; s < N; ++s)
                    ord[((uint64_t)k * N + s) * Gr + j] =
                        !r ? kNoAck : ((r->confirmed >> s) & 1) ? 0 : r->ord[s];
            }
        }
        uint8_t *gr = H(v_gr), *rj = H(v_rj), *vnv = H(v_nv);
        for (uint64_t j = 0; j < Gv; ++j) {
            const Group &g = groups[l_vote[j]];
            gr[j] = g.granted;
            rj[j] = g.rejected;
            vnv[j] = g.n_voting;
        }
        uint8_t *act = H(q_act), *qnv = H(q_nv);
        for (uint64_t j = 0; j < Gq; ++j) {
            const Group &g = groups[l_cq[j]];
            const Member *m = pool.data() + g.mem;
            uint8_t a = 0;
            for (uint32_t s = 0; s < g.n_voting; ++s) a |= (uint8_t)(m[s].active << s);
            act[j] = a;
            qnv[j] = g.n_voting;
        }
    }

    // one H2D, the decisions, one D2H, one sync
    const uint64_t t1 = now_ns();
    t_pack += t1 - t0;
    rc = hq(hq_memcpy_async(ctx, dev, host, in_bytes, 0), "hq_memcpy_async(H2D)");
    if (!rc && Gc) {
        hq_commit_args a{};
        a.G = Gc;
        a.n_max = N;
        a.form = HQ_FORM_TERM_START;
        a.match_stride = sc;
        a.match = reinterpret_cast<const uint64_t *>(D(c_match));
        a.n_voting = D(c_nv);
        a.committed_in = reinterpret_cast<const uint64_t *>(D(c_cin));
        a.committed_out = reinterpret_cast<uint64_t *>(D(c_out));
        a.last_index = reinterpret_cast<const uint64_t *>(D(c_last));
        a.term_start = reinterpret_cast<const uint64_t *>(D(c_ts));
        a.changed = reinterpret_cast<uint64_t *>(D(c_chg));
        a.fallback = reinterpret_cast<uint64_t *>(D(c_fb));
        rc = hq(hq_commit_dev(ctx, &a), "hq_commit_dev");
    }
    if (!rc && Gr)
        rc = hq(hq_readindex_multi_dev(ctx, Gr, K, N, reinterpret_cast<const uint16_t *>(D(r_ord)),
                                       reinterpret_cast<const uint64_t *>(D(r_idx)), D(r_np),
                                       D(r_nv), 0, nullptr, D(r_cnt), D(r_be),
                                       reinterpret_cast<uint64_t *>(D(r_fb))),
                "hq_readindex_multi_dev");
    if (!rc && Gv)
        rc = hq(hq_vote_dev(ctx, Gv, D(v_gr), D(v_rj), D(v_nv), 0,
                            reinterpret_cast<uint64_t *>(D(v_out)),
                            reinterpret_cast<uint64_t *>(D(v_fb))),
                "hq_vote_dev");
    if (!rc && Gq)
        rc = hq(hq_check_quorum_dev(ctx, Gq, D(q_act), D(q_nv), 0, 0,
                                    reinterpret_cast<uint64_t *>(D(q_hq)),
                                    reinterpret_cast<uint64_t *>(D(q_fb))),
                "hq_check_quorum_dev");
    if (!rc) rc = hq(hq_memcpy_async(ctx, H(in_bytes), D(in_bytes), total - in_bytes, 1),
                     "hq_memcpy_async(D2H)");
    if (!rc) rc = hq(hq_sync(ctx), "hq_sync");
    if (rc) return rc;
    decisions += Gc + Gr + Gv + Gq;
    const uint64_t t2 = now_ns();
    t_device += t2 - t1;

    // every group handed to a kernel satisfies its contract; a fallback bit is an internal error
    auto any = [&](size_t o, uint64_t G) {
        const uint64_t *w = reinterpret_cast<const uint64_t *>(H(o));
        for (uint64_t i = 0; i < (G + 63) / 64; ++i)
            if (w[i]) return true;
        return false;
    };
    if (any(c_fb, Gc) || any(r_fb, Gr) || any(v_fb, Gv) || any(q_fb, Gq))
        return fail(HQ_E_STATE, "a kernel refused a packed group (worker contract bug)");

    // apply, per group in the reference's order: commit, ReadIndex release, vote, CheckQuorum
    const uint64_t *cout = reinterpret_cast<const uint64_t *>(H(c_out));
    for (uint64_t j = 0; j < Gc; ++j) {
        Group &g = groups[l_commit[j]];
        g.committed = cout[j];                      // commitTo (logentry.go:323-332)
        g.clear(kCommitDue);
    }
    const uint8_t *cnt = H(r_cnt), *be = H(r_be);
    for (uint64_t j = 0; j < Gr; ++j) {
        Group &g = groups[l_ri[j]];
        ReadQueue &q = rqs[g.rq];
        const uint32_t c = cnt[j];
        for (uint32_t i = 0; i < c; ++i) {
            uint32_t k = i;                         // the ctx whose confirm() released entry i
            while (k < c && !((be[j] >> k) & 1)) ++k;
            if (k >= c) return fail(HQ_E_STATE, "ReadIndex release without a closing ctx");
            const ReadStatus &s = q.r[i];
            // confirm() rewrites every released entry's index to the closing ctx's
            // (readindex.go:96-104): what the kernel's released_index column would hold
            const uint64_t index = q.r[k].index;
            if (s.from == 0 || s.from == g.node_id)
                ready.push_back({g.cluster_id, index, s.low, s.high});
            else
                resps.push_back({g.cluster_id, s.from, index, q.r[k].low, q.r[k].high});
        }
        std::copy(q.r + c, q.r + q.n, q.r);         // r.queue = r.queue[done:]
        q.n -= c;
        for (uint32_t i = 0; i < q.n; ++i) {        // carry the run's confirmations over
            ReadStatus &r = q.r[i];
            for (uint32_t s = 0; s < HQ_MAX_VOTERS; ++s) {
                if (r.ord[s] != kNoAck) r.confirmed |= (uint8_t)(1u << s);
                r.ord[s] = kNoAck;
            }
        }
        if (q.n == 0) rq_release(g);
        g.ord = 0;
        g.clear(kRiDue);
    }
    const uint64_t *outc = reinterpret_cast<const uint64_t *>(H(v_out));
    for (uint64_t j = 0; j < Gv; ++j) {
        Group &g = groups[l_vote[j]];
        g.clear(kVoteDue);
        const uint32_t o = (uint32_t)((outc[j >> 5] >> (2 * (j & 31))) & 3);
        if (o == HQ_OUTCOME_LEADER) become_leader(g);
        else if (o == HQ_OUTCOME_FOLLOWER) become_follower(g, g.term, HQ_REASON_VOTE);
    }
    const uint64_t *hqb = reinterpret_cast<const uint64_t *>(H(q_hq));
    for (uint64_t j = 0; j < Gq; ++j) {
        Group &g = groups[l_cq[j]];
        g.clear(kCqDue);
        Member *m = members(g);
        for (uint32_t s = 0; s < g.n_voting; ++s) m[s].active = 0;   // setNotActive
        if (!((hqb[j >> 6] >> (j & 63)) & 1)) become_follower(g, g.term, HQ_REASON_CHECK_QUORUM);
    }
    t_apply += now_ns() - t2;
    return HQ_OK;
}

// ------------------------------------------------------------------------------ step -------
int hq_worker::step(const hq_step_input *inp, hq_step_output *out) {
    const uint64_t t0 = now_ns();
    uint64_t t_pass = 0;
    in = inp;
    commits.clear();
    ready.clear();
    resps.clear();
    states.clear();
    dropped.clear();
    deferred.clear();
    fallback.clear();
    decisions = 0;
    t_pack = t_device = t_apply = 0;
    uint64_t passes = 0;

    // the groups with events, each with its slice of the event array (node.mq per node)
    work.clear();
    touched.clear();
    int rc = HQ_OK;
    for (uint64_t i = 0; i < in->n_groups; ++i) {
        const uint32_t gi = in->groups[i];
        const uint64_t b = in->offsets[i], e = in->offsets[i + 1];
        if (gi >= groups.size()) { rc = fail(HQ_E_INVAL, "hq_worker_step: unknown group handle"); break; }
        if (e < b) { rc = fail(HQ_E_INVAL, "hq_worker_step: offsets decrease"); break; }
        Group &g = groups[gi];
        if (g.has(kTouched)) { rc = fail(HQ_E_INVAL, "hq_worker_step: a group is listed twice"); break; }
        g.set(kTouched);
        g.committed0 = g.committed;
        touched.push_back(gi);
        if (b == e) continue;
        g.cursor = b;
        g.ev_end = e;
        g.set(kInWork);
        work.push_back(gi);
    }

    while (!rc && !work.empty()) {
        l_commit.clear();
        l_ri.clear();
        l_vote.clear();
        l_cq.clear();
        for (uint32_t gi : work) {
            Group &g = groups[gi];
            g.clear(kInWork);
            advance(g);
            if (g.has(kCommitDue)) l_commit.push_back(gi);
            if (g.has(kRiDue)) l_ri.push_back(gi);
            if (g.has(kVoteDue)) l_vote.push_back(gi);
            if (g.has(kCqDue)) l_cq.push_back(gi);
        }
        if (l_commit.empty() && l_ri.empty() && l_vote.empty() && l_cq.empty()) break;
        const uint64_t tp = now_ns();
        rc = run_pass();
        t_pass += now_ns() - tp;
        if (rc) break;
        ++passes;
        next_work.clear();
        for (const auto *l : {&l_commit, &l_ri, &l_vote, &l_cq})
            for (uint32_t gi : *l) {
                Group &g = groups[gi];
                if (g.has(kInWork)) continue;
                if (g.cursor < g.ev_end || g.pending()) {
                    g.set(kInWork);
                    next_work.push_back(gi);
                }
            }
        work.swap(next_work);
    }
    for (uint32_t gi : touched) {
        Group &g = groups[gi];
        g.clear(kTouched | kInWork);
        if (g.committed != g.committed0) commits.push_back({g.cluster_id, g.committed});
    }
    if (rc) return rc;

    out->commits = commits.data();
    out->n_commits = commits.size();
    out->ready = ready.data();
    out->n_ready = ready.size();
    out->read_resps = resps.data();
    out->n_read_resps = resps.size();
    out->state_changes = states.data();
    out->n_state_changes = states.size();
    out->dropped_reads = dropped.data();
    out->n_dropped_reads = dropped.size();
    out->deferred = deferred.data();
    out->n_deferred = deferred.size();
    out->fallback_groups = fallback.data();
    out->n_fallback_groups = fallback.size();
    out->gpu_passes = passes;
    out->decisions = decisions;
    out->pass_ns = t_pass;
    out->pack_ns = t_pack;
    out->device_ns = t_device;
    out->apply_ns = t_apply;
    out->handle_ns = now_ns() - t0 - t_pass;
    return HQ_OK;
}

// ------------------------------------------------------------------------------ device mode ---
void hq_worker::to_device_record(const Group &g, hq_dgroup &d, hq_dread *r) const {
    d = hq_dgroup{};
    d.cluster_id = g.cluster_id;
    d.node_id = g.node_id;
    d.term = g.term;
    d.committed = g.committed;
    d.last = g.last;
    d.term_start = g.term_start;
    d.mem = g.mem;
    d.n_members = g.n_members;
    d.n_voting = g.n_voting;
    d.state = g.state;
    d.granted = g.granted;
    d.rejected = g.rejected;
    d.flags = g.has(kSuspended) ? kDSuspended : 0;
    const ReadQueue *q = g.rq == kNone ? nullptr : &rqs[g.rq];
    d.n_reads = q ? (uint8_t)q->n : 0;
    for (uint32_t k = 0; k < kDReads; ++k) {
        r[k] = hq_dread{};
        if (q && k < q->n) {
            const ReadStatus &s = q->r[k];
            r[k].index = s.index;
            r[k].from = s.from;
            r[k].low = s.low;
            r[k].high = s.high;
            uint8_t c = s.confirmed;
            for (uint32_t v = 0; v < HQ_MAX_VOTERS; ++v)
                if (s.ord[v] != kNoAck) c |= (uint8_t)(1u << v);
            r[k].confirmed = c;
        }
    }
}

// new groups (and their members) in one upload; groups changed by set_group one by one
int hq_worker::sync_to_device() {
    const uint64_t G = groups.size();
    if (dev_groups < G || dev_members < pool.size()) {
        const uint64_t ng = G - dev_groups, nm = pool.size() - dev_members;
        std::vector<hq_dgroup> dg(ng);
        std::vector<hq_dread> dr(ng * kDReads);
        for (uint64_t i = 0; i < ng; ++i)
            to_device_record(groups[dev_groups + i], dg[i], dr.data() + i * kDReads);
        std::vector<hq_dmember> dm(nm);
        for (uint64_t i = 0; i < nm; ++i) {
            const Member &m = pool[dev_members + i];
            dm[i] = hq_dmember{m.node_id, m.match, m.role, m.active, m.order, {0, 0, 0, 0, 0}};
        }
        int rc = hq(hq_dstep_put(dstep, dev_groups, ng, dg.data(), dr.data(), dev_members, nm,
                                 dm.data()), "hq_dstep_put");
        if (rc) return rc;
        dev_groups = G;
        dev_members = pool.size();
    }
    for (uint32_t h : dirty) {
        const Group &g = groups[h];
        hq_dgroup dg;
        hq_dread dr[kDReads];
        to_device_record(g, dg, dr);
        std::vector<hq_dmember> dm(g.n_members);
        for (uint32_t i = 0; i < g.n_members; ++i) {
            const Member &m = pool[g.mem + i];
            dm[i] = hq_dmember{m.node_id, m.match, m.role, m.active, m.order, {0, 0, 0, 0, 0}};
        }
        int rc = hq(hq_dstep_put(dstep, h, 1, &dg, dr, g.mem, g.n_members, dm.data()),
                    "hq_dstep_put");
        if (rc) return rc;
    }
    dirty.clear();
    return HQ_OK;
}

// the whole device state back into the host records
int hq_worker::sync_from_device() {
    if (!host_stale) return HQ_OK;
    const uint64_t G = dev_groups, M = dev_members;
    std::vector<hq_dgroup> dg(G);
    std::vector<hq_dread> dr(G * kDReads);
    std::vector<hq_dmember> dm(M);
    int rc = hq(hq_dstep_get(dstep, G, dg.data(), dr.data(), M, dm.data()), "hq_dstep_get");
    if (rc) return rc;
    for (uint64_t h = 0; h < G; ++h) {
        Group &g = groups[h];
        const hq_dgroup &d = dg[h];
        g.term = d.term;
        g.committed = d.committed;
        g.last = d.last;
        g.term_start = d.term_start;
        g.state = d.state;
        g.granted = d.granted;
        g.rejected = d.rejected;
        if (d.flags & kDSuspended) g.set(kSuspended);
        else g.clear(kSuspended);
        if (d.n_reads == 0) {
            rq_release(g);
        } else {
            if (g.rq == kNone) g.rq = rq_alloc();
            ReadQueue &q = rqs[g.rq];
            q.n = d.n_reads;
            for (uint32_t k = 0; k < q.n; ++k) {
                const hq_dread &r = dr[h * kDReads + k];
                ReadStatus &s = q.r[k];
                s.index = r.index;
                s.from = r.from;
                s.low = r.low;
                s.high = r.high;
                s.confirmed = r.confirmed;
                std::fill(std::begin(s.ord), std::end(s.ord), kNoAck);
            }
        }
    }
    for (uint64_t i = 0; i < M; ++i) {
        pool[i].match = dm[i].match;
        pool[i].active = dm[i].active;
    }
    host_stale = false;
    return HQ_OK;
}

int hq_worker::step_on_device(const hq_dstep_in &inp, hq_step_output *out) {
    const uint64_t t0 = now_ns();
    // the per-group input checks (handles, offsets, a group listed twice) run in the engine's
    // first kernel, which writes each group's new state in place; a failed step takes that state
    // back (k_step_restore). The device copy is the authoritative one from here on, whatever the
    // outcome: the host copy is reloaded from it before the host reads a group.
    int rc = sync_to_device();
    if (rc) return rc;
    const uint64_t t1 = now_ns();
    host_stale = true;
    rc = hq_dstep_run(dstep, &inp, &dout);
    return device_step_done(rc, inp, out, t0, t1);
}

// the outputs of a device step (hq_dstep_run or hq_dstep_run_jobs) in the worker's terms
int hq_worker::device_step_done(int rc, const hq_dstep_in &inp, hq_step_output *out, uint64_t t0,
                                uint64_t t1) {
    if (rc == HQ_E_INVAL && dout.input_error) {
        const uint32_t e = dout.input_error;
        if (e & (16 | 32))        // (hq_dstep.hip kErrScan / kErrTicket: not the input's fault)
            return fail(HQ_E_STATE, "hq_worker_step: the device step's scan of the ReadyToRead "
                                    "places or its launch order failed (internal); no group "
                                    "state was written");
        return fail(HQ_E_INVAL, e & 1 ? "hq_worker_step: unknown group handle"
                                : e & 8 ? "hq_worker_step: a group is listed twice"
                                : e & 2 ? "hq_worker_step: offsets decrease"
                                        : "hq_worker_step_stream: boffsets decrease or out of range, sizes "
                                          "not summing to the totals, or a group's bytes not used up by its "
                                          "events (malformed event stream)");
    }
    rc = hq(rc, "hq_dstep_run");
    if (rc) return rc;
    const uint64_t t2 = now_ns();
    out->commits = dout.commits;
    out->n_commits = dout.n_commits;
    out->committed_column = dout.commit_col;
    out->committed_advance = dout.commit_adv;
    out->ready = dout.ready;
    out->ready_compact = dout.ready_compact;
    out->n_ready = dout.n_ready;
    out->read_resps = dout.resps;
    out->n_read_resps = dout.n_resps;
    out->state_changes = dout.states;
    out->n_state_changes = dout.n_states;
    out->dropped_reads = dout.dropped;
    out->n_dropped_reads = dout.n_dropped;
    out->deferred = dout.deferred;
    out->n_deferred = dout.n_deferred;
    out->fallback_groups = dout.fallback;
    out->n_fallback_groups = dout.n_fallback;
    out->gpu_passes = inp.n ? 1 : 0;
    out->decisions = dout.decisions;
    // (device path: pack = the host's submit, device = the GPU's time between its events, apply
    // = the outputs mapped after the wait; pass less the three is the wait the GPU does not
    // explain: queueing ahead of the step's work and the waiting thread's wake-up)
    out->ready_slots = dout.ready_slots;
    out->ready_slot_counts = dout.slot_counts;
    out->n_ready_tiles = dout.n_tiles;
    out->n_ready_slotted = dout.n_slotted;
    // (device path: pack = the host's submit, device = the thread's wait for the device, apply =
    // the outputs mapped after the wait, gpu = the GPU's time between the step's events)
    out->pass_ns = t2 - t1;
    out->pack_ns = dout.submit_ns;
    out->device_ns = dout.wait.t_end_ns > dout.wait.t_begin_ns
                         ? dout.wait.t_end_ns - dout.wait.t_begin_ns : 0;
    out->apply_ns = dout.d2h_ns;
    out->handle_ns = t1 - t0;
    out->gpu_ns = dout.gpu_ns;
    out->gpu_jobs = dout.gpu_jobs;
    out->wait_sleeps = (uint32_t)dout.wait.sleeps;
    out->wait_poll_ns = dout.wait.poll_ns;
    out->wait_sleep_ns = dout.wait.sleep_ns;
    out->wait_end_ns = dout.wait.t_end_ns;
    out->device_end_ticks = dout.wait.device_end_ticks;
    out->device_start_ticks = dout.wait.device_start_ticks;
    return HQ_OK;
}

// ------------------------------------------------------------------------------ C-ABI ------
extern "C" {

int hq_worker_open(int device, uint32_t n_max, hq_worker **out) {
    return hq_worker_open_ex(device, n_max, 0, out);
}

int hq_worker_open_ex(int device, uint32_t n_max, uint32_t flags, hq_worker **out) {
    if (!out) return HQ_E_INVAL;
    if (flags & ~(HQ_WORKER_ON_DEVICE | HQ_WORKER_COMMIT_COLUMN | HQ_WORKER_COMMIT_ADVANCE |
                  HQ_WORKER_READY_COMPACT | HQ_WORKER_READY_SLOTS))
        return HQ_E_INVAL;
    if ((flags & (HQ_WORKER_READY_COMPACT | HQ_WORKER_READY_SLOTS)) && !(flags & HQ_WORKER_ON_DEVICE))
        return HQ_E_INVAL;            // (the compact records are the device step's form)
    if ((flags & HQ_WORKER_READY_SLOTS) && !(flags & HQ_WORKER_COMMIT_ADVANCE))
        return HQ_E_INVAL;            // (the slots follow the advance column in the region)
    *out = nullptr;
    if (n_max < 1 || n_max > HQ_MAX_VOTERS) return HQ_E_INVAL;
    hq_worker *w = new (std::nothrow) hq_worker();
    if (!w) return HQ_E_NOMEM;
    int rc = hq_open(device, 0, &w->ctx);
    if (rc) {
        delete w;
        return rc;   // message: hq_last_error(NULL)
    }
    w->n_max = n_max;
    w->device = device;
    if (flags & HQ_WORKER_ON_DEVICE) {
        rc = hq_dstep_open(w->ctx, &w->dstep,
                           ((flags & HQ_WORKER_COMMIT_COLUMN) ? 1u : 0u) |
                               ((flags & HQ_WORKER_COMMIT_ADVANCE) ? 2u : 0u) |
                               ((flags & HQ_WORKER_READY_COMPACT) ? 4u : 0u) |
                               ((flags & HQ_WORKER_READY_SLOTS) ? 8u : 0u));
        if (rc) {
            hq_close(w->ctx);
            delete w;
            return rc;
        }
    }
    *out = w;
    return HQ_OK;
}

void hq_worker_close(hq_worker *w) {
    if (!w) return;
    if (w->dstep) hq_dstep_close(w->dstep);
    if (w->ctx) {
        hq_sync(w->ctx);
        if (w->host) hq_free_pinned(w->ctx, w->host);
        if (w->dev) hq_free_dev(w->ctx, w->dev);
        hq_close(w->ctx);
    }
    delete w;
}

const char *hq_worker_last_error(const hq_worker *w) {
    return w ? w->err.c_str() : hq_last_error(nullptr);
}

int hq_worker_add_group(hq_worker *w, const hq_worker_group *g, const hq_member *members,
                        uint32_t *handle) {
    if (!w) return HQ_E_INVAL;
    if (!g) return w->fail(HQ_E_INVAL, "hq_worker_add_group: group is NULL");
    if (w->index.count(g->cluster_id)) return w->fail(HQ_E_INVAL, "hq_worker_add_group: cluster exists");
    if (w->host_stale) {                            // new pool entries append to a fresh mirror
        int rc = w->sync_from_device();
        if (rc) return rc;
    }
    if (w->groups.size() >= UINT32_MAX) return w->fail(HQ_E_NOMEM, "hq_worker_add_group: too many groups");
    Group n{};
    n.rq = kNone;
    const size_t pool0 = w->pool.size();
    int rc = w->load_group(n, g, members, true);
    if (rc) {
        w->pool.resize(pool0);
        return rc;
    }
    const uint32_t h = (uint32_t)w->groups.size();
    w->index.emplace(g->cluster_id, h);
    w->groups.push_back(n);
    if (handle) *handle = h;
    return HQ_OK;
}

int hq_worker_add_groups(hq_worker *w, const hq_worker_group *groups, uint64_t count,
                         const hq_member *members) {
    if (!w) return HQ_E_INVAL;
    if (count && (!groups || !members))
        return w->fail(HQ_E_INVAL, "hq_worker_add_groups: NULL argument");
    w->groups.reserve(w->groups.size() + count);
    w->index.reserve(w->groups.size() + count);
    uint64_t off = 0, nm = 0;
    for (uint64_t i = 0; i < count; ++i) nm += groups[i].n_members;
    w->pool.reserve(w->pool.size() + nm);
    for (uint64_t i = 0; i < count; ++i) {
        int rc = hq_worker_add_group(w, groups + i, members + off, nullptr);
        if (rc) return rc;
        off += groups[i].n_members;
    }
    return HQ_OK;
}

int hq_worker_group_count(hq_worker *w, uint64_t *n) {
    if (!w || !n) return HQ_E_INVAL;
    *n = w->groups.size();
    return HQ_OK;
}

int hq_worker_find(hq_worker *w, uint64_t cluster_id, uint32_t *handle) {
    if (!w) return HQ_E_INVAL;
    auto it = w->index.find(cluster_id);
    if (it == w->index.end()) return w->fail(HQ_E_INVAL, "hq_worker_find: unknown cluster");
    if (handle) *handle = it->second;
    return HQ_OK;
}

int hq_worker_set_group(hq_worker *w, const hq_worker_group *g, const hq_member *members) {
    if (!w) return HQ_E_INVAL;
    if (!g) return w->fail(HQ_E_INVAL, "hq_worker_set_group: group is NULL");
    auto it = w->index.find(g->cluster_id);
    if (it == w->index.end()) return w->fail(HQ_E_INVAL, "hq_worker_set_group: unknown cluster");
    int rc = w->sync_from_device();
    if (rc) return rc;
    Group n = w->groups[it->second];
    rc = w->load_group(n, g, members, false);
    if (rc) return rc;
    w->groups[it->second] = n;
    if (w->dstep && it->second < w->dev_groups) w->dirty.push_back(it->second);
    return HQ_OK;
}

int hq_worker_get_group(hq_worker *w, uint64_t cluster_id, hq_worker_group *out,
                        hq_member *members, uint32_t cap, hq_read_status *reads,
                        uint32_t reads_cap) {
    if (!w) return HQ_E_INVAL;
    auto it = w->index.find(cluster_id);
    if (it == w->index.end()) return w->fail(HQ_E_INVAL, "hq_worker_get_group: unknown cluster");
    int rc = w->sync_from_device();
    if (rc) return rc;
    const Group &g = w->groups[it->second];
    const ReadQueue *q = g.rq == kNone ? nullptr : &w->rqs[g.rq];
    if (out) {
        out->cluster_id = g.cluster_id;
        out->node_id = g.node_id;
        out->term = g.term;
        out->committed = g.committed;
        out->last_index = g.last;
        out->term_start = g.term_start;
        out->state = g.state;
        out->n_members = g.n_members;
        out->n_pending_reads = q ? q->n : 0;
        out->suspended = g.has(kSuspended);
    }
    if (members) {                                  // back in the caller's order
        const Member *m = w->pool.data() + g.mem;
        for (uint32_t i = 0; i < g.n_members; ++i)
            if (m[i].order < cap)
                members[m[i].order] = hq_member{m[i].node_id, m[i].match, m[i].role, m[i].active};
    }
    if (reads && q)
        for (uint32_t i = 0; i < reads_cap && i < q->n; ++i) {
            const ReadStatus &r = q->r[i];
            uint32_t n = 0;
            for (uint32_t s = 0; s < HQ_MAX_VOTERS; ++s)
                n += ((r.confirmed >> s) & 1) || r.ord[s] != kNoAck;
            reads[i] = {r.index, r.from, r.low, r.high, n, 0};
        }
    return HQ_OK;
}

int hq_worker_set_wait(hq_worker *w, uint32_t mode, uint32_t poll_us, uint32_t sleep_us) {
    if (!w) return HQ_E_INVAL;
    if (!w->dstep) return w->fail(HQ_E_INVAL, "hq_worker_set_wait: not a device worker");
    const int rc = hq_dstep_set_wait(w->dstep, mode, poll_us, sleep_us);
    if (rc == HQ_E_INVAL) return w->fail(rc, "hq_worker_set_wait: unknown mode (or sleep_us 0)");
    return w->hq(rc, "hq_worker_set_wait");
}

int hq_worker_step(hq_worker *w, const hq_step_input *in, hq_step_output *out) {
    if (!w) return HQ_E_INVAL;
    if (!in || !out) return w->fail(HQ_E_INVAL, "hq_worker_step: NULL argument");
    if (in->n_groups && (!in->groups || !in->offsets))
        return w->fail(HQ_E_INVAL, "hq_worker_step: NULL groups/offsets");
    if (in->n_groups && in->offsets[in->n_groups] > in->offsets[0] && !in->events)
        return w->fail(HQ_E_INVAL, "hq_worker_step: NULL events");
    std::memset(out, 0, sizeof *out);
    if (w->dstep)
        return w->step_on_device(hq_dstep_in{in->n_groups, in->groups, in->offsets, in->events,
                                             nullptr, nullptr}, out);
    return w->step(in, out);
}

}  // extern "C"

// hq_worker_step_jobs (hq_jobs.cpp): jobs that are all sized event streams for distinct device
// workers on one GPU are stepped through shared launches (hq_dstep_run_jobs: one pass A per
// input chunk, one layout, one k_step_lite and one pass B for all of them, one wait) instead of
// one launch sequence per worker on its own thread. Returns kJobsNotFused, having done nothing,
// for any other set of jobs; else the first job's failure (each job's in its rc).
int hq_worker_step_jobs_fused(hq_step_job *jobs, uint32_t count) {
    if (count < 2 || count > kDStepMaxJobs) return kJobsNotFused;
    if (const char *v = std::getenv("HQ_STEP_JOBS_FUSED"))
        if (std::atoi(v) == 0) return kJobsNotFused;
    int device = -1;
    for (uint32_t j = 0; j < count; ++j) {
        const hq_step_job &b = jobs[j];
        const hq_step_stream *in = b.stream;
        if (!b.worker || !b.worker->dstep || !b.out || b.rows || !in || !(in->sizes || in->sizes16) ||
            (in->n_bytes && !in->bytes) || in->n_groups == 0)
            return kJobsNotFused;
        if (device >= 0 && b.worker->device != device) return kJobsNotFused;
        device = b.worker->device;
    }
    static const uint8_t none = 0;
    hq_dstep *ds[kDStepMaxJobs];
    hq_dstep_in ins[kDStepMaxJobs];
    hq_dstep_out outs[kDStepMaxJobs];
    int rcs[kDStepMaxJobs];
    uint32_t idx[kDStepMaxJobs], nl = 0;
    const uint64_t t0 = now_ns();
    for (uint32_t j = 0; j < count; ++j) {
        hq_worker *w = jobs[j].worker;
        const hq_step_stream *in = jobs[j].stream;
        std::memset(jobs[j].out, 0, sizeof *jobs[j].out);
        jobs[j].rc = w->sync_to_device();
        if (jobs[j].rc) continue;
        w->host_stale = true;
        hq_dstep_in d{in->n_groups, in->groups, nullptr, nullptr, nullptr,
                      in->bytes ? in->bytes : &none};
        d.sizes = in->sizes16 ? nullptr : in->sizes;
        d.sizes16 = in->sizes16;
        d.n_events = in->n_events;
        d.n_bytes = in->n_bytes;
        ds[nl] = w->dstep;
        ins[nl] = d;
        idx[nl++] = j;
    }
    const uint64_t t1 = now_ns();
    if (nl) (void)hq_dstep_run_jobs(ds, ins, outs, rcs, nl);
    int first = HQ_OK;
    for (uint32_t x = 0; x < nl; ++x) {
        hq_step_job &b = jobs[idx[x]];
        b.worker->dout = outs[x];
        b.rc = b.worker->device_step_done(rcs[x], ins[x], b.out, t0, t1);
    }
    for (uint32_t j = 0; j < count; ++j)
        if (jobs[j].rc && !first) first = jobs[j].rc;
    return first;
}

extern "C" {

int hq_worker_step_stream(hq_worker *w, const hq_step_stream *in, hq_step_output *out) {
    if (!w) return HQ_E_INVAL;
    if (!in || !out) return w->fail(HQ_E_INVAL, "hq_worker_step_stream: NULL argument");
    if (in->sizes || in->sizes16 || (in->n_groups && !in->offsets && !in->boffsets)) {
        // the sized form: the device engine scans the sizes; a host worker (or a check) makes
        // the prefix arrays here
        if (in->n_groups && !in->sizes && !in->sizes16)
            return w->fail(HQ_E_INVAL, "hq_worker_step_stream: NULL sizes");
        if (in->n_bytes && !in->bytes)
            return w->fail(HQ_E_INVAL, "hq_worker_step_stream: NULL bytes");
        std::memset(out, 0, sizeof *out);
        static const uint8_t none = 0;
        if (w->dstep) {
            hq_dstep_in d{in->n_groups, in->groups, nullptr, nullptr, nullptr,
                          in->bytes ? in->bytes : &none};
            d.sizes = in->sizes16 ? nullptr : in->sizes;
            d.sizes16 = in->sizes16;
            d.n_events = in->n_events;
            d.n_bytes = in->n_bytes;
            return w->step_on_device(d, out);
        }
        const uint32_t *groups = in->groups;
        if (!groups) {                    // the step lists handles 0 .. n_groups - 1
            w->sized_groups.resize(in->n_groups);
            for (uint64_t i = 0; i < in->n_groups; ++i) w->sized_groups[i] = (uint32_t)i;
            groups = w->sized_groups.data();
        }
        w->sized_off.resize(in->n_groups + 1);
        w->sized_boff.resize(in->n_groups + 1);
        w->sized_off[0] = w->sized_boff[0] = 0;
        if (in->sizes16) {        // bytes only: the events counted from the bytes
            for (uint64_t i = 0; i < in->n_groups; ++i)
                w->sized_boff[i + 1] = w->sized_boff[i] + in->sizes16[i];
            if (w->sized_boff[in->n_groups] != in->n_bytes)
                return w->fail(HQ_E_INVAL, "hq_worker_step_stream: sizes do not sum to the totals");
            if (hq_events_count(in->n_groups, w->sized_boff.data(), in->bytes ? in->bytes : &none,
                                w->sized_off.data()) != HQ_OK)
                return w->fail(HQ_E_INVAL, "hq_worker_step_stream: malformed event stream");
        } else {
            for (uint64_t i = 0; i < in->n_groups; ++i) {
                w->sized_off[i + 1] = w->sized_off[i] + (in->sizes[i] & 0xFFFFu);
                w->sized_boff[i + 1] = w->sized_boff[i] + (in->sizes[i] >> 16);
            }
        }
        if (w->sized_off[in->n_groups] != in->n_events || w->sized_boff[in->n_groups] != in->n_bytes)
            return w->fail(HQ_E_INVAL, "hq_worker_step_stream: sizes do not sum to the totals");
        const hq_step_stream full{in->n_groups, groups, w->sized_off.data(),
                                  w->sized_boff.data(), in->bytes ? in->bytes : &none,
                                  nullptr, 0, 0, nullptr};
        return hq_worker_step_stream(w, &full, out);
    }
    if (in->n_groups && (!in->groups || !in->offsets || !in->boffsets))
        return w->fail(HQ_E_INVAL, "hq_worker_step_stream: NULL groups/offsets/boffsets");
    if (in->n_groups && in->boffsets[in->n_groups] > in->boffsets[0] && !in->bytes)
        return w->fail(HQ_E_INVAL, "hq_worker_step_stream: NULL bytes");
    std::memset(out, 0, sizeof *out);
    static const uint8_t none = 0;
    if (w->dstep)
        return w->step_on_device(hq_dstep_in{in->n_groups, in->groups, in->offsets, nullptr,
                                             in->boffsets, in->bytes ? in->bytes : &none}, out);
    for (uint64_t i = 0; i < in->n_groups; ++i)
        if (in->offsets[i + 1] < in->offsets[i])
            return w->fail(HQ_E_INVAL, "hq_worker_step: offsets decrease");
    const uint64_t ne = in->n_groups ? in->offsets[in->n_groups] : 0;
    w->decoded.resize(ne);
    if (in->n_groups && hq_events_decode(in->n_groups, in->offsets, in->boffsets, in->bytes,
                                         w->decoded.data()) != HQ_OK)
        return w->fail(HQ_E_INVAL, "hq_worker_step_stream: malformed event stream");
    const hq_step_input rows{in->n_groups, in->groups, in->offsets, w->decoded.data()};
    return w->step(&rows, out);
}

}  // extern "C"
