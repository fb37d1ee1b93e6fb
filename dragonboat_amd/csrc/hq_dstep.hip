// hq_dstep.hip — the step worker's device engine (hq_worker_open_ex, HQ_WORKER_ON_DEVICE): the
// whole quorum side of execEngine.processSteps / node.handleEvents (execengine.go:923-1000,
// node.go:1113-1157) for many Raft groups in one launch, their state resident in HBM.
//
// One thread owns one group of the step and takes its events in order, exactly as the reference
// takes a node's queue one message at a time: Peer.Handle's membership filter (peer.go:186-198),
// onMessageTermNotMatched (raft.go:1416-1452), remote.tryUpdate + tryCommit per ReplicateResp
// (remote.go:123-133, raft.go:888-909, 1671-1700), the confirmed-set insert and readIndex.confirm
// per HeartbeatResp (readindex.go:77-116, raft.go:1702-1760), handleLeaderReadIndex
// (raft.go:1636-1669), the first-wins vote tally (raft.go:1062-1080, 1968-1985), CheckQuorum
// (raft.go:380-390, 1582-1588), campaign (raft.go:1082-1117), appendEntries (raft.go:911-922)
// and the state transitions (raft.go:949-1010). Every decision is taken at the event that
// triggers it, so no event waits for another's decision and a step is one launch, whatever the
// events (the host worker cuts runs at such barriers and needs several passes).
//
// The outputs are lists whose lengths are not known in advance: the kernel runs twice. Pass A
// takes every group's events, counts its records (and adds each wave's counts into per-wave
// sums), saves the state it found and writes the new state in place; the per-wave sums are
// scanned (hipcub, or k_scan_layout for a small step), k_step_lite scans the lanes of each wave
// by shuffles, and pass B replays, from the saved state, only the groups that have records other
// than their commit and one ReadyToRead — with the commits as a column (k_step_lite writes every
// group's word from the saved and the new committed index, and copies out the single
// ReadyToReads pass A kept) no group of a steady step is replayed — writing every record at its
// place, in input group order, as the host worker lists them. A step with an input error writes
// no state: k_step_restore puts the saved state back.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <new>
#include <thread>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "hq_dstep.h"
#include "hq_internal.h"

namespace {

// kRerun: 1 for a group with records other than its commit; kEvents: the group's events (pass A
// counts them as it decodes: with 2-byte size words the event prefix pass B needs is their scan);
// kSlotted: 1 for a group whose single ReadyToRead went to its tile's slot (HQ_WORKER_READY_SLOTS)
enum List { kCommits, kReady, kResps, kStates, kDropped, kDeferred, kFallback, kDecisions,
            kRerun, kEvents, kSlotted, kLists };
// the worker's input checks, taken by pass A (which writes no group state) before pass B runs;
// kErrScan: pass A's chained scan of the ReadyToRead places gave up on a tile's word (a stalled
// predecessor: the step re-runs the copy-out through k_step_lite, finish()); kErrTicket: a pass A
// launch found its ticket word not zeroed (an internal fault: nothing of that launch stepped)
enum InputError : uint32_t { kErrHandle = 1, kErrOffsets = 2, kErrBoffsets = 4, kErrTwice = 8,
                             kErrScan = 16, kErrTicket = 32 };
constexpr uint32_t kTickets = 8;  // pass A launches per step (chunks) with their own ticket word

struct StepK {
    hq_dgroup *groups;
    hq_dmember *members;
    hq_dread *reads;
    uint64_t n;                   // groups listed in this step
    uint64_t i_begin, i_end;      // the chunk of them this launch takes
    uint64_t n_handles;           // groups on the device (valid handles)
    uint64_t n_events, n_bytes;   // input sizes (rows or stream bytes)
    uint32_t *stamp;              // per handle: the last step that listed it
    uint32_t step_no;
    uint32_t *error;              // pass A: input errors (kErr* bits)
    uint32_t *wide;               // pass A: a committed index advanced by 2^32 or more (or NULL)
    const uint32_t *handles;
    const uint64_t *offsets;
    const hq_event *events;       // rows, or
    const uint64_t *boffsets;     // an event stream (include/hipquorum.h "event streams")
    const uint8_t *bytes;
    // sized streams: prefix[i] = events before group i << 32 | bytes before it (the scan of the
    // sizes); pass A of byte chunk c takes the groups whose bytes end in [own_lo, own_hi)
    const uint64_t *prefix;
    uint64_t own_lo, own_hi;
    uint32_t *counts;             // [kLists][n]: pass A output (the group's records per list)
    uint32_t *wsum;               // [kLists][nw] + 1 zero: pass A adds each wave's counts (zero
    uint64_t ws;                  //   between steps: k_step_lite clears the ws it used, after the scan)
    const uint32_t *scan;         // exclusive scan of wsum: a wave's first record per list
    uint64_t nw;
    uint32_t *pre;                // [kLists][n] k_step_lite: the counts of the lanes before in the
                                  //   wave, for the groups pass B replays (with scan: their places)
    char *out;                    // pass B: the lists, written straight into pinned host memory
    const struct Layout *layout;  //   at layout->off[list]
    // pass A writes each group's new state in place and its state before the step here (same
    // indexing as groups / members / reads): pass B replays the step from it, and a step with an
    // input error puts it back (k_step_restore)
    hq_dgroup *groups_old;        // (pad1 holds the members' active flags, bit s = member s)
    uint64_t *match_old;
    hq_dread *reads_old;
    // pass A also writes every group's 4-byte advance where the advance column goes (offset 0
    // of the host region) when spec_col is set: those PCIe writes then overlap the later chunks'
    // input copies, and k_step_lite skips them when the layout picks that column (spec_valid)
    uint32_t spec_col, spec_valid;
    uint8_t *rerun;               // [n] pass A: bit 0 the group has records other than its
                                  //   commit (and not just one ReadyToRead), bit 1 pass A stepped
                                  //   it (0: an input error), bit 2 its only record besides the
                                  //   commit is one ReadyToRead, kept in ready_slot
    hq_ready_to_read *ready_slot; // [n] pass A: a group's first ReadyToRead of the step
    uint32_t *rerun_list;         // [n] k_step_lite: the positions of those groups, in order
    // the jobs path (hq_dstep_run_jobs: several workers' steps in shared launches): the layout's
    // arguments, the sizes of a sized stream and the per-1024-group sums of their scan
    uint64_t out_cap;
    uint32_t allow_column, pad_j;
    struct Layout *host_layout;
    const uint32_t *sizes;
    const uint32_t *sizes_src;    // the caller's sizes when in pinned host memory (read over the
                                  //   link by k_size_sums, which writes `sizes`), else NULL
    uint64_t *bsum;
    // pass A over a stream with the advance column speculated (spec_ready): the ReadyToRead
    // records of the groups pass B does not replay go straight to their places in the host region
    // (ready_off: the list's offset when the commits are the 4-byte column), each tile of 256
    // groups finding its first place by a chained scan over `tiles` in start order (`tickets`,
    // one word per pass A launch `chunk`; k_step_lite zeroes them)
    uint32_t spec_ready, chunk;
    uint64_t ready_off;
    // HQ_WORKER_READY_COMPACT: pass A flags a ReadyToRead whose index - the group's committed
    // index before the step does not fit 32 bits (the step then keeps the 32-byte records)
    uint32_t *ready_wide;
    uint64_t *tiles;              // per tile: step_no << 32 | chunk << 29 | inclusive << 28 | count
    uint32_t *tickets;            // [kTickets]
    // 2-byte size words (hq_step_stream.sizes16: a group's byte count only): the prefixes hold
    // bytes alone, pass A counts each group's events as it decodes them (kEvents) and a group's
    // bytes that do not decode are an input error (kErrBoffsets); sizes16_src as sizes_src
    const uint16_t *sizes16;
    const uint16_t *sizes16_src;
    uint32_t bytes_only;
    // HQ_WORKER_READY_SLOTS: pass A writes the single ReadyToRead of every group that has no other
    // record (and whose index - committed fits 32 bits) as an hq_ready_compact into its tile's slot
    // in the host region — tile t (256 groups) at out + slot_off + 6144 t, in group order, its
    // count at out + cnt_off + 4 t — in the link's write direction while pass A reads the stream;
    // those groups leave the list (kSlotted instead of kReady)
    uint32_t slots;
    uint64_t slot_off, cnt_off;
    uint32_t test_scan_fail, pad_t;   // HQ_TEST_SCAN_FAIL at open: every look-back gives up (tests)
};

constexpr uint32_t kSlotTile = 256;   // groups per slot tile (pass A's workgroup)
constexpr uint64_t kSlotTileBytes = kSlotTile * sizeof(hq_ready_compact);
static_assert(kSlotTileBytes % 256 == 0, "slot tiles keep the region's 256-byte alignment");

struct PackSize {                 // group i's size word -> events << 32 | bytes; i = n: 0 (the
    const uint32_t *sizes;        // scan's last element is the totals; no memset on the copy
    uint64_t n;                   // stream between the sizes' copy and the bytes')
    const uint16_t *sizes16 = nullptr;   // 2-byte words: bytes only
    __host__ __device__ uint64_t operator()(uint64_t i) const {
        if (sizes16) return i < n ? sizes16[i] : 0;
        const uint32_t s = i < n ? sizes[i] : 0;
        return (uint64_t)(s & 0xFFFFu) << 32 | (s >> 16);
    }
};

// where the lists go in the host output region (k_layout, from the scanned counts); a step with
// an input error or a region too small has pass B write nothing, not even state
struct Layout {
    uint64_t off[kLists];
    uint32_t len[kLists];
    uint64_t total;
    uint32_t error, overflow;
    uint32_t commit_column;       // the commits list is a column: one word per listed group
                                  // (kColumn64: the committed index, kColumn32: its advance)
    uint32_t ready_compact;       // the ReadyToReads are hq_ready_compact records
    uint32_t pad;
    uint64_t reserve;             // bytes ahead of the lists (the slot form's column + slots)
};
constexpr uint32_t kColumn64 = 1, kColumn32 = 2;
constexpr uint32_t kReadyCompact = 4;   // allow_column bit: HQ_WORKER_READY_COMPACT
constexpr uint32_t kReadySlots = 8;     // allow_column bit: this step writes slots (ready slots)

__device__ __forceinline__ bool is_response(uint32_t t) {   // internal/raft/utils.go
    return t == HQ_MSG_REPLICATE_RESP || t == HQ_MSG_REQUEST_VOTE_RESP ||
           t == HQ_MSG_HEARTBEAT_RESP || t == 20 || t == 8 || t == 9;
}

// A group's bytes read through one cached aligned 8-byte word: a varint byte costs a shift
// instead of a dependent byte load (a group's ~24 bytes take 3-4 loads instead of ~24; the
// input region keeps 8 bytes of slack past its last byte, so the aligned word never leaves it)
struct ByteReader {
    const uint8_t *p, *end;
    uintptr_t wa = 1;             // address of the cached word (never a valid aligned one at start)
    uint64_t w = 0;

    __device__ __forceinline__ bool more() const { return p < end; }
    __device__ __forceinline__ uint32_t next() {
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        if ((a & ~uintptr_t(7)) != wa) {
            wa = a & ~uintptr_t(7);
            w = *reinterpret_cast<const uint64_t *>(wa);
        }
        ++p;
        return (uint32_t)(w >> (8 * (a & 7))) & 0xFF;
    }
};

// the device twin of hq_stream.cpp's decoder: one LEB128 varint
__device__ __forceinline__ bool dvar(ByteReader &r, uint64_t &v) {
    v = 0;
    for (int sh = 0; sh < 64; sh += 7) {
        if (!r.more()) return false;
        const uint32_t b = r.next();
        v |= (uint64_t)(b & 0x7F) << sh;
        if (b < 0x80) return true;
    }
    return false;
}

// a group's stream state the codes refer back to (hq_stream.cpp's Prev): its previous message
// term, its previous ReplicateResp's log_index (code 4), its previous HeartbeatResp's ctx (code
// 5), the previous message a run repeats (code 6; last 1 ReplicateResp, 2 HeartbeatResp, bit 2
// its reject, bit 3 a run in the consecutive form) and the run's events still to come (and, in
// the consecutive form, the next member's sender)
struct DPrev {
    uint64_t term = 0, index = 0, hint = 0, high = 0;
    bool have_index = false;
    uint32_t last = 0, run = 0, run_from = 0;
};

// one event of a group's stream
__device__ bool decode_event(ByteReader &r, DPrev &pv, hq_event &v) {
    v = hq_event{};
    if (pv.run == 0) {
        if (!r.more()) return false;
        // (peek: a run header is taken here, any other header below)
        const uintptr_t a = reinterpret_cast<uintptr_t>(r.p);
        if ((a & ~uintptr_t(7)) != r.wa) {
            r.wa = a & ~uintptr_t(7);
            r.w = *reinterpret_cast<const uint64_t *>(r.wa);
        }
        const uint32_t h0 = (uint32_t)(r.w >> (8 * (a & 7))) & 0xFF;
        if ((h0 & 7) == HQ_EV_MESSAGE && ((h0 >> 3) & 7) == 6) {
            (void)r.next();
            uint64_t m;
            if (!(pv.last & 3) || !dvar(r, m) || m == 0 || m > 0xFFFF) return false;
            pv.run = (uint32_t)m;
            pv.last &= 7u;
            if (h0 & 0x80) {       // the consecutive form: the first sender, the rest follow
                uint64_t f0;
                if (!dvar(r, f0) || f0 + m > 0xFFFFFFFFull) return false;
                pv.run_from = (uint32_t)f0;
                pv.last |= 8u;
            }
        }
    }
    if (pv.run) {                  // a run member: the previous message with another sender
        --pv.run;
        v.kind = HQ_EV_MESSAGE;
        v.type = (pv.last & 3) == 1 ? HQ_MSG_REPLICATE_RESP : HQ_MSG_HEARTBEAT_RESP;
        v.reject = (pv.last >> 2) & 1;
        v.term = pv.term;
        if ((pv.last & 3) == 1) {
            v.log_index = pv.index;
        } else {
            v.hint = pv.hint;
            v.hint_high = pv.high;
        }
        if (pv.last & 8u) {
            v.from = pv.run_from++;
            return true;
        }
        return dvar(r, v.from);
    }
    const uint32_t h = r.next();
    v.kind = h & 7;
    if (v.kind == HQ_EV_READ) return dvar(r, v.hint) && dvar(r, v.hint_high);
    if (v.kind == HQ_EV_PROPOSE) return dvar(r, v.log_index);
    if (v.kind != HQ_EV_MESSAGE) return true;
    const uint32_t code = (h >> 3) & 7;
    uint64_t t = code == 0 || code == 4 ? HQ_MSG_REPLICATE_RESP
               : code == 1 ? HQ_MSG_REQUEST_VOTE_RESP
               : code == 2 || code == 5 ? HQ_MSG_HEARTBEAT_RESP
               : code == 3 ? HQ_MSG_READ_INDEX : 0;
    if (code == 7 && !dvar(r, t)) return false;
    if (code == 4 && !pv.have_index) return false;  // repeats an index the group has not sent
    v.type = (uint32_t)t;
    v.reject = (h >> 6) & 1;
    if (!dvar(r, v.from)) return false;
    if (!(h & 0x80) && !dvar(r, pv.term)) return false;
    v.term = pv.term;
    if ((code == 0 || code == 7) && !dvar(r, v.log_index)) return false;
    if (code == 4) v.log_index = pv.index;
    if ((code == 2 || code == 3 || code == 7) && !(dvar(r, v.hint) && dvar(r, v.hint_high)))
        return false;
    if (code == 5) {
        v.hint = pv.hint;
        v.hint_high = pv.high;
    }
    if (code == 0 || code == 4) {
        pv.index = v.log_index;
        pv.have_index = true;
    }
    if (code == 2 || code == 5) {
        pv.hint = v.hint;
        pv.high = v.hint_high;
    }
    pv.last = (code == 0 || code == 4 ? 1u : code == 2 || code == 5 ? 2u : 0u) | v.reject << 2;
    return true;
}

// One group's state and its output cursor. WRITE = false: counting pass on a private copy;
// WRITE = true: the same sequence writing records and, at the end, the new state.
constexpr uint32_t kStageReady = 64;   // ReadyToRead records staged per wave in pass B
constexpr uint32_t kStageBytes = 16384;  // pass A: a workgroup's stream bytes staged in LDS

// pass A's chained scan of the ReadyToRead places (StepK::tiles): a tile publishes its count
// (aggregate) and then its inclusive prefix, tagged with the step and the launch's chunk so that
// words of earlier launches and steps are never taken for this one's
constexpr uint32_t kTileVal = (1u << 28) - 1;
// how long a tile waits for a predecessor's word before it gives up (kErrScan; the host then
// re-runs the copy-out without pass A's records): 0.1 s of the device's 100-MHz constant clock
// (wall_clock64, hipDeviceAttributeWallClockRate), whatever each poll costs
constexpr uint64_t kScanWaitTicks = 10000000;
__device__ __forceinline__ uint64_t tile_word(uint32_t step, uint32_t chunk, bool incl, uint32_t v) {
    return (uint64_t)step << 32 | (uint64_t)(chunk & 7) << 29 | (uint64_t)incl << 28 | (v & kTileVal);
}
__device__ __forceinline__ uint64_t tile_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void tile_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A workgroup's place in its launch: a ticket drawn at its start, so that a tile's predecessor in
// the chained scan has always started before it (resident or done: no wait on a workgroup not yet
// dispatched)
__device__ __forceinline__ uint32_t draw_ticket(uint32_t *ctr) {
    __shared__ uint32_t t;
    if (threadIdx.x == 0) t = atomicAdd(ctr, 1u);
    __syncthreads();
    return t;
}

template <bool WRITE, int MC>   // MC: member slots held in registers (8 or MC)
struct Engine {
    const StepK &a;
    uint64_t i;                   // position of the group in the step's list
    hq_dgroup g;
    const hq_dmember *gm;         // the group's member records (node ids and roles read-only)
    // member state in registers: every index below is a compile-time constant (unrolled loops,
    // selects), so nothing of it lives in scratch; only the pending reads (rd) are indexed at run
    // time, and they are touched only while a group has reads pending
    uint64_t match[MC];
    uint64_t ids[MC];
    uint32_t active;              // bit s = member s active
    hq_dread *rd;                 // the pending reads: a separate local array (run-time indexed)
    uint32_t cnt[kLists];
    uint32_t base[kLists];
    // pass B: the wave's ReadyToRead records are staged in LDS from record stage_lo on (the
    // records of a wave's groups are consecutive) and written out by the wave as one contiguous
    // run of 16-byte lane stores: a 32-byte record stored per lane leaves half-filled lines
    // whose writes cross PCIe as small packets
    hq_ready_to_read *stage = nullptr;
    uint32_t stage_lo = 0;
    uint64_t c0 = 0;              // the group's committed index before the step
    // pass B over a group whose single ReadyToRead pass A put in its tile's slot (a step in list
    // mode replays every group): the record is not written again nor counted in the list
    bool slotted = false;

    __device__ __forceinline__ Engine(const StepK &k, uint64_t idx, uint32_t h, hq_dread *reads)
        : a(k), i(idx), rd(reads) {
        // pass A: the group's state (then saved, and overwritten by its new state); pass B: the
        // state pass A saved (node ids and roles never change in a step: the live records)
        g = WRITE ? k.groups_old[h] : k.groups[h];
        gm = k.members + g.mem;
        active = 0;
#pragma unroll
        for (uint32_t s = 0; s < MC; ++s) {
            match[s] = 0;
            ids[s] = 0;
            if (s < g.n_members) {
                match[s] = WRITE ? k.match_old[g.mem + s] : gm[s].match;
                ids[s] = gm[s].node_id;
                active |= (uint32_t)(WRITE ? (g.pad1 >> s) & 1 : gm[s].active != 0) << s;
            }
        }
        const hq_dread *rs = (WRITE ? k.reads_old : k.reads) + (uint64_t)h * kDReads;
        for (uint32_t r = 0; r < g.n_reads; ++r) rd[r] = rs[r];
        for (int l = 0; l < kLists; ++l) {
            cnt[l] = 0;           // pass B: the wave's base + the counts of the lanes before
            base[l] = WRITE ? k.scan[(uint64_t)l * k.nw + (idx >> 6)] - k.scan[(uint64_t)l * k.nw] +
                                  k.pre[(uint64_t)l * k.n + idx]
                            : 0;
        }
    }

    __device__ __forceinline__ uint32_t quorum() const { return g.n_voting / 2 + 1; }   // raft.go:372-374
    __device__ __forceinline__ int member_of(uint64_t id) const {
        int m = -1;
#pragma unroll
        for (int s = MC - 1; s >= 0; --s)           // the first match wins
            m = (s < (int)g.n_members && ids[s] == id) ? s : m;
        return m;
    }
    __device__ __forceinline__ uint64_t match_of(int mi) const {
        uint64_t v = 0;
#pragma unroll
        for (int s = 0; s < (int)MC; ++s) v = s == mi ? match[s] : v;
        return v;
    }
    __device__ __forceinline__ void set_match(int mi, uint64_t v) {
#pragma unroll
        for (int s = 0; s < (int)MC; ++s) match[s] = s == mi ? v : match[s];
    }
    __device__ __forceinline__ uint32_t slot(int l) { return base[l] + cnt[l]++; }
    template <class T>
    __device__ __forceinline__ T *list(int l) const {   // (uniform: scalar loads of the layout)
        return reinterpret_cast<T *>(a.out + a.layout->off[l]);
    }

    // -- outputs ----------------------------------------------------------------------------
    __device__ __forceinline__ void ready(uint64_t index, uint64_t low, uint64_t high) {
        if (WRITE && slotted) return;
        const uint32_t p = slot(kReady);
        const hq_ready_to_read r{g.cluster_id, index, low, high};
        const int64_t delta = (int64_t)(index - c0);
        if (!WRITE) {
            if (p == 0) a.ready_slot[i] = r;              // k_step_lite copies it out
            if (a.ready_wide && delta != (int64_t)(int32_t)delta) atomicOr(a.ready_wide, 1u);
        } else if (a.layout->ready_compact) {
            list<hq_ready_compact>(kReady)[p] =
                hq_ready_compact{low, high, (uint32_t)i, (int32_t)delta};
        } else if (stage && p - stage_lo < kStageReady) {
            stage[p - stage_lo] = r;
        } else {
            list<hq_ready_to_read>(kReady)[p] = r;
        }
    }
    __device__ __forceinline__ void resp(uint64_t to, uint64_t index, uint64_t hint, uint64_t high) {
        const uint32_t p = slot(kResps);
        if (WRITE)
            list<hq_read_index_resp>(kResps)[p] = hq_read_index_resp{g.cluster_id, to, index, hint, high};
    }
    __device__ __forceinline__ void state_change(uint32_t reason) {
        const uint32_t p = slot(kStates);
        if (WRITE) list<hq_state_change>(kStates)[p] = hq_state_change{g.cluster_id, g.term, g.state, reason};
    }
    __device__ __forceinline__ void dropped(uint64_t low, uint64_t high, uint64_t from, uint32_t reason) {
        const uint32_t p = slot(kDropped);
        if (WRITE)
            list<hq_dropped_read>(kDropped)[p] = hq_dropped_read{g.cluster_id, low, high, from, reason, 0};
    }
    __device__ __forceinline__ void defer(uint64_t e) {
        const uint32_t p = slot(kDeferred);
        if (WRITE) list<uint64_t>(kDeferred)[p] = e;
    }

    // -- reference state transitions (raft.go:949-1010) --------------------------------------
    __device__ __forceinline__ void reset(uint64_t term) {
        g.term = term;
        g.granted = g.rejected = 0;
        g.n_reads = 0;                                   // r.readIndex = newReadIndex()
#pragma unroll
        for (uint32_t s = 0; s < MC; ++s)         // resetRemotes/Observers/Witnesses
            match[s] = s < g.n_members && ids[s] == g.node_id ? g.last : 0;
        active = 0;
    }
    __device__ __forceinline__ void become_follower(uint64_t term, uint32_t reason) {
        g.state = HQ_STATE_FOLLOWER;
        reset(term);
        state_change(reason);
    }
    __device__ __forceinline__ void become_leader() {
        g.state = HQ_STATE_LEADER;
        reset(g.term);
        state_change(HQ_REASON_VOTE);
        // the no-op of p72: the first entry of the new term; the node's own remote follows it
        g.term_start = g.last + 1;
        g.last += 1;
        match[0] = g.last;
        if (g.n_voting == 1) try_commit();               // appendEntries: single-node tryCommit
    }

    // raft.tryCommit (raft.go:888-909): the quorum-th largest match of the voting members, then
    // entryLog.tryCommit (logentry.go:378-393) with term(q) == term <=> term_start <= q <= last
    // (the leader's entries carry its term and terms never decrease, entryutils.go:44-47)
    // The quorum-th largest by an 8-input sorting network (19 compare-exchanges; the slots past
    // n_voting enter as 0, below or tied with every voting match, so the q-th largest of the 8
    // is that of the n, q <= n) instead of counting, for every slot, the slots at or above it
    // (64 compares): the same value, a third of the instructions on every updating ack.
    __device__ __forceinline__ void try_commit() {
        static_assert(HQ_MAX_VOTERS == 8, "the network sorts 8 voting slots");
        cnt[kDecisions]++;
        const uint32_t n = g.n_voting, q = quorum();
        uint64_t v[8];
#pragma unroll
        for (uint32_t s = 0; s < 8; ++s) v[s] = s < n ? match[s] : 0;
        auto cx = [&](int i, int j) {                    // v[i] >= v[j] afterwards
            const uint64_t a = v[i], b = v[j];
            const bool gt = a > b;
            v[i] = gt ? a : b;
            v[j] = gt ? b : a;
        };
        cx(0, 2); cx(1, 3); cx(4, 6); cx(5, 7);
        cx(0, 4); cx(1, 5); cx(2, 6); cx(3, 7);
        cx(0, 1); cx(2, 3); cx(4, 5); cx(6, 7);
        cx(2, 4); cx(3, 5);
        cx(1, 4); cx(3, 6);
        cx(1, 2); cx(3, 4); cx(5, 6);
        uint64_t best = 0;
#pragma unroll
        for (uint32_t s = 0; s < 8; ++s) best = s + 1 == q ? v[s] : best;
        if (best > g.committed && best >= g.term_start && best <= g.last)
            g.committed = best;                          // commitTo (logentry.go:323-332)
    }

    // handleLeaderReadIndex (raft.go:1636-1669) and readIndex.addRequest (readindex.go:43-67);
    // returns false for the worker's fallback contract (see include/hipquorum.h)
    __device__ __forceinline__ bool read_index(uint64_t from, uint64_t low, uint64_t high, uint64_t e) {
        if (g.state != HQ_STATE_LEADER) {
            defer(e);                                    // forwarded / dropped (raft.go:1875, 1937)
            return true;
        }
        const int fm = member_of(from);
        const uint32_t role = fm >= 0 ? gm[fm].role : 0xFF;
        if (role == HQ_ROLE_WITNESS) {
            dropped(low, high, from, HQ_DROP_WITNESS);
            return true;
        }
        if (g.n_voting == 1) {                           // isSingleNodeQuorum
            ready(g.committed, low, high);
            if (from != g.node_id && role == HQ_ROLE_OBSERVER) resp(from, g.committed, low, high);
            return true;
        }
        // hasCommittedEntryAtCurrentTerm (raft.go:1612-1621)
        if (!(g.committed >= g.term_start && g.committed <= g.last)) {
            dropped(low, high, from, HQ_DROP_NOT_READY);
            return true;
        }
        for (uint32_t k = 0; k < g.n_reads; ++k)
            if (rd[k].low == low && rd[k].high == high) return true;   // already pending
        if (g.n_reads && g.committed < rd[g.n_reads - 1].index) return false;  // reference panics
        if (g.n_reads >= kDReads) return false;
        hq_dread &r = rd[g.n_reads++];
        r = hq_dread{};
        r.index = g.committed;
        r.from = from;
        r.low = low;
        r.high = high;
        return true;
    }

    // readIndex.confirm (readindex.go:77-116) + handleReadIndexLeaderConfirmation
    // (raft.go:1740-1760) for the ack of voting slot mi
    __device__ __forceinline__ bool confirm(uint64_t hint, uint64_t high, int mi) {
        uint32_t k = 0;
        while (k < g.n_reads && !(rd[k].low == hint && rd[k].high == high)) ++k;
        if (k == g.n_reads) return true;                 // not pending
        if (mi >= (int)g.n_voting) return false;         // an observer acking a ctx
        rd[k].confirmed |= (uint8_t)(1u << mi);          // p.confirmed[from] = struct{}{}
        cnt[kDecisions]++;
        if ((uint32_t)__popc(rd[k].confirmed) + 1 < quorum()) return true;
        const uint64_t index = rd[k].index;              // the rewrite of readindex.go:97-105
        for (uint32_t r = 0; r <= k; ++r) {
            if (rd[r].from == 0 || rd[r].from == g.node_id) ready(index, rd[r].low, rd[r].high);
            else resp(rd[r].from, index, hint, high);
        }
        for (uint32_t r = k + 1; r < g.n_reads; ++r) rd[r - k - 1] = rd[r];
        g.n_reads -= (uint8_t)(k + 1);
        return true;
    }

    // one event; false: the group leaves the device path at this event (fallback)
    __device__ __forceinline__ bool handle(const hq_event &ev, uint64_t e) {
        switch (ev.kind) {
        case HQ_EV_READ:
            return read_index(0, ev.hint, ev.hint_high, e);
        case HQ_EV_CHECK_QUORUM: {                       // raft.go:1582-1588, 380-390
            if (g.state != HQ_STATE_LEADER) return true;
            cnt[kDecisions]++;
            const uint32_t vm = (1u << g.n_voting) - 1u;
            const bool has = (uint32_t)__popc((active | 1u) & vm) >= quorum();
            active &= ~vm;                               // setNotActive (remote.go:196-198)
            if (!has) become_follower(g.term, HQ_REASON_CHECK_QUORUM);
            return true;
        }
        case HQ_EV_ELECTION:                             // raft.go:1485-1515, campaign 1082-1117
            if (g.state == HQ_STATE_LEADER) return true;
            g.state = HQ_STATE_CANDIDATE;
            reset(g.term + 1);
            state_change(HQ_REASON_CAMPAIGN);
            g.granted = 1;                               // the self vote
            cnt[kDecisions]++;
            if (g.n_voting == 1) become_leader();        // isSingleNodeQuorum
            return true;
        case HQ_EV_PROPOSE:                              // handleLeaderPropose -> appendEntries
            if (g.state != HQ_STATE_LEADER) {
                defer(e);                                // forwarded / dropped (raft.go:1845, 1932)
                return true;
            }
            g.last += ev.log_index;
            if (match[0] < g.last) match[0] = g.last;
            if (g.n_voting == 1) try_commit();
            return true;
        case HQ_EV_MESSAGE:
            break;
        default:
            return false;
        }
        const uint32_t type = ev.type;
        if (type != HQ_MSG_REPLICATE_RESP && type != HQ_MSG_HEARTBEAT_RESP &&
            type != HQ_MSG_REQUEST_VOTE_RESP && type != HQ_MSG_READ_INDEX)
            return false;
        const int mi = member_of(ev.from);
        if (mi < 0 && is_response(type)) return true;    // Peer.Handle drop (peer.go:191-197)
        if (ev.term != 0 && ev.term != g.term) {         // onMessageTermNotMatched
            if (ev.term < g.term) return true;
            become_follower(ev.term, HQ_REASON_HIGHER_TERM);
        }
        if (g.state == HQ_STATE_LEADER) {
            switch (type) {
            case HQ_MSG_REPLICATE_RESP:                  // handleLeaderReplicateResp
                if (!ev.reject && match_of(mi) < ev.log_index) {
                    if (ev.log_index > g.last) return false;   // a follower acks only what it got
                    set_match(mi, ev.log_index);         // remote.tryUpdate
                    try_commit();
                }
                active |= 1u << mi;
                return true;
            case HQ_MSG_HEARTBEAT_RESP:                  // handleLeaderHeartbeatResp
                if (ev.hint != 0 && !confirm(ev.hint, ev.hint_high, mi)) return false;
                active |= 1u << mi;
                return true;
            case HQ_MSG_READ_INDEX:
                return read_index(ev.from, ev.hint, ev.hint_high, e);
            default:
                return true;                             // RequestVoteResp: no leader handler
            }
        }
        if (g.state == HQ_STATE_CANDIDATE && type == HQ_MSG_REQUEST_VOTE_RESP) {
            if (mi >= (int)g.n_voting) return true;      // observer vote dropped (:1969-1972)
            const uint8_t bit = (uint8_t)(1u << mi);
            if (!((g.granted | g.rejected) & bit)) {     // first response wins (:1071-1073)
                if (ev.reject) g.rejected |= bit;
                else g.granted |= bit;
            }
            cnt[kDecisions]++;
            const uint32_t q = quorum();
            if ((uint32_t)__popc(g.granted) == q) become_leader();            // :1977-1980
            else if ((uint32_t)__popc(g.rejected) == q)                      // :1981-1984
                become_follower(g.term, HQ_REASON_VOTE);
            return true;
        }
        if (type == HQ_MSG_READ_INDEX) return read_index(ev.from, ev.hint, ev.hint_high, e);
        return true;                                     // no handler in this state
    }

    // the group's events: rows (STREAM = false) or its bytes [p, end) of the stream; an event
    // that does not decode is a fallback like one the path does not take
    // (2-byte size words, a.bytes_only: the events are the group's bytes decoded to their end —
    // e1 is not known and a suspended group's events are still decoded to be counted; bytes that
    // do not decode are an input error, as the host worker's decoder makes them, not a fallback)
    template <bool STREAM>
    __device__ __forceinline__ void run(uint64_t e0, uint64_t e1, const uint8_t *p, const uint8_t *end) {
        const uint64_t committed0 = c0 = g.committed;
        DPrev pv;
        ByteReader br{p, end};
        const bool by_bytes = STREAM && a.bytes_only;
        uint64_t e = e0;
        for (;; ++e) {
            if (by_bytes ? !(br.more() || pv.run) : e >= e1) break;
            hq_event ev;
            bool dec = true;
            if (STREAM && (by_bytes || !(g.flags & kDSuspended))) dec = decode_event(br, pv, ev);
            if (by_bytes && !dec) {
                if (!WRITE) atomicOr(a.error, (uint32_t)kErrBoffsets);
                break;
            }
            if (g.flags & kDSuspended) {
                defer(e);
                continue;
            }
            bool ok;
            if (STREAM) {
                ok = dec && handle(ev, e);
            } else {
                ev = a.events[e];
                ok = handle(ev, e);
            }
            if (!ok) {                                   // this event and the rest are deferred
                g.flags |= kDSuspended;
                const uint32_t p = slot(kFallback);
                if (WRITE) list<uint64_t>(kFallback)[p] = g.cluster_id;
                defer(e);
            } else if (STREAM && pv.run) {               // the run's other members at once
#ifndef HQ_NO_TAKE_RUN
                e += take_run(pv, by_bytes ? ~0ull : e1 - e - 1);
#endif
            }
        }
        cnt[kEvents] = (uint32_t)(e - e0);
        // a group that took all its events must have used all its bytes: left-over bytes mean the
        // sizes were split wrongly between groups, which the host decoder rejects as HQ_E_INVAL
        // (hq_stream.cpp); pass A makes it an input error, so no state is written
        if (STREAM && !WRITE && !by_bytes && !(g.flags & kDSuspended) && (br.p != br.end || pv.run))
            atomicOr(a.error, (uint32_t)kErrBoffsets);
        if (!WRITE && g.committed - committed0 > 0xFFFFFFFFull && a.wide)
            atomicOr(a.wide, 1u);                        // no 4-byte advance column this step
        if (!WRITE && a.spec_col)                        // the advance column, ahead of the layout
            reinterpret_cast<uint32_t *>(a.out)[i] = (uint32_t)(g.committed - committed0);
        if (WRITE && a.layout->commit_column) {
            // every listed group's word: k_step_lite wrote it (from the saved and the new state)
        } else if (g.committed != committed0) {
            const uint32_t p = slot(kCommits);
            if (WRITE) list<hq_commit_event>(kCommits)[p] = hq_commit_event{g.cluster_id, g.committed};
        }
    }

    // The rest of a run whose members are consecutive node ids (the event just handled was its
    // first or an earlier member) taken at once where each member could only raise its match
    // (ReplicateResp) and mark its member active: a leader at the run's term, a ReplicateResp
    // run within the log (or rejecting) or a HeartbeatResp run without a ctx. Each member that
    // raises its match is a tryCommit decision; tryCommit runs once after the last: the quorum-th
    // largest match only rises as matches rise, so it ends where the member-by-member calls end
    // (and the run holds no event that reads the committed index). Returns the members taken;
    // otherwise (0) the loop takes them one at a time (also when the run claims more events than
    // the group has left, `room`: the loop then reports the bad sizes).
    __device__ __forceinline__ uint32_t take_run(DPrev &pv, uint64_t room) {
        const uint32_t kind = pv.last & 3;
        const bool rej = (pv.last >> 2) & 1;
        if (!(pv.last & 8u) || pv.run > room || g.state != HQ_STATE_LEADER || (g.flags & kDSuspended) ||
            (pv.term != 0 && pv.term != g.term) ||
            !(kind == 2 ? pv.hint == 0 : (rej || pv.index <= g.last)))
            return 0;
        const uint32_t m = pv.run;
        uint32_t upd = 0;
        for (uint32_t j = 0; j < m; ++j) {
            const int mi = member_of(pv.run_from + j);
            if (mi < 0) continue;                        // Peer.Handle drop (peer.go:191-197)
            if (kind == 1 && !rej && match_of(mi) < pv.index) {
                set_match(mi, pv.index);                 // remote.tryUpdate
                ++upd;
            }
            active |= 1u << mi;
        }
        pv.run_from += m;
        pv.run = 0;
        if (upd) {
            try_commit();
            cnt[kDecisions] += upd - 1;
        }
        return m;
    }

    // pass A, before the group's events: its state as the step found it
    __device__ __forceinline__ void save_old(uint32_t h) {
        hq_dgroup o = g;
        o.pad1 = active;
        a.groups_old[h] = o;
#pragma unroll
        for (uint32_t s = 0; s < MC; ++s)
            if (s < g.n_members) a.match_old[g.mem + s] = match[s];
        for (uint32_t r = 0; r < g.n_reads; ++r) a.reads_old[(uint64_t)h * kDReads + r] = rd[r];
    }

    __device__ __forceinline__ void store(uint32_t h) {
        a.groups[h] = g;
        hq_dmember *m = a.members + g.mem;
#pragma unroll
        for (uint32_t s = 0; s < MC; ++s) {
            if (s < g.n_members) {
                m[s].match = match[s];
                m[s].active = (uint8_t)((active >> s) & 1);
            }
        }
        for (uint32_t r = 0; r < g.n_reads; ++r) a.reads[(uint64_t)h * kDReads + r] = rd[r];
    }
};

// HQ_STEP_WAVES: waves per SIMD asked of the compiler (0: its own choice, 2-3 waves at 157-177
// VGPRs); a group's events are one serial dependency chain, so resident waves hide its latency
#ifndef HQ_STEP_WAVES
#define HQ_STEP_WAVES 0
#endif
#if HQ_STEP_WAVES
#define HQ_STEP_OCC __attribute__((amdgpu_waves_per_eu(HQ_STEP_WAVES)))
#else
#define HQ_STEP_OCC
#endif
// Pass A over a stream, the advance column speculated (StepK::spec_ready): the ReadyToRead records
// of the tile's groups that pass B does not replay (one record, kept in ready_slot), written at
// their final places in the host region during pass A — their PCIe writes then overlap the step's
// input reads instead of following pass A as k_step_lite's. A record's place is the count of
// records of the groups before it in input order: the tile's first place comes from a chained
// scan over the launch's tiles in start order (a tile publishes its count, looks back over its
// predecessors' words until an inclusive one, publishes its own inclusive prefix); the launch's
// first tile takes the inclusive prefix an earlier launch of the step left in the tile of the
// group before its first (0 for group 0). The records are staged in LDS at their places (the
// holes, the places of groups pass B replays, are written by pass B afterwards) and stored as
// one contiguous run of 16-byte stores. All threads of the workgroup call this.
__device__ void ready_tail(const StepK &a, uint64_t tile, uint32_t chunk, bool member, bool first,
                          uint64_t i, uint32_t cnt, bool one, uint4 *sbuf) {
    __shared__ uint32_t s_w[256 / 64], s_excl, s_any, s_first, s_ok;
    __shared__ unsigned long long s_first_i;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x == 0) {
        s_any = 0;
        s_first = 0;
    }
    uint32_t x = cnt;             // inclusive scan over the wave's lanes
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        x += lane >= d ? y : 0u;
    }
    if (lane == 63) s_w[wv] = x;
    __syncthreads();              // (also: every thread is done with the staged bytes in sbuf)
    if (member) s_any = 1;
    if (first) {                  // (one group of the launch is its first)
        s_first = 1;
        s_first_i = i;
    }
    uint32_t before = 0, agg = 0;
#pragma unroll
    for (int w = 0; w < 256 / 64; ++w) {
        before += w < wv ? s_w[w] : 0u;
        agg += s_w[w];
    }
    __syncthreads();
    if (!s_any) return;           // no group of this launch: no tile waits for this one
    if (wv == 0) {                // the first wave looks back, 64 tiles per round trip
        const uint32_t step = a.step_no;
        uint32_t excl = 0;
        bool ok = true;
        if (s_first) {
            if (s_first_i > 0) {  // written by an earlier launch of this step
                const uint64_t w = tile_load(a.tiles + (s_first_i - 1) / 256);
                ok = (uint32_t)(w >> 32) == step && ((w >> 28) & 1) &&
                     (uint32_t)((w >> 29) & 7) < chunk;
                excl = (uint32_t)w & kTileVal;
            }
        } else if (tile == 0 || a.test_scan_fail) {
            ok = false;
        } else {
            if (lane == 0) tile_store(a.tiles + tile, tile_word(step, chunk, false, agg));
            // lane k reads tile hi - k; a window is taken once every tile up to the nearest
            // inclusive word (or all 64) has published for this launch
            int64_t hi = (int64_t)tile - 1;
            const uint64_t t_wait = wall_clock64();
            for (;;) {
                const int64_t p = hi - lane;
                const uint64_t w = p >= 0 ? tile_load(a.tiles + p) : 0;
                const bool ready = p >= 0 && (uint32_t)(w >> 32) == step &&
                                   (uint32_t)((w >> 29) & 7) == (chunk & 7);
                const uint64_t rdy = __ballot(ready), inc = __ballot(ready && ((w >> 28) & 1));
                const uint64_t need = inc ? (inc & (0 - inc)) * 2 - 1 : ~0ull;   // lanes 0 .. k
                if ((rdy & need) == need) {
                    uint32_t v = (lane < 64 - __clzll((long long)need) || !inc) && ready
                                     ? (uint32_t)w & kTileVal : 0u;
#pragma unroll
                    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
                    excl += v;
                    if (inc) break;
                    hi -= 64;
                    if (hi < 0) {     // no inclusive word before: cannot be
                        ok = false;
                        break;
                    }
                    continue;
                }
                if (wall_clock64() - t_wait > kScanWaitTicks) {
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        if (lane == 0) {
            if (!ok) atomicOr(a.error, (uint32_t)kErrScan);
            tile_store(a.tiles + tile, tile_word(step, chunk, true, excl + agg));
            s_excl = excl;
            s_ok = ok;
        }
    }
    __syncthreads();
    const uint32_t lo = s_excl;
    // (a region too small: the layout reports the overflow and the regrown step's k_step_lite
    // writes every record)
    if (!s_ok || agg == 0 || a.ready_off + (uint64_t)(lo + agg) * sizeof(hq_ready_to_read) > a.out_cap)
        return;
    constexpr uint32_t kCap = kStageBytes / sizeof(hq_ready_to_read);
    hq_ready_to_read *stage = reinterpret_cast<hq_ready_to_read *>(sbuf);
    hq_ready_to_read *dst = reinterpret_cast<hq_ready_to_read *>(a.out + a.ready_off) + lo;
    const uint32_t pos = before + x - cnt;   // the tile's records before this group's
    if (one) {
        const hq_ready_to_read r = a.ready_slot[i];
        if (pos < kCap) stage[pos] = r;
        else dst[pos] = r;
    }
    __syncthreads();
    const uint32_t nq = 2 * min(agg, kCap);
    const uint4 *src = reinterpret_cast<const uint4 *>(stage);
    uint4 *out = reinterpret_cast<uint4 *>(dst);
    for (uint32_t q = threadIdx.x; q < nq; q += 256) out[q] = src[q];
}

// HQ_WORKER_READY_SLOTS: tile `tile`'s slotted records (one per slotted thread, the thread's
// group = the tile's 256-group block in order) staged in LDS in group order and stored as one
// contiguous run of 16-byte stores at the tile's slot, the count beside it. No place depends on
// another tile, so pass A writes them while it still reads the stream (the link's other
// direction). buf: >= kSlotTileBytes of LDS no thread still reads. All threads of the workgroup
// call this.
__device__ void slot_store(const StepK &a, uint64_t tile, bool slotted, const hq_ready_compact &rec,
                           uint4 *buf) {
    __shared__ uint32_t s_w[256 / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t bal = __ballot(slotted);
    if (lane == 0) s_w[wv] = (uint32_t)__popcll(bal);
    __syncthreads();              // (also: every thread is done with what buf held)
    uint32_t before = 0, agg = 0;
#pragma unroll
    for (int w = 0; w < 256 / 64; ++w) {
        before += w < wv ? s_w[w] : 0u;
        agg += s_w[w];
    }
    hq_ready_compact *stage = reinterpret_cast<hq_ready_compact *>(buf);
    if (slotted) stage[before + __popcll(bal & ((1ull << lane) - 1))] = rec;
    __syncthreads();
    char *dst = a.out + a.slot_off + tile * kSlotTileBytes;
    const uint32_t nbytes = agg * (uint32_t)sizeof(hq_ready_compact);
    for (uint32_t q = threadIdx.x; q < nbytes / 16; q += 256)
        reinterpret_cast<uint4 *>(dst)[q] = buf[q];
    if (threadIdx.x == 0) {
        if (nbytes & 8)           // (an odd record count: the last 8 bytes)
            reinterpret_cast<uint2 *>(dst)[nbytes / 8 - 1] =
                reinterpret_cast<const uint2 *>(buf)[nbytes / 8 - 1];
        reinterpret_cast<uint32_t *>(a.out + a.cnt_off)[tile] = agg;
    }
}

template <bool WRITE, bool STREAM, int MC>
__device__ __forceinline__ void step_groups(const StepK &a, uint64_t blk, uint32_t chunk = 0) {
    // pass A: the wave's counts summed in LDS, added to wsum by one lane (i_begin is a multiple
    // of 64: the wave's groups are one wave of the scan)
    __shared__ uint32_t wtot[WRITE ? 1 : 256 / 64][kLists];
    if (!WRITE && (threadIdx.x & 63) < kLists) wtot[threadIdx.x >> 6][threadIdx.x & 63] = 0;
    uint64_t i = a.i_begin + blk * 256 + threadIdx.x;
    // pass A over a stream stages the workgroup's bytes in LDS first (below): every thread takes
    // part in that, so until then a thread with no group to step clears `act` instead of leaving
    constexpr bool STAGE = !WRITE && STREAM;
    bool act = true;
    if (WRITE && (a.layout->error | a.layout->overflow)) return;   // nothing written this time
    if (WRITE && a.layout->commit_column) {
        // the commits are a column (k_step_lite wrote it from pass A's state): pass B takes
        // only the groups with other records, packed at the front of the grid
        if (i >= a.layout->len[kRerun]) return;
        i = a.rerun_list[i];
    } else if (i >= a.i_end) {
        if (!STAGE) return;
        act = false;
    }
    uint64_t e0 = 0, e1 = 0, b0 = 0, b1 = 0;
    if (act && STREAM && a.prefix) {
        const uint64_t x0 = a.prefix[i], x1 = a.prefix[i + 1];
        e0 = x0 >> 32;
        e1 = x1 >> 32;
        b0 = x0 & 0xFFFFFFFFu;
        b1 = x1 & 0xFFFFFFFFu;
        if (!WRITE) {
            // the sizes' totals must be the ones the copies were sized by (checked once)
            // (2-byte words carry no events: the layout checks the events pass A counted)
            if (i + 1 == a.n && a.own_lo == 0 &&
                ((!a.bytes_only && e1 != a.n_events) || b1 != a.n_bytes))
                atomicOr(a.error, (uint32_t)kErrBoffsets);
            if (b1 < a.own_lo || b1 >= a.own_hi) act = false;   // another chunk's group
        }
    } else if (act) {
        e0 = a.offsets[i];
        e1 = a.offsets[i + 1];
        if (STREAM) {
            b0 = a.boffsets[i];
            b1 = a.boffsets[i + 1];
        }
    }
    if (!STAGE && !act) return;
    // (pass A over a stream: a group of this launch, input errors or not, and the launch's first)
    const bool member = act;
    const bool first = member && (a.prefix ? i == 0 || b0 < a.own_lo : i == a.i_begin);
    const uint32_t h = !act ? 0u : a.handles ? a.handles[i] : (uint32_t)i;   // NULL: 0 .. n - 1
    if (!WRITE && act) {          // validate this group's entry; a bad one is not stepped
        uint32_t err = 0;
        if (h >= a.n_handles) err |= kErrHandle;
        if (e1 < e0 || (!STREAM && e1 > a.n_events) || (STREAM && a.prefix && e1 > a.n_events))
            err |= kErrOffsets;
        if (STREAM && (b1 < b0 || b1 > a.n_bytes)) err |= kErrBoffsets;
        if (!(err & kErrHandle) && atomicExch(a.stamp + h, a.step_no) == a.step_no)
            err |= kErrTwice;
        if (err) {
            atomicOr(a.error, err);
            for (int l = 0; l < kLists; ++l) a.counts[(uint64_t)l * a.n + i] = 0;
            a.rerun[i] = 0;       // not stepped: nothing to restore
            act = false;
        }
    }
    // Pass A reads each group's bytes once, a thread per group: the workgroup's groups' bytes
    // are one contiguous range, loaded into LDS by all its threads in coalesced 16-byte loads
    // (a zero-copy stream in pinned host memory read lane by lane in 8-byte words crossed the
    // link at 41 GB/s), each thread then decoding its own from LDS; a range larger than the
    // buffer is read in place. The aligned 16-byte blocks around the range never leave the
    // pages of its bytes.
    const uint8_t *src0 = a.bytes + b0;
    __shared__ uint4 sbuf[STAGE ? kStageBytes / 16 : 1];
    if constexpr (STAGE) {
        __shared__ unsigned long long s_lo, s_hi;
        if (threadIdx.x == 0) {
            s_lo = ~0ull;
            s_hi = 0;
        }
        __syncthreads();
        const uint64_t base = reinterpret_cast<uint64_t>(a.bytes);
        if (act && b1 > b0) {
            atomicMin(&s_lo, (unsigned long long)(base + b0));
            atomicMax(&s_hi, (unsigned long long)(base + b1));
        }
        __syncthreads();
        const uint64_t lo = s_lo & ~15ull, hi = (s_hi + 15) & ~15ull;
        const bool fits = s_hi > s_lo && hi - lo <= kStageBytes;
        if (fits) {               // every load issued before the first LDS store: one round
            constexpr int kU = kStageBytes / (256 * 16);   // trip over the link, not kU
            uint4 v[kU];
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const uint64_t o = (threadIdx.x + 256ull * u) * 16;
                if (o < hi - lo) v[u] = *reinterpret_cast<const uint4 *>(lo + o);
            }
#pragma unroll
            for (int u = 0; u < kU; ++u) {
                const uint64_t o = (threadIdx.x + 256ull * u) * 16;
                if (o < hi - lo) sbuf[o / 16] = v[u];
            }
        }
        __syncthreads();
        if (act && fits) src0 = reinterpret_cast<const uint8_t *>(sbuf) + (base + b0 - lo);
    }
    uint32_t n_ready = 0;
    bool one_ready = false, slotted = false;
    hq_ready_compact srec{};
    if (act) {
        hq_dread reads[kDReads];
        Engine<WRITE, MC> eng(a, i, h, reads);   // (pass B: i_begin = 0, i / 64 is its wave)
        if (!WRITE) eng.save_old(h);
        if (WRITE && STREAM && a.bytes_only) e0 = eng.base[kEvents];   // (the events' scan)
        if (WRITE && a.slots) eng.slotted = (a.rerun[i] & 8) != 0;
        __shared__ hq_ready_to_read stage[WRITE ? 256 / 64 : 1][WRITE ? kStageReady : 1];
        // list mode: the wave's groups are consecutive and so are their records, staged from its
        // first active lane's on; column mode: the groups replayed are a sparse subset whose records
        // lie between k_step_lite's, so each is stored where it goes
        const bool staged = WRITE && !a.layout->commit_column && !a.layout->ready_compact;
        if (staged) {
            eng.stage = stage[threadIdx.x >> 6];
            eng.stage_lo = __builtin_amdgcn_readfirstlane(eng.base[kReady]);
        }
        if (STREAM)
            eng.template run<true>(e0, e1, src0, src0 + (b1 - b0));
        else
            eng.template run<false>(e0, e1, nullptr, nullptr);
        if (staged) {                 // the staged records out, 16 contiguous bytes per lane
            const uint64_t act = __ballot(1);
            const int last = 63 - __clzll((long long)act);
            const uint32_t end = __shfl(eng.base[kReady] + eng.cnt[kReady], last);
            const uint32_t nrec = min(end - eng.stage_lo, kStageReady);
            const uint32_t rank = __popcll(act & ((1ull << (threadIdx.x & 63)) - 1));
            const uint32_t nact = __popcll(act);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's LDS stores landed
            __builtin_amdgcn_wave_barrier();
            const uint4 *src = reinterpret_cast<const uint4 *>(eng.stage);
            uint4 *dst = reinterpret_cast<uint4 *>(eng.template list<hq_ready_to_read>(kReady) +
                                                   eng.stage_lo);
            for (uint32_t q = rank; q < 2 * nrec; q += nact) dst[q] = src[q];
        }
        if (!WRITE) {                 // the new state in place (pass B replays from the saved one)
            const bool others = (eng.cnt[kResps] | eng.cnt[kStates] | eng.cnt[kDropped] |
                                 eng.cnt[kDeferred] | eng.cnt[kFallback]) != 0;
            const bool rerun = others || eng.cnt[kReady] > 1;
            one_ready = !rerun && eng.cnt[kReady] == 1;
            if (a.slots && one_ready) {   // the record goes to the tile's slot, out of the list
                const hq_ready_to_read r = a.ready_slot[i];
                const int64_t delta = (int64_t)(r.index - eng.c0);
                if (delta == (int64_t)(int32_t)delta) {
                    slotted = true;
                    one_ready = false;
                    srec = hq_ready_compact{r.ctx_low, r.ctx_high, (uint32_t)i, (int32_t)delta};
                    eng.cnt[kReady] = 0;
                    eng.cnt[kSlotted] = 1;
                }
            }
            n_ready = eng.cnt[kReady];
            eng.cnt[kRerun] = rerun;
            for (int l = 0; l < kLists; ++l) a.counts[(uint64_t)l * a.n + i] = eng.cnt[l];
            a.rerun[i] = (uint8_t)(2 | rerun | (one_ready ? 4 : 0) | (slotted ? 8 : 0));
            eng.store(h);
            uint32_t *wt = wtot[threadIdx.x >> 6];   // (the lanes that left early add nothing)
            for (int l = 0; l < kLists; ++l)
                if (eng.cnt[l]) atomicAdd(wt + l, eng.cnt[l]);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            if ((int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1) {
                for (int l = 0; l < kLists; ++l) {
                    const uint32_t v = wt[l];
                    if (v) atomicAdd(a.wsum + (uint64_t)l * a.nw + (i >> 6), v);
                }
            }
        }
    }
    if constexpr (STAGE) {
        if (a.spec_ready)
            ready_tail(a, (a.i_begin >> 8) + blk, chunk, member, first, i, n_ready, one_ready, sbuf);
        else if (a.slots)
            slot_store(a, (a.i_begin >> 8) + blk, slotted, srec, sbuf);
    }
}

template <bool WRITE, bool STREAM, int MC>
__global__ __launch_bounds__(256) HQ_STEP_OCC void k_step(const StepK a) {
    if constexpr (!WRITE && STREAM) {   // tiles in start order (ready_tail's chained scan)
        const uint32_t b = draw_ticket(a.tickets + a.chunk);
        if (b >= gridDim.x) {     // tickets not zeroed: report, step nothing
            if (threadIdx.x == 0) atomicOr(a.error, (uint32_t)kErrTicket);
            return;
        }
        step_groups<WRITE, STREAM, MC>(a, b, a.chunk);
    } else {
        step_groups<WRITE, STREAM, MC>(a, blockIdx.x);
    }
}

// The jobs path: one launch over several workers' steps, each job's groups in consecutive
// workgroups (blk0[j] .. blk0[j + 1]) and its StepK in device memory
constexpr uint32_t kMaxJobs = 64;
struct JobMap {
    const StepK *ks;              // the jobs' StepK, job0 .. job0 + count - 1 in this launch
    uint32_t job0, count;
    uint32_t blk0[kMaxJobs + 1];  // relative to job0
    uint32_t *tickets;            // pass A: the launch's ticket word is tickets[chunk]; k_step_lite_jobs
    uint32_t chunk;               //   zeroes them
    StepK *table_out;             // k_size_sums (reading `ks` from its pinned copy): workgroup 0
                                  //   writes the jobs' StepK there for the later launches
    uint32_t bsum_scanned, pad;   // k_size_apply: the tiles' totals were scanned (k_bsum_scan_jobs)
};
static_assert(sizeof(StepK) % 8 == 0, "k_size_sums copies the table in 8-byte words");

__device__ __forceinline__ uint32_t job_of(const JobMap &m, uint32_t b) {
    uint32_t j = 0;               // (uniform: kernel arguments and blockIdx)
    while (j + 1 < m.count && b >= m.blk0[j + 1]) ++j;
    return j;
}

template <bool WRITE, bool STREAM, int MC>
__global__ __launch_bounds__(256) HQ_STEP_OCC void k_step_jobs(const JobMap m) {
    uint32_t b = blockIdx.x;
    if constexpr (!WRITE && STREAM) {
        b = draw_ticket(m.tickets + m.chunk);
        if (b >= gridDim.x) {
            if (threadIdx.x == 0) atomicOr(m.ks[m.job0].error, (uint32_t)kErrTicket);
            return;
        }
    }
    const uint32_t j = job_of(m, b);
    step_groups<WRITE, STREAM, MC>(m.ks[m.job0 + j], b - m.blk0[j], m.chunk);
}

// Between the layout and pass B: with the commits as a column, every listed group's word from
// the committed index pass A saved and the one it wrote (the advance, or the new index), and the
// positions of the groups with other records packed in order for pass B; in list mode nothing
__device__ __forceinline__ void lite_groups(const StepK &a, uint64_t blk, uint32_t *tickets) {
    const uint64_t i = blk * 256 + threadIdx.x;
    if (tickets && threadIdx.x < kTickets) tickets[threadIdx.x] = 0;   // (pass A's are done)
    if (i < a.ws) a.wsum[i] = 0;  // (scanned already; the grid covers ws: 11 n / 64 + 12 <= max(n, 256))
    __shared__ __align__(16) hq_ready_to_read stage[256 / 64][kStageReady];
    static_assert(sizeof(stage) >= kSlotTileBytes, "the slot staging fits the list's");
    if (a.slots && !a.spec_valid && !(a.layout->error | a.layout->overflow)) {
        // the output region grew after pass A wrote the slots into the old one: this tile's
        // slots again, from the records pass A kept (whole workgroup; the tiles are pass A's)
        const bool s = i < a.n && (a.rerun[i] & 8);
        hq_ready_compact rec{};
        if (s) {
            const hq_ready_to_read r = a.ready_slot[i];
            const uint32_t h = a.handles ? a.handles[i] : (uint32_t)i;
            rec = hq_ready_compact{r.ctx_low, r.ctx_high, (uint32_t)i,
                                   (int32_t)(int64_t)(r.index - a.groups_old[h].committed)};
        }
        slot_store(a, blk, s, rec, reinterpret_cast<uint4 *>(&stage[0][0]));
        __syncthreads();          // (stage is the list's staging below)
    }
    const bool in = i < a.n;
    if ((a.layout->error | a.layout->overflow) || !__ballot(in)) return;   // (whole waves)
    const uint32_t col = a.layout->commit_column;
    const uint8_t rr = in ? a.rerun[i] : 0;
    const int lane = threadIdx.x & 63;
    // the counts of the lanes before in the wave (pass A's counts, scanned across the wave):
    // stored for the groups pass B replays (with the column: those with other records; in list
    // mode: all), kReady's and kRerun's kept for below; a wave with no replayed group scans those two
    const bool replay = in && (!col || (rr & 1));
    const bool any = __ballot(replay) != 0;
    uint32_t pre_ready = 0, pre_rerun = 0;
    for (int l = 0; l < kLists; ++l) {
        if (!any && l != kReady && l != kRerun) continue;
        const uint32_t c = in ? a.counts[(uint64_t)l * a.n + i] : 0;
        uint32_t x = c;           // inclusive scan over the wave's lanes
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            x += lane >= d ? y : 0u;
        }
        if (replay) a.pre[(uint64_t)l * a.n + i] = x - c;
        if (l == kReady) pre_ready = x - c;
        if (l == kRerun) pre_rerun = x - c;
    }
    if (!col) return;
    const bool col32 = col == kColumn32;
    // the single ReadyToReads pass A kept: the wave's records are consecutive in the list (its
    // groups are), staged in LDS at their places and stored as one contiguous run of 16-byte
    // lane stores; the places of the replayed groups' records are holes pass B fills afterwards
    // (stage: declared above)
    if (!(col32 && a.spec_valid && a.spec_ready)) {   // (else pass A wrote them: ready_tail)
        constexpr uint64_t l = kReady;
        const uint64_t w = i >> 6;
        const uint32_t lo = a.scan[l * a.nw + w] - a.scan[l * a.nw];
        const uint32_t cnt = a.scan[l * a.nw + w + 1] - a.scan[l * a.nw + w];   // the wave's
        hq_ready_to_read *st = stage[threadIdx.x >> 6];
        const uint32_t pos = lo + pre_ready;
        const uint32_t nrec = min(cnt, kStageReady);
        if (a.layout->ready_compact) {
            // 24-byte records (the group's position and index - its committed index before the
            // step, which pass A saved), stored as 8-byte lane words
            hq_ready_compact *stc = reinterpret_cast<hq_ready_compact *>(st);
            hq_ready_compact *dst = reinterpret_cast<hq_ready_compact *>(a.out + a.layout->off[kReady]);
            if (rr & 4) {
                const hq_ready_to_read r = a.ready_slot[i];
                const uint32_t h = a.handles ? a.handles[i] : (uint32_t)i;
                const hq_ready_compact c{r.ctx_low, r.ctx_high, (uint32_t)i,
                                         (int32_t)(int64_t)(r.index - a.groups_old[h].committed)};
                if (pos - lo < kStageReady) stc[pos - lo] = c;
                else dst[pos] = c;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            const uint2 *src = reinterpret_cast<const uint2 *>(stc);
            uint2 *out = reinterpret_cast<uint2 *>(dst + lo);
            for (uint32_t q = lane; q < 3 * nrec; q += 64) out[q] = src[q];
        } else {
            hq_ready_to_read *dst = reinterpret_cast<hq_ready_to_read *>(a.out + a.layout->off[kReady]);
            if (rr & 4) {
                if (pos - lo < kStageReady) st[pos - lo] = a.ready_slot[i];
                else dst[pos] = a.ready_slot[i];
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            const uint4 *src = reinterpret_cast<const uint4 *>(st);
            uint4 *out = reinterpret_cast<uint4 *>(dst + lo);
            for (uint32_t q = lane; q < 2 * nrec; q += 64) out[q] = src[q];
        }
    }
    if (!in) return;
    if (!(col32 && a.spec_valid)) {   // (pass A wrote the advance words)
        const uint32_t h = a.handles ? a.handles[i] : (uint32_t)i;
        const uint64_t c0 = a.groups_old[h].committed, c1 = a.groups[h].committed;
        char *cw = a.out + a.layout->off[kCommits];
        if (col32)
            reinterpret_cast<uint32_t *>(cw)[i] = (uint32_t)(c1 - c0);
        else
            reinterpret_cast<uint64_t *>(cw)[i] = c1 != c0 ? c1 : 0;
    }
    if (rr & 1) {                 // the wave's base + the lanes before
        const uint64_t l = kRerun;
        a.rerun_list[a.scan[l * a.nw + (i >> 6)] - a.scan[l * a.nw] + pre_rerun] = (uint32_t)i;
    }
}

__global__ __launch_bounds__(256) void k_step_lite(const StepK a) {
    lite_groups(a, blockIdx.x, blockIdx.x == 0 ? a.tickets : nullptr);
}

__global__ __launch_bounds__(256) void k_step_lite_jobs(const JobMap m) {
    const uint32_t j = job_of(m, blockIdx.x);
    lite_groups(m.ks[m.job0 + j], blockIdx.x - m.blk0[j], blockIdx.x == 0 ? m.tickets : nullptr);
}

// A step with an input error writes no group state: the groups pass A stepped get back the
// state it saved (the host launches this only when k_layout reported an error)
__global__ __launch_bounds__(256) void k_step_restore(const StepK a) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n || !(a.rerun[i] & 2)) return;
    const uint32_t h = a.handles ? a.handles[i] : (uint32_t)i;
    hq_dgroup g = a.groups_old[h];
    const uint32_t act = g.pad1;
    g.pad1 = 0;
    a.groups[h] = g;
    for (uint32_t s = 0; s < g.n_members; ++s) {
        a.members[g.mem + s].match = a.match_old[g.mem + s];
        a.members[g.mem + s].active = (uint8_t)((act >> s) & 1);
    }
    for (uint32_t r = 0; r < g.n_reads; ++r)
        a.reads[(uint64_t)h * kDReads + r] = a.reads_old[(uint64_t)h * kDReads + r];
}

// the lists' place in the host output region (of cap bytes) from the scanned per-wave sums, and
// the input errors of pass A (reset for the next step)
// input chunks of a large step (at least kChunkGroups groups each): chunk c's copy overlaps pass A
// of chunk c - 1, and the last chunk's pass A is the step's tail (8 chunks: no faster, profiles/r03e/ab_step_chunks.log)
#ifndef HQ_STEP_CHUNKS
#define HQ_STEP_CHUNKS 4
#endif
constexpr int kMaxChunks = HQ_STEP_CHUNKS;
constexpr int kMaxJobChunks = 8;   // the jobs path's chunks of whole jobs (events per copy stream)
static_assert(kMaxChunks <= kMaxJobChunks, "the chunk events serve both paths");
static_assert(kMaxJobChunks <= kTickets, "a ticket word per pass A launch");
constexpr uint64_t kChunkGroups = 65536;
// the slot form's part of the host region ahead of the lists: the 4-byte column at 0, tile t's
// slots at slot_off + 6144 t, the tiles' counts at cnt_off; returns its size (the lists' start)
__host__ __device__ inline uint64_t slot_layout(uint64_t n, uint64_t *slot_off, uint64_t *cnt_off) {
    const uint64_t tiles = (n + kSlotTile - 1) / kSlotTile;
    const uint64_t so = (n * 4 + 255) & ~uint64_t(255);
    const uint64_t co = so + tiles * kSlotTileBytes;
    if (slot_off) *slot_off = so;
    if (cnt_off) *cnt_off = co;
    return co + ((tiles * 4 + 255) & ~uint64_t(255));
}

// bnd[l] = the scan at l * nw (list l's first record), l = 0 .. kLists; want_events: the step's
// event total when pass A counted the events (2-byte size words), else ~0
__device__ void layout_from(const uint32_t *bnd, uint64_t n, uint32_t *error, uint64_t cap,
                            uint32_t allow_column, uint64_t want_events, Layout *lay,
                            Layout *host_lay) {
    uint32_t *wide = error + 1;   // pass A: an advance of 2^32 or more
    uint32_t *ready_wide = error + 2;   // pass A: a ReadyToRead delta beyond 32 bits
    if (want_events != ~uint64_t(0) && (uint64_t)(bnd[kEvents + 1] - bnd[kEvents]) != want_events)
        *error |= kErrBoffsets;   // (the events decoded are not the totals the caller gave)
    lay->ready_compact = (allow_column & kReadyCompact) && !*ready_wide;
    const uint64_t rec[kLists] = {sizeof(hq_commit_event),
                                  lay->ready_compact ? sizeof(hq_ready_compact) : sizeof(hq_ready_to_read),
                                  sizeof(hq_read_index_resp), sizeof(hq_state_change),
                                  sizeof(hq_dropped_read), 8, 8, 0, 0, 0, 0};
    const uint32_t commits = bnd[1] - bnd[0];
    // the commits as a column when that moves fewer bytes (16 per commit in the list against 8
    // per listed group, or 4 when every advance fits)
    // (allow_column: bit kColumn64 HQ_WORKER_COMMIT_COLUMN, bit kColumn32 _ADVANCE)
    lay->commit_column = (allow_column & kColumn32) && !*wide && 4 * (uint64_t)commits > n
                             ? kColumn32
                         : (allow_column & kColumn64) && 2 * (uint64_t)commits > n ? kColumn64 : 0;
    // the slot form: the column and the slots pass A wrote come first, the lists after them
    const bool slots = (allow_column & kReadySlots) != 0;
    const uint64_t reserve = slots ? slot_layout(n, nullptr, nullptr) : 0;
    uint64_t total = reserve;
    for (int l = 0; l < kLists; ++l) {
        const uint32_t len = bnd[l + 1] - bnd[l];
        lay->len[l] = len;
        if (l == kCommits && slots && lay->commit_column == kColumn32) {
            lay->off[l] = 0;      // (where pass A wrote the advance words)
            continue;
        }
        lay->off[l] = total;
        const uint64_t bytes = l == kCommits && lay->commit_column
                                   ? n * (lay->commit_column == kColumn32 ? 4 : 8)
                                   : len * rec[l];
        total += (bytes + 255) & ~uint64_t(255);
    }
    lay->total = total;
    lay->reserve = reserve;
    lay->error = *error;
    lay->overflow = total > cap;
    // pass A's flags are reset for the next step, except when the host will run this layout again
    // for the same step and the re-run must see the same flags (or it could choose the 4-byte
    // advance column for a 2^32 advance): an overflow without an input error (the region grows),
    // or kErrScan alone (the copy-out runs again without pass A's records; the host clears it)
    if (!((lay->overflow && !*error) || *error == kErrScan)) {
        *error = 0;
        *wide = 0;
        *ready_wide = 0;
    }
    *host_lay = *lay;             // the host's copy, written into pinned memory (no copy launch)
}

__global__ void k_layout(const uint32_t *scan, uint64_t n, uint64_t nw, uint32_t *error,
                         uint64_t cap, uint32_t allow_column, uint64_t want_events, Layout *lay,
                         Layout *host_lay) {
    if (threadIdx.x != 0) return;
    uint32_t bnd[kLists + 1];
    for (int l = 0; l <= kLists; ++l) bnd[l] = scan[(uint64_t)l * nw];
    layout_from(bnd, n, error, cap, allow_column, want_events, lay, host_lay);
}

// A small step's scan of the per-wave sums and its layout in one workgroup (hipcub's scan is two
// launches, then k_layout a third: 16 workers pay 48 such launches per step): tiles of 11 Ki sums,
// each thread scanning 11 consecutive ones from LDS (an odd stride: no bank conflicts), the
// threads' totals scanned across the waves, with the carry of the tiles before
constexpr int kScanT = 1024, kScanE = 11;
constexpr uint64_t kScanSmall = 2 * kScanT * kScanE;   // sums taken this way (2 tiles)
__device__ __forceinline__ void scan_layout(const uint32_t *wsum, uint32_t *scan, uint64_t ws,
                                            uint64_t n, uint64_t nw, uint32_t *error, uint64_t cap,
                                            uint32_t allow_column, uint64_t want_events, Layout *lay,
                                            Layout *host_lay) {
    __shared__ uint32_t tile[kScanT * kScanE];
    __shared__ uint32_t wtot[kScanT / 64];
    __shared__ uint32_t bnd[kLists + 1];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    uint32_t carry = 0;
    for (uint64_t base = 0; base < ws; base += (uint64_t)kScanT * kScanE) {
        for (int k = 0; k < kScanE; ++k) {
            const uint64_t j = base + (uint64_t)k * kScanT + t;
            tile[k * kScanT + t] = j < ws ? wsum[j] : 0u;
        }
        __syncthreads();
        uint32_t v[kScanE], sum = 0;
        for (int k = 0; k < kScanE; ++k) {
            v[k] = tile[t * kScanE + k];
            sum += v[k];
        }
        uint32_t x = sum;         // inclusive scan of the threads' totals over the wave
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(x, d, 64);
            x += lane >= d ? y : 0u;
        }
        if (lane == 63) wtot[wv] = x;
        __syncthreads();
        uint32_t before = 0, all = 0;
        for (int w = 0; w < kScanT / 64; ++w) {
            const uint32_t z = wtot[w];
            before += w < wv ? z : 0u;
            all += z;
        }
        uint32_t run = carry + before + x - sum;
        for (int k = 0; k < kScanE; ++k) {
            tile[t * kScanE + k] = run;
            run += v[k];
        }
        __syncthreads();
        for (int k = 0; k < kScanE; ++k) {
            const uint64_t j = base + (uint64_t)k * kScanT + t;
            if (j < ws) {
                const uint32_t e = tile[k * kScanT + t];
                scan[j] = e;
                if (j % nw == 0 && j / nw <= kLists) bnd[j / nw] = e;
            }
        }
        carry += all;
        __syncthreads();          // (the next tile overwrites tile and wtot)
    }
    if (t == 0) layout_from(bnd, n, error, cap, allow_column, want_events, lay, host_lay);
}

__global__ __launch_bounds__(kScanT) void k_scan_layout(const uint32_t *wsum, uint32_t *scan,
                                                        uint64_t ws, uint64_t n, uint64_t nw,
                                                        uint32_t *error, uint64_t cap,
                                                        uint32_t allow_column, uint64_t want_events,
                                                        Layout *lay, Layout *host_lay) {
    scan_layout(wsum, scan, ws, n, nw, error, cap, allow_column, want_events, lay, host_lay);
}

__host__ __device__ inline uint64_t want_events_of(const StepK &a) {
    return a.bytes_only ? a.n_events : ~uint64_t(0);
}

// the jobs path: one workgroup per job (grid = the jobs)
__global__ __launch_bounds__(kScanT) void k_scan_layout_jobs(const StepK *ks) {
    const StepK &a = ks[blockIdx.x];
    scan_layout(a.wsum, const_cast<uint32_t *>(a.scan), a.ws, a.n, a.nw, a.error, a.out_cap,
                a.allow_column, want_events_of(a), const_cast<Layout *>(a.layout), a.host_layout);
}

// The jobs path's scan of a sized stream's sizes (the single path: hipcub over PackSize), in
// two launches for all jobs: each 1024 groups' packed total (k_size_sums), then each 1024 groups
// scanned in a workgroup from the sum of the totals before it (k_size_apply); prefix[i] = events
// before group i << 32 | bytes before it, prefix[n] the totals (n + 1 elements, as the single
// path's scan)
constexpr uint32_t kSizeTile = 1024;   // groups per workgroup of 256 threads (4 each)
// a job of more size tiles than this has its tiles' totals scanned by a launch of their own
// (k_bsum_scan_jobs) instead of each k_size_apply workgroup summing the totals before it (the
// sum's work grows with the square of the tiles: ~134 M L2 loads at 16 M groups)
constexpr uint64_t kSizeApplyDirect = 2048;
__device__ __forceinline__ uint64_t packed_size(const StepK &a, uint64_t i) {
    if (i >= a.n) return 0;
    if (a.bytes_only) return a.sizes16[i];
    const uint32_t s = a.sizes[i];
    return (uint64_t)(s & 0xFFFFu) << 32 | (s >> 16);
}

__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t *total) {
    __shared__ uint64_t wt[1024 / 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        x += lane >= d ? y : 0ull;
    }
    if (lane == 63) wt[wv] = x;
    __syncthreads();
    uint64_t before = 0, all = 0;
    for (int w = 0; w < (int)(blockDim.x / 64); ++w) {
        before += w < wv ? wt[w] : 0ull;
        all += wt[w];
    }
    __syncthreads();              // (wt is reused by the next call)
    *total = all;
    return before + x - v;
}

__global__ __launch_bounds__(256) void k_size_sums(const JobMap m) {
    if (m.table_out && blockIdx.x == 0) {   // the table for the launches behind this one
        const uint64_t *src = reinterpret_cast<const uint64_t *>(m.ks + m.job0);
        uint64_t *dst = reinterpret_cast<uint64_t *>(m.table_out + m.job0);
        for (uint32_t q = threadIdx.x; q < m.count * (uint32_t)(sizeof(StepK) / 8); q += 256)
            dst[q] = src[q];
    }
    const uint32_t j = job_of(m, blockIdx.x);
    const StepK &a = m.ks[m.job0 + j];
    const uint64_t b = blockIdx.x - m.blk0[j], i0 = b * kSizeTile + threadIdx.x * 4;
    uint64_t v = 0;
    if (a.bytes_only && a.sizes16_src) {
        // 2-byte words straight from pinned host memory (one 8-byte load of a thread's 4 where
        // aligned and whole), kept on device for k_size_apply
        uint16_t *dst = const_cast<uint16_t *>(a.sizes16);
        uint16_t z[4];
        if (i0 + 4 <= a.n && !(reinterpret_cast<uintptr_t>(a.sizes16_src) & 7)) {
            const uint64_t w = *reinterpret_cast<const uint64_t *>(a.sizes16_src + i0);
#pragma unroll
            for (int k = 0; k < 4; ++k) z[k] = (uint16_t)(w >> (16 * k));
            *reinterpret_cast<uint64_t *>(dst + i0) = w;   // (dst: a 256-byte aligned region)
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint64_t i = i0 + k;
                z[k] = i < a.n ? a.sizes16_src[i] : 0;
                if (i < a.n) dst[i] = z[k];
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) v += z[k];
    } else if (!a.bytes_only && a.sizes_src) {   // the sizes straight from pinned host memory
        uint32_t *dst = const_cast<uint32_t *>(a.sizes);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t i = i0 + k;
            const uint32_t z = i < a.n ? a.sizes_src[i] : 0;
            if (i < a.n) dst[i] = z;
            v += (uint64_t)(z & 0xFFFFu) << 32 | (z >> 16);
        }
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) v += packed_size(a, i0 + k);
    }
    uint64_t tot;
    (void)block_excl_scan(v, &tot);
    if (threadIdx.x == 0) a.bsum[b] = tot;
}

// the size tiles' totals of every job scanned in place (exclusive), one workgroup per job: the
// large steps' form (k_size_apply then reads its tile's prefix)
__global__ __launch_bounds__(1024) void k_bsum_scan_jobs(const JobMap m) {
    const StepK &a = m.ks[m.job0 + blockIdx.x];
    const uint64_t nb = (a.n + 1 + kSizeTile - 1) / kSizeTile;
    uint64_t carry = 0;
    for (uint64_t base = 0; base < nb; base += 1024) {
        const uint64_t k = base + threadIdx.x;
        const uint64_t v = k < nb ? a.bsum[k] : 0;
        uint64_t tot;
        const uint64_t ex = block_excl_scan(v, &tot);
        if (k < nb) a.bsum[k] = carry + ex;
        carry += tot;
    }
}

// (a small job's workgroups each sum the totals of the tiles before their own: at most a few
// thousand words from L2, in place of a scan launch between the two passes)
__global__ __launch_bounds__(256) void k_size_apply(const JobMap m) {
    const uint32_t j = job_of(m, blockIdx.x);
    const StepK &a = m.ks[m.job0 + j];
    const uint64_t b = blockIdx.x - m.blk0[j], i0 = b * kSizeTile + threadIdx.x * 4;
    uint64_t base;
    if (m.bsum_scanned) {
        base = a.bsum[b];
    } else {
        uint64_t before = 0;
        for (uint64_t k = threadIdx.x; k < b; k += 256) before += a.bsum[k];
        (void)block_excl_scan(before, &base);
    }
    uint64_t v[4], sum = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[k] = packed_size(a, i0 + k);
        sum += v[k];
    }
    uint64_t tot;
    uint64_t run = base + block_excl_scan(sum, &tot);
    uint64_t *prefix = const_cast<uint64_t *>(a.prefix);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (i0 + k <= a.n) prefix[i0 + k] = run;
        run += v[k];
    }
}

uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

}  // namespace

struct hq_dstep {
    hq_ctx *ctx = nullptr;
    // HQ_TEST_FAIL_REGROW=1 in the environment at open: the output region's regrow fails (the
    // failure path's test, tests/test_gpu_worker.py)
    bool test_fail_regrow = false;
    bool test_scan_fail = false;  // HQ_TEST_SCAN_FAIL=1 at open: pass A's look-backs give up
    hq_dgroup *groups = nullptr;
    hq_dread *reads = nullptr;
    hq_dmember *members = nullptr;
    // the state pass A saved (StepK::groups_old ...), as large as the state
    hq_dgroup *groups_old = nullptr;
    hq_dread *reads_old = nullptr;
    uint64_t *match_old = nullptr;
    uint8_t *rerun = nullptr;     // [rcap] per listed group
    uint32_t *rerun_list = nullptr;
    hq_ready_to_read *ready_slot = nullptr;
    size_t rcap = 0;
    uint32_t *stamp = nullptr;    // [gcap] step stamps (duplicate handles)
    uint64_t gcap = 0, mcap = 0;
    uint64_t n_groups = 0;        // group records uploaded (valid handles)
    uint32_t max_members = 0;     // the most members of any uploaded group
    uint32_t step_no = 0;
    uint32_t commit_column = 0;   // bits: kColumn64 HQ_WORKER_COMMIT_COLUMN, kColumn32 _ADVANCE
    // step staging
    void *in = nullptr;
    size_t in_cap = 0;
    uint32_t *counts = nullptr, *scan = nullptr, *bases = nullptr;
    size_t cnt_cap = 0;
    uint32_t *wsum = nullptr;     // pass A's per-wave sums (StepK::wsum), zero between steps
    size_t wsum_cap = 0;          //   (bytes)
    bool wsum_dirty = true;
    void *scan_tmp = nullptr;
    size_t scan_tmp_cap = 0;
    void *host_out = nullptr;     // pinned host region pass B writes the lists into
    size_t host_out_cap = 0;
    Layout *layout = nullptr;     // device: the lists' places (k_layout)
    Layout *host_layout = nullptr;  // pinned mirror, copied back at the end of the step
    // a large step runs in chunks of groups: chunk c's input copy (copy stream) overlaps pass A
    // of chunk c - 1, and its result copy overlaps pass B of chunk c + 1 (compute stream); the
    // copy stream is created by the first such step
    hipStream_t copy = nullptr;
    hipEvent_t ev_in[kMaxJobChunks] = {};
    // the jobs path's second copy stream (jobs' byte copies alternate between the two, so that
    // one copy's start-up gap overlaps the other's transfer) and its events
    hipStream_t copy2 = nullptr;
    hipEvent_t ev_in2[kMaxJobChunks] = {};
    // the pinned bounce buffer of hq_dstep_put / _get (two halves) and each half's last copy
    char *bounce = nullptr;
    hipEvent_t bounce_ev[2] = {nullptr, nullptr};
    hipEvent_t ev_sync = nullptr;  // blocking-sync event: a waiting worker thread sleeps
    // timing events around a step's device work (hq_dstep_out::gpu_ns): the host's wait for a
    // step, less the GPU's time, is its wake-up and queueing delay
    hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr;
    // the jobs path (hq_dstep_run_jobs, this engine first): the jobs' StepK, pinned and on device
    StepK *jobs_host = nullptr, *jobs_dev = nullptr;
    const StepK *jobs_host_dev = nullptr;   // jobs_host's device address (k_size_sums reads it)
    uint32_t jobs_cap = 0;
    // pass A's ticket words (StepK::tickets), zeroed by k_step_lite; a step that stopped before
    // it leaves them to clear (dirty), and pass A's chained-scan words per tile of 256 groups
    uint32_t *tickets = nullptr;
    bool tickets_dirty = false;
    uint64_t *tiles = nullptr;
    size_t tiles_cap = 0;         // (bytes)
    // how the step's thread waits for the device (hq_dstep_set_wait; HQ_WAIT_*) and the clock of
    // the last wait: the device's 100-MHz stamp after the step's last kernel (HQ_WAIT_CLOCK), in
    // pinned memory
    uint32_t wait_mode = HQ_WAIT_BLOCK, wait_poll_us = 50, wait_sleep_us = 20;
    uint64_t wait_pred_ns = 0;    // HQ_WAIT_ADAPT: the last step's wait, start to seen done
    bool wait_clock = false;
    uint64_t *clock_host = nullptr;
    hq_wait_clock last_wait{};
};

namespace {

int grow(hq_ctx *ctx, void **p, size_t *cap, size_t need, bool keep, const char *what) {
    if (need <= *cap) return HQ_OK;
    size_t want = need + need / 2;
    // HQ_GROW_TRACE=1: each device regrowth on stderr (a hipMalloc + hipFree in a step's
    // submission: the device synchronizes for the free)
    static const bool trace = [] {
        const char *v = std::getenv("HQ_GROW_TRACE");
        return v && std::atoi(v) != 0;
    }();
    if (trace)
        std::fprintf(stderr, "[hq grow] %s %zu -> %zu bytes at %.3f ms\n", what, *cap, want,
                     now_ns() / 1e6);
    void *n = nullptr;
    int rc = hq::check_hip(ctx, hipMalloc(&n, want), what);
    if (rc) return rc;
    if (*p && keep) rc = hq::check_hip(ctx, hipMemcpyAsync(n, *p, *cap, hipMemcpyDeviceToDevice,
                                                           ctx->stream), what);
    if (!rc) rc = hq::check_hip(ctx, hipStreamSynchronize(ctx->stream), what);
    if (*p) (void)hipFree(*p);
    *p = n;
    *cap = want;
    return rc;
}

}  // namespace

namespace {

// Wait for a stream on the step's thread, as d's policy says (hq_dstep_set_wait), its clock in
// d->last_wait:
//   HQ_WAIT_BLOCK  poll for poll_us, then sleep on a blocking-sync event (the runtime's interrupt
//                  wait): 16 workers waiting at once do not spin 16 host cores (a spinning wait
//                  under a CPU quota stalls every thread of the process for the rest of the
//                  period); spin_us > 50 (the jobs path's one waiter, HQ_STEP_JOBS_SPIN_US) polls
//                  longer, yielding now and then
//   HQ_WAIT_SLEEP  poll for poll_us, then query the event every sleep_us, asleep in between (a
//                  timer wake-up: its lateness is bounded by the timer's slack, not by the
//                  runtime's interrupt path)
//   HQ_WAIT_SPIN   poll with yields until done (a core held for the step)
//   HQ_WAIT_ADAPT  one timed sleep until max(poll_us, 100) before the end the last step's wait
//                  predicts (its length from the wait's start to the step seen done), then poll
//                  with yields: a spinning wait's lateness for ~100 us of a core per step; past
//                  twice the prediction (+ 1 ms) it sleeps on the blocking-sync event
// With HQ_WAIT_CLOCK a one-thread kernel behind the step writes the device's constant clock into
// pinned memory: the step's end on the device's clock, against which the host's wake-up is read
__global__ void k_clock_stamp(uint64_t *dst) {
    if (threadIdx.x == 0) *dst = wall_clock64();
}

int wait_stream(hq_dstep *d, hipStream_t s, const char *what, uint32_t spin_us = 0) {
    hq_ctx *ctx = d->ctx;
    hq_wait_clock &wc = d->last_wait;
    wc = hq_wait_clock{};
    int rc = HQ_OK;
    if (d->wait_clock) {
        d->clock_host[0] = 0;
        hipLaunchKernelGGL(k_clock_stamp, dim3(1), dim3(64), 0, s, d->clock_host);
        rc = hq::check_hip(ctx, hipGetLastError(), "k_clock_stamp");
    }
    if (!rc) rc = hq::check_hip(ctx, hipEventRecord(d->ev_sync, s), what);
    if (rc) return rc;
    const uint32_t mode = d->wait_mode;
    const uint32_t poll_us = spin_us ? spin_us : d->wait_poll_us;
    const uint64_t t0 = now_ns();
    wc.t_begin_ns = t0;
    auto done = [&](int r) {
        wc.t_end_ns = now_ns();
        if (d->wait_clock && !r) {
            wc.device_end_ticks = d->clock_host[0];
            wc.device_start_ticks = d->clock_host[1];
        }
        return r;
    };
    if (mode == HQ_WAIT_ADAPT && d->wait_pred_ns) {
        const uint64_t pred = d->wait_pred_ns;
        const uint64_t margin = (uint64_t)std::max<uint32_t>(poll_us, 100) * 1000;
        if (pred > margin) {
            std::this_thread::sleep_for(std::chrono::nanoseconds(pred - margin));
            wc.sleeps = 1;
            wc.sleep_ns = now_ns() - t0;
        }
        const uint64_t t1 = now_ns();
        for (uint32_t k = 0;; ++k) {
            const hipError_t q = hipEventQuery(d->ev_sync);
            if (q == hipSuccess) {
                wc.poll_ns = now_ns() - t1;
                d->wait_pred_ns = now_ns() - t0;
                return done(HQ_OK);
            }
            if (q != hipErrorNotReady) return done(hq::check_hip(ctx, q, what));
            if (now_ns() - t0 > 2 * pred + 1000000) break;    // far past the prediction
            if ((k & 15) == 15) std::this_thread::yield();
        }
        const uint64_t t2 = now_ns();
        wc.poll_ns = t2 - t1;
        ++wc.sleeps;
        rc = hq::check_hip(ctx, hipEventSynchronize(d->ev_sync), what);
        wc.sleep_ns += now_ns() - t2;
        if (!rc) d->wait_pred_ns = now_ns() - t0;
        return done(rc);
    }
    for (uint32_t k = 0;; ++k) {
        const hipError_t q = hipEventQuery(d->ev_sync);
        if (q == hipSuccess) {
            wc.poll_ns = now_ns() - t0;
            return done(HQ_OK);
        }
        if (q != hipErrorNotReady) return done(hq::check_hip(ctx, q, what));
        if (mode != HQ_WAIT_SPIN && now_ns() - t0 > (uint64_t)poll_us * 1000) break;
        if ((mode == HQ_WAIT_SPIN || poll_us > 50) && (k & 15) == 15) std::this_thread::yield();
    }
    const uint64_t t1 = now_ns();
    wc.poll_ns = t1 - t0;
    if (mode == HQ_WAIT_SLEEP) {
        for (;;) {
            std::this_thread::sleep_for(std::chrono::microseconds(d->wait_sleep_us));
            ++wc.sleeps;
            const hipError_t q = hipEventQuery(d->ev_sync);
            if (q == hipSuccess) break;
            if (q != hipErrorNotReady) return done(hq::check_hip(ctx, q, what));
        }
        wc.sleep_ns = now_ns() - t1;
        return done(HQ_OK);
    }
    wc.sleeps = 1;
    rc = hq::check_hip(ctx, hipEventSynchronize(d->ev_sync), what);
    wc.sleep_ns = now_ns() - t1;
    if (!rc) d->wait_pred_ns = now_ns() - t0;   // (HQ_WAIT_ADAPT's first step)
    return done(rc);
}

}  // namespace

int hq_dstep_set_wait(hq_dstep *d, uint32_t mode, uint32_t poll_us, uint32_t sleep_us) {
    const uint32_t m = mode & ~HQ_WAIT_CLOCK;
    if (m != HQ_WAIT_BLOCK && m != HQ_WAIT_SLEEP && m != HQ_WAIT_SPIN && m != HQ_WAIT_ADAPT)
        return HQ_E_INVAL;
    if (m == HQ_WAIT_SLEEP && sleep_us == 0) return HQ_E_INVAL;
    if ((mode & HQ_WAIT_CLOCK) && !d->clock_host) {
        int rc = hq::check_hip(d->ctx, hipHostMalloc(&d->clock_host, 64, hipHostMallocDefault),
                               "hq_dstep clock");
        if (rc) return rc;
    }
    d->wait_mode = m;
    d->wait_poll_us = poll_us;
    d->wait_sleep_us = sleep_us;
    d->wait_clock = (mode & HQ_WAIT_CLOCK) != 0;
    return HQ_OK;
}

int hq_dstep_open(hq_ctx *ctx, hq_dstep **out, uint32_t commit_column) {
    *out = new (std::nothrow) hq_dstep();
    if (!*out) return HQ_E_NOMEM;
    hq_dstep *d = *out;
    d->ctx = ctx;
    d->commit_column = commit_column;
    if (const char *f = std::getenv("HQ_TEST_FAIL_REGROW")) d->test_fail_regrow = std::atoi(f) != 0;
    if (const char *f = std::getenv("HQ_TEST_SCAN_FAIL")) d->test_scan_fail = std::atoi(f) != 0;
    int rc = hq::check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (!rc)
        rc = hq::check_hip(ctx, hipEventCreateWithFlags(&d->ev_sync, hipEventDisableTiming |
                                                                          hipEventBlockingSync),
                           "event");
    for (hipEvent_t *e : {&d->ev_t0, &d->ev_t1})
        if (!rc) rc = hq::check_hip(ctx, hipEventCreate(e), "event");
    for (int c = 0; c < kMaxJobChunks && !rc; ++c) {
        rc = hq::check_hip(ctx, hipEventCreateWithFlags(&d->ev_in[c], hipEventDisableTiming), "event");
        if (!rc)
            rc = hq::check_hip(ctx, hipEventCreateWithFlags(&d->ev_in2[c], hipEventDisableTiming),
                               "event");
    }
    if (!rc) rc = hq::check_hip(ctx, hipMalloc(&d->layout, sizeof(Layout)), "hq_dstep layout");
    if (!rc) rc = hq::check_hip(ctx, hipMalloc(&d->tickets, kTickets * 4), "hq_dstep tickets");
    if (!rc) rc = hq::check_hip(ctx, hipMemset(d->tickets, 0, kTickets * 4), "hq_dstep tickets");
    if (!rc)
        rc = hq::check_hip(ctx, hipHostMalloc(&d->host_layout, sizeof(Layout), hipHostMallocDefault),
                           "hq_dstep layout");
    if (rc) {
        hq_dstep_close(d);
        *out = nullptr;
    }
    return rc;
}

void hq_dstep_close(hq_dstep *d) {
    if (!d) return;
    (void)hipSetDevice(d->ctx->device);
    (void)hipStreamSynchronize(d->ctx->stream);
    for (void *p : {(void *)d->groups, (void *)d->reads, (void *)d->members, (void *)d->stamp, d->in,
                    (void *)d->counts, (void *)d->scan, (void *)d->bases, d->scan_tmp,
                    (void *)d->layout, (void *)d->groups_old, (void *)d->reads_old,
                    (void *)d->match_old, (void *)d->rerun, (void *)d->ready_slot,
                    (void *)d->rerun_list, (void *)d->wsum, (void *)d->jobs_dev,
                    (void *)d->tickets, (void *)d->tiles})
        if (p) (void)hipFree(p);
    if (d->host_out) (void)hipHostFree(d->host_out);
    if (d->jobs_host) (void)hipHostFree(d->jobs_host);
    if (d->host_layout) (void)hipHostFree(d->host_layout);
    if (d->clock_host) (void)hipHostFree(d->clock_host);
    if (d->bounce) (void)hipHostFree(d->bounce);
    for (hipEvent_t e : d->bounce_ev)
        if (e) (void)hipEventDestroy(e);
    for (hipStream_t cs : {d->copy, d->copy2}) {
        if (cs) {
            (void)hipStreamSynchronize(cs);
            (void)hipStreamDestroy(cs);
        }
    }
    for (hipEvent_t e : {d->ev_sync, d->ev_t0, d->ev_t1})
        if (e) (void)hipEventDestroy(e);
    for (int c = 0; c < kMaxJobChunks; ++c) {
        if (d->ev_in[c]) (void)hipEventDestroy(d->ev_in[c]);
        if (d->ev_in2[c]) (void)hipEventDestroy(d->ev_in2[c]);
    }
    delete d;
}

namespace {

// The groups' state moves between the worker's own (pageable) vectors and the device through a
// pinned bounce buffer, in halves of kBounce bytes: for a large pageable copy the HIP runtime pins
// the caller's pages in place, and when those pages' mappings later change (the allocator handing
// them back) the driver evicts and restores the process's queues — a device step queued meanwhile
// started 5-24 ms late (profiles/r06l/)
constexpr size_t kBounce = size_t(8) << 20;

int bounce_ready(hq_dstep *d) {
    if (d->bounce) return HQ_OK;
    hq_ctx *ctx = d->ctx;
    int rc = hq::check_hip(ctx, hipHostMalloc(reinterpret_cast<void **>(&d->bounce), 2 * kBounce,
                                              hipHostMallocDefault), "hq_dstep bounce");
    for (hipEvent_t &e : d->bounce_ev)
        if (!rc) rc = hq::check_hip(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming), "event");
    return rc;
}

int put_staged(hq_dstep *d, void *dst, const void *src, size_t bytes, uint64_t *half) {
    hq_ctx *ctx = d->ctx;
    int rc = bounce_ready(d);
    for (size_t off = 0; !rc && off < bytes; off += kBounce, ++*half) {
        const size_t n = std::min(kBounce, bytes - off);
        const int h = (int)(*half & 1);
        char *b = d->bounce + h * kBounce;
        // (the half's previous copy must have read it: its event, recorded behind that copy)
        if (*half >= 2) rc = hq::check_hip(ctx, hipEventSynchronize(d->bounce_ev[h]), "hq_dstep_put");
        if (rc) break;
        std::memcpy(b, static_cast<const char *>(src) + off, n);
        rc = hq::check_hip(ctx, hipMemcpyAsync(static_cast<char *>(dst) + off, b, n,
                                               hipMemcpyHostToDevice, ctx->stream), "hq_dstep_put");
        if (!rc) rc = hq::check_hip(ctx, hipEventRecord(d->bounce_ev[h], ctx->stream), "hq_dstep_put");
    }
    return rc;
}

int get_staged(hq_dstep *d, void *dst, const void *src, size_t bytes) {
    hq_ctx *ctx = d->ctx;
    int rc = bounce_ready(d);
    for (size_t off = 0; !rc && off < bytes; off += kBounce) {
        const size_t n = std::min(kBounce, bytes - off);
        rc = hq::check_hip(ctx, hipMemcpyAsync(d->bounce, static_cast<const char *>(src) + off, n,
                                               hipMemcpyDeviceToHost, ctx->stream), "hq_dstep_get");
        if (!rc) rc = hq::check_hip(ctx, hipStreamSynchronize(ctx->stream), "hq_dstep_get");
        if (!rc) std::memcpy(static_cast<char *>(dst) + off, d->bounce, n);
    }
    return rc;
}

}  // namespace

int hq_dstep_put(hq_dstep *d, uint64_t g0, uint64_t ng, const hq_dgroup *g, const hq_dread *r,
                 uint64_t m0, uint64_t nm, const hq_dmember *m) {
    hq_ctx *ctx = d->ctx;
    int rc = hq::check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    size_t gc = d->gcap * sizeof(hq_dgroup), rcap = d->gcap * kDReads * sizeof(hq_dread),
           mc = d->mcap * sizeof(hq_dmember);
    if (!rc && (g0 + ng) > d->gcap) {
        rc = grow(ctx, reinterpret_cast<void **>(&d->groups), &gc, (g0 + ng) * sizeof(hq_dgroup),
                  true, "hq_dstep groups");
        if (!rc)
            rc = grow(ctx, reinterpret_cast<void **>(&d->reads), &rcap,
                      (g0 + ng) * kDReads * sizeof(hq_dread), true, "hq_dstep reads");
        size_t sc = d->gcap * 4;
        if (!rc)
            rc = grow(ctx, reinterpret_cast<void **>(&d->stamp), &sc, (g0 + ng) * 4, true,
                      "hq_dstep stamps");
        // the saved-state buffers only live within a step: grown without their contents
        size_t gn = d->gcap * sizeof(hq_dgroup), rn = d->gcap * kDReads * sizeof(hq_dread);
        if (!rc)
            rc = grow(ctx, reinterpret_cast<void **>(&d->groups_old), &gn,
                      (g0 + ng) * sizeof(hq_dgroup), false, "hq_dstep saved groups");
        if (!rc)
            rc = grow(ctx, reinterpret_cast<void **>(&d->reads_old), &rn,
                      (g0 + ng) * kDReads * sizeof(hq_dread), false, "hq_dstep saved reads");
        if (!rc) d->gcap = std::min({gc / sizeof(hq_dgroup), rcap / (kDReads * sizeof(hq_dread)),
                                     sc / 4, gn / sizeof(hq_dgroup),
                                     rn / (kDReads * sizeof(hq_dread))});
    }
    for (uint64_t i = 0; i < ng; ++i)
        if (g[i].n_members > d->max_members) d->max_members = g[i].n_members;
    if (!rc && ng) {              // new stamps start at 0 (no step has listed them)
        rc = hq::check_hip(ctx, hipMemsetAsync(d->stamp + g0, 0, ng * 4, ctx->stream), "memset");
        if (!rc && g0 + ng > d->n_groups) d->n_groups = g0 + ng;
    }
    if (!rc && (m0 + nm) > d->mcap) {
        size_t xn = d->mcap * 8;
        rc = grow(ctx, reinterpret_cast<void **>(&d->members), &mc,
                  (m0 + nm) * sizeof(hq_dmember), true, "hq_dstep members");
        if (!rc)
            rc = grow(ctx, reinterpret_cast<void **>(&d->match_old), &xn, (m0 + nm) * 8, false,
                      "hq_dstep saved matches");
        if (!rc) d->mcap = std::min(mc / sizeof(hq_dmember), xn / 8);
    }
    uint64_t half = 0;
    if (!rc && ng) rc = put_staged(d, d->groups + g0, g, ng * sizeof(hq_dgroup), &half);
    if (!rc && ng) rc = put_staged(d, d->reads + g0 * kDReads, r, ng * kDReads * sizeof(hq_dread), &half);
    if (!rc && nm) rc = put_staged(d, d->members + m0, m, nm * sizeof(hq_dmember), &half);
    if (!rc) rc = hq::check_hip(ctx, hipStreamSynchronize(ctx->stream), "hq_dstep_put");
    return rc;
}

int hq_dstep_get(hq_dstep *d, uint64_t ng, hq_dgroup *g, hq_dread *r, uint64_t nm, hq_dmember *m) {
    hq_ctx *ctx = d->ctx;
    int rc = hq::check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (!rc && ng) rc = get_staged(d, g, d->groups, ng * sizeof(hq_dgroup));
    if (!rc && ng) rc = get_staged(d, r, d->reads, ng * kDReads * sizeof(hq_dread));
    if (!rc && nm) rc = get_staged(d, m, d->members, nm * sizeof(hq_dmember));
    return rc;
}

namespace {

// One worker's step from its preparation to its outputs (hq_dstep_run; hq_dstep_run_jobs runs
// several of them through shared launches)
struct Run {
    hq_dstep *d = nullptr;
    const hq_dstep_in *in = nullptr;
    hq_dstep_out *out = nullptr;
    StepK k{};
    uint64_t n = 0, ne = 0, nb = 0, nw = 0;
    size_t ws = 0, tmp = 0, tmp2 = 0;
    size_t o_off = 0, o_boff = 0, o_ev = 0;
    int chunks = 1;
    bool stream = false, sized = false, small = false, small_scan = false;
    bool stepped = false, first = true;
    bool timing = false;          // ev_t0 recorded: pass B records ev_t1 before its wait
    uint64_t t0 = 0, t1 = 0, t_sub = 0, gpu_ns = 0;
    int rc = HQ_OK;
};

// GPU time between two completed events (0 if it cannot be read)
uint64_t elapsed_ns(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return (uint64_t)((double)ms * 1e6);
}

// HQ_STEP_SPEC_READY=0 in the environment: pass A leaves the ReadyToReads to k_step_lite (A/B)
bool spec_ready_allowed() {
    static const bool on = [] {
        const char *v = std::getenv("HQ_STEP_SPEC_READY");
        return !v || std::atoi(v) != 0;
    }();
    return on;
}

// The step's buffers (grown as needed) and its StepK, with the memsets it needs queued on s; no
// launch. in->n > 0.
int prepare(Run &r, hipStream_t s, bool jobs = false) {
    hq_dstep *d = r.d;
    hq_ctx *ctx = d->ctx;
    const hq_dstep_in *in = r.in;
    const uint64_t n = r.n = in->n;
    r.stream = in->bytes != nullptr;
    r.sized = r.stream && (in->sizes != nullptr || in->sizes16 != nullptr);   // scanned here
    const bool stream = r.stream, sized = r.sized;
    const bool s16 = sized && in->sizes16 != nullptr;   // 2-byte words: bytes only
    const uint64_t ne = r.ne = sized ? in->n_events : in->offsets[n];
    const uint64_t nb = r.nb = !stream ? 0 : sized ? in->n_bytes : in->boffsets[n];
    if (sized && (ne >> 32 || nb >> 32))     // the scanned prefixes pack both totals in 64 bits
        return hq::fail(ctx, HQ_E_INVAL, "hq_dstep: a sized step holds < 2^32 events and bytes");
    r.t0 = now_ns();
    int rc = hq::check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    // chunks of groups (at least 64 Ki each): chunk c's input copy overlaps pass A of chunk c - 1
    while (r.chunks * 2 <= kMaxChunks && n >= (uint64_t)r.chunks * 2 * kChunkGroups) r.chunks *= 2;
    // the step's input in one device region: handles, offsets, [boffsets,] events or bytes, each
    // at the offsets it has on the host; a sized stream: handles, sizes (+ a zero), their scan,
    // bytes
    auto up = [](size_t x) { return (x + 255) & ~size_t(255); };
    r.o_off = up(n * 4);
    r.o_boff = r.o_off + up((n + 1) * 8);
    r.o_ev = r.o_boff + (stream ? up((n + 1) * 8) : 0);   // (sized: prefix at o_boff)
    // + 8: slack for ByteReader's aligned word past the last byte
    const size_t in_bytes = r.o_ev + (stream ? nb : ne * sizeof(hq_event)) + 8;
    if (!rc) rc = grow(ctx, &d->in, &d->in_cap, in_bytes, false, "hq_dstep input");
    char *din = static_cast<char *>(d->in);
    // counts [kLists][n] and the prefixes pass B reads, [kLists][n]; the scan buffer holds the
    // per-wave sums [kLists][nw] + 1 (a zero: the scan's last element is the grand total) and
    // their scan (one size covers both)
    const uint64_t nw = r.nw = (n + 63) / 64;
    const size_t ws = r.ws = (size_t)kLists * nw + 1;
    r.small_scan = ws <= kScanSmall;
    const size_t cn = (size_t)2 * kLists * n + 2 * ws;
    size_t cc = d->cnt_cap * 4, sc = d->cnt_cap * 4, bc = d->cnt_cap ? 256 : 0;
    if (!rc && cn > d->cnt_cap) {
        rc = grow(ctx, reinterpret_cast<void **>(&d->counts), &cc, cn * 4, false, "hq_dstep counts");
        if (!rc) rc = grow(ctx, reinterpret_cast<void **>(&d->scan), &sc, cn * 4, false, "hq_dstep scan");
        if (!rc && !d->bases) {
            rc = grow(ctx, reinterpret_cast<void **>(&d->bases), &bc, 256, false, "hq_dstep error");
            if (!rc) rc = hq::check_hip(ctx, hipMemsetAsync(d->bases, 0, 256, s), "memset");
        }
        if (!rc) d->cnt_cap = std::min(cc, sc) / 4;
    }
    // pass A's chained-scan words: zeroed when allocated (their tags then never match a step)
    const size_t tiles_bytes = ((n + 255) / 256 + 1) * 8;
    if (!rc && tiles_bytes > d->tiles_cap) {
        rc = grow(ctx, reinterpret_cast<void **>(&d->tiles), &d->tiles_cap, tiles_bytes, false,
                  "hq_dstep tiles");
        if (!rc) rc = hq::check_hip(ctx, hipMemsetAsync(d->tiles, 0, d->tiles_cap, s), "memset");
    }
    if (!rc && ws * 4 > d->wsum_cap) {
        rc = grow(ctx, reinterpret_cast<void **>(&d->wsum), &d->wsum_cap, ws * 4, false,
                  "hq_dstep wave sums");
        d->wsum_dirty = true;
    }
    if (!rc && n > d->rcap) {
        size_t fc = d->rcap, lc = d->rcap * 4;
        rc = grow(ctx, reinterpret_cast<void **>(&d->rerun), &fc, n, false, "hq_dstep rerun");
        if (!rc)
            rc = grow(ctx, reinterpret_cast<void **>(&d->rerun_list), &lc, n * 4, false,
                      "hq_dstep rerun list");
        size_t sc = d->rcap * sizeof(hq_ready_to_read);
        if (!rc)
            rc = grow(ctx, reinterpret_cast<void **>(&d->ready_slot), &sc,
                      n * sizeof(hq_ready_to_read), false, "hq_dstep ready slots");
        if (!rc) d->rcap = std::min({fc, lc / 4, sc / sizeof(hq_ready_to_read)});
    }
    // the host region the lists go to: last step's size with room to spare (a step that needs
    // more runs pass B again after growing it)
    if (!rc && !d->host_out) {
        const size_t want = std::max<size_t>(n * 64, 1 << 16);
        rc = hq::check_hip(ctx, hipHostMalloc(&d->host_out, want, hipHostMallocDefault),
                           "hq_dstep pinned output");
        if (!rc) d->host_out_cap = want;
    }
    const hipcub::TransformInputIterator<uint64_t, PackSize, hipcub::CountingInputIterator<uint64_t>>
        packed_sizes(hipcub::CountingInputIterator<uint64_t>(0),
                     PackSize{reinterpret_cast<const uint32_t *>(din + r.o_off), n,
                              s16 ? reinterpret_cast<const uint16_t *>(din + r.o_off) : nullptr});
    uint64_t *prefix = reinterpret_cast<uint64_t *>(din + r.o_boff);
    uint32_t *wsum = d->wsum;
    // (the jobs path scans with its own kernels: no hipcub temporary, whose size query costs
    // microseconds of host time per job before the first launch)
    if (!rc && !jobs)
        rc = hq::check_hip(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, r.tmp, wsum, d->scan,
                                                                  ws, s),
                           "hipcub scan size");
    if (!rc && sized && !jobs)
        rc = hq::check_hip(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, r.tmp2, packed_sizes,
                                                                  prefix, n + 1, s),
                           "hipcub scan size");
    // (the jobs path's per-1024-group size totals live there too)
    const size_t bsum_bytes = sized ? (n + 1 + kSizeTile - 1) / kSizeTile * 8 : 0;
    if (!rc) rc = grow(ctx, &d->scan_tmp, &d->scan_tmp_cap, std::max({r.tmp, r.tmp2, bsum_bytes}),
                       false, "hq_dstep scan tmp");
    if (rc) return rc;
    StepK &k = r.k;
    k = StepK{};
    k.groups = d->groups;
    k.members = d->members;
    k.reads = d->reads;
    k.n = n;
    k.i_begin = 0;
    k.i_end = n;
    k.own_lo = 0;
    k.own_hi = UINT64_MAX;
    k.handles = sized && !in->groups ? nullptr : reinterpret_cast<const uint32_t *>(din);
    k.offsets = reinterpret_cast<const uint64_t *>(din + r.o_off);
    if (sized) {
        k.prefix = prefix;
        k.bytes = reinterpret_cast<const uint8_t *>(din + r.o_ev);
        k.sizes = reinterpret_cast<const uint32_t *>(din + r.o_off);
        k.sizes16 = reinterpret_cast<const uint16_t *>(din + r.o_off);   // (one of the two)
        k.bytes_only = s16;
        k.bsum = static_cast<uint64_t *>(d->scan_tmp);
    } else if (stream) {
        k.boffsets = reinterpret_cast<const uint64_t *>(din + r.o_boff);
        k.bytes = reinterpret_cast<const uint8_t *>(din + r.o_ev);
    } else {
        k.events = reinterpret_cast<const hq_event *>(din + r.o_ev);
    }
    k.counts = d->counts;
    k.pre = d->counts + (size_t)kLists * n;
    k.wsum = wsum;
    k.ws = ws;
    k.scan = d->scan;
    k.nw = nw;
    k.n_handles = d->n_groups;
    k.n_events = ne;
    k.n_bytes = nb;
    k.stamp = d->stamp;
    if (++d->step_no == 0) {      // stamps wrap: forget them, and the chained-scan words
        rc = hq::check_hip(ctx, hipMemsetAsync(d->stamp, 0, d->gcap * 4, s), "memset");   // (tagged
        if (!rc && d->tiles)                                                               // with it)
            rc = hq::check_hip(ctx, hipMemsetAsync(d->tiles, 0, d->tiles_cap, s), "memset");
        d->step_no = 1;
        if (rc) return rc;
    }
    k.step_no = d->step_no;
    // pass A adds each wave's counts into wsum, which k_step_lite leaves zero; a step that
    // stopped before it (or a new buffer) leaves it to clear here
    if (d->wsum_dirty) {
        rc = hq::check_hip(ctx, hipMemsetAsync(wsum, 0, d->wsum_cap, s), "memset");
        if (rc) return rc;
    }
    d->wsum_dirty = true;
    k.error = d->bases;           // zero here: reset by the previous step's k_layout
    k.wide = d->commit_column & kColumn32 ? d->bases + 1 : nullptr;   // likewise
    k.out = static_cast<char *>(d->host_out);
    k.layout = d->layout;
    k.groups_old = d->groups_old;
    k.match_old = d->match_old;
    // pass A's advance words need the column allowed and the region to hold n of them (its
    // offset 0 is the commits list's in every layout)
    k.spec_col = (d->commit_column & kColumn32) && n * 4 <= d->host_out_cap;
    k.spec_valid = k.spec_col;
    // pass A writes the single ReadyToReads at their places too (ready_tail): stream input, the
    // column speculated, the counts within a tile word (HQ_STEP_SPEC_READY=0: k_step_lite, A/B)
    // (not the jobs path: there pass A reads the streams over the link in place, and these
    // writes beside its reads slowed it by more than k_step_lite's copy takes, 981 vs 693 + 158
    // us for the 16-worker step5, profiles/r05e)
    // (nor with compact ReadyToReads, whose record size the layout picks after pass A)
    k.spec_ready = !jobs && stream && k.spec_col && ne < kTileVal && spec_ready_allowed() &&
                   !(d->commit_column & kReadyCompact);
    k.ready_wide = (d->commit_column & kReadyCompact) ? d->bases + 2 : nullptr;   // (zero: k_layout)
    k.ready_off = (n * 4 + 255) & ~uint64_t(255);   // layout_from's offset of the list after the column
    k.tiles = d->tiles;
    k.tickets = d->tickets;
    k.chunk = 0;
    k.reads_old = d->reads_old;
    k.rerun = d->rerun;
    k.rerun_list = d->rerun_list;
    k.ready_slot = d->ready_slot;
    k.out_cap = d->host_out_cap;
    k.test_scan_fail = d->test_scan_fail;
    k.allow_column = d->commit_column & ~kReadySlots;
    k.host_layout = d->host_layout;
    r.small = d->max_members <= 8;   // member slots in registers: 8 or kDMembers
    // HQ_WORKER_READY_SLOTS: a stream step of the jobs path (pass A's tiles are whole 256-group
    // blocks of one launch there) with the advance column allowed writes the slots; the host region
    // is grown ahead of pass A to hold the column, the slots and room for the lists
    if (jobs && stream && (d->commit_column & kReadySlots) && (d->commit_column & kColumn32)) {
        const uint64_t reserve = slot_layout(n, &k.slot_off, &k.cnt_off);
        const size_t want = reserve + std::max<size_t>(n * 16, 1 << 16);
        if (d->host_out_cap < want) {
            void *grown = nullptr;
            rc = hq::check_hip(ctx, hipHostMalloc(&grown, want, hipHostMallocDefault),
                               "hq_dstep pinned output");
            if (rc) return rc;
            if (d->host_out) (void)hipHostFree(d->host_out);
            d->host_out = grown;
            d->host_out_cap = want;
            k.out = static_cast<char *>(d->host_out);
            k.out_cap = want;
            k.spec_col = n * 4 <= want;
            k.spec_valid = k.spec_col;
        }
        k.slots = 1;
        k.allow_column |= kReadySlots;
    }
    return HQ_OK;
}

// one pass over groups [i0, i1) of the step on its worker's stream
void launch_pass(Run &r, bool write, uint64_t i0, uint64_t i1) {
    hq_ctx *ctx = r.d->ctx;
    StepK &k = r.k;
    k.i_begin = i0;
    k.i_end = i1;
    const dim3 grid((unsigned)((i1 - i0 + 255) / 256)), blk(256);
    if (r.rc || i1 == i0) return;
    r.rc = hq::pre_launch(ctx);
    if (r.rc) return;
    const bool stream = r.stream, small = r.small;
#define HQ_STEP_LAUNCH(W)                                                                        \
    if (stream && small) hipLaunchKernelGGL((k_step<W, true, 8>), grid, blk, 0, ctx->stream, k); \
    else if (stream) hipLaunchKernelGGL((k_step<W, true, kDMembers>), grid, blk, 0, ctx->stream, k); \
    else if (small) hipLaunchKernelGGL((k_step<W, false, 8>), grid, blk, 0, ctx->stream, k); \
    else hipLaunchKernelGGL((k_step<W, false, kDMembers>), grid, blk, 0, ctx->stream, k);
    if (write) {
        HQ_STEP_LAUNCH(true)
    } else {
        HQ_STEP_LAUNCH(false)
    }
#undef HQ_STEP_LAUNCH
    r.rc = hq::post_launch(ctx, write ? "k_step<write>" : "k_step<count>");
}

// layout, pass B (straight into the pinned region), the layout back: one wait per step. The
// first layout of a small step scans the wave sums in one workgroup; a re-run after an overflow
// (or a step whose sums hipcub scanned) takes k_layout: k_step_lite has cleared the sums
void pass_b(Run &r) {
    hq_dstep *d = r.d;
    hq_ctx *ctx = d->ctx;
    StepK &k = r.k;
    if (!r.rc && r.small_scan && r.first) {
        hipLaunchKernelGGL(k_scan_layout, dim3(1), dim3(kScanT), 0, ctx->stream, d->wsum, d->scan,
                           (uint64_t)r.ws, r.n, r.nw, k.error, (uint64_t)d->host_out_cap,
                           k.allow_column, want_events_of(k), d->layout, d->host_layout);
        r.rc = hq::check_hip(ctx, hipGetLastError(), "k_scan_layout");
    } else if (!r.rc) {
        hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, ctx->stream, d->scan, r.n, r.nw, k.error,
                           (uint64_t)d->host_out_cap, k.allow_column, want_events_of(k), d->layout,
                           d->host_layout);
        r.rc = hq::check_hip(ctx, hipGetLastError(), "k_layout");
    }
    r.first = false;
    const dim3 grid((unsigned)((r.n + 255) / 256)), blk(256);
    if (!r.rc) {
        hipLaunchKernelGGL(k_step_lite, grid, blk, 0, ctx->stream, k);
        r.rc = hq::check_hip(ctx, hipGetLastError(), "k_step_lite");
        if (!r.rc) d->wsum_dirty = d->tickets_dirty = false;
    }
    launch_pass(r, true, 0, r.n);
    if (!r.rc && r.timing) {
        r.rc = hq::check_hip(ctx, hipEventRecord(d->ev_t1, ctx->stream), "event");
        r.t_sub = now_ns();
    }
    if (!r.rc) r.rc = wait_stream(d, ctx->stream, "hq_dstep sync");
    if (!r.rc && r.timing) r.gpu_ns = elapsed_ns(d->ev_t0, d->ev_t1);
    r.timing = false;             // (a second pass B, after the output region grew: untimed)
}

// Pass A has written every listed group's new state in place (the state it found is saved).
// From there on a step that fails returns with that state taken back (k_step_restore), so a
// failed step leaves the groups as they were, whatever failed: an input error found by the
// kernels, a HIP error, the output region that could not grow, a second layout failure. (A
// pass A launch that itself fails leaves rc set before that point; the context is then
// unusable and the caller reloads the groups from the device, hq_worker.cpp.)
int restore(Run &r, int code) {
    if (!r.stepped) return code;
    hq_ctx *ctx = r.d->ctx;
    hipLaunchKernelGGL(k_step_restore, dim3((unsigned)((r.n + 255) / 256)), dim3(256), 0,
                       ctx->stream, r.k);
    int r2 = hq::check_hip(ctx, hipGetLastError(), "k_step_restore");
    if (!r2) r2 = wait_stream(r.d, ctx->stream, "hq_dstep restore");
    return code ? code : r2;
}

// the device's address of host memory it can read (pinned by hipHostMalloc / registered), or
// NULL (pageable memory: copied instead)
template <class T>
const T *pinned_on_device(const T *p) {
    hipPointerAttribute_t at;
    if (!p || hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();  // pageable host memory reports an error: clear it
        return nullptr;
    }
    if (at.type != hipMemoryTypeHost || !at.devicePointer) return nullptr;
    const char *hp = static_cast<const char *>(at.hostPointer ? at.hostPointer : (const void *)p);
    return reinterpret_cast<const T *>(static_cast<const char *>(at.devicePointer) +
                                       (reinterpret_cast<const char *>(p) - hp));
}

// HQ_STEP_JOBS_SPIN_US: how long the jobs path's one waiting thread polls before it waits as the
// policy says (unset: the policy's poll, hq_worker_set_wait). Polling through the whole step
// (5000) gained nothing device-only and cost end to end: the poller takes a core from the
// producer's encode (tools/ab_spin.sh, step5 e2e 5.16 -> 5.37 ms)
uint32_t jobs_spin_us() {
    static const uint32_t us = [] {
        const char *v = std::getenv("HQ_STEP_JOBS_SPIN_US");
        return v ? (uint32_t)std::atoi(v) : 0u;
    }();
    return us;
}

// HQ_STEP_SINGLE_JOBS=0 in the environment: a single pinned sized step takes the copy path (A/B)
bool single_as_job_allowed() {
    static const bool on = [] {
        const char *v = std::getenv("HQ_STEP_SINGLE_JOBS");
        return !v || std::atoi(v) != 0;
    }();
    return on;
}

// HQ_STEP_ZERO_COPY=0 in the environment: pinned streams are copied like pageable ones (A/B)
bool zero_copy_allowed() {
    static const bool on = [] {
        const char *v = std::getenv("HQ_STEP_ZERO_COPY");
        return !v || std::atoi(v) != 0;
    }();
    return on;
}

// after the first pass B and its wait: input errors, an output region too small, the outputs
int finish(Run &r) {
    hq_dstep *d = r.d;
    hq_ctx *ctx = d->ctx;
    hq_dstep_out *out = r.out;
    if (r.rc) return restore(r, r.rc);
    const Layout &lay = *d->host_layout;
    if (lay.error == kErrScan) {
        // pass A's chained scan of the ReadyToRead places gave up on a stalled predecessor
        // (only the copy-out is affected, not a group's step): the layout again, and k_step_lite
        // writes every single ReadyToRead, as when pass A does not (spec_ready off). The layout
        // kept pass A's flags for this; its error word is cleared here
        r.k.spec_ready = 0;
        int rc = hq::check_hip(ctx, hipMemsetAsync(r.k.error, 0, 4, ctx->stream), "memset");
        if (rc) return restore(r, rc);
        pass_b(r);
        if (r.rc) return restore(r, r.rc);
    }
    if (lay.error) {              // no group state is written: pass A's is taken back
        const int rc = restore(r, HQ_OK);
        if (rc) return rc;
        out->input_error = lay.error;
        return HQ_E_INVAL;
    }
    if (lay.overflow) {           // grow the region and write the lists again
        // the new region first: if it cannot be had, the old one stays and the step is undone
        const size_t want = lay.total + lay.total / 2;
        void *grown = nullptr;
        int rc = hq::check_hip(ctx, hipHostMalloc(&grown, want, hipHostMallocDefault),
                               "hq_dstep pinned output");
        if (d->test_fail_regrow) {   // tests: the allocation failure path
            if (grown) (void)hipHostFree(grown);
            grown = nullptr;
            rc = hq::fail(ctx, HQ_E_NOMEM, "hq_dstep pinned output: injected failure");
        }
        if (rc) return restore(r, rc);
        if (d->host_out) (void)hipHostFree(d->host_out);
        d->host_out = grown;
        d->host_out_cap = want;
        r.k.out = static_cast<char *>(d->host_out);
        r.k.out_cap = want;
        r.k.spec_valid = 0;       // pass A's advance words went with the old region
        pass_b(r);
        if (r.rc) return restore(r, r.rc);
        if (lay.overflow || lay.error)
            return restore(r, hq::fail(ctx, HQ_E_STATE, "hq_dstep: output layout"));
    }
    const char *ho = static_cast<const char *>(d->host_out);
    if (lay.reserve) {            // the slot form (pass A's, or k_step_lite's after a regrow)
        out->ready_slots = reinterpret_cast<const hq_ready_compact *>(ho + r.k.slot_off);
        out->slot_counts = reinterpret_cast<const uint32_t *>(ho + r.k.cnt_off);
        out->n_tiles = (r.n + kSlotTile - 1) / kSlotTile;
        out->n_slotted = lay.len[kSlotted];
    }
    out->wait = d->last_wait;
    out->commits = lay.commit_column ? nullptr
                                     : reinterpret_cast<const hq_commit_event *>(ho + lay.off[kCommits]);
    out->commit_col = lay.commit_column == kColumn64
                          ? reinterpret_cast<const uint64_t *>(ho + lay.off[kCommits]) : nullptr;
    out->commit_adv = lay.commit_column == kColumn32
                          ? reinterpret_cast<const uint32_t *>(ho + lay.off[kCommits]) : nullptr;
    out->ready = lay.ready_compact ? nullptr
                                   : reinterpret_cast<const hq_ready_to_read *>(ho + lay.off[kReady]);
    out->ready_compact = lay.ready_compact
                             ? reinterpret_cast<const hq_ready_compact *>(ho + lay.off[kReady])
                             : nullptr;
    out->resps = reinterpret_cast<const hq_read_index_resp *>(ho + lay.off[kResps]);
    out->states = reinterpret_cast<const hq_state_change *>(ho + lay.off[kStates]);
    out->dropped = reinterpret_cast<const hq_dropped_read *>(ho + lay.off[kDropped]);
    out->deferred = reinterpret_cast<const uint64_t *>(ho + lay.off[kDeferred]);
    out->fallback = reinterpret_cast<const uint64_t *>(ho + lay.off[kFallback]);
    out->n_commits = lay.len[kCommits];
    out->n_ready = lay.len[kReady];
    out->n_resps = lay.len[kResps];
    out->n_states = lay.len[kStates];
    out->n_dropped = lay.len[kDropped];
    out->n_deferred = lay.len[kDeferred];
    out->n_fallback = lay.len[kFallback];
    out->decisions = lay.len[kDecisions];
    out->kernel_ns = r.t1 - r.t0;
    out->d2h_ns = now_ns() - r.t1;
    out->submit_ns = r.t_sub > r.t0 ? r.t_sub - r.t0 : 0;
    out->gpu_ns = r.gpu_ns;
    out->gpu_jobs = 1;
    return HQ_OK;
}

}  // namespace

int hq_dstep_run(hq_dstep *d, const hq_dstep_in *in, hq_dstep_out *out) {
    *out = hq_dstep_out{};
    if (in->n == 0) return HQ_OK;
    // A sized stream in pinned memory takes the jobs path as one job: pass A reads it in place in
    // one launch (the stream staged through LDS), where this path's chunked copies put the
    // first chunk's copy ahead of pass A and the last chunk's pass A behind the copies
    // (HQ_STEP_SINGLE_JOBS=0: this path, A/B)
    if ((in->sizes || in->sizes16) && in->bytes && single_as_job_allowed() &&
        pinned_on_device(in->bytes)) {
        int rc1 = HQ_OK;
        const int rc = hq_dstep_run_jobs(&d, in, out, &rc1, 1);
        return rc1 ? rc1 : rc;
    }
    Run r;
    r.d = d;
    r.in = in;
    r.out = out;
    hq_ctx *ctx = d->ctx;
    int rc = prepare(r, ctx->stream);
    if (rc) return rc;
    rc = hq::check_hip(ctx, hipEventRecord(d->ev_t0, ctx->stream), "event");
    if (!rc && d->tickets_dirty)
        rc = hq::check_hip(ctx, hipMemsetAsync(d->tickets, 0, kTickets * 4, ctx->stream), "memset");
    if (rc) return rc;
    d->tickets_dirty = true;
    r.timing = true;
    const uint64_t n = r.n, ne = r.ne, nb = r.nb;
    const bool stream = r.stream, sized = r.sized;
    const int chunks = r.chunks;
    uint64_t bound[kMaxChunks + 1];
    // (multiples of 256 inside: pass A's waves are the scan's, its tiles ready_tail's)
    for (int c = 0; c <= chunks; ++c)
        bound[c] = c == chunks ? n : (n * c / chunks) & ~uint64_t(255);
    if (chunks > 1 && !d->copy)       // the copy stream of the first chunked step
        rc = hq::check_hip(ctx, hipStreamCreateWithFlags(&d->copy, hipStreamNonBlocking),
                           "hq_dstep copy stream");
    // one chunk: every copy on the compute stream (nothing to overlap, no cross-stream waits)
    hipStream_t cs = chunks > 1 ? d->copy : ctx->stream;
    char *din = static_cast<char *>(d->in);
    auto h2d = [&](size_t off, const void *src, size_t bytes, hipStream_t s = nullptr) {
        if (!rc && bytes)
            rc = hq::check_hip(ctx, hipMemcpyAsync(din + off, src, bytes, hipMemcpyHostToDevice,
                                                   s ? s : cs), "hq_dstep H2D");
    };
    if (sized) {
        // handles and sizes, their scan (PackSize adds the totals as element n); then
        // the bytes in equal byte chunks, each followed by pass A over the groups whose bytes end
        // inside what has landed
        // every copy is queued before the first launch, event c behind chunk c's bytes; the
        // handles and sizes go on the compute stream ahead of their scan, the bytes on the copy
        // stream beside them (behind the sizes on one stream the first bytes copy started
        // 50-65 us after the sizes' copy ended)
        if (in->groups) h2d(0, in->groups, n * 4, ctx->stream);   // NULL: handles 0 .. n - 1
        if (in->sizes16) h2d(r.o_off, in->sizes16, n * 2, ctx->stream);
        else h2d(r.o_off, in->sizes, n * 4, ctx->stream);
        for (int c = 0; c < chunks && !rc; ++c) {
            const uint64_t lo = nb * c / chunks, hi = nb * (c + 1) / chunks;
            h2d(r.o_ev + lo, in->bytes + lo, hi - lo);
            if (chunks > 1 && !rc) rc = hq::check_hip(ctx, hipEventRecord(d->ev_in[c], cs), "event");
        }
        const hipcub::TransformInputIterator<uint64_t, PackSize,
                                             hipcub::CountingInputIterator<uint64_t>>
            packed_sizes(hipcub::CountingInputIterator<uint64_t>(0),
                         PackSize{reinterpret_cast<const uint32_t *>(din + r.o_off), n,
                                  in->sizes16 ? reinterpret_cast<const uint16_t *>(din + r.o_off)
                                              : nullptr});
        if (!rc) rc = hq::check_hip(ctx, hipcub::DeviceScan::ExclusiveSum(
                                              d->scan_tmp, r.tmp2, packed_sizes,
                                              const_cast<uint64_t *>(r.k.prefix), n + 1,
                                              ctx->stream),
                                    "hipcub scan");
        r.rc = rc;
        for (int c = 0; c < chunks && !r.rc; ++c) {
            const uint64_t lo = nb * c / chunks, hi = nb * (c + 1) / chunks;
            if (chunks > 1)
                r.rc = hq::check_hip(ctx, hipStreamWaitEvent(ctx->stream, d->ev_in[c], 0), "wait");
            r.k.own_lo = c == 0 ? 0 : lo + 1;
            r.k.own_hi = c + 1 == chunks ? UINT64_MAX : hi + 1;
            r.k.chunk = (uint32_t)c;
            launch_pass(r, false, 0, n);
        }
        rc = r.rc;
    }
    // inputs chunk by chunk, pass A of each chunk once it has landed
    for (int c = 0; c < chunks && !rc && !sized; ++c) {
        const uint64_t i0 = bound[c], i1 = bound[c + 1];
        h2d(i0 * 4, in->groups + i0, (i1 - i0) * 4);
        h2d(r.o_off + i0 * 8, in->offsets + i0, (i1 - i0 + 1) * 8);
        if (stream) {
            h2d(r.o_boff + i0 * 8, in->boffsets + i0, (i1 - i0 + 1) * 8);
            // the chunk's bytes (garbage offsets are the kernel's to reject: clamp the copy)
            const uint64_t lo = std::min(in->boffsets[i0], nb);
            const uint64_t hi = std::min(std::max(in->boffsets[i1], lo), nb);
            h2d(r.o_ev + lo, in->bytes + lo, hi - lo);
        } else {
            const uint64_t lo = std::min(in->offsets[i0], ne);
            const uint64_t hi = std::min(std::max(in->offsets[i1], lo), ne);
            h2d(r.o_ev + lo * sizeof(hq_event), in->events + lo, (hi - lo) * sizeof(hq_event));
        }
        if (chunks > 1) {
            if (!rc) rc = hq::check_hip(ctx, hipEventRecord(d->ev_in[c], cs), "event");
            if (!rc) rc = hq::check_hip(ctx, hipStreamWaitEvent(ctx->stream, d->ev_in[c], 0), "wait");
        }
        r.rc = rc;
        r.k.chunk = (uint32_t)c;
        launch_pass(r, false, i0, i1);
        rc = r.rc;
    }
    r.k.own_lo = 0;
    r.k.own_hi = UINT64_MAX;
    r.k.chunk = 0;
    // the wave sums' scan (hipcub for a large step; a small one's is the layout's workgroup)
    if (!rc && !r.small_scan)
        rc = hq::check_hip(ctx, hipcub::DeviceScan::ExclusiveSum(d->scan_tmp, r.tmp, d->wsum,
                                                                  d->scan, r.ws, ctx->stream),
                           "hipcub scan");
    r.rc = rc;
    r.stepped = !rc;
    pass_b(r);
    r.t1 = now_ns();
    return finish(r);
}

int hq_dstep_run_jobs(hq_dstep *const *ds, const hq_dstep_in *ins, hq_dstep_out *outs, int *rcs,
                      uint32_t count) {
    if (count == 0) return HQ_OK;
    if (count > kMaxJobs) return HQ_E_INVAL;
    hq_dstep *d0 = ds[0];
    hq_ctx *ctx = d0->ctx;
    hipStream_t s = ctx->stream;
    // HQ_STEP_JOBS_TRACE=1: the host phases of each call to stderr (where a step's time goes)
    static const bool trace = [] {
        const char *v = std::getenv("HQ_STEP_JOBS_TRACE");
        return v && std::atoi(v) != 0;
    }();
    uint64_t tp[6] = {now_ns(), 0, 0, 0, 0, 0};
    int rc = hq::check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    Run runs[kMaxJobs];
    uint32_t live[kMaxJobs], nl = 0;
    for (uint32_t j = 0; j < count; ++j) {
        outs[j] = hq_dstep_out{};
        rcs[j] = HQ_OK;
        if (ds[j]->ctx->device != ctx->device || !(ins[j].sizes || ins[j].sizes16) || !ins[j].bytes) {
            rcs[j] = hq::fail(ds[j]->ctx, HQ_E_INVAL, "hq_dstep_run_jobs: a sized stream step "
                                                      "on the first job's device");
            continue;
        }
        if (rc || ins[j].n == 0) {
            rcs[j] = rc;
            continue;
        }
        Run &r = runs[j];
        r.d = ds[j];
        r.in = &ins[j];
        r.out = &outs[j];
        rcs[j] = prepare(r, s, true);
        if (!rcs[j]) live[nl++] = j;
    }
    if (!nl) return rc;
    tp[1] = now_ns();
    if (!rc && d0->wait_clock) {  // (HQ_WAIT_CLOCK: the device's clock ahead of the step)
        d0->clock_host[1] = 0;
        hipLaunchKernelGGL(k_clock_stamp, dim3(1), dim3(64), 0, s, d0->clock_host + 1);
        rc = hq::check_hip(ctx, hipGetLastError(), "k_clock_stamp");
    }
    if (!rc) rc = hq::check_hip(ctx, hipEventRecord(d0->ev_t0, s), "event");
    if (!rc && d0->tickets_dirty)
        rc = hq::check_hip(ctx, hipMemsetAsync(d0->tickets, 0, kTickets * 4, s), "memset");
    d0->tickets_dirty = true;
    // the jobs' StepK, pinned and copied to the device ahead of the launches
    if (!rc && nl > d0->jobs_cap) {
        if (d0->jobs_host) (void)hipHostFree(d0->jobs_host);
        if (d0->jobs_dev) (void)hipFree(d0->jobs_dev);
        d0->jobs_host = d0->jobs_dev = nullptr;
        d0->jobs_host_dev = nullptr;
        d0->jobs_cap = 0;
        rc = hq::check_hip(ctx, hipHostMalloc(&d0->jobs_host, kMaxJobs * sizeof(StepK),
                                              hipHostMallocDefault), "hq_dstep jobs");
        if (!rc) rc = hq::check_hip(ctx, hipMalloc(&d0->jobs_dev, kMaxJobs * sizeof(StepK)),
                                    "hq_dstep jobs");
        if (!rc) {
            d0->jobs_cap = kMaxJobs;
            d0->jobs_host_dev = pinned_on_device(d0->jobs_host);
        }
    }
    bool small = true;
    uint64_t total_bytes = 0;
    // (a stream read in place: ByteReader's aligned 8-byte words and the staging's aligned 16-byte
    // blocks never cross a page, so no read leaves the caller's pages; a kernel launch acquires
    // at system scope, so the host's writes before the call are seen)
    // (the streams' pointers are checked after the sizes' scan is queued: the checks cost the
    // host ~1 us each, and the scan does not read the streams)
    for (uint32_t x = 0; x < nl && !rc; ++x) {
        Run &r = runs[live[x]];
        // sizes in pinned host memory are read by k_size_sums over the link: no copy per job
        // (16 workers' 256 KB size copies took 340 us one after another, with their gaps)
        if (r.in->sizes16) r.k.sizes16_src = pinned_on_device(r.in->sizes16);
        else r.k.sizes_src = pinned_on_device(r.in->sizes);
        d0->jobs_host[x] = r.k;
        small = small && r.small;
        total_bytes += r.nb;
    }
    // (k_size_sums reads the table from the pinned copy and writes it to the device: no copy is
    // queued ahead of the first launch, ~25 us of host time for a one-worker step)
    const bool table_first = !d0->jobs_host_dev;
    if (!rc && table_first)
        rc = hq::check_hip(ctx, hipMemcpyAsync(d0->jobs_dev, d0->jobs_host, nl * sizeof(StepK),
                                               hipMemcpyHostToDevice, s), "hq_dstep jobs");
    tp[2] = now_ns();
    // maps of jobs [x0, x1) onto workgroups of `per` groups (+ extra elements per job)
    auto map = [&](uint32_t x0, uint32_t x1, uint64_t per, uint64_t extra) {
        JobMap m{};
        m.ks = d0->jobs_dev;
        m.job0 = x0;
        m.count = x1 - x0;
        m.tickets = d0->tickets;
        m.blk0[0] = 0;
        for (uint32_t x = x0; x < x1; ++x)
            m.blk0[x - x0 + 1] = m.blk0[x - x0] + (uint32_t)((runs[live[x]].n + extra + per - 1) / per);
        return m;
    };
    auto launched = [&](const char *what) {
        if (!rc) rc = hq::check_hip(ctx, hipGetLastError(), what);
    };
    auto h2d = [&](void *dst, const void *src, size_t bytes, hipStream_t st) {
        if (!rc && bytes)
            rc = hq::check_hip(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st),
                               "hq_dstep H2D");
    };
    // The jobs' bytes in up to kMaxJobChunks chunks of whole jobs, copied on two copy streams
    // (jobs alternating: one copy's start-up gap overlaps the other's transfer), event c behind
    // chunk c on each. Queued in the order the device needs them, since each call takes the host
    // microseconds: the sizes' scan first (it reads pinned sizes over the link), the copies of
    // chunks 0 and 1, then pass A of chunk c (once its bytes have landed) before the copies of
    // chunk c + 2.
    for (hipStream_t *cs : {&d0->copy, &d0->copy2})
        if (!rc && !*cs)
            rc = hq::check_hip(ctx, hipStreamCreateWithFlags(cs, hipStreamNonBlocking),
                               "hq_dstep copy stream");
    uint32_t cend[kMaxJobChunks + 1] = {0};
    int nchunks = 0;
    bool zero_copy = false;
    // the sizes' first pass before anything else the device can start on
    for (uint32_t x = 0; x < nl; ++x) {
        const Run &r = runs[live[x]];
        char *din = static_cast<char *>(r.d->in);
        if (r.in->groups) h2d(din, r.in->groups, r.n * 4, s);
        if (r.in->sizes16) {
            if (!r.k.sizes16_src) h2d(din + r.o_off, r.in->sizes16, r.n * 2, s);
        } else if (!r.k.sizes_src) {
            h2d(din + r.o_off, r.in->sizes, r.n * 4, s);
        }
    }
    if (!rc) {
        // every job's stream in pinned host memory: pass A (and pass B) read it in place, in one
        // launch for all jobs, with no copy (HQ_STEP_ZERO_COPY=0: copied in chunks). The
        // streams' device addresses go into the table before the first launch, which carries it
        // to the device
        zero_copy = zero_copy_allowed();
        const uint8_t *zbytes[kMaxJobs] = {};
        for (uint32_t x = 0; x < nl && zero_copy; ++x) {
            zbytes[x] = pinned_on_device(runs[live[x]].in->bytes);
            zero_copy = zbytes[x] != nullptr || runs[live[x]].nb == 0;
        }
        if (zero_copy) {
            for (uint32_t x = 0; x < nl; ++x) {
                Run &r = runs[live[x]];
                if (zbytes[x]) r.k.bytes = zbytes[x];
                d0->jobs_host[x].bytes = r.k.bytes;
            }
        }
        if (zero_copy && table_first)   // (no device alias of the pinned table: copied again)
            rc = hq::check_hip(ctx, hipMemcpyAsync(d0->jobs_dev, d0->jobs_host, nl * sizeof(StepK),
                                                   hipMemcpyHostToDevice, s), "hq_dstep jobs");
    }
    JobMap sm = map(0, nl, kSizeTile, 1);
    for (uint32_t x = 0; x < nl; ++x)   // (a large job: its size tiles' totals get their own scan)
        if ((runs[live[x]].n + kSizeTile) / kSizeTile > kSizeApplyDirect) sm.bsum_scanned = 1;
    if (!rc) {
        // k_size_sums reads the table from its pinned copy and writes it to the device for the
        // launches behind it: no copy of its own (a blit launch and ~10 us of host time)
        JobMap pm = sm;
        if (!table_first) {
            pm.ks = d0->jobs_host_dev;
            pm.table_out = d0->jobs_dev;
        }
        hipLaunchKernelGGL(k_size_sums, dim3(pm.blk0[nl]), dim3(256), 0, s, pm);
        launched("k_size_sums");
    }
    if (zero_copy) {              // one chunk of all jobs, nothing to copy
        cend[nchunks = 1] = nl;
    } else {
        uint64_t acc = 0;
        uint32_t x = 0;
        while (nchunks < kMaxJobChunks && x < nl) {
            const uint64_t want = total_bytes * (uint64_t)(nchunks + 1) / kMaxJobChunks;
            do acc += runs[live[x++]].nb;
            while (x < nl && (nchunks + 1 == kMaxJobChunks || acc < want));
            cend[++nchunks] = x;
        }
    }
    auto copies = [&](int c) {
        if (c >= nchunks || zero_copy) return;
        for (uint32_t x = cend[c]; x < cend[c + 1]; ++x) {
            const Run &r = runs[live[x]];
            h2d(static_cast<char *>(r.d->in) + r.o_ev, r.in->bytes, r.nb,
                x % 2 ? d0->copy2 : d0->copy);
        }
        if (!rc) rc = hq::check_hip(ctx, hipEventRecord(d0->ev_in[c], d0->copy), "event");
        if (!rc) rc = hq::check_hip(ctx, hipEventRecord(d0->ev_in2[c], d0->copy2), "event");
    };
    copies(0);
    if (!rc && sm.bsum_scanned) {
        hipLaunchKernelGGL(k_bsum_scan_jobs, dim3(nl), dim3(1024), 0, s, sm);
        launched("k_bsum_scan_jobs");
    }
    if (!rc) {
        hipLaunchKernelGGL(k_size_apply, dim3(sm.blk0[nl]), dim3(256), 0, s, sm);
        launched("k_size_apply");
    }
    copies(1);
    for (int c = 0; c < nchunks && !rc; ++c) {
        const uint32_t x0 = cend[c], x1 = cend[c + 1];
        if (!zero_copy) {
            rc = hq::check_hip(ctx, hipStreamWaitEvent(s, d0->ev_in[c], 0), "wait");
            if (!rc) rc = hq::check_hip(ctx, hipStreamWaitEvent(s, d0->ev_in2[c], 0), "wait");
        }
        JobMap m = map(x0, x1, 256, 0);
        m.chunk = (uint32_t)c;
        if (!rc) rc = hq::pre_launch(ctx);
        if (!rc) {
            if (small) hipLaunchKernelGGL((k_step_jobs<false, true, 8>), dim3(m.blk0[x1 - x0]),
                                          dim3(256), 0, s, m);
            else hipLaunchKernelGGL((k_step_jobs<false, true, kDMembers>), dim3(m.blk0[x1 - x0]),
                                    dim3(256), 0, s, m);
            rc = hq::post_launch(ctx, "k_step_jobs<count>");
            for (uint32_t x = x0; x < x1 && !rc; ++x) runs[live[x]].stepped = true;
        }
        copies(c + 2);
    }
    // every job's layout (one workgroup each), k_step_lite and pass B over all jobs, one wait;
    // one large job (a single worker's step) scans its wave sums with hipcub, whose two launches
    // take ~14 us where the one workgroup took 117 for 1 M groups (147 Ki sums, profiles/r05e)
    const JobMap am = map(0, nl, 256, 0);
    Run &r0 = runs[live[0]];
    hq_dstep *dj = r0.d;          // (the one job's engine: not d0 when job 0 listed no group)
    if (!rc && nl == 1 && !r0.small_scan) {
        size_t tmp = 0;
        rc = hq::check_hip(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, dj->wsum, dj->scan,
                                                                  r0.ws, s), "hipcub scan size");
        // (scan_tmp holds the sizes' block totals, done with once pass A has its prefixes)
        if (!rc) rc = grow(ctx, &dj->scan_tmp, &dj->scan_tmp_cap, tmp, false, "hq_dstep scan tmp");
        if (!rc)
            rc = hq::check_hip(ctx, hipcub::DeviceScan::ExclusiveSum(dj->scan_tmp, tmp, dj->wsum,
                                                                      dj->scan, r0.ws, s),
                               "hipcub scan");
        if (!rc) {
            hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, s, dj->scan, r0.n, r0.nw, r0.k.error,
                               (uint64_t)dj->host_out_cap, r0.k.allow_column, want_events_of(r0.k),
                               dj->layout, dj->host_layout);
            launched("k_layout");
        }
    } else if (!rc) {
        hipLaunchKernelGGL(k_scan_layout_jobs, dim3(nl), dim3(kScanT), 0, s, d0->jobs_dev);
        launched("k_scan_layout_jobs");
    }
    if (!rc) {
        hipLaunchKernelGGL(k_step_lite_jobs, dim3(am.blk0[nl]), dim3(256), 0, s, am);
        launched("k_step_lite_jobs");
        for (uint32_t x = 0; x < nl && !rc; ++x) runs[live[x]].d->wsum_dirty = false;
        if (!rc) d0->tickets_dirty = false;
    }
    if (!rc) rc = hq::pre_launch(ctx);
    if (!rc) {
        if (small) hipLaunchKernelGGL((k_step_jobs<true, true, 8>), dim3(am.blk0[nl]), dim3(256),
                                      0, s, am);
        else hipLaunchKernelGGL((k_step_jobs<true, true, kDMembers>), dim3(am.blk0[nl]),
                                dim3(256), 0, s, am);
        rc = hq::post_launch(ctx, "k_step_jobs<write>");
    }
    if (!rc) rc = hq::check_hip(ctx, hipEventRecord(d0->ev_t1, s), "event");
    tp[3] = now_ns();
    uint64_t gpu_ns = 0;
    if (!rc) {
        rc = wait_stream(d0, s, "hq_dstep jobs sync", jobs_spin_us());
        if (!rc) gpu_ns = elapsed_ns(d0->ev_t0, d0->ev_t1);
    } else {                      // (a failed launch sequence leaves no copy behind either)
        (void)hipStreamSynchronize(s);
        for (hipStream_t cs : {d0->copy, d0->copy2})
            if (cs) (void)hipStreamSynchronize(cs);
    }
    const uint64_t t1 = now_ns();
    const hq_wait_clock w = d0->last_wait;   // (the one wait, before any job's own re-run)
    int first_rc = HQ_OK;
    for (uint32_t x = 0; x < nl; ++x) {
        Run &r = runs[live[x]];
        r.rc = rc;                // (restore: only the jobs whose pass A was launched)
        r.first = false;
        r.t1 = t1;
        r.t_sub = tp[3];
        r.gpu_ns = gpu_ns;
        rcs[live[x]] = finish(r);
        outs[live[x]].wait = w;
        outs[live[x]].gpu_jobs = nl;
        if (rcs[live[x]] && !first_rc) first_rc = rcs[live[x]];
    }
    if (trace) {
        tp[4] = t1;
        tp[5] = now_ns();
        std::fprintf(stderr, "hq_dstep_run_jobs %u jobs: prepare %.1f us, pointers + table %.1f, "
                             "submit %.1f, wait %.1f, outputs %.1f\n", nl,
                     (tp[1] - tp[0]) / 1e3, (tp[2] - tp[1]) / 1e3, (tp[3] - tp[2]) / 1e3,
                     (tp[4] - tp[3]) / 1e3, (tp[5] - tp[4]) / 1e3);
    }
    return first_rc;
}
