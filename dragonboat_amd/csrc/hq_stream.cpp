// hq_stream.cpp — the compact event stream of the device step worker (include/hipquorum.h
// "event streams"): a step's hq_event rows as one byte string per group, each event a header
// byte and LEB128 varints of only the fields its handler reads. The steady-state leader step
// (ReplicateResp / HeartbeatResp / proposals at the current term) takes 3-7 bytes per event
// instead of the 56-byte row, so that a host-fed step crosses PCIe ~10x faster. Host code: the
// encoder a producer holding rows can call (the wire decoder and a caller's own producer can
// write the stream directly) and the decoder the host worker uses for stream input; the device
// twin of the decoder is in hq_dstep.hip.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/hipquorum.h"
#include "hq_stream.h"

namespace {

// message types with a code of their own in the header (bits 3-5); 7 = the type follows
inline uint32_t type_code(uint32_t t) {
    switch (t) {
    case HQ_MSG_REPLICATE_RESP: return 0;
    case HQ_MSG_REQUEST_VOTE_RESP: return 1;
    case HQ_MSG_HEARTBEAT_RESP: return 2;
    case HQ_MSG_READ_INDEX: return 3;
    default: return 7;
    }
}
inline uint32_t code_type(uint32_t c) {
    static const uint32_t t[6] = {HQ_MSG_REPLICATE_RESP, HQ_MSG_REQUEST_VOTE_RESP,
                                  HQ_MSG_HEARTBEAT_RESP, HQ_MSG_READ_INDEX,
                                  HQ_MSG_REPLICATE_RESP, HQ_MSG_HEARTBEAT_RESP};
    return c < 6 ? t[c] : 0;
}

inline uint8_t *put(uint8_t *p, uint64_t v) {
    while (v >= 0x80) {
        *p++ = (uint8_t)(v | 0x80);
        v >>= 7;
    }
    *p++ = (uint8_t)v;
    return p;
}

inline bool get(const uint8_t *&p, const uint8_t *end, uint64_t &v) {
    v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
        if (p >= end) return false;
        const uint8_t b = *p++;
        v |= (uint64_t)(b & 0x7F) << shift;
        if (b < 0x80) return true;
    }
    return false;
}

// a group's stream state the codes refer back to: its previous message term, its previous
// ReplicateResp's log_index (code 4), its previous HeartbeatResp's ctx (code 5; 0 / 0 at first),
// and the previous message a run (code 6) repeats: last 1 = a ReplicateResp, 2 = a HeartbeatResp
// (written with codes 0 / 4 / 2 / 5 or in a run), 0 = none or another type; last_reject its bit
struct Prev {
    uint64_t term = 0, index = 0, hint = 0, high = 0;
    bool have_index = false;
    uint8_t last = 0, last_reject = 0;
    bool run_seq = false;          // (decoder) the current run's senders are run_from, + 1, ..
    uint32_t run_from = 0;
};

// Runs (code 6): the acks of a steady leader's followers repeat one another but for the sender
// (every follower acks the same index, every follower's heartbeat ack carries the same ctx). A
// run of 3..kRunMax messages that repeat the group's previous message (its type, term, reject
// and index / ctx) is one header, a count and the senders: 2 + m bytes for 1-byte senders
// instead of 2 m. At most kRunMax events per run, so that a run with 10-byte senders still fits
// the HQ_EVENT_STREAM_MAX bytes the encoder asks for before each unit.
constexpr uint32_t kRunMin = 3, kRunMax = 6;
constexpr uint32_t kCodeRun = 6;

inline uint8_t last_of(uint32_t code) {
    return code == 0 || code == 4 ? 1 : code == 2 || code == 5 ? 2 : 0;
}

// does row e repeat the group's previous message (a run member)?
template <class Ev>
inline bool repeats(const Ev &e, const Prev &pv) {
    if (!pv.last || e.kind != HQ_EV_MESSAGE || (e.reject != 0) != (pv.last_reject != 0) ||
        e.term != pv.term)
        return false;
    if (pv.last == 1) return e.type == HQ_MSG_REPLICATE_RESP && e.log_index == pv.index;
    return e.type == HQ_MSG_HEARTBEAT_RESP && e.hint == pv.hint && e.hint_high == pv.high;
}

// a run of m messages repeating the previous one, senders from[0..m); senders s0, s0 + 1, ..
// (a leader's followers acking in node order) as the consecutive form: header bit 7, m, s0
template <class From>
inline uint8_t *put_run(uint8_t *p, uint32_t m, From from) {
    const uint64_t f0 = from(0);
    bool seq = f0 + m <= 0xFFFFFFFFull;
    for (uint32_t j = 1; j < m && seq; ++j) seq = from(j) == f0 + j;
    if (seq) {
        *p++ = (uint8_t)(HQ_EV_MESSAGE | kCodeRun << 3 | 0x80);
        *p++ = (uint8_t)m;
        if (f0 < 0x80) *p++ = (uint8_t)f0;
        else p = put(p, f0);
        return p;
    }
    *p++ = (uint8_t)(HQ_EV_MESSAGE | kCodeRun << 3);
    *p++ = (uint8_t)m;                  // m <= kRunMax: one byte
    for (uint32_t j = 0; j < m; ++j) {
        const uint64_t f = from(j);
        if (f < 0x80) *p++ = (uint8_t)f;   // (a node id: one byte in the steady state)
        else p = put(p, f);
    }
    return p;
}

// the 1- and 2-byte varints inline
__attribute__((always_inline)) inline uint8_t *put_fast(uint8_t *p, uint64_t v) {
    if (v < 0x80) {
        *p = (uint8_t)v;
        return p + 1;
    }
    if (v < 0x4000) {
        p[0] = (uint8_t)(v | 0x80);
        p[1] = (uint8_t)(v >> 7);
        return p + 2;
    }
    return put(p, v);
}

// one event; returns the write position
template <class Ev>
inline uint8_t *encode(uint8_t *p, const Ev &e, Prev &pv) {
    const uint32_t kind = e.kind >= 1 && e.kind <= 5 ? e.kind : 0;   // 0: not a valid kind
    if (kind != HQ_EV_MESSAGE) {
        *p++ = (uint8_t)kind;
        if (kind == HQ_EV_READ) {
            p = put(p, e.hint);
            p = put_fast(p, e.hint_high);
        } else if (kind == HQ_EV_PROPOSE) {
            p = put_fast(p, e.log_index);
        }
        return p;
    }
    uint32_t code = type_code(e.type);
    if (code == 0) {
        if (pv.have_index && e.log_index == pv.index) code = 4;
        pv.index = e.log_index;
        pv.have_index = true;
    } else if (code == 2) {
        if (e.hint == pv.hint && e.hint_high == pv.high) code = 5;
        pv.hint = e.hint;
        pv.high = e.hint_high;
    }
    const bool same = e.term == pv.term;
    pv.last = last_of(code);
    pv.last_reject = e.reject ? 1 : 0;
    *p++ = (uint8_t)(HQ_EV_MESSAGE | code << 3 | (e.reject ? 0x40 : 0) | (same ? 0x80 : 0));
    if (code == 7) p = put(p, e.type);
    p = put_fast(p, e.from);
    if (!same) p = put(p, e.term);
    pv.term = e.term;
    if (code == 0 || code == 7) p = put_fast(p, e.log_index);
    if (code == 2 || code == 3 || code == 7) {
        p = put(p, e.hint);
        p = put_fast(p, e.hint_high);
    }
    return p;
}

// The event a compact record stands for. rc: records taken (1, or 5 for an escape), 0 when a
// record is malformed (an escape without its 4 records). ctx: the group's latest READ ctx.
inline int from16(const hq_event16 *r, uint64_t left, uint64_t ctx[2], hq_event &e) {
    if (r->kind & HQ_EV16_FULL) {
        if (left < 5) return 0;
        std::memcpy(&e, r + 1, sizeof e);
        if (e.kind == HQ_EV_READ) {
            ctx[0] = e.hint;
            ctx[1] = e.hint_high;
        }
        return 5;
    }
    e = hq_event{};
    e.kind = r->kind & 7;
    e.reject = (r->kind >> 3) & 1;
    if (e.kind == HQ_EV_READ) {
        e.hint = ctx[0] = r->value;
        e.hint_high = ctx[1] = r->term;
    } else if (e.kind == HQ_EV_PROPOSE) {
        e.log_index = r->value;
    } else if (e.kind == HQ_EV_MESSAGE) {
        e.type = r->type;
        e.from = r->from;
        e.term = r->term;
        if (e.type == HQ_MSG_HEARTBEAT_RESP || e.type == HQ_MSG_READ_INDEX) {
            if (r->kind & HQ_EV16_READ_CTX) {
                e.hint = ctx[0];
                e.hint_high = ctx[1];
            } else {
                e.hint = r->value;
            }
        } else {
            e.log_index = r->value;
        }
    }
    return 1;
}

// type_code of the types below 32
constexpr uint8_t kCode16[32] = {7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 0, 7, 1,
                                 7, 7, 2, 3, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7, 7};
static_assert(HQ_MSG_REPLICATE_RESP == 13 && HQ_MSG_REQUEST_VOTE_RESP == 15 &&
                  HQ_MSG_HEARTBEAT_RESP == 18 && HQ_MSG_READ_INDEX == 19,
              "kCode16 follows the message type numbers");

// one compact record (not an escape) straight into bytes: encode() of the event from16() makes
// of it, without the row
__attribute__((always_inline)) inline uint8_t *encode16(uint8_t *p, const hq_event16 &r, Prev &pv,
                                                       uint64_t ctx[2]) {
    const uint32_t k = r.kind & 7;
    if (k != HQ_EV_MESSAGE) {
        const uint32_t kind = k >= 1 && k <= 5 ? k : 0;
        *p++ = (uint8_t)kind;
        if (kind == HQ_EV_READ) {
            ctx[0] = r.value;
            ctx[1] = r.term;
            p = put(p, r.value);
            p = put_fast(p, r.term);
        } else if (kind == HQ_EV_PROPOSE) {
            p = put_fast(p, r.value);
        }
        return p;
    }
    uint32_t code = r.type < 32 ? kCode16[r.type] : 7u;
    uint64_t hint = 0, high = 0;
    if (code == 0) {
        if (pv.have_index && r.value == pv.index) code = 4;
        pv.index = r.value;
        pv.have_index = true;
    } else if (code == 2 || code == 3) {
        if (r.kind & HQ_EV16_READ_CTX) {
            hint = ctx[0];
            high = ctx[1];
        } else {
            hint = r.value;
        }
        if (code == 2) {
            if (hint == pv.hint && high == pv.high) code = 5;
            pv.hint = hint;
            pv.high = high;
        }
    }
    const bool same = r.term == pv.term;
    pv.last = last_of(code);
    pv.last_reject = (r.kind & 8) ? 1 : 0;
    const uint32_t hdr =
        HQ_EV_MESSAGE | code << 3 | ((r.kind & 8) ? 0x40u : 0u) | (same ? 0x80u : 0u);
    if (code != 7 && r.from < 0x80) {   // header and a 1-byte sender in one store
        const uint16_t w = (uint16_t)(hdr | (uint32_t)r.from << 8);
        std::memcpy(p, &w, 2);
        p += 2;
    } else {
        *p++ = (uint8_t)hdr;
        if (code == 7) p = put(p, r.type);
        p = put_fast(p, r.from);
    }
    if (!same) p = put(p, r.term);
    pv.term = r.term;
    if (code == 0 || code == 7) p = put_fast(p, r.value);
    if (code == 2 || code == 3 || code == 7) {
        p = put(p, hint);
        p = put_fast(p, high);
    }
    return p;
}

// does record r (not an escape) repeat the group's previous message? (repeats() of the event
// from16 makes of it, without the row)
__attribute__((always_inline)) inline bool repeats16(const hq_event16 &r, const Prev &pv,
                                                    const uint64_t ctx[2]) {
    if (!pv.last || (r.kind & 7) != HQ_EV_MESSAGE || ((r.kind >> 3) & 1) != pv.last_reject ||
        r.term != pv.term)
        return false;
    if (pv.last == 1) return r.type == HQ_MSG_REPLICATE_RESP && r.value == pv.index;
    if (r.type != HQ_MSG_HEARTBEAT_RESP) return false;
    return (r.kind & HQ_EV16_READ_CTX) ? ctx[0] == pv.hint && ctx[1] == pv.high
                                       : r.value == pv.hint && pv.high == 0;
}

// the records recs[k .. r1) that open with a run: its length (0 below kRunMin), the senders in
// from[] and the records it takes in *used (an escaped event is 5 records)
inline uint32_t run16(const hq_event16 *recs, uint64_t k, uint64_t r1, const Prev &pv,
                      const uint64_t ctx[2], uint64_t from[kRunMax], uint64_t *used) {
    uint32_t m = 0;
    uint64_t q = k;
    while (m < kRunMax && q < r1) {
        const hq_event16 &r = recs[q];
        if (r.kind & HQ_EV16_FULL) {      // an escaped event: its row
            if (r1 - q < 5) break;
            hq_event e;
            std::memcpy(&e, &r + 1, sizeof e);
            if (!repeats(e, pv)) break;
            from[m++] = e.from;
            q += 5;
            continue;
        }
        if (!repeats16(r, pv, ctx)) break;
        from[m++] = r.from;
        ++q;
    }
    *used = q - k;
    return m >= kRunMin ? m : 0;
}

// the rows events[e .. e1) that open with a run: its length (0 below kRunMin)
template <class Ev>
inline uint32_t run_rows(const Ev *events, uint64_t e, uint64_t e1, const Prev &pv) {
    uint32_t m = 0;
    while (m < kRunMax && e + m < e1 && repeats(events[e + m], pv)) ++m;
    return m >= kRunMin ? m : 0;
}

// the unit at row e of a group's rows [.., e1): a run of repeats of the previous message, or
// row e alone; returns the next row
template <class Ev>
inline uint64_t encode_unit(uint8_t *&p, const Ev *events, uint64_t e, uint64_t e1, Prev &pv) {
    if (pv.last) {
        const uint32_t m = run_rows(events, e, e1, pv);
        if (m) {
            p = put_run(p, m, [&](uint32_t j) { return events[e + j].from; });
            return e + m;
        }
    }
    p = encode(p, events[e], pv);
    return e + 1;
}

// groups [g0, g1) encoded at out (cap bytes), or into a growing scratch (grow != nullptr) from
// its byte pos0 on (a thread's later pieces follow its earlier ones there); the range's event
// count and byte count out, its last event's start relative to the range's first byte (locals
// until the end: threads encoding neighbouring ranges share no written cache line but their ends
// of `sizes`)
int enc16_range(const uint64_t *off, const hq_event16 *recs, uint32_t *sizes, uint64_t g0,
                uint64_t g1, std::vector<uint8_t> *grow, uint8_t *out, uint64_t cap,
                uint64_t *n_events, uint64_t *n_bytes, uint64_t *last_start = nullptr,
                uint64_t pos0 = 0, uint16_t *sizes16 = nullptr) {
    uint64_t pos = pos0, events = 0, ls = ~0ull;
    uint8_t *base = grow ? grow->data() : out;
    for (uint64_t i = g0; i < g1; ++i) {
        const uint64_t r0 = off[i], r1 = off[i + 1];
        if (r1 < r0) return HQ_E_INVAL;
        // room for the group's records at HQ_EVENT_STREAM_MAX each: no check per event
        const uint64_t need = (r1 - r0) * HQ_EVENT_STREAM_MAX;
        if (grow && grow->size() < pos + need) {
            grow->resize(std::max<size_t>(2 * grow->size(), pos + need + (1 << 20)));
            base = grow->data();
        }
        const bool roomy = grow || (cap >= pos && cap - pos >= need);
        const uint64_t p0 = pos;
        uint64_t ne = 0, ctx[2] = {0, 0};
        Prev pv;
        uint8_t *p = base + pos;
        uint8_t *lp = nullptr;
        for (uint64_t k = r0; k < r1; ++ne) {
            if (!roomy && (cap < (uint64_t)(p - base) || cap - (uint64_t)(p - base) <
                                                             HQ_EVENT_STREAM_MAX))
                return HQ_E_STATE;
            lp = p;
            if (pv.last) {                  // the next events repeat the previous message: a run
                uint64_t from[kRunMax], used = 0;
                const uint32_t m = run16(recs, k, r1, pv, ctx, from, &used);
                if (m) {
                    p = put_run(p, m, [&](uint32_t j) { return from[j]; });
                    k += used;
                    ne += m - 1;
                    continue;
                }
            }
            if (!(recs[k].kind & HQ_EV16_FULL)) {
                p = encode16(p, recs[k], pv, ctx);
                ++k;
                continue;
            }
            hq_event e;
            const int used = from16(recs + k, r1 - k, ctx, e);
            if (!used) return HQ_E_INVAL;
            k += used;
            p = encode(p, e, pv);
        }
        pos = (uint64_t)(p - base);
        if (lp) ls = (uint64_t)(lp - base) - pos0;
        if (ne > 0xFFFF || pos - p0 > 0xFFFF) return HQ_E_INVAL;
        if (sizes16) sizes16[i] = (uint16_t)(pos - p0);   // (2-byte words: bytes only)
        else sizes[i] = (uint32_t)ne | (uint32_t)(pos - p0) << 16;
        events += ne;
    }
    *n_events = events;
    *n_bytes = pos - pos0;
    if (last_start) *last_start = ls;
    return HQ_OK;
}

uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// phase clocks of the threaded encodes (hq_encode_stats_read)
struct EncodeClocks {
    std::atomic<uint64_t> calls{0}, tasks{0}, helped{0}, wall_ns{0}, encode_ns{0}, copy_ns{0},
        lag_ns{0}, max_lag_ns{0}, run_ns{0};
    void max_lag(uint64_t v) {
        uint64_t m = max_lag_ns.load(std::memory_order_relaxed);
        while (v > m && !max_lag_ns.compare_exchange_weak(m, v, std::memory_order_relaxed)) {
        }
    }
};
EncodeClocks g_clk;

// The threaded encodes' workers: created once and kept (a call spawning its T - 1 threads for
// each of its two phases paid tens of microseconds per thread in a process holding the GPU
// runtime's mappings). A call is one Job: indexes 1..T-1 are queued for the pool, the caller runs
// index 0 and then takes its own job's remaining indexes from the job's counter — never another
// call's tasks, so concurrent callers (one per step worker, execengine.go:675-690) do not wait
// behind each other's work. The Job is shared with every queue entry, so a pool thread that
// finishes the last index signals through memory the caller no longer owns alone (the caller
// returns only once every index has finished; an entry popped after that finds no index left).
class TaskPool {
public:
    ~TaskPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto &t : th_) t.join();
    }
    // gang: the T indexes run at the same time (each may wait for the others: a barrier inside
    // fn); the caller runs index 0 only and every other index gets a pool thread of its own (the
    // pool holds a thread per queued index of every live call, so the gang always assembles).
    // The pool holds at most kMaxThreads threads: a call whose indexes would need more waits
    // until earlier calls have finished (T - 1 <= kMaxThreads: callers clamp T). HQ_E_NOMEM when
    // a thread cannot be started (nothing of the call run).
    static constexpr uint32_t kMaxThreads = 256;
    int parallel_for(uint32_t T, const std::function<void(uint32_t)> &fn, bool gang = false) {
        if (T <= 1) {
            if (T) fn(0);
            return HQ_OK;
        }
        if (T - 1 > kMaxThreads) return HQ_E_INVAL;
#ifdef HQ_ENCODE_SPAWN          // A/B (tools/lib_encspawn): fresh threads for every phase
        std::vector<std::thread> th;
        for (uint32_t t = 1; t < T; ++t) th.emplace_back(fn, t);
        fn(0);
        for (auto &x : th) x.join();
        return HQ_OK;
#endif
        auto job = std::make_shared<Job>();
        job->fn = &fn;
        job->T = T;
        {
            std::unique_lock<std::mutex> lk(mu_);
            room_.wait(lk, [&] { return demand_ + (T - 1) <= kMaxThreads; });
            demand_ += T - 1;
            try {
                while (th_.size() < demand_) th_.emplace_back([this] { loop(); });
            } catch (const std::system_error &) {   // (no thread: the call does not start)
                demand_ -= T - 1;
                room_.notify_all();
                return HQ_E_NOMEM;
            }
            job->queued = now_ns();
            for (uint32_t t = 1; t < T; ++t) q_.push_back(job);
        }
        cv_.notify_all();
        run(*job, 0);
        for (; !gang;) {
            const uint32_t i = job->next.fetch_add(1);
            if (i >= T) break;
            run(*job, i);
        }
        {
            std::unique_lock<std::mutex> l(job->m);
            job->cv.wait(l, [&] { return job->done == job->T; });
        }
        std::lock_guard<std::mutex> lk(mu_);
        demand_ -= T - 1;
        room_.notify_all();
        return HQ_OK;
    }

private:
    struct Job {
        const std::function<void(uint32_t)> *fn = nullptr;
        uint32_t T = 0;
        std::atomic<uint32_t> next{1};
        uint64_t queued = 0;
        std::mutex m;
        std::condition_variable cv;
        uint32_t done = 0;
    };
    static void run(Job &j, uint32_t i) {
        const uint64_t t0 = now_ns();
        (*j.fn)(i);
        g_clk.run_ns += now_ns() - t0;
        g_clk.tasks++;
        std::lock_guard<std::mutex> l(j.m);
        if (++j.done == j.T) j.cv.notify_all();
    }
    void loop() {
        for (;;) {
            std::shared_ptr<Job> job;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;          // stop_ and nothing left
                job = std::move(q_.front());
                q_.pop_front();
            }
            const uint32_t i = job->next.fetch_add(1);
            if (i >= job->T) continue;           // the caller took it
            const uint64_t lag = now_ns() - job->queued;
            g_clk.lag_ns += lag;
            g_clk.max_lag(lag);
            g_clk.helped++;
            run(*job, i);
        }
    }
    std::mutex mu_;
    std::condition_variable cv_, room_;
    std::deque<std::shared_ptr<Job>> q_;
    std::vector<std::thread> th_;
    size_t demand_ = 0;
    bool stop_ = false;
};

// One event of a group's bytes at p (pv, run_left: the group's decoder state, as the encoder
// left it); false when the bytes do not hold a whole event
bool decode_one(const uint8_t *&p, const uint8_t *end, Prev &pv, uint64_t &run_left, hq_event &v) {
    std::memset(&v, 0, sizeof v);
    if (p >= end && !run_left) return false;
    const uint8_t h = run_left ? (uint8_t)0 : *p;
    if (run_left || ((h & 7) == HQ_EV_MESSAGE && ((h >> 3) & 7) == kCodeRun)) {
        // a run member: the group's previous message with another sender
        if (!run_left) {
            ++p;
            if (!pv.last || !get(p, end, run_left) || run_left == 0) return false;
            pv.run_seq = (h & 0x80) != 0;
            if (pv.run_seq) {          // the consecutive form: the first sender, the rest follow
                uint64_t f0;
                if (!get(p, end, f0) || f0 + run_left > 0xFFFFFFFFull) return false;
                pv.run_from = (uint32_t)f0;
            }
        }
        --run_left;
        v.kind = HQ_EV_MESSAGE;
        v.type = pv.last == 1 ? HQ_MSG_REPLICATE_RESP : HQ_MSG_HEARTBEAT_RESP;
        v.reject = pv.last_reject;
        v.term = pv.term;
        if (pv.last == 1) {
            v.log_index = pv.index;
        } else {
            v.hint = pv.hint;
            v.hint_high = pv.high;
        }
        if (pv.run_seq) {
            v.from = pv.run_from++;
            return true;
        }
        return get(p, end, v.from);
    }
    ++p;
    v.kind = h & 7;
    bool ok = true;
    if (v.kind == HQ_EV_READ) {
        ok = get(p, end, v.hint) && get(p, end, v.hint_high);
    } else if (v.kind == HQ_EV_PROPOSE) {
        ok = get(p, end, v.log_index);
    } else if (v.kind == HQ_EV_MESSAGE) {
        const uint32_t code = (h >> 3) & 7;
        uint64_t t = code_type(code);
        if (code == 7) ok = get(p, end, t);
        if (code == 4) ok = pv.have_index;  // repeats an index the group has not sent
        v.type = (uint32_t)t;
        v.reject = (h >> 6) & 1;
        ok = ok && get(p, end, v.from);
        if (ok && !(h & 0x80)) ok = get(p, end, pv.term);
        v.term = pv.term;
        if (ok && (code == 0 || code == 7)) ok = get(p, end, v.log_index);
        if (code == 4) v.log_index = pv.index;
        if (ok && (code == 2 || code == 3 || code == 7))
            ok = get(p, end, v.hint) && get(p, end, v.hint_high);
        if (code == 5) {
            v.hint = pv.hint;
            v.hint_high = pv.high;
        }
        if (ok && (code == 0 || code == 4)) {
            pv.index = v.log_index;
            pv.have_index = true;
        }
        if (ok && (code == 2 || code == 5)) {
            pv.hint = v.hint;
            pv.high = v.hint_high;
        }
        pv.last = last_of(code);
        pv.last_reject = (uint8_t)v.reject;
    }
    return ok;
}

// a pool thread's encode scratch is kept for its next call (first touched on its memory node),
// unless a call grew it past kKeepScratch: then it is released
constexpr size_t kKeepScratch = size_t(256) << 20;
// hq_events16_encode_sized_multi: chunks per encode thread (taken from a shared counter);
// HQ_ENC_CHUNKS overrides (1: one range per thread, the static split of round 5, for A/B)
uint64_t chunks_per_thread() {
    auto read = [] {
        const char *v = std::getenv("HQ_ENC_CHUNKS");
        return v && std::atoi(v) > 0 ? (uint64_t)std::atoi(v) : uint64_t(8);
    };
#ifdef HQ_ENC_PROF
    return read();                  // (probe builds: read at every call, for step-by-step A/B)
#else
    static const uint64_t k = read();
    return k;
#endif
}
inline void shrink_scratch(std::vector<uint8_t> &v) {
    if (v.capacity() > kKeepScratch) std::vector<uint8_t>().swap(v);
}

TaskPool &task_pool() {
    static TaskPool p;
    return p;
}

}  // namespace

extern "C" {

int hq_events16_encode_sized(uint64_t n_groups, const uint64_t *offsets16, const hq_event16 *recs,
                             uint8_t *out, uint64_t cap, uint32_t *sizes, uint64_t *n_events,
                             uint64_t *n_bytes, uint32_t threads) {
    if (!offsets16 || !n_events || !n_bytes || (n_groups && !sizes) ||
        (n_groups && offsets16[n_groups] > offsets16[0] && !recs))
        return HQ_E_INVAL;
    *n_events = *n_bytes = 0;
    if (n_groups && offsets16[n_groups] > offsets16[0] && !out) return HQ_E_STATE;
    const uint64_t nrec = n_groups ? offsets16[n_groups] - offsets16[0] : 0;
    const uint32_t T = (uint32_t)std::min<uint64_t>(
        {std::max(threads, 1u), std::max<uint64_t>(1, nrec / 4096), TaskPool::kMaxThreads + 1});
    // one thread encodes straight into out (through a scratch of its own it was slower: 59
    // against 38 ms for the step5 producer on one fresh thread, profiles/r05b/enc_probe.log)
    if (T <= 1)
        return enc16_range(offsets16, recs, sizes, 0, n_groups, nullptr, out, cap, n_events,
                           n_bytes);
    // the threads take chunks of the records as hq_events16_encode_sized_multi does (one job):
    // each chunk encoded into the taking thread's own scratch (first touched, so held on its
    // memory node, and reused by later calls), then copied into place once every chunk's byte
    // count is known (scratch handed from thread to thread ran the encode 2.5 x slower per record
    // on a 256-CPU host, profiles/r05b/enc_probe.log)
    hq_encode16_job job{};
    job.n_groups = n_groups;
    job.offsets16 = offsets16;
    job.recs = recs;
    job.out = out;
    job.cap = cap;
    job.sizes = sizes;
    const int rc = hq_events16_encode_sized_multi(&job, 1, T);
    if (rc) return rc;
    *n_events = job.n_events;
    *n_bytes = job.n_bytes;
    return HQ_OK;
}

int hq_events16_encode_sized_multi(hq_encode16_job *jobs, uint32_t count, uint32_t threads) {
    if (count && !jobs) return HQ_E_INVAL;
    // each job checked as its own call would; the records of the valid ones laid end to end
    std::vector<uint64_t> rec0(count + 1, 0);
    std::vector<uint32_t> live;
    int first = HQ_OK;
    for (uint32_t j = 0; j < count; ++j) {
        hq_encode16_job &b = jobs[j];
        b.n_events = b.n_bytes = 0;
        b.rc = HQ_OK;
        const uint64_t n = b.n_groups;
        if (!b.offsets16 || (n && !b.sizes && !b.sizes16) ||
            (n && b.offsets16[n] > b.offsets16[0] && !b.recs))
            b.rc = HQ_E_INVAL;
        else if (n && b.offsets16[n] > b.offsets16[0] && !b.out)
            b.rc = HQ_E_STATE;
        else if (n && b.offsets16[n] < b.offsets16[0])
            b.rc = HQ_E_INVAL;
        rec0[j + 1] = rec0[j] + (b.rc || !n ? 0 : b.offsets16[n] - b.offsets16[0]);
        if (!b.rc && n) live.push_back(j);
        if (b.rc && !first) first = b.rc;
    }
    const uint64_t R = rec0[count];
    const uint32_t T = (uint32_t)std::min<uint64_t>(
        {std::max(threads, 1u), std::max<uint64_t>(1, R / 4096), TaskPool::kMaxThreads + 1});
    if (live.empty()) return first;
    const uint64_t c0 = now_ns();
    // C chunks of about equal records, taken by the T threads from a shared counter: a thread
    // slowed by its core (a busy SMT sibling or a crowded host) takes fewer chunks instead of
    // holding the call back by a whole 1/T share
    const uint32_t C = (uint32_t)std::min<uint64_t>((uint64_t)T * chunks_per_thread(),
                                                    std::max<uint64_t>(T, R / 4096));
    // job j's groups split at the global record cuts R c / C (group boundaries): chunk c of the
    // job is groups [gc[j][c], gc[j][c + 1]), empty unless the job's records meet chunk c
    std::vector<std::vector<uint64_t>> gc(count);
    for (uint32_t j : live) {
        const hq_encode16_job &b = jobs[j];
        std::vector<uint64_t> &c = gc[j];
        c.assign(C + 1, 0);
        c[C] = b.n_groups;
        for (uint32_t t = 1; t < C; ++t) {
            const uint64_t cut = R * t / C;
            const uint64_t rel = cut <= rec0[j] ? 0 : std::min(cut - rec0[j], rec0[j + 1] - rec0[j]);
            const uint64_t want = b.offsets16[0] + rel;
            const uint64_t g = (uint64_t)(std::lower_bound(b.offsets16, b.offsets16 + b.n_groups, want) -
                                          b.offsets16);
            c[t] = std::min<uint64_t>(std::max<uint64_t>(c[t - 1], g), b.n_groups);
        }
    }
    struct Piece {
        uint32_t job, thread;                          // thread: whose scratch holds it
        uint64_t at, events, bytes, last_start, dst;   // at: offset in that scratch; dst: in out
        int rc;
    };
    std::vector<std::vector<Piece>> pieces(C);         // per chunk, one per job it meets
    std::atomic<uint32_t> next{0};
    std::mutex bm;
    std::condition_variable bcv;
    uint32_t arrived = 0;
    uint64_t c1 = 0;
    std::vector<uint8_t> fits(count, 1);
#ifdef HQ_ENC_PROF   // probe builds only: each range's start and arrival at the barrier (stderr)
    std::vector<uint64_t> p_start(T, 0), p_arrive(T, 0);
#endif
    const int prc = task_pool().parallel_for(T, [&](uint32_t t) {
        thread_local std::vector<uint8_t> scratch;
        uint64_t pos = 0;
#ifdef HQ_ENC_PROF
        p_start[t] = now_ns();
#endif
        for (;;) {
            const uint32_t c = next.fetch_add(1, std::memory_order_relaxed);
            if (c >= C) break;
            std::vector<Piece> &ps = pieces[c];
            for (uint32_t j : live) {
                const uint64_t g0 = gc[j][c], g1 = gc[j][c + 1];
                if (g0 >= g1) continue;
                const hq_encode16_job &b = jobs[j];
                Piece pc{j, t, pos, 0, 0, ~0ull, 0, HQ_OK};
                // (the piece follows the thread's earlier pieces in its scratch)
                pc.rc = enc16_range(b.offsets16, b.recs, b.sizes, g0, g1, &scratch, nullptr, 0,
                                    &pc.events, &pc.bytes, &pc.last_start, pos, b.sizes16);
                if (pc.rc) pc.bytes = 0;
                pos += pc.bytes;
                ps.push_back(pc);
            }
        }
#ifdef HQ_ENC_PROF
        p_arrive[t] = now_ns();
#endif
        {
            std::unique_lock<std::mutex> lk(bm);
            if (++arrived == T) {
                // every piece in: each job's totals, its capacity rule and its pieces' places
                c1 = now_ns();
                std::vector<uint64_t> total(count, 0), last(count, ~0ull);
                for (uint32_t u = 0; u < C; ++u) {       // (chunk order: each job's byte order)
                    for (Piece &pc : pieces[u]) {
                        hq_encode16_job &b = jobs[pc.job];
                        if (pc.rc && !b.rc) b.rc = pc.rc;
                        if (pc.last_start != ~0ull) last[pc.job] = total[pc.job] + pc.last_start;
                        pc.dst = total[pc.job];
                        total[pc.job] += pc.bytes;
                        b.n_events += pc.events;
                    }
                }
                for (uint32_t j : live) {
                    hq_encode16_job &b = jobs[j];
                    fits[j] = last[j] == ~0ull ||
                              (b.cap >= last[j] && b.cap - last[j] >= HQ_EVENT_STREAM_MAX);
                    if (!b.rc && !fits[j]) b.rc = HQ_E_STATE;
                    b.n_bytes = b.rc ? 0 : total[j];
                    if (b.rc) b.n_events = 0;
                }
                bcv.notify_all();
            } else {
                bcv.wait(lk, [&] { return arrived == T; });
            }
        }
        for (uint32_t c = 0; c < C; ++c)                // the pieces this thread encoded
            for (const Piece &pc : pieces[c]) {
                const hq_encode16_job &b = jobs[pc.job];
                if (pc.thread == t && !b.rc && pc.bytes)
                    std::memcpy(b.out + pc.dst, scratch.data() + pc.at, pc.bytes);
            }
        shrink_scratch(scratch);
    }, true);
    if (prc) {                    // (nothing encoded)
        for (uint32_t j : live) jobs[j].rc = prc;
        return prc;
    }
    first = HQ_OK;
    for (uint32_t j = 0; j < count && !first; ++j) first = jobs[j].rc;
    const uint64_t c2 = now_ns();
#ifdef HQ_ENC_PROF
    {   // per call: wall, phase 1, the ranges' latest start and earliest / latest arrival (us
        // after the call's start), and the slowest range's own encode time
        uint64_t s_max = 0, a_min = ~0ull, a_max = 0, d_max = 0, d_min = ~0ull;
        for (uint32_t t = 0; t < T; ++t) {
            s_max = std::max(s_max, p_start[t] - c0);
            a_min = std::min(a_min, p_arrive[t] - c0);
            a_max = std::max(a_max, p_arrive[t] - c0);
            d_max = std::max(d_max, p_arrive[t] - p_start[t]);
            d_min = std::min(d_min, p_arrive[t] - p_start[t]);
        }
        std::fprintf(stderr, "encprof T=%u wall=%.1f phase1=%.1f start_max=%.1f arrive=%.1f..%.1f "
                             "range_us=%.1f..%.1f\n", T, (c2 - c0) / 1e3, (c1 - c0) / 1e3,
                     s_max / 1e3, a_min / 1e3, a_max / 1e3, d_min / 1e3, d_max / 1e3);
    }
#endif
    g_clk.calls++;
    g_clk.encode_ns += c1 - c0;
    g_clk.copy_ns += c2 - c1;
    g_clk.wall_ns += c2 - c0;
    return first;
}

int hq_encode_stats_read(hq_encode_stats *out, int reset) {
    if (!out) return HQ_E_INVAL;
    auto take = [&](std::atomic<uint64_t> &a) { return reset ? a.exchange(0) : a.load(); };
    out->calls = take(g_clk.calls);
    out->tasks = take(g_clk.tasks);
    out->helped = take(g_clk.helped);
    out->wall_ns = take(g_clk.wall_ns);
    out->encode_ns = take(g_clk.encode_ns);
    out->copy_ns = take(g_clk.copy_ns);
    out->lag_ns = take(g_clk.lag_ns);
    out->max_lag_ns = take(g_clk.max_lag_ns);
    out->run_ns = take(g_clk.run_ns);
    return HQ_OK;
}

int hq_events_to16(uint64_t n_groups, const uint64_t *offsets, const hq_event *events,
                   hq_event16 *out, uint64_t cap, uint64_t *offsets16) {
    if (!offsets || !offsets16 || (n_groups && offsets[n_groups] > offsets[0] && !events))
        return HQ_E_INVAL;
    uint64_t k = 0;
    offsets16[0] = 0;
    for (uint64_t i = 0; i < n_groups; ++i) {
        if (offsets[i + 1] < offsets[i]) return HQ_E_INVAL;
        uint64_t ctx[2] = {0, 0};
        for (uint64_t j = offsets[i]; j < offsets[i + 1]; ++j) {
            const hq_event &e = events[j];
            hq_event16 r{};
            bool fits = e.kind >= 1 && e.kind <= 5 && e.reject <= 1;
            r.kind = (uint8_t)(e.kind | (e.reject ? 8u : 0u));
            if (fits && e.kind == HQ_EV_READ) {
                fits = e.hint_high >> 32 == 0;
                r.value = e.hint;
                r.term = (uint32_t)e.hint_high;
            } else if (fits && e.kind == HQ_EV_PROPOSE) {
                r.value = e.log_index;
            } else if (fits && e.kind == HQ_EV_MESSAGE) {
                fits = e.type < 256 && e.from >> 16 == 0 && e.term >> 32 == 0;
                r.type = (uint8_t)e.type;
                r.from = (uint16_t)e.from;
                r.term = (uint32_t)e.term;
                if (e.type == HQ_MSG_HEARTBEAT_RESP || e.type == HQ_MSG_READ_INDEX) {
                    if (e.hint == ctx[0] && e.hint_high == ctx[1] && (e.hint | e.hint_high)) {
                        r.kind |= HQ_EV16_READ_CTX;
                    } else {
                        fits = fits && e.hint_high == 0;
                        r.value = e.hint;
                    }
                } else if (e.type == HQ_MSG_REPLICATE_RESP || e.type == HQ_MSG_REQUEST_VOTE_RESP) {
                    r.value = e.log_index;   // (a RequestVoteResp carries nothing more)
                } else {                     // another type: log_index, hint, hint_high
                    fits = fits && e.hint == 0 && e.hint_high == 0;
                    r.value = e.log_index;
                }
            }
            if (fits) {
                if (k + 1 > cap) return HQ_E_STATE;
                out[k++] = r;
            } else {
                if (k + 5 > cap) return HQ_E_STATE;
                out[k] = hq_event16{};
                out[k].kind = (uint8_t)HQ_EV16_FULL;
                std::memset(out + k + 1, 0, 4 * sizeof(hq_event16));
                std::memcpy(out + k + 1, &e, sizeof e);
                k += 5;
            }
            if (e.kind == HQ_EV_READ) {
                ctx[0] = e.hint;
                ctx[1] = e.hint_high;
            }
        }
        offsets16[i + 1] = k;
    }
    return HQ_OK;
}

}  // extern "C"

namespace hqs {
namespace {
template <class Ev>
uint8_t *encode_events_of(uint8_t *p, const uint8_t *end, const Ev *ev, uint64_t n) {
    Prev pv;
    for (uint64_t e = 0; e < n;) {
        if ((uint64_t)(end - p) < HQ_EVENT_STREAM_MAX) return nullptr;
        e = encode_unit(p, ev, e, n, pv);
    }
    return p;
}
}  // namespace
uint8_t *encode_group(uint8_t *p, const uint8_t *end, const hq_event *ev, uint64_t n) {
    return encode_events_of(p, end, ev, n);
}
uint8_t *encode_group(uint8_t *p, const uint8_t *end, const WireEvent *ev, uint64_t n) {
    return encode_events_of(p, end, ev, n);
}
}  // namespace hqs

extern "C" {

int hq_events_encode(uint64_t n_groups, const uint64_t *offsets, const hq_event *events,
                     uint8_t *out, uint64_t cap, uint64_t *boffsets) {
    if (!offsets || !boffsets || (n_groups && offsets[n_groups] > offsets[0] && !events))
        return HQ_E_INVAL;
    uint8_t *p = out, *const end = out ? out + cap : nullptr;
    boffsets[0] = 0;
    for (uint64_t i = 0; i < n_groups; ++i) {
        Prev pv;
        for (uint64_t e = offsets[i]; e < offsets[i + 1];) {
            if (!out || (uint64_t)(end - p) < HQ_EVENT_STREAM_MAX) return HQ_E_STATE;
            e = encode_unit(p, events, e, offsets[i + 1], pv);
        }
        boffsets[i + 1] = (uint64_t)(p - out);
    }
    return HQ_OK;
}

int hq_events_encode_sized(uint64_t n_groups, const uint64_t *offsets, const hq_event *events,
                           uint8_t *out, uint64_t cap, uint32_t *sizes, uint64_t *n_bytes) {
    if (!offsets || !sizes || !n_bytes || (n_groups && offsets[n_groups] > offsets[0] && !events))
        return HQ_E_INVAL;
    uint8_t *p = out, *const end = out ? out + cap : nullptr;
    for (uint64_t i = 0; i < n_groups; ++i) {
        if (offsets[i + 1] < offsets[i] || offsets[i + 1] - offsets[i] > 0xFFFF) return HQ_E_INVAL;
        uint8_t *const g0 = p;
        Prev pv;
        for (uint64_t e = offsets[i]; e < offsets[i + 1];) {
            if (!out || (uint64_t)(end - p) < HQ_EVENT_STREAM_MAX) return HQ_E_STATE;
            e = encode_unit(p, events, e, offsets[i + 1], pv);
        }
        if (p - g0 > 0xFFFF) return HQ_E_INVAL;
        sizes[i] = (uint32_t)(offsets[i + 1] - offsets[i]) | (uint32_t)(p - g0) << 16;
    }
    *n_bytes = (uint64_t)(p - out);
    return HQ_OK;
}

int hq_events_decode(uint64_t n_groups, const uint64_t *offsets, const uint64_t *boffsets,
                     const uint8_t *bytes, hq_event *events) {
    if (!offsets || !boffsets || !events) return HQ_E_INVAL;
    for (uint64_t i = 0; i < n_groups; ++i) {
        const uint8_t *p = bytes + boffsets[i], *const end = bytes + boffsets[i + 1];
        Prev pv;
        uint64_t run_left = 0;          // events still to come in the current run
        for (uint64_t e = offsets[i]; e < offsets[i + 1]; ++e)
            if (!decode_one(p, end, pv, run_left, events[e])) return HQ_E_INVAL;
        if (p != end || run_left) return HQ_E_INVAL;
    }
    return HQ_OK;
}

int hq_events_count(uint64_t n_groups, const uint64_t *boffsets, const uint8_t *bytes,
                    uint64_t *offsets) {
    if (!boffsets || !offsets || (n_groups && boffsets[n_groups] > boffsets[0] && !bytes))
        return HQ_E_INVAL;
    offsets[0] = 0;
    for (uint64_t i = 0; i < n_groups; ++i) {
        if (boffsets[i + 1] < boffsets[i]) return HQ_E_INVAL;
        const uint8_t *p = bytes + boffsets[i], *const end = bytes + boffsets[i + 1];
        Prev pv;
        uint64_t run_left = 0, n = 0;
        hq_event v;
        while (p < end || run_left) {
            if (!decode_one(p, end, pv, run_left, v)) return HQ_E_INVAL;
            ++n;
        }
        offsets[i + 1] = offsets[i] + n;
    }
    return HQ_OK;
}

}  // extern "C"
