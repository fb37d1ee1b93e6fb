// hq_wire.cpp — the step worker's input from the wire: raftpb.MessageBatch bytes decoded into
// hq_event rows (include/hipquorum.h "wire decode").
//
// The reference path is TCPTransport.serveConn -> Transport.handleRequest
// (internal/transport/transport.go:289-316: deployment id and binary version checks) ->
// messageHandler.HandleMessageBatch (nodehost.go:2021-2061: SnapshotReceived handled aside, a
// message for a cluster this host does not run dropped, the rest queued per cluster) ->
// node.handleReceivedMessages (node.go:1257-1287) draining the queue into Peer.Handle in arrival
// order, inside node.handleEvents' order (node.go:1113-1157: the local ReadIndex first, then the
// received messages, then the ticks, then the proposals). The bytes are the protobuf encoding of
// raftpb/raft.proto:154-168 (Message) and :191-196 (MessageBatch) as raft.pb.go marshals them
// (Message.MarshalTo raft.pb.go:2232-2300, MessageBatch.MarshalTo :2417-2445); the decoder
// accepts any valid proto2 encoding of them (fields in any order, unknown fields skipped, as
// Message.Unmarshal raft.pb.go:4831 / raft_optimized.go:654 do).
#include <cstring>
#include <new>
#include <string>
#include <utility>
#include <vector>

#include "../../include/hipquorum.h"
#include "hq_stream.h"

namespace {

constexpr uint32_t kSnapshotReceived = 22;   // raft.proto MessageType

struct Reader {
    const uint8_t *p, *end;
    const char *err = nullptr;

    bool varint(uint64_t &v) {
        if (p < end && *p < 0x80) {                   // the common one-byte varint
            v = *p++;
            return true;
        }
        v = 0;
        for (int shift = 0; shift < 64; shift += 7) {
            if (p >= end) {
                err = "unexpected end of data in a varint";
                return false;
            }
            const uint8_t b = *p++;
            v |= (uint64_t)(b & 0x7F) << shift;
            if (b < 0x80) return true;
        }
        err = "varint overflows 64 bits";
        return false;
    }
    // skip a field of the given wire type (skipRaft, raft.pb.go:6293)
    bool skip(uint32_t wt) {
        uint64_t n = 0;
        switch (wt) {
        case 0: return varint(n);
        case 1: n = 8; break;
        case 2:
            if (!varint(n)) return false;
            break;
        case 5: n = 4; break;
        default:
            err = "unsupported wire type (groups are not part of raft.proto)";
            return false;
        }
        if ((uint64_t)(end - p) < n) {
            err = "unexpected end of data in a field";
            return false;
        }
        p += n;
        return true;
    }
    bool bytes(const uint8_t *&b, uint64_t &n) {
        if (!varint(n)) return false;
        if ((uint64_t)(end - p) < n) {
            err = "unexpected end of data in a length-delimited field";
            return false;
        }
        b = p;
        p += n;
        return true;
    }
};

// raftpb.Message (raft.proto:154-168) into the fields the quorum path reads
int decode_message(const uint8_t *b, size_t len, hq_wire_message *m, std::string &err) {
    std::memset(m, 0, sizeof(*m));
    m->ev.kind = HQ_EV_MESSAGE;
    Reader r{b, b + len};
    while (r.p < r.end) {
        uint64_t tag;
        if (!r.varint(tag)) break;
        const uint32_t field = (uint32_t)(tag >> 3), wt = (uint32_t)(tag & 7);
        if (field == 0) {
            r.err = "illegal field number 0";
            break;
        }
        uint64_t v = 0;
        if (field <= 10 || field == 13) {              // the varint fields
            if (wt != 0) {
                err = "Message: wrong wire type " + std::to_string(wt) + " for field " +
                      std::to_string(field);
                return HQ_E_INVAL;
            }
            if (!r.varint(v)) break;
        }
        switch (field) {
        case 1: m->ev.type = (uint32_t)v; break;      // type
        case 2: m->to = v; break;
        case 3: m->ev.from = v; break;
        case 4: m->cluster_id = v; break;
        case 5: m->ev.term = v; break;
        case 6: m->log_term = v; break;
        case 7: m->ev.log_index = v; break;
        case 8: m->commit = v; break;
        case 9: m->ev.reject = v != 0; break;
        case 10: m->ev.hint = v; break;
        case 13: m->ev.hint_high = v; break;
        case 11:                                       // repeated Entry entries
        case 12: {                                     // Snapshot snapshot
            if (wt != 2) {
                err = "Message: wrong wire type " + std::to_string(wt) + " for field " +
                      std::to_string(field);
                return HQ_E_INVAL;
            }
            const uint8_t *x;
            uint64_t n;
            if (!r.bytes(x, n)) break;
            if (field == 11) m->n_entries++;
            else m->has_snapshot = 1;
            break;
        }
        default:
            r.skip(wt);
        }
        if (r.err) break;
    }
    if (r.err) {
        err = std::string("Message: ") + r.err;
        return HQ_E_INVAL;
    }
    return HQ_OK;
}

// one event of the step as the wire keeps it (hq_stream.h): a decoded message's fields, or a
// local event's
struct Rec : hqs::WireEvent {
    hq_event event() const {
        hq_event e{};
        e.kind = kind;
        e.type = type;
        e.from = from;
        e.term = term;
        e.log_index = log_index;
        e.hint = hint;
        e.hint_high = hint_high;
        e.reject = reject;
        return e;
    }
};
static_assert(sizeof(Rec) == 56, "56-byte wire records");

// the one-byte varint, else the loop; p < end on entry
inline bool varint_at(const uint8_t *&p, const uint8_t *end, uint64_t &v) {
    if (*p < 0x80) {
        v = *p++;
        return true;
    }
    v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
        if (p >= end) return false;
        const uint8_t b = *p++;
        v |= (uint64_t)(b & 0x7F) << shift;
        if (b < 0x80) return true;
    }
    return false;
}

// A Message in the field order raft.pb.go Message.MarshalTo writes (:2232-2296): every field of
// 1-10 with its tag in order, entries (11) repeated, the snapshot (12, always: nullable=false),
// hint_high (13), nothing else. false: not that layout (the general decoder takes it from the
// start, any field order); *entries counts field 11
inline bool decode_marshal_order(const uint8_t *p, const uint8_t *end, Rec &r, uint64_t &cluster,
                                 uint32_t &entries) {
    uint64_t v[10];
    // fields 1-10: tag (f + 1) << 3, a varint — unrolled, so that each field's tag is a constant
    // and each field's varint length has a branch of its own to predict (the lengths differ by
    // field and repeat from message to message)
#pragma GCC unroll 10
    for (uint32_t f = 0; f < 10; ++f) {
        if (p >= end || *p != (uint8_t)((f + 1) << 3)) return false;
        if (++p >= end || !varint_at(p, end, v[f])) return false;
    }
    entries = 0;
    while (p < end && *p == 0x5a) {                // entries: counted, not decoded
        uint64_t n;
        if (++p >= end || !varint_at(p, end, n) || (uint64_t)(end - p) < n) return false;
        p += n;
        ++entries;
    }
    uint64_t n, high;
    if (p >= end || *p != 0x62) return false;      // the snapshot
    if (++p >= end || !varint_at(p, end, n) || (uint64_t)(end - p) < n) return false;
    p += n;
    if (p >= end || *p != 0x68) return false;      // hint_high, the last field
    if (++p >= end || !varint_at(p, end, high) || p != end) return false;
    r.kind = HQ_EV_MESSAGE;
    r.type = (uint32_t)v[0];
    r.from = v[2];
    cluster = v[3];
    r.term = v[4];
    r.log_index = v[6];
    r.reject = v[8] != 0;
    r.hint = v[9];
    r.hint_high = high;
    return true;
}

// MessageBatch (raft.proto:191-196): every Message handed to sink(bytes, len) in order (sink
// returns an HQ_ status), the other fields into *bi. Any field order; unknown fields skipped.
template <class Sink>
int parse_batch(const uint8_t *bytes, size_t len, hq_wire_batch_info *bi, uint64_t *count,
                Sink &&sink) {
    *bi = hq_wire_batch_info{};
    *count = 0;
    Reader r{bytes, bytes + len};
    while (r.p < r.end) {
        // the common case first: a Message (tag 0x0a) shorter than 128 bytes
        if (r.end - r.p >= 2 && r.p[0] == 0x0a && r.p[1] < 0x80) {
            const uint64_t n = r.p[1];
            if ((uint64_t)(r.end - r.p - 2) < n) {
                r.err = "unexpected end of data in a length-delimited field";
                break;
            }
            const uint8_t *m = r.p + 2;
            r.p = m + n;
            const int rc = sink(m, (size_t)n);
            if (rc) return rc;
            ++*count;
            continue;
        }
        uint64_t tag;
        if (!r.varint(tag)) break;
        const uint32_t field = (uint32_t)(tag >> 3), wt = (uint32_t)(tag & 7);
        if (field == 1 && wt == 2) {                  // repeated Message requests
            const uint8_t *m;
            uint64_t n;
            if (!r.bytes(m, n)) break;
            const int rc = sink(m, (size_t)n);
            if (rc) return rc;
            ++*count;
        } else if (field == 2 && wt == 0) {           // deployment_id
            if (!r.varint(bi->deployment_id)) break;
        } else if (field == 3 && wt == 2) {           // source_address
            const uint8_t *a;
            uint64_t n;
            if (!r.bytes(a, n)) break;
            bi->source_address_len = n;
        } else if (field == 4 && wt == 0) {           // bin_ver
            uint64_t v;
            if (!r.varint(v)) break;
            bi->bin_ver = (uint32_t)v;
        } else if (field == 0) {
            r.err = "illegal field number 0";
            break;
        } else if (field <= 4) {
            r.err = "wrong wire type for a MessageBatch field";
            break;
        } else if (!r.skip(wt)) {
            break;
        }
    }
    if (r.err) return HQ_E_INVAL;
    bi->n_messages = *count;
    return HQ_OK;
}

// cluster id -> index in order of first appearance: open addressing, linear probing (a step
// looks every message's cluster up once; a node-based map costs more than the decode)
class ClusterIndex {
  public:
    void clear() {
        for (uint32_t i : used_) slots_[i].key = kEmpty;
        used_.clear();
        has_empty_ = false;
    }
    // the value of id, or false
    bool find(uint64_t id, uint32_t *v) const {
        if (id == kEmpty) {
            if (has_empty_) *v = empty_val_;
            return has_empty_;
        }
        if (slots_.empty()) return false;
        const uint64_t mask = slots_.size() - 1;
        for (uint64_t i = hash(id) & mask;; i = (i + 1) & mask) {
            if (slots_[i].key == id) {
                *v = slots_[i].val;
                return true;
            }
            if (slots_[i].key == kEmpty) return false;
        }
    }
    void prefetch(uint64_t id) const {
        if (!slots_.empty()) __builtin_prefetch(&slots_[hash(id) & (slots_.size() - 1)]);
    }
    size_t size() const { return used_.size() + has_empty_; }
    // the index of id, inserting next if new (*fresh = true)
    uint32_t find_or_add(uint64_t id, uint32_t next, bool *fresh) {
        if ((used_.size() + 1) * 2 > slots_.size()) rehash(slots_.empty() ? 1024 : slots_.size() * 2);
        const uint64_t mask = slots_.size() - 1;
        for (uint64_t i = hash(id) & mask;; i = (i + 1) & mask) {
            if (slots_[i].key == id && id != kEmpty) {
                *fresh = false;
                return slots_[i].val;
            }
            if (slots_[i].key == kEmpty) {
                if (id == kEmpty) {                   // the one key the table cannot hold
                    if (!has_empty_) {
                        has_empty_ = true;
                        empty_val_ = next;
                        *fresh = true;
                        return next;
                    }
                    *fresh = false;
                    return empty_val_;
                }
                slots_[i].key = id;
                slots_[i].val = next;
                used_.push_back((uint32_t)i);
                *fresh = true;
                return next;
            }
        }
    }
  private:
    static constexpr uint64_t kEmpty = ~0ull;
    static uint64_t hash(uint64_t x) {
        x ^= x >> 33;
        x *= 0xff51afd7ed558ccdull;
        return x ^ (x >> 33);
    }
    // key and value side by side: a lookup touches one 16-byte slot
    struct Slot {
        uint64_t key;
        uint32_t val, pad;
    };
    void rehash(size_t cap) {
        std::vector<Slot> k(cap, Slot{kEmpty, 0, 0});
        std::vector<uint32_t> u;
        u.reserve(used_.size());
        for (uint32_t i : used_) {
            const uint64_t id = slots_[i].key;
            uint64_t j = hash(id) & (cap - 1);
            while (k[j].key != kEmpty) j = (j + 1) & (cap - 1);
            k[j] = slots_[i];
            u.push_back((uint32_t)j);
        }
        slots_.swap(k);
        used_.swap(u);
    }
    std::vector<Slot> slots_;
    std::vector<uint32_t> used_;
    bool has_empty_ = false;
    uint32_t empty_val_ = 0;
};

}  // namespace

struct hq_wire {
    uint64_t deployment_id = 0;
    std::string err;
    std::vector<Rec> recs;
    std::vector<uint64_t> clusters;
    ClusterIndex cluster_index;
    // attached (hq_wire_attach): a record's key is the worker's handle, resolved as it is
    // decoded through handle_of (cluster id -> handle, kept across steps: handles never change;
    // only clusters the worker runs are kept in it)
    hq_worker *worker = nullptr;
    ClusterIndex handle_of;
    std::vector<uint64_t> pending;     // the cluster ids of a batch's records, before their keys
    hq_wire_stats stats{};
    // the assembled step input (valid until the next reset)
    std::vector<uint32_t> groups;
    std::vector<uint64_t> offsets;
    std::vector<hq_event> events;
    std::vector<uint64_t> boffsets;    // hq_wire_step_stream
    std::vector<uint8_t> bytes;
    std::vector<uint32_t> cnt, perm, pos;   // hq_wire_step_sized's counting sort
    std::vector<uint32_t> kcnt;        // attached: the records queued per handle (at h + 1)

    void count_key(uint32_t k) {
        if ((size_t)k + 2 > kcnt.size()) kcnt.resize(std::max<size_t>((size_t)k + 2, 2 * kcnt.size()), 0);
        kcnt[(size_t)k + 1]++;
    }
    static constexpr uint32_t kNoKey = UINT32_MAX;   // a record of a cluster the worker does not run
    // records r0.. leave the queue (a batch dropped after its decode)
    void drop_from(size_t r0) {
        if (worker)
            for (size_t i = r0; i < recs.size(); ++i)
                if (recs[i].key != kNoKey) kcnt[(size_t)recs[i].key + 1]--;
        recs.resize(r0);
    }
    std::vector<Rec> grp;              //   and one group's events

    int fail(int code, const std::string &m) {
        err = m;
        return code;
    }
    uint32_t cluster(uint64_t id) {
        bool fresh;
        const uint32_t k = cluster_index.find_or_add(id, (uint32_t)clusters.size(), &fresh);
        if (fresh) clusters.push_back(id);
        return k;
    }
    // the key of a cluster: its handle when attached (false: the worker does not run it), else
    // its index of first appearance
    bool key(uint64_t id, uint32_t *k) {
        if (!worker) {
            *k = cluster(id);
            return true;
        }
        if (handle_of.find(id, k)) return true;
        uint32_t h;
        if (hq_worker_find(worker, id, &h) != HQ_OK) return false;
        bool fresh;
        handle_of.find_or_add(id, h, &fresh);
        *k = h;
        return true;
    }
    // the records from r0 on got their cluster ids in `pending`: their keys, dropping (in place)
    // those of clusters the attached worker does not run; the handle table prefetched 8 ahead
    void resolve(size_t r0) {
        const size_t n = recs.size() - r0;
        size_t i = 0;
        for (; i < n; ++i) {                   // (no record dropped: keys set in place)
            if (worker && i + 8 < n) handle_of.prefetch(pending[i + 8]);
            if (!key(pending[i], &recs[r0 + i].key)) break;
        }
        if (i == n) return;
        size_t o = r0 + i;
        for (; i < n; ++i) {
            if (worker && i + 8 < n) handle_of.prefetch(pending[i + 8]);
            uint32_t k;
            if (!key(pending[i], &k)) {
                stats.dropped_no_cluster++;
                continue;
            }
            recs[o] = recs[r0 + i];
            recs[o++].key = k;
        }
        recs.resize(o);
    }
};

extern "C" {

int hq_wire_decode_batch(const uint8_t *bytes, size_t len, hq_wire_message *out, uint64_t cap,
                         uint64_t *count, hq_wire_batch_info *info) {
    if ((!bytes && len) || !count) return HQ_E_INVAL;
    std::string err;
    hq_wire_batch_info bi;
    uint64_t k = 0;
    const int rc = parse_batch(bytes, len, &bi, count, [&](const uint8_t *m, size_t n) {
        hq_wire_message tmp;
        hq_wire_message *dst = out && k < cap ? out + k : &tmp;
        ++k;
        return decode_message(m, n, dst, err);
    });
    if (rc) return rc;
    if (info) *info = bi;
    return *count > cap && out ? HQ_E_STATE : HQ_OK;
}

// The sending node's side (bench and tests): MessageBatch.MarshalTo (raft.pb.go:2417-2445) over
// Message.MarshalTo (:2232-2296) of the fields hq_wire_message carries, every nullable=false
// field written, the empty Snapshot's 24 bytes (Snapshot.MarshalTo :2142, Membership :2019)
int hq_wire_encode_batch(const hq_wire_message *msgs, uint64_t n, uint64_t deployment_id,
                         const uint8_t *source, size_t source_len, uint8_t *out, uint64_t cap,
                         uint64_t *len) {
    if ((n && !msgs) || !len || (source_len && !source) || (cap && !out)) return HQ_E_INVAL;
    static const uint8_t kSnap[24] = {0x12, 0, 0x18, 0, 0x20, 0, 0x28, 0, 0x32, 2, 0x08, 0,
                                      0x48, 0, 0x50, 0, 0x58, 0, 0x60, 0, 0x68, 0, 0x70, 0};
    auto vlen = [](uint64_t v) {
        uint32_t k = 1;
        while (v >= 0x80) {
            v >>= 7;
            ++k;
        }
        return k;
    };
    auto put = [](uint8_t *p, uint64_t v) {
        while (v >= 0x80) {
            *p++ = (uint8_t)(v | 0x80);
            v >>= 7;
        }
        *p++ = (uint8_t)v;
        return p;
    };
    uint8_t *p = out, *const end = out + cap;
    for (uint64_t i = 0; i < n; ++i) {
        const hq_wire_message &m = msgs[i];
        if (m.n_entries) return HQ_E_INVAL;      // (entries are not marshalled here)
        const uint64_t f[10] = {m.ev.type, m.to, m.ev.from, m.cluster_id, m.ev.term, m.log_term,
                                m.ev.log_index, m.commit, m.ev.reject ? 1u : 0u, m.ev.hint};
        uint64_t size = 2 + sizeof kSnap + 1 + vlen(m.ev.hint_high);
        for (uint64_t v : f) size += 1 + vlen(v);
        if ((uint64_t)(end - p) < size + 1 + vlen(size)) return HQ_E_STATE;
        *p++ = 0x0a;                              // requests (1), length-delimited
        p = put(p, size);
        for (uint32_t k = 0; k < 10; ++k) {
            *p++ = (uint8_t)((k + 1) << 3);
            p = put(p, f[k]);
        }
        *p++ = 0x62;
        *p++ = (uint8_t)sizeof kSnap;
        std::memcpy(p, kSnap, sizeof kSnap);
        p += sizeof kSnap;
        *p++ = 0x68;
        p = put(p, m.ev.hint_high);
    }
    if ((uint64_t)(end - p) < 1 + 10 + 1 + 10 + source_len + 1 + 10) return HQ_E_STATE;
    *p++ = 0x10;                                  // deployment_id (2)
    p = put(p, deployment_id);
    *p++ = 0x1a;                                  // source_address (3)
    p = put(p, source_len);
    if (source_len) std::memcpy(p, source, source_len);
    p += source_len;
    *p++ = 0x20;                                  // bin_ver (4)
    p = put(p, HQ_RPC_BIN_VERSION);
    *len = (uint64_t)(p - out);
    return HQ_OK;
}

int hq_wire_open(uint64_t deployment_id, hq_wire **out) {
    if (!out) return HQ_E_INVAL;
    *out = new (std::nothrow) hq_wire();
    if (!*out) return HQ_E_NOMEM;
    (*out)->deployment_id = deployment_id;
    return HQ_OK;
}

void hq_wire_close(hq_wire *w) { delete w; }

const char *hq_wire_last_error(const hq_wire *w) { return w ? w->err.c_str() : ""; }

int hq_wire_attach(hq_wire *w, hq_worker *worker) {
    if (!w) return HQ_E_INVAL;
    if (!w->recs.empty()) return w->fail(HQ_E_STATE, "hq_wire_attach: events queued (reset first)");
    w->worker = worker;
    w->handle_of = ClusterIndex();
    w->kcnt.clear();
    return HQ_OK;
}

int hq_wire_reset(hq_wire *w) {
    if (!w) return HQ_E_INVAL;
    w->recs.clear();
    std::fill(w->kcnt.begin(), w->kcnt.end(), 0u);
    w->clusters.clear();
    w->cluster_index.clear();
    w->stats = hq_wire_stats{};
    return HQ_OK;
}

int hq_wire_add_local(hq_wire *w, uint64_t cluster_id, const hq_event *events, uint64_t count) {
    if (!w || (count && !events)) return HQ_E_INVAL;
    const uint64_t off[2] = {0, count};
    return hq_wire_add_locals(w, 1, &cluster_id, off, events);
}

int hq_wire_add_locals(hq_wire *w, uint64_t n, const uint64_t *cluster_ids, const uint64_t *offsets,
                       const hq_event *events) {
    if (!w || (n && (!cluster_ids || !offsets))) return HQ_E_INVAL;
    if (n && offsets[n] > offsets[0] && !events) return HQ_E_INVAL;
    for (uint64_t c = 0; c < n; ++c) {
        if (offsets[c + 1] < offsets[c]) return w->fail(HQ_E_INVAL, "hq_wire_add_locals: offsets decrease");
        for (uint64_t i = offsets[c]; i < offsets[c + 1]; ++i) {
            switch (events[i].kind) {
            case HQ_EV_READ: case HQ_EV_CHECK_QUORUM: case HQ_EV_ELECTION: case HQ_EV_PROPOSE: break;
            default: return w->fail(HQ_E_INVAL, "hq_wire_add_local: kind must be a local event");
            }
        }
    }
    for (uint64_t c = 0; c < n; ++c) {
        if (offsets[c + 1] == offsets[c]) continue;
        uint32_t k;
        if (!w->key(cluster_ids[c], &k)) {      // (a cluster the attached worker does not run)
            w->stats.dropped_no_cluster += offsets[c + 1] - offsets[c];
            continue;
        }
        for (uint64_t i = offsets[c]; i < offsets[c + 1]; ++i) {
            const hq_event &e = events[i];
            Rec r{};
            r.key = k;
            r.cat = e.kind == HQ_EV_READ ? 0 : e.kind == HQ_EV_PROPOSE ? 3 : 2;
            r.kind = (uint8_t)e.kind;
            r.reject = e.reject != 0;
            r.type = e.type;
            r.from = e.from;
            r.term = e.term;
            r.log_index = e.log_index;
            r.hint = e.hint;
            r.hint_high = e.hint_high;
            w->recs.push_back(r);
            if (w->worker) w->count_key(k);
        }
    }
    return HQ_OK;
}

int hq_wire_add_batch(hq_wire *w, const uint8_t *bytes, size_t len) {
    if (!w) return HQ_E_INVAL;
    if (!bytes && len) return w->fail(HQ_E_INVAL, "hq_wire_add_batch: NULL bytes");
    // one pass: every message straight into a record (Message.MarshalTo's field order on the fast
    // path, any order on the general one) with its cluster id aside; the batch's own fields
    // (they follow the messages in the marshalled order) then decide whether the records stay
    // and their clusters are resolved to keys
    const size_t r0 = w->recs.size();
    w->pending.clear();
    uint64_t entries = 0, snap = 0, no_cluster = 0;
    // attached: each record's key (the worker's handle) looked up while the batch decodes, kAhead
    // messages behind the decode (the handle table's slot prefetched when the message is decoded;
    // a batch the deployment check drops afterwards only leaves its clusters' handles cached);
    // else the keys wait for that check (an index of first appearance must not see a dropped
    // batch)
    const bool now = w->worker != nullptr;
    constexpr size_t kAhead = 8;
    size_t looked = 0;
    auto look_up = [&]() {
        Rec &x = w->recs[r0 + looked];
        const uint64_t id = w->pending[looked++];
        if (w->handle_of.find(id, &x.key) || w->key(id, &x.key)) {
            w->count_key(x.key);
        } else {
            x.key = hq_wire::kNoKey;
            ++no_cluster;
        }
    };
    std::string err;
    hq_wire_batch_info bi;
    uint64_t n = 0;
    const int rc = parse_batch(bytes, len, &bi, &n, [&](const uint8_t *m, size_t k) {
        Rec r;
        r.key = 0;
        r.pad = 0;
        r.pad2 = 0;
        uint64_t cid;
        uint32_t ent;
        if (!decode_marshal_order(m, m + k, r, cid, ent)) {
            hq_wire_message x;
            const int e = decode_message(m, k, &x, err);
            if (e) return e;
            r.kind = HQ_EV_MESSAGE;
            r.type = x.ev.type;
            r.from = x.ev.from;
            r.term = x.ev.term;
            r.log_index = x.ev.log_index;
            r.hint = x.ev.hint;
            r.hint_high = x.ev.hint_high;
            r.reject = x.ev.reject != 0;
            cid = x.cluster_id;
            ent = x.n_entries;
        }
        entries += ent;
        // HandleMessageBatch (nodehost.go:2039-2044): snapshot confirmations go aside
        if (r.type == kSnapshotReceived) {
            ++snap;
            return HQ_OK;
        }
        r.cat = 1;
        w->recs.push_back(r);
        w->pending.push_back(cid);
        if (now) {
            w->handle_of.prefetch(cid);
            if (w->pending.size() - looked > kAhead) look_up();
        }
        return HQ_OK;
    });
    if (now) {
        while (looked < w->pending.size()) look_up();
        if (no_cluster && !rc) {       // the records of clusters the worker does not run leave
            size_t o = r0;
            for (size_t i = r0; i < w->recs.size(); ++i)
                if (w->recs[i].key != hq_wire::kNoKey) w->recs[o++] = w->recs[i];
            w->recs.resize(o);
        }
    }
    if (rc) {
        w->drop_from(r0);
        return w->fail(HQ_E_INVAL, "hq_wire_add_batch: malformed MessageBatch" +
                                       (err.empty() ? std::string() : ": " + err));
    }
    w->stats.batches++;
    w->stats.bytes += len;
    // Transport.handleRequest (transport.go:289-300): the whole batch is dropped on a foreign
    // deployment id or binary version (none of its clusters is looked at)
    if (bi.deployment_id != w->deployment_id || bi.bin_ver != HQ_RPC_BIN_VERSION) {
        w->drop_from(r0);
        w->stats.dropped_batches++;
        w->stats.dropped_messages += n;
        return HQ_OK;
    }
    w->stats.messages += n;
    w->stats.entries += entries;
    w->stats.snapshot_received += snap;
    w->stats.dropped_no_cluster += no_cluster;
    if (!now) w->resolve(r0);
    return HQ_OK;
}

int hq_wire_step_input(hq_wire *w, hq_worker *worker, hq_step_input *out, hq_wire_stats *stats) {
    if (!w || !worker || !out) return HQ_E_INVAL;
    if (w->worker) return w->fail(HQ_E_STATE, "hq_wire_step_input: attached (hq_wire_step_sized)");
    const uint32_t nc = (uint32_t)w->clusters.size();
    // handles; clusters this worker does not run are dropped (nodehost.go:2045-2046)
    std::vector<uint32_t> handle(nc);
    std::vector<uint64_t> cnt((size_t)nc * 4 + 1, 0);
    for (uint32_t k = 0; k < nc; ++k)
        if (hq_worker_find(worker, w->clusters[k], &handle[k]) != HQ_OK) handle[k] = UINT32_MAX;
    // counting sort by (cluster order of first appearance, category), stable in arrival order
    for (const auto &r : w->recs) cnt[(size_t)r.key * 4 + r.cat + 1]++;
    for (size_t i = 1; i < cnt.size(); ++i) cnt[i] += cnt[i - 1];
    std::vector<uint32_t> perm(w->recs.size());
    std::vector<uint64_t> pos(cnt.begin(), cnt.end() - 1);
    for (uint32_t i = 0; i < (uint32_t)w->recs.size(); ++i) {
        const Rec &r = w->recs[i];
        perm[pos[(size_t)r.key * 4 + r.cat]++] = i;
    }
    w->groups.clear();
    w->offsets.assign(1, 0);
    w->events.clear();
    for (uint32_t k = 0; k < nc; ++k) {
        const uint64_t b = cnt[(size_t)k * 4], e = cnt[(size_t)k * 4 + 4];
        if (handle[k] == UINT32_MAX) {
            w->stats.dropped_no_cluster += e - b;
            continue;
        }
        if (b == e) continue;
        w->groups.push_back(handle[k]);
        for (uint64_t j = b; j < e; ++j) w->events.push_back(w->recs[perm[j]].event());
        w->offsets.push_back(w->events.size());
    }
    out->n_groups = w->groups.size();
    out->groups = w->groups.data();
    out->offsets = w->offsets.data();
    out->events = w->events.data();
    if (stats) *stats = w->stats;
    return HQ_OK;
}

int hq_wire_step_stream(hq_wire *w, hq_worker *worker, hq_step_stream *out, hq_wire_stats *stats) {
    if (!w || !out) return HQ_E_INVAL;
    hq_step_input in;
    int rc = hq_wire_step_input(w, worker, &in, stats);
    if (rc) return rc;
    w->boffsets.resize(in.n_groups + 1);
    w->bytes.resize((size_t)w->events.size() * HQ_EVENT_STREAM_MAX);
    rc = hq_events_encode(in.n_groups, in.offsets, in.events, w->bytes.data(), w->bytes.size(),
                          w->boffsets.data());
    if (rc) return w->fail(rc, "hq_wire_step_stream: encode");
    out->n_groups = in.n_groups;
    out->groups = in.groups;
    out->offsets = in.offsets;
    out->boffsets = w->boffsets.data();
    out->bytes = w->bytes.data();
    out->sizes = nullptr;
    out->n_events = out->n_bytes = 0;
    out->sizes16 = nullptr;
    return HQ_OK;
}

int hq_wire_step_sized(hq_wire *w, uint8_t *bytes, uint64_t cap, uint16_t *sizes16, uint64_t n_cap,
                       hq_step_stream *out, hq_wire_stats *stats) {
    if (!w || !out || (cap && !bytes)) return HQ_E_INVAL;
    if (!w->worker) return w->fail(HQ_E_STATE, "hq_wire_step_sized: no worker attached");
    uint64_t n = 0;
    if (hq_worker_group_count(w->worker, &n) != HQ_OK) return HQ_E_INVAL;
    if (n > n_cap || (n && !sizes16))
        return w->fail(HQ_E_INVAL, "hq_wire_step_sized: sizes16 holds fewer words than the worker's groups");
    // counting sort of the records by handle, stable in arrival order; each handle's records
    // then taken category by category (node.handleEvents: local ReadIndex, received messages,
    // ticks, proposals)
    const uint32_t nr = (uint32_t)w->recs.size();
    // (the counts per handle were kept as the records were queued; handles only grow, so every
    // queued key is below n)
    w->cnt.assign(n + 1, 0);
    std::copy(w->kcnt.begin(), w->kcnt.begin() + std::min<size_t>(w->kcnt.size(), n + 1), w->cnt.begin());
    for (uint64_t h = 0; h < n; ++h) w->cnt[h + 1] += w->cnt[h];
    if (w->cnt[n] != nr) return w->fail(HQ_E_STATE, "hq_wire_step_sized: a queued record's handle is past the worker's groups");
    w->perm.resize(nr);
    w->pos.assign(w->cnt.begin(), w->cnt.end() - 1);
    for (uint32_t i = 0; i < nr; ++i) w->perm[w->pos[w->recs[i].key]++] = i;
    uint8_t *p = bytes, *const end = bytes + cap;
    uint64_t events = 0;
    for (uint64_t h = 0; h < n; ++h) {
        const uint32_t b = w->cnt[h], e = w->cnt[h + 1];
        uint8_t *const g0 = p;
        if (e > b) {
            // the group's events gathered in arrival order; put in category order (a stable
            // insertion sort of the few out of place) when they are not already
            w->grp.resize(e - b);
            Rec *g = w->grp.data();
            bool sorted = true;
            for (uint32_t j = b; j < e; ++j) {
                g[j - b] = w->recs[w->perm[j]];
                sorted = sorted && (j == b || g[j - b - 1].cat <= g[j - b].cat);
            }
            if (!sorted)
                for (uint32_t x = 1; x < e - b; ++x)
                    for (uint32_t y = x; y > 0 && g[y - 1].cat > g[y].cat; --y) std::swap(g[y - 1], g[y]);
            p = hqs::encode_group(p, end, static_cast<const hqs::WireEvent *>(g), e - b);
            if (!p) return w->fail(HQ_E_STATE, "hq_wire_step_sized: the stream does not fit cap");
            if (p - g0 > 0xFFFF || e - b > 0xFFFF)
                return w->fail(HQ_E_INVAL, "hq_wire_step_sized: a group of 2^16 events or bytes");
            events += e - b;
        }
        sizes16[h] = (uint16_t)(p - g0);
    }
    *out = hq_step_stream{};
    out->n_groups = n;
    out->bytes = bytes;
    out->sizes16 = sizes16;
    out->n_events = events;
    out->n_bytes = (uint64_t)(p - bytes);
    if (stats) *stats = w->stats;
    return HQ_OK;
}

}  // extern "C"
