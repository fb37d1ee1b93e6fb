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
#include <vector>

#include "../../include/hipquorum.h"

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

// MessageBatch (raft.proto:191-196): every Message handed to sink(bytes, len) in order (sink
// returns an HQ_ status), the other fields into *bi. Any field order; unknown fields skipped.
template <class Sink>
int parse_batch(const uint8_t *bytes, size_t len, hq_wire_batch_info *bi, uint64_t *count,
                Sink &&sink) {
    *bi = hq_wire_batch_info{};
    *count = 0;
    Reader r{bytes, bytes + len};
    while (r.p < r.end) {
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
        for (uint32_t i : used_) keys_[i] = kEmpty;
        used_.clear();
        has_empty_ = false;
    }
    // the index of id, inserting next if new (*fresh = true)
    uint32_t find_or_add(uint64_t id, uint32_t next, bool *fresh) {
        if ((used_.size() + 1) * 2 > keys_.size()) rehash(keys_.empty() ? 1024 : keys_.size() * 2);
        const uint64_t mask = keys_.size() - 1;
        for (uint64_t i = hash(id) & mask;; i = (i + 1) & mask) {
            if (keys_[i] == id && id != kEmpty) {
                *fresh = false;
                return vals_[i];
            }
            if (keys_[i] == kEmpty) {
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
                keys_[i] = id;
                vals_[i] = next;
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
    void rehash(size_t cap) {
        std::vector<uint64_t> k(cap, kEmpty);
        std::vector<uint32_t> v(cap);
        std::vector<uint32_t> u;
        u.reserve(used_.size());
        for (uint32_t i : used_) {
            const uint64_t id = keys_[i];
            uint64_t j = hash(id) & (cap - 1);
            while (k[j] != kEmpty) j = (j + 1) & (cap - 1);
            k[j] = id;
            v[j] = vals_[i];
            u.push_back((uint32_t)j);
        }
        keys_.swap(k);
        vals_.swap(v);
        used_.swap(u);
    }
    std::vector<uint64_t> keys_;
    std::vector<uint32_t> vals_;
    std::vector<uint32_t> used_;
    bool has_empty_ = false;
    uint32_t empty_val_ = 0;
};

}  // namespace

struct hq_wire {
    uint64_t deployment_id = 0;
    std::string err;
    struct Rec {
        uint32_t cluster;   // index into clusters (order of first appearance)
        uint32_t cat;       // 0 local ReadIndex, 1 received message, 2 tick, 3 proposal
        hq_event ev;
    };
    std::vector<Rec> recs;
    std::vector<uint64_t> clusters;
    ClusterIndex cluster_index;
    std::vector<hq_wire_message> scratch;
    hq_wire_stats stats{};
    // the assembled step input (valid until the next reset)
    std::vector<uint32_t> groups;
    std::vector<uint64_t> offsets;
    std::vector<hq_event> events;
    std::vector<uint64_t> boffsets;    // hq_wire_step_stream
    std::vector<uint8_t> bytes;

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

int hq_wire_open(uint64_t deployment_id, hq_wire **out) {
    if (!out) return HQ_E_INVAL;
    *out = new (std::nothrow) hq_wire();
    if (!*out) return HQ_E_NOMEM;
    (*out)->deployment_id = deployment_id;
    return HQ_OK;
}

void hq_wire_close(hq_wire *w) { delete w; }

const char *hq_wire_last_error(const hq_wire *w) { return w ? w->err.c_str() : ""; }

int hq_wire_reset(hq_wire *w) {
    if (!w) return HQ_E_INVAL;
    w->recs.clear();
    w->clusters.clear();
    w->cluster_index.clear();
    w->stats = hq_wire_stats{};
    return HQ_OK;
}

int hq_wire_add_local(hq_wire *w, uint64_t cluster_id, const hq_event *events, uint64_t count) {
    if (!w || (count && !events)) return HQ_E_INVAL;
    const uint32_t k = w->cluster(cluster_id);
    for (uint64_t i = 0; i < count; ++i) {
        const hq_event &e = events[i];
        uint32_t cat;
        switch (e.kind) {
        case HQ_EV_READ: cat = 0; break;
        case HQ_EV_CHECK_QUORUM:
        case HQ_EV_ELECTION: cat = 2; break;
        case HQ_EV_PROPOSE: cat = 3; break;
        default: return w->fail(HQ_E_INVAL, "hq_wire_add_local: kind must be a local event");
        }
        w->recs.push_back({k, cat, e});
    }
    return HQ_OK;
}

int hq_wire_add_batch(hq_wire *w, const uint8_t *bytes, size_t len) {
    if (!w) return HQ_E_INVAL;
    if (!bytes && len) return w->fail(HQ_E_INVAL, "hq_wire_add_batch: NULL bytes");
    // one pass: every message decoded into the scratch list; the batch's own fields (they follow
    // the messages in the marshalled order) decide afterwards whether it is kept
    w->scratch.clear();
    std::string err;
    hq_wire_batch_info bi;
    uint64_t n = 0;
    const int rc = parse_batch(bytes, len, &bi, &n, [&](const uint8_t *m, size_t k) {
        w->scratch.emplace_back();
        return decode_message(m, k, &w->scratch.back(), err);
    });
    if (rc) return w->fail(HQ_E_INVAL, "hq_wire_add_batch: malformed MessageBatch" +
                                           (err.empty() ? std::string() : ": " + err));
    w->stats.batches++;
    w->stats.bytes += len;
    // Transport.handleRequest (transport.go:289-300): the whole batch is dropped on a foreign
    // deployment id or binary version
    if (bi.deployment_id != w->deployment_id || bi.bin_ver != HQ_RPC_BIN_VERSION) {
        w->stats.dropped_batches++;
        w->stats.dropped_messages += n;
        return HQ_OK;
    }
    w->recs.reserve(w->recs.size() + n);
    for (const hq_wire_message &x : w->scratch) {
        w->stats.messages++;
        w->stats.entries += x.n_entries;
        // HandleMessageBatch (nodehost.go:2039-2044): snapshot confirmations go aside
        if (x.ev.type == kSnapshotReceived) {
            w->stats.snapshot_received++;
            continue;
        }
        w->recs.push_back({w->cluster(x.cluster_id), 1, x.ev});
    }
    return HQ_OK;
}

int hq_wire_step_input(hq_wire *w, hq_worker *worker, hq_step_input *out, hq_wire_stats *stats) {
    if (!w || !worker || !out) return HQ_E_INVAL;
    const uint32_t nc = (uint32_t)w->clusters.size();
    // handles; clusters this worker does not run are dropped (nodehost.go:2045-2046)
    std::vector<uint32_t> handle(nc);
    std::vector<uint64_t> cnt((size_t)nc * 4 + 1, 0);
    for (uint32_t k = 0; k < nc; ++k)
        if (hq_worker_find(worker, w->clusters[k], &handle[k]) != HQ_OK) handle[k] = UINT32_MAX;
    // counting sort by (cluster order of first appearance, category), stable in arrival order
    for (const auto &r : w->recs) cnt[(size_t)r.cluster * 4 + r.cat + 1]++;
    for (size_t i = 1; i < cnt.size(); ++i) cnt[i] += cnt[i - 1];
    std::vector<hq_event> sorted(w->recs.size());
    std::vector<uint64_t> pos(cnt.begin(), cnt.end() - 1);
    for (const auto &r : w->recs) sorted[pos[(size_t)r.cluster * 4 + r.cat]++] = r.ev;
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
        w->events.insert(w->events.end(), sorted.begin() + b, sorted.begin() + e);
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
    return HQ_OK;
}

}  // extern "C"
