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
#include <unordered_map>
#include <vector>

#include "../../include/hipquorum.h"

namespace {

constexpr uint32_t kSnapshotReceived = 22;   // raft.proto MessageType

struct Reader {
    const uint8_t *p, *end;
    const char *err = nullptr;

    bool varint(uint64_t &v) {
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
    std::unordered_map<uint64_t, uint32_t> cluster_index;
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
        auto it = cluster_index.find(id);
        if (it != cluster_index.end()) return it->second;
        const uint32_t k = (uint32_t)clusters.size();
        cluster_index.emplace(id, k);
        clusters.push_back(id);
        return k;
    }
};

extern "C" {

int hq_wire_decode_batch(const uint8_t *bytes, size_t len, hq_wire_message *out, uint64_t cap,
                         uint64_t *count, hq_wire_batch_info *info) {
    if ((!bytes && len) || !count) return HQ_E_INVAL;
    *count = 0;
    hq_wire_batch_info bi{};
    Reader r{bytes, bytes + len};
    std::string err;
    while (r.p < r.end) {
        uint64_t tag;
        if (!r.varint(tag)) break;
        const uint32_t field = (uint32_t)(tag >> 3), wt = (uint32_t)(tag & 7);
        if (field == 1 && wt == 2) {                  // repeated Message requests
            const uint8_t *m;
            uint64_t n;
            if (!r.bytes(m, n)) break;
            if (*count < cap && out) {
                if (decode_message(m, n, out + *count, err) != HQ_OK) return HQ_E_INVAL;
            } else {
                hq_wire_message tmp;
                if (decode_message(m, n, &tmp, err) != HQ_OK) return HQ_E_INVAL;
            }
            ++*count;
        } else if (field == 2 && wt == 0) {           // deployment_id
            if (!r.varint(bi.deployment_id)) break;
        } else if (field == 3 && wt == 2) {           // source_address
            const uint8_t *s;
            uint64_t n;
            if (!r.bytes(s, n)) break;
            bi.source_address_len = n;
        } else if (field == 4 && wt == 0) {           // bin_ver
            uint64_t v;
            if (!r.varint(v)) break;
            bi.bin_ver = (uint32_t)v;
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
    bi.n_messages = *count;
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
    uint64_t n = 0;
    hq_wire_batch_info bi;
    if (hq_wire_decode_batch(bytes, len, nullptr, 0, &n, &bi) != HQ_OK)
        return w->fail(HQ_E_INVAL, "hq_wire_add_batch: malformed MessageBatch");
    w->stats.batches++;
    w->stats.bytes += len;
    // Transport.handleRequest (transport.go:289-300): the whole batch is dropped on a foreign
    // deployment id or binary version
    if (bi.deployment_id != w->deployment_id || bi.bin_ver != HQ_RPC_BIN_VERSION) {
        w->stats.dropped_batches++;
        w->stats.dropped_messages += n;
        return HQ_OK;
    }
    w->scratch.resize(n);
    uint64_t m = 0;
    if (hq_wire_decode_batch(bytes, len, w->scratch.data(), n, &m, nullptr) != HQ_OK)
        return w->fail(HQ_E_INVAL, "hq_wire_add_batch: malformed MessageBatch");
    for (uint64_t i = 0; i < m; ++i) {
        const hq_wire_message &x = w->scratch[i];
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
    return HQ_OK;
}

}  // extern "C"
