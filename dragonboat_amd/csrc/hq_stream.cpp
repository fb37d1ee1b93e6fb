// hq_stream.cpp — the compact event stream of the device step worker (include/hipquorum.h
// "event streams"): a step's hq_event rows as one byte string per group, each event a header
// byte and LEB128 varints of only the fields its handler reads. The steady-state leader step
// (ReplicateResp / HeartbeatResp / proposals at the current term) takes 3-7 bytes per event
// instead of the 56-byte row, so that a host-fed step crosses PCIe ~10x faster. Host code: the
// encoder a producer holding rows can call (the wire decoder and a caller's own producer can
// write the stream directly) and the decoder the host worker uses for stream input; the device
// twin of the decoder is in hq_dstep.hip.
#include <cstring>

#include "../../include/hipquorum.h"

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
// ReplicateResp's log_index (code 4), its previous HeartbeatResp's ctx (code 5; 0 / 0 at first)
struct Prev {
    uint64_t term = 0, index = 0, hint = 0, high = 0;
    bool have_index = false;
};

// one event; returns the write position
inline uint8_t *encode(uint8_t *p, const hq_event &e, Prev &pv) {
    const uint32_t kind = e.kind >= 1 && e.kind <= 5 ? e.kind : 0;   // 0: not a valid kind
    if (kind != HQ_EV_MESSAGE) {
        *p++ = (uint8_t)kind;
        if (kind == HQ_EV_READ) {
            p = put(p, e.hint);
            p = put(p, e.hint_high);
        } else if (kind == HQ_EV_PROPOSE) {
            p = put(p, e.log_index);
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
    *p++ = (uint8_t)(HQ_EV_MESSAGE | code << 3 | (e.reject ? 0x40 : 0) | (same ? 0x80 : 0));
    if (code == 7) p = put(p, e.type);
    p = put(p, e.from);
    if (!same) p = put(p, e.term);
    pv.term = e.term;
    if (code == 0 || code == 7) p = put(p, e.log_index);
    if (code == 2 || code == 3 || code == 7) {
        p = put(p, e.hint);
        p = put(p, e.hint_high);
    }
    return p;
}

}  // namespace

extern "C" {

int hq_events_encode(uint64_t n_groups, const uint64_t *offsets, const hq_event *events,
                     uint8_t *out, uint64_t cap, uint64_t *boffsets) {
    if (!offsets || !boffsets || (n_groups && offsets[n_groups] > offsets[0] && !events))
        return HQ_E_INVAL;
    uint8_t *p = out, *const end = out ? out + cap : nullptr;
    boffsets[0] = 0;
    for (uint64_t i = 0; i < n_groups; ++i) {
        Prev pv;
        for (uint64_t e = offsets[i]; e < offsets[i + 1]; ++e) {
            if (!out || (uint64_t)(end - p) < HQ_EVENT_STREAM_MAX) return HQ_E_STATE;
            p = encode(p, events[e], pv);
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
        for (uint64_t e = offsets[i]; e < offsets[i + 1]; ++e) {
            if (!out || (uint64_t)(end - p) < HQ_EVENT_STREAM_MAX) return HQ_E_STATE;
            p = encode(p, events[e], pv);
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
        for (uint64_t e = offsets[i]; e < offsets[i + 1]; ++e) {
            hq_event &v = events[e];
            std::memset(&v, 0, sizeof v);
            if (p >= end) return HQ_E_INVAL;
            const uint8_t h = *p++;
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
            }
            if (!ok) return HQ_E_INVAL;
        }
        if (p != end) return HQ_E_INVAL;
    }
    return HQ_OK;
}

}  // extern "C"
