// hq_stream.h — internal: the event-stream encoder shared by hq_stream.cpp (rows, compact
// records) and hq_wire.cpp (events decoded from the wire). Internal to libhipquorum.so.
#pragma once

#include <cstdint>

#include "../../include/hipquorum.h"

namespace hqs {

// One event as the wire decoder keeps it: the fields the quorum path reads (the hq_event's,
// narrowed) with the wire's bookkeeping. key: the attached worker's handle, or the cluster's index
// of first appearance; cat: 0 local ReadIndex, 1 received message, 2 tick, 3 proposal
struct WireEvent {
    uint32_t key;
    uint8_t cat, kind, reject, pad;
    uint32_t type, pad2;
    uint64_t from, term, log_index, hint, hint_high;
};
static_assert(sizeof(WireEvent) == 56, "56-byte wire records");

// one group's events ev[0 .. n) encoded at p as hq_events_encode does (its runs and repeat
// codes); NULL when fewer than HQ_EVENT_STREAM_MAX bytes are left before an event
uint8_t *encode_group(uint8_t *p, const uint8_t *end, const hq_event *ev, uint64_t n);
uint8_t *encode_group(uint8_t *p, const uint8_t *end, const WireEvent *ev, uint64_t n);

}  // namespace hqs
