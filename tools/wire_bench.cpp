// wire_bench.cpp — host-only timing of the wire feed (hq_wire.cpp) in the shape of bench.py's
// `wire` leg: one steady-state step of G leader groups (3 voters: a ReplicateResp and a
// HeartbeatResp from each of the 2 followers, every 4th group a local ReadIndex whose heartbeats
// carry the ctx, one proposal per group), marshalled as one MessageBatch per (message type,
// sender); per rep on one thread hq_wire_reset + hq_wire_add_batch of every batch +
// hq_wire_add_locals + hq_wire_step_sized, each phase timed. The worker is a stub (cluster id ->
// handle = its position), so no GPU is needed: it is for A/B of decoder builds on the box's CPU
// (profiles/r06w/). Build it as the library builds its host sources (g++ -O3):
//   g++ -O3 -std=c++17 -fPIC -o wire_bench tools/wire_bench.cpp dragonboat_amd/csrc/hq_wire.cpp \
//       dragonboat_amd/csrc/hq_stream.cpp -pthread
//   wire_bench [G] [reps]      (WB_REVERSE=1: one batch in reverse group order)
// The line ends with a digest of the stream: two decoders must print the same one.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <vector>

#include "../include/hipquorum.h"

// the stub worker: G groups, cluster id base + i * stride at handle i
struct hq_worker {
    uint64_t n;
    std::unordered_map<uint64_t, uint32_t> h;
};
extern "C" int hq_worker_find(hq_worker *w, uint64_t cid, uint32_t *handle) {
    auto it = w->h.find(cid);
    if (it == w->h.end()) return HQ_E_INVAL;
    *handle = it->second;
    return HQ_OK;
}
extern "C" int hq_worker_group_count(hq_worker *w, uint64_t *n) {
    *n = w->n;
    return HQ_OK;
}

static double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const uint64_t G = argc > 1 ? std::strtoull(argv[1], nullptr, 0) : 16384;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 200;
    const uint64_t dep = 0x5EED, cid0 = 1, stride = 1, s = 0, last = 1000 + s;
    hq_worker wk{G, {}};
    for (uint64_t i = 0; i < G; ++i) wk.h[cid0 + i * stride] = (uint32_t)i;
    // the batches: (ReplicateResp, HeartbeatResp) x (from 2, from 3), in group order
    std::vector<std::vector<uint8_t>> bufs;
    uint64_t n_msg = 0, n_bytes = 0;
    for (uint32_t typ : {13u, 18u})
        for (uint64_t frm = 2; frm <= 3; ++frm) {
            std::vector<hq_wire_message> m(G);
            for (uint64_t i = 0; i < G; ++i) {
                hq_wire_message &x = m[i];
                std::memset(&x, 0, sizeof x);
                x.ev.kind = HQ_EV_MESSAGE;
                x.ev.type = typ;
                x.ev.from = frm;
                x.ev.term = 5;
                x.to = 1;
                x.cluster_id = cid0 + i * stride;
                if (typ == 13) {
                    x.ev.log_index = last;
                } else if (i % 4 == 0) {
                    x.ev.hint = ((s + 1) << 32) | i;
                    x.ev.hint_high = s + 1;
                }
            }
            if (std::getenv("WB_REVERSE") && typ == 13 && frm == 3) std::reverse(m.begin(), m.end());
            std::vector<uint8_t> b(G * 128 + 256);
            uint64_t len = 0;
            const char src[] = "n2:63000";
            if (hq_wire_encode_batch(m.data(), G, dep, (const uint8_t *)src, 8, b.data(), b.size(),
                                     &len) != HQ_OK) {
                std::fprintf(stderr, "encode failed\n");
                return 1;
            }
            b.resize(len);
            n_msg += G;
            n_bytes += len;
            bufs.push_back(std::move(b));
        }
    // the locals: every 4th group a ReadIndex, every group a proposal
    std::vector<uint64_t> lc(G), lo(G + 1, 0);
    std::vector<hq_event> lev;
    for (uint64_t i = 0; i < G; ++i) {
        lc[i] = cid0 + i * stride;
        if (i % 4 == 0) {
            hq_event e{};
            e.kind = HQ_EV_READ;
            e.hint = ((s + 1) << 32) | i;
            e.hint_high = s + 1;
            lev.push_back(e);
        }
        hq_event p{};
        p.kind = HQ_EV_PROPOSE;
        p.log_index = 1;
        lev.push_back(p);
        lo[i + 1] = lev.size();
    }
    hq_wire *w = nullptr;
    hq_wire_open(dep, &w);
    hq_wire_attach(w, &wk);
    std::vector<uint8_t> out(lev.size() * HQ_EVENT_STREAM_MAX + n_msg * HQ_EVENT_STREAM_MAX + 64);
    std::vector<uint16_t> sizes(G);
    std::vector<double> ts, pa, pb, pc;
    hq_step_stream ss{};
    hq_wire_stats st{};
    for (int r = 0; r < reps + 3; ++r) {
        const double t0 = now_s();
        hq_wire_reset(w);
        for (auto &b : bufs)
            if (hq_wire_add_batch(w, b.data(), b.size()) != HQ_OK) {
                std::fprintf(stderr, "add_batch: %s\n", hq_wire_last_error(w));
                return 1;
            }
        const double ta = now_s();
        hq_wire_add_locals(w, G, lc.data(), lo.data(), lev.data());
        const double tb = now_s();
        if (hq_wire_step_sized(w, out.data(), out.size(), sizes.data(), G, &ss, &st) != HQ_OK) {
            std::fprintf(stderr, "step_sized: %s\n", hq_wire_last_error(w));
            return 1;
        }
        const double t1 = now_s();
        if (r >= 3) { ts.push_back(t1 - t0); pa.push_back(ta-t0); pb.push_back(tb-ta); pc.push_back(t1-tb);} 
    }
    // a digest of the stream (the same tree must give the same bytes before and after a change)
    uint64_t h = 1469598103934665603ull;
    for (uint64_t i = 0; i < ss.n_bytes; ++i) h = (h ^ out[i]) * 1099511628211ull;
    for (uint64_t i = 0; i < G; ++i) h = (h ^ sizes[i]) * 1099511628211ull;
    std::sort(ts.begin(), ts.end()); std::sort(pa.begin(),pa.end()); std::sort(pb.begin(),pb.end()); std::sort(pc.begin(),pc.end()); std::printf("batches %.3f locals %.3f sized %.3f ms (medians)\n", pa[pa.size()/2]*1e3, pb[pb.size()/2]*1e3, pc[pc.size()/2]*1e3);
    const double med = ts[ts.size() / 2], best = ts[0];
    std::printf("G %llu: %llu messages in %zu batches (%llu bytes), %llu events, %llu stream bytes; "
                "median %.3f ms = %.2f ns/message (best %.2f); digest %016llx\n",
                (unsigned long long)G, (unsigned long long)n_msg, bufs.size(),
                (unsigned long long)n_bytes, (unsigned long long)ss.n_events,
                (unsigned long long)ss.n_bytes, med * 1e3, med / n_msg * 1e9, best / n_msg * 1e9,
                (unsigned long long)h);
    hq_wire_close(w);
    return st.messages == n_msg ? 0 : 1;
}
