// binprof.hip — phase timestamps of the binned table ingest (hq_table.hip k_bin / k_apply,
// compiled here with HQ_BIN_PROF): the bench's `ing` shape (4 Mi random 16-byte match records
// into a 4 Mi x 3 leader-row table), one warm-up and one measured launch pair; prints, per kernel,
// the spread of workgroup start times and each phase's mean / max duration over the workgroups.
// Build: make tools/binprof (links the library's other objects).
#define HQ_BIN_PROF 1
#include "../dragonboat_amd/csrc/hq_table.hip"

#include <cstdio>
#include <random>
#include <vector>

int main() {
    const uint64_t G = 4 << 20, U = 4 << 20;
    const uint32_t n = 3, form = HQ_FORM_TERM_MASK;
    hq_ctx *ctx = nullptr;
    if (hq_open(0, 0, &ctx)) return 1;
    const uint64_t words = hq_commit_tiles(G) * hq_commit_tile_words_for(n, form, HQ_LAYOUT_TILES_LEADER);
    uint64_t *tiles = nullptr, *upd = nullptr;
    (void)hipMalloc(&tiles, words * 8);
    (void)hipMalloc(&upd, U * 16);
    (void)hipMemset(tiles, 0, words * 8);
    std::vector<uint64_t> h(U * 2);
    std::mt19937_64 rng(7);
    for (uint64_t i = 0; i < U; ++i) {
        h[2 * i] = (rng() % G) << 8 | (1 + rng() % (n - 1));
        h[2 * i + 1] = (1ull << 30) + rng() % 64;
    }
    (void)hipMemcpy(upd, h.data(), U * 16, hipMemcpyHostToDevice);
    int rate_khz = 0;
    (void)hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0);
    for (int rep = 0; rep < 2; ++rep) {
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bin_prof), std::vector<unsigned long long>(2 * 8192 * 8).data(),
                                sizeof(unsigned long long) * 2 * 8192 * 8);
        if (hq_table_ingest_match_dev(ctx, reinterpret_cast<const hq_match_update *>(upd), U, tiles,
                                      G, n, form, HQ_INGEST_BINNED, nullptr))
            return 2;
        if (hq_sync(ctx)) return 3;
    }
    std::vector<unsigned long long> p(2 * 8192 * 8);
    (void)hipMemcpyFromSymbol(p.data(), HIP_SYMBOL(g_bin_prof), p.size() * 8);
    const double us = 1e3 / rate_khz;
    const char *names[2] = {"k_bin", "k_apply"};
    const int nmark[2] = {4, 4};   // markers 0..3 of the first iteration, 7 = the workgroup's end
    for (int k = 0; k < 2; ++k) {
        unsigned long long t0 = ~0ull, t1 = 0, s_last = 0, t_end = 0;
        double sum[8] = {}, mx[8] = {};
        int nwg = 0;
        const int L = nmark[k] - 1;
        for (int b = 0; b < 8192; ++b) {
            const unsigned long long *q = &p[(k * 8192 + b) * 8];
            if (!q[0] || !q[L]) continue;
            ++nwg;
            t0 = std::min(t0, q[0]);
            t1 = std::max(t1, q[L]);
            s_last = std::max(s_last, q[0]);
            t_end = std::max(t_end, q[7]);
            for (int ph = 0; ph < L; ++ph) {
                const double d = (double)(q[ph + 1] - q[ph]) * us;
                sum[ph] += d;
                mx[ph] = std::max(mx[ph], d);
            }
        }
        if (!nwg) continue;
        std::printf("%s: %d workgroups timed, first start -> last end of the first iteration %.2f us, "
                    "-> kernel end %.2f us, starts spread %.2f us\n",
                    names[k], nwg, (double)(t1 - t0) * us, (double)(t_end - t0) * us,
                    (double)(s_last - t0) * us);
        for (int ph = 0; ph < L; ++ph)
            std::printf("  phase %d: mean %.2f us, max %.2f us\n", ph, sum[ph] / nwg, mx[ph]);
    }
    hq_close(ctx);
    return 0;
}
