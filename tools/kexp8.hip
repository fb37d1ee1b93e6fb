// kexp8.hip — c4 / c4u (16M groups x 7 voters, fused ReadIndex + vote) over a TILED bitmap layout:
// 1024 consecutive groups (one wave, 16 per lane) stored as one contiguous block of rows
// [n (per-group form only)] [ack] [granted] [rejected], 1 KiB each, so a wave reads ONE stream
// instead of 3-4 column streams. Decision kernels and copy floors for both layouts, each decision
// checked bit-exact against the library's hq_readindex_vote_dev; 200 launches back to back over
// rotating sets (> 1 GiB). Not shipped.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "hipquorum.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
#define HQ(x) do { int r_ = (x); if (r_) { fprintf(stderr, "%s:%d hq %d %s\n", __FILE__, __LINE__, r_, hq_last_error(ctx)); exit(1); } } while (0)

typedef uint64_t u64;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kB80 = 0x80808080u, kB01 = 0x01010101u;

__device__ __forceinline__ uint32_t popc_bytes(uint32_t x) {
    x = x - ((x >> 1) & 0x55555555u);
    x = (x & 0x33333333u) + ((x >> 2) & 0x33333333u);
    return (x + (x >> 4)) & 0x0F0F0F0Fu;
}
__device__ __forceinline__ uint32_t ge_bytes(uint32_t a, uint32_t b) { return ((a | kB80) - b) & kB80; }
__device__ __forceinline__ uint32_t pack4(uint32_t f) { return (((f >> 7) & kB01) * 0x01020408u) >> 24; }
__device__ __forceinline__ uint32_t pack4x2(uint32_t f) { return (((f >> 7) & kB01) * 0x01041040u) >> 24; }
__device__ __forceinline__ uint32_t valid_n(uint32_t n) {
    const uint32_t lo = n & 0x0F0F0F0Fu, hi = (n >> 4) & 0x0F0F0F0Fu;
    return (lo + 0x7F7F7F7Fu) & ~(lo + 0x77777777u) & ~(hi + 0x7F7F7F7Fu) & kB80;
}
__device__ __forceinline__ uint32_t mask_n(uint32_t n) {
    const uint32_t sel = n | (((n >> 3) & kB01) * 0x0Du);
    return __builtin_amdgcn_perm(0x7F3F1F0Fu, 0x07030100u, sel);
}
__device__ __forceinline__ u32x4 ld16(const uint8_t *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
}

struct K {
    const uint8_t *ack, *gr, *rj, *nv;   // columns
    const uint8_t *tiles;                // tiled
    uint16_t *conf; uint32_t *outc; u64 nslots; uint32_t nu;
};

template <bool PERN>
__device__ __forceinline__ void decide(u32x4 nv, u32x4 ac, u32x4 gr, u32x4 rj, uint32_t nu,
                                       uint32_t &conf, uint32_t &outc) {
    conf = 0; outc = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t n = PERN ? nv[w] : nu;
        const uint32_t ok = valid_n(n);
        const uint32_t mask = mask_n(n);
        const uint32_t quorum = ((n >> 1) & 0x7F7F7F7Fu) + kB01;
        const uint32_t c = popc_bytes(ac[w] & mask);
        conf |= pack4(ge_bytes(c, quorum - kB01) & ok) << (4 * w);
        const uint32_t gm = gr[w] & mask;
        const uint32_t rm = rj[w] & mask & ~gm;
        const uint32_t lead = ge_bytes(popc_bytes(gm), quorum) & ok;
        const uint32_t foll = ge_bytes(popc_bytes(rm), quorum) & ok & ~lead;
        const uint32_t cand = kB80 & ~lead & ~foll;
        outc |= (pack4x2(cand) | (pack4x2(lead) << 1)) << (8 * w);
    }
}

// columns: slot t = groups [16t, 16t + 16)
template <int BLK, bool PERN, bool COPY>
__global__ __launch_bounds__(BLK) void col(K a) {
    const u64 lanes = (u64)gridDim.x * BLK;
    for (u64 t = (u64)blockIdx.x * BLK + threadIdx.x; t < a.nslots; t += lanes) {
        const u32x4 nv = PERN ? ld16(a.nv + 16 * t) : u32x4{0, 0, 0, 0};
        const u32x4 ac = ld16(a.ack + 16 * t), gr = ld16(a.gr + 16 * t), rj = ld16(a.rj + 16 * t);
        uint32_t conf, outc;
        if (COPY) { const u32x4 x = nv ^ ac ^ gr ^ rj; conf = x.x ^ x.y; outc = x.z ^ x.w; }
        else decide<PERN>(nv, ac, gr, rj, a.nu, conf, outc);
        a.conf[t] = (uint16_t)conf;
        a.outc[t] = outc;
    }
}

// tiles: wave w owns tile w (1024 groups); lane i holds groups [1024 w + 16 i, +16)
template <int BLK, bool PERN, bool COPY>
__global__ __launch_bounds__(BLK) void tile(K a) {
    constexpr int R = PERN ? 4 : 3;
    const u64 lane = threadIdx.x & 63;
    const u64 nw = (u64)gridDim.x * (BLK / 64);
    const u64 ntiles = a.nslots / 64;
    for (u64 w = (u64)blockIdx.x * (BLK / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
         w < ntiles; w += nw) {
        const uint8_t *p = a.tiles + w * (R * 1024) + lane * 16;
        const u32x4 nv = PERN ? ld16(p) : u32x4{0, 0, 0, 0};
        const u32x4 ac = ld16(p + (R - 3) * 1024), gr = ld16(p + (R - 2) * 1024), rj = ld16(p + (R - 1) * 1024);
        uint32_t conf, outc;
        if (COPY) { const u32x4 x = nv ^ ac ^ gr ^ rj; conf = x.x ^ x.y; outc = x.z ^ x.w; }
        else decide<PERN>(nv, ac, gr, rj, a.nu, conf, outc);
        const u64 t = w * 64 + lane;
        a.conf[t] = (uint16_t)conf;
        a.outc[t] = outc;
    }
}

template <bool PERN>
__global__ void pack(K a, uint8_t *tiles) {
    constexpr int R = PERN ? 4 : 3;
    const u64 G = a.nslots * 16;
    for (u64 g = (u64)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += (u64)gridDim.x * blockDim.x) {
        uint8_t *t = tiles + (g / 1024) * (R * 1024) + (g % 1024);
        if (PERN) t[0] = a.nv[g];
        t[(R - 3) * 1024] = a.ack[g];
        t[(R - 2) * 1024] = a.gr[g];
        t[(R - 1) * 1024] = a.rj[g];
    }
}

int main() {
    const u64 G = 16ull << 20, nsl = G / 16;
    hq_ctx *ctx = nullptr;
    HQ(hq_open(0, 0, &ctx));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const int nsets = 17;
    struct S { uint8_t *a, *g, *r, *n, *t3, *t4; u64 *conf, *outc; };
    std::vector<S> sets(nsets);
    for (int s = 0; s < nsets; ++s) {
        void *p;
        HQ(hq_malloc_dev(ctx, G, &p)); sets[s].a = (uint8_t *)p;
        HQ(hq_malloc_dev(ctx, G, &p)); sets[s].g = (uint8_t *)p;
        HQ(hq_malloc_dev(ctx, G, &p)); sets[s].r = (uint8_t *)p;
        HQ(hq_malloc_dev(ctx, G, &p)); sets[s].n = (uint8_t *)p;
        HQ(hq_malloc_dev(ctx, 3 * G, &p)); sets[s].t3 = (uint8_t *)p;
        HQ(hq_malloc_dev(ctx, 4 * G, &p)); sets[s].t4 = (uint8_t *)p;
        HQ(hq_malloc_dev(ctx, G / 8, &p)); sets[s].conf = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G / 4, &p)); sets[s].outc = (u64 *)p;
        hq_synth_spec sp = {0x5EED0003ull + ((u64)s << 40), G, 1, 1, 7, 0, 16, 0};
        HQ(hq_synth_bitmaps_dev(ctx, &sp, sets[s].a, sets[s].g, sets[s].r, sets[s].n));
    }
    HQ(hq_sync(ctx));
    auto mk = [&](int s, bool pern, bool tiled) {
        return K{sets[s].a, sets[s].g, sets[s].r, sets[s].n, pern ? sets[s].t4 : sets[s].t3,
                 (uint16_t *)sets[s].conf, (uint32_t *)sets[s].outc, nsl, 7u * kB01};
    };
    for (int s = 0; s < nsets; ++s) {
        hipLaunchKernelGGL(pack<true>, 4096, 256, 0, st, mk(s, true, true), sets[s].t4);
        hipLaunchKernelGGL(pack<false>, 4096, 256, 0, st, mk(s, false, true), sets[s].t3);
    }
    CK(hipStreamSynchronize(st));
    std::vector<u64> rc[2], ro[2], c(G / 64), o(G / 32);
    for (int pern = 0; pern < 2; ++pern) {
        rc[pern].resize(G / 64); ro[pern].resize(G / 32);
        HQ(hq_readindex_vote_dev(ctx, G, sets[0].a, sets[0].g, sets[0].r, pern ? sets[0].n : nullptr,
                                 pern ? 0 : 7, sets[0].conf, sets[0].outc, nullptr));
        HQ(hq_sync(ctx));
        CK(hipMemcpy(rc[pern].data(), sets[0].conf, G / 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(ro[pern].data(), sets[0].outc, G / 4, hipMemcpyDeviceToHost));
    }
    typedef void (*KF)(K);
    struct V { const char *name; KF k; int blk; bool pern, tiled, copy; };
    V vs[] = {
        {"c4  col  b256", col<256, true, false>, 256, true, false, false},
        {"c4  tile b256", tile<256, true, false>, 256, true, true, false},
        {"c4  tile b512", tile<512, true, false>, 512, true, true, false},
        {"c4  col  copy", col<256, true, true>, 256, true, false, true},
        {"c4  tile copy", tile<256, true, true>, 256, true, true, true},
        {"c4u col  b256", col<256, false, false>, 256, false, false, false},
        {"c4u tile b256", tile<256, false, false>, 256, false, true, false},
        {"c4u tile b512", tile<512, false, false>, 512, false, true, false},
        {"c4u col  copy", col<256, false, true>, 256, false, false, true},
        {"c4u tile copy", tile<256, false, true>, 256, false, true, true},
    };
    for (int rep = 0; rep < 3; ++rep) {
        for (int pern = 1; pern >= 0; --pern) {
            auto lib = [&](int s) {
                HQ(hq_readindex_vote_dev(ctx, G, sets[s].a, sets[s].g, sets[s].r, pern ? sets[s].n : nullptr,
                                         pern ? 0 : 7, sets[s].conf, sets[s].outc, nullptr));
            };
            for (int i = 0; i < 20; ++i) lib(i % nsets);
            HQ(hq_sync(ctx));
            double ms; u64 n;
            HQ(hq_timing_reset(ctx)); HQ(hq_timing_enable(ctx, 1));
            for (int i = 0; i < 200; ++i) lib(i % nsets);
            HQ(hq_sync(ctx)); HQ(hq_timing_enable(ctx, 0));
            HQ(hq_timing_read(ctx, &ms, &n));
            printf("%-16s per launch %.2f us\n", pern ? "c4  library" : "c4u library", ms * 1e3 / n);
            auto libt = [&](int s) {
                HQ(hq_readindex_vote_tiles_dev(ctx, G, pern ? sets[s].t4 : sets[s].t3, pern, pern ? 0 : 7,
                                               sets[s].conf, sets[s].outc, nullptr));
            };
            libt(0);
            HQ(hq_sync(ctx));
            CK(hipMemcpy(c.data(), sets[0].conf, G / 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(o.data(), sets[0].outc, G / 4, hipMemcpyDeviceToHost));
            const bool okt = c == rc[pern] && o == ro[pern];
            for (int i = 0; i < 20; ++i) libt(i % nsets);
            HQ(hq_sync(ctx));
            HQ(hq_timing_reset(ctx)); HQ(hq_timing_enable(ctx, 1));
            for (int i = 0; i < 200; ++i) libt(i % nsets);
            HQ(hq_sync(ctx)); HQ(hq_timing_enable(ctx, 0));
            HQ(hq_timing_read(ctx, &ms, &n));
            printf("%-16s per launch %.2f us  %s\n", pern ? "c4  lib tiles" : "c4u lib tiles", ms * 1e3 / n, okt ? "exact" : "MISMATCH");
        }
        for (const V &v : vs) {
            const unsigned grid = (unsigned)(v.tiled ? nsl / v.blk : nsl / v.blk);
            CK(hipMemsetAsync(sets[0].conf, 0, G / 8, st));
            CK(hipMemsetAsync(sets[0].outc, 0, G / 4, st));
            hipLaunchKernelGGL(v.k, grid, v.blk, 0, st, mk(0, v.pern, v.tiled));
            CK(hipStreamSynchronize(st));
            CK(hipMemcpy(c.data(), sets[0].conf, G / 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(o.data(), sets[0].outc, G / 4, hipMemcpyDeviceToHost));
            const bool ok = c == rc[v.pern] && o == ro[v.pern];
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
            for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(v.k, grid, v.blk, 0, st, mk(i % nsets, v.pern, v.tiled));
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(v.k, grid, v.blk, 0, st, mk(i % nsets, v.pern, v.tiled));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("%-16s per launch %.2f us  %s\n", v.name, ms * 1e3 / 200,
                   v.copy ? "(no decision)" : ok ? "exact" : "MISMATCH");
        }
    }
    hq_close(ctx);
    return 0;
}
