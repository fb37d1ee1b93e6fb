// kexp4.hip — c4 (16M groups x 7 voters, fused ReadIndex + vote, per-group n) bitmap-kernel
// variants: load policy (nt / plain) x 16-group slots per lane (1 or 2, all loads issued first)
// x block size. Each variant is checked bit-exact against the library's hq_readindex_vote_dev,
// then launched 200 times back to back over 17 rotating input sets (> 1 GiB). Not shipped.
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
template <bool NT> __device__ __forceinline__ u32x4 ld16(const uint8_t *p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return *reinterpret_cast<const u32x4 *>(p);
}

struct K { const uint8_t *ack, *gr, *rj, *nv; uint16_t *conf; uint32_t *outc; u64 nslots; };

// G a multiple of 16 here (16M); SLOTS 16-group slots per lane, slot j = tid + k * lanes
template <int BLK, int SLOTS, bool NT>
__global__ __launch_bounds__(BLK) void bits(K a) {
    const u64 lanes = (u64)gridDim.x * BLK;
    for (u64 t = (u64)blockIdx.x * BLK + threadIdx.x; t < a.nslots; t += lanes * SLOTS) {
        u32x4 nv[SLOTS], ac[SLOTS], gr[SLOTS], rj[SLOTS];
#pragma unroll
        for (int k = 0; k < SLOTS; ++k) {
            const u64 s = t + k * lanes;
            if (s < a.nslots) {
                nv[k] = ld16<NT>(a.nv + 16 * s);
                ac[k] = ld16<NT>(a.ack + 16 * s);
                gr[k] = ld16<NT>(a.gr + 16 * s);
                rj[k] = ld16<NT>(a.rj + 16 * s);
            }
        }
#pragma unroll
        for (int k = 0; k < SLOTS; ++k) {
            const u64 s = t + k * lanes;
            if (s >= a.nslots) continue;
            uint32_t conf = 0, outc = 0;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const uint32_t n = nv[k][w];
                const uint32_t ok = valid_n(n);
                const uint32_t mask = mask_n(n);
                const uint32_t quorum = ((n >> 1) & 0x7F7F7F7Fu) + kB01;
                const uint32_t c = popc_bytes(ac[k][w] & mask);
                conf |= pack4(ge_bytes(c, quorum - kB01) & ok) << (4 * w);
                const uint32_t gm = gr[k][w] & mask;
                const uint32_t rm = rj[k][w] & mask & ~gm;
                const uint32_t lead = ge_bytes(popc_bytes(gm), quorum) & ok;
                const uint32_t foll = ge_bytes(popc_bytes(rm), quorum) & ok & ~lead;
                const uint32_t cand = kB80 & ~lead & ~foll;
                outc |= (pack4x2(cand) | (pack4x2(lead) << 1)) << (8 * w);
            }
            a.conf[s] = (uint16_t)conf;
            a.outc[s] = outc;
        }
    }
}

// the same bytes with no decision: four 16-B loads, a 2-B and a 4-B store per lane
template <int BLK>
__global__ __launch_bounds__(BLK) void copy_like(K a) {
    const u64 lanes = (u64)gridDim.x * BLK;
    for (u64 t = (u64)blockIdx.x * BLK + threadIdx.x; t < a.nslots; t += lanes) {
        const u32x4 x = ld16<true>(a.nv + 16 * t) ^ ld16<true>(a.ack + 16 * t) ^
                        ld16<true>(a.gr + 16 * t) ^ ld16<true>(a.rj + 16 * t);
        a.conf[t] = (uint16_t)(x.x ^ x.y);
        a.outc[t] = x.z ^ x.w;
    }
}

int main() {
    const u64 G = 16ull << 20, nsl = G / 16;
    hq_ctx *ctx = nullptr;
    HQ(hq_open(0, 0, &ctx));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const int nsets = 17;
    struct S { uint8_t *a, *g, *r, *n; u64 *conf, *outc; };
    std::vector<S> sets(nsets);
    for (int s = 0; s < nsets; ++s) {
        void *p;
        HQ(hq_malloc_dev(ctx, G, &p)); sets[s].a = (uint8_t *)p;
        HQ(hq_malloc_dev(ctx, G, &p)); sets[s].g = (uint8_t *)p;
        HQ(hq_malloc_dev(ctx, G, &p)); sets[s].r = (uint8_t *)p;
        HQ(hq_malloc_dev(ctx, G, &p)); sets[s].n = (uint8_t *)p;
        HQ(hq_malloc_dev(ctx, G / 8, &p)); sets[s].conf = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G / 4, &p)); sets[s].outc = (u64 *)p;
        hq_synth_spec sp = {0x5EED0003ull + ((u64)s << 40), G, 1, 1, 7, 0, 16, 0};
        HQ(hq_synth_bitmaps_dev(ctx, &sp, sets[s].a, sets[s].g, sets[s].r, sets[s].n));
    }
    HQ(hq_sync(ctx));
    std::vector<u64> rc(G / 64), ro(G / 32), c(G / 64), o(G / 32);
    auto lib = [&](int s) {
        HQ(hq_readindex_vote_dev(ctx, G, sets[s].a, sets[s].g, sets[s].r, sets[s].n, 0, sets[s].conf, sets[s].outc, nullptr));
    };
    lib(0);
    HQ(hq_sync(ctx));
    CK(hipMemcpy(rc.data(), sets[0].conf, G / 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ro.data(), sets[0].outc, G / 4, hipMemcpyDeviceToHost));
    auto mk = [&](int s) { return K{sets[s].a, sets[s].g, sets[s].r, sets[s].n, (uint16_t *)sets[s].conf, (uint32_t *)sets[s].outc, nsl}; };
    typedef void (*KF)(K);
    struct V { const char *name; KF k; int blk, slots; unsigned grid; };
    V vs[] = {
        {"copy-like b256", copy_like<256>, 256, 1, (unsigned)(nsl / 256)},
        {"copy-like b512", copy_like<512>, 512, 1, (unsigned)(nsl / 512)},
        {"b256 s1 nt  full", bits<256, 1, true>, 256, 1, (unsigned)(nsl / 256)},
        {"b256 s1 pl  full", bits<256, 1, false>, 256, 1, (unsigned)(nsl / 256)},
        {"b512 s1 nt  full", bits<512, 1, true>, 512, 1, (unsigned)(nsl / 512)},
        {"b256 s2 nt  full", bits<256, 2, true>, 256, 2, (unsigned)(nsl / 512)},
        {"b256 s2 pl  full", bits<256, 2, false>, 256, 2, (unsigned)(nsl / 512)},
        {"b512 s2 nt  full", bits<512, 2, true>, 512, 2, (unsigned)(nsl / 1024)},
        {"b256 s1 nt  2048", bits<256, 1, true>, 256, 1, 2048},
        {"b256 s2 nt  1024", bits<256, 2, true>, 256, 2, 1024},
        {"b512 s2 nt  512", bits<512, 2, true>, 512, 2, 512},
        {"b256 s4 nt  full", bits<256, 4, true>, 256, 4, (unsigned)(nsl / 1024)},
    };
    for (int rep = 0; rep < 2; ++rep) {
        {
            for (int i = 0; i < 20; ++i) lib(i % nsets);
            HQ(hq_sync(ctx));
            double ms; u64 n;
            HQ(hq_timing_reset(ctx)); HQ(hq_timing_enable(ctx, 1));
            for (int i = 0; i < 200; ++i) lib(i % nsets);
            HQ(hq_sync(ctx)); HQ(hq_timing_enable(ctx, 0));
            HQ(hq_timing_read(ctx, &ms, &n));
            printf("%-18s per launch %.2f us  (%.0f GB/s)\n", "library", ms * 1e3 / n, G * 4.375 / (ms * 1e-3 / n) / 1e9);
        }
        for (const V &v : vs) {
            CK(hipMemsetAsync(sets[0].conf, 0, G / 8, st));
            CK(hipMemsetAsync(sets[0].outc, 0, G / 4, st));
            hipLaunchKernelGGL(v.k, v.grid, v.blk, 0, st, mk(0));
            CK(hipStreamSynchronize(st));
            CK(hipMemcpy(c.data(), sets[0].conf, G / 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(o.data(), sets[0].outc, G / 4, hipMemcpyDeviceToHost));
            const bool ok = c == rc && o == ro;
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
            for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(v.k, v.grid, v.blk, 0, st, mk(i % nsets));
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(v.k, v.grid, v.blk, 0, st, mk(i % nsets));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("%-18s per launch %.2f us  (%.0f GB/s)  %s\n", v.name, ms * 1e3 / 200, G * 4.375 / (ms * 1e-3 / 200) / 1e9, ok ? "exact" : (strncmp(v.name, "copy", 4) == 0 ? "(no decision)" : "MISMATCH"));
        }
    }
    hq_close(ctx);
    return 0;
}
