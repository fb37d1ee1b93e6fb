// kexp3.hip — C2 (term-start, n = 3, 1M groups) store-policy variants: the end-of-kernel release
// writes back the launch's dirty L2 lines (MI355X_MICROARCH.md "boundary": + B / 6 TB/s), so a
// write-through store (sc1) may shorten the dependent-launch boundary. Each variant is checked
// bit-exact against hq_commit_dev, then launched 400 times back to back (rotating 24 input sets
// > 1 GiB), timed with events. Not shipped.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "hipquorum.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
#define HQ(x) do { int r_ = (x); if (r_) { fprintf(stderr, "%s:%d hq %d %s\n", __FILE__, __LINE__, r_, hq_last_error(ctx)); exit(1); } } while (0)

typedef uint64_t u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

enum { ST_NT = 0, ST_PLAIN = 1, ST_SC1 = 2, ST_SC0SC1 = 3, ST_NTSC1 = 4, ST_SC0 = 5 };

__device__ __forceinline__ u64x2 ld2(const u64 *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(p));
}
template <int ST> __device__ __forceinline__ void st2(u64 *p, u64x2 v) {
    if constexpr (ST == ST_NT) __builtin_nontemporal_store(v, reinterpret_cast<u64x2 *>(p));
    else if constexpr (ST == ST_PLAIN) *reinterpret_cast<u64x2 *>(p) = v;
    else if constexpr (ST == ST_SC1) asm volatile("global_store_dwordx4 %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
    else if constexpr (ST == ST_SC0SC1) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" :: "v"(p), "v"(v) : "memory");
    else if constexpr (ST == ST_NTSC1) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" :: "v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc0" :: "v"(p), "v"(v) : "memory");
}
template <int ST> __device__ __forceinline__ void st1(u64 *p, u64 v) {
    if constexpr (ST == ST_NT) __builtin_nontemporal_store(v, p);
    else if constexpr (ST == ST_PLAIN) *p = v;
    else if constexpr (ST == ST_SC1) asm volatile("global_store_dwordx2 %0, %1, off sc1" :: "v"(p), "v"(v) : "memory");
    else if constexpr (ST == ST_SC0SC1) asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" :: "v"(p), "v"(v) : "memory");
    else if constexpr (ST == ST_NTSC1) asm volatile("global_store_dwordx2 %0, %1, off sc1 nt" :: "v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx2 %0, %1, off sc0" :: "v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ u64 med3(u64 a, u64 b, u64 c) {
    u64 lo = a < b ? a : b, hi = a < b ? b : a;
    u64 m = hi < c ? hi : c;
    return lo > m ? lo : m;
}
__device__ __forceinline__ u64 spread32(unsigned x) {
    u64 v = x;
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;
    v = (v | (v << 1)) & 0x5555555555555555ull;
    return v;
}

struct C2 { const u64 *m; u64 stride; const u64 *cin, *last, *ts; u64 *cout, *chg; u64 G, nwords; };

template <int ST, int BLK = 512, bool XCD = false>
__global__ __launch_bounds__(BLK) void c2(C2 a) {
    const int lane = threadIdx.x & 63;
    // XCD-aware: workgroups are dealt round-robin over the 8 XCDs (blockIdx % 8); remap so that
    // each XCD streams one contiguous eighth of the batch
    const u64 nb = gridDim.x;
    const u64 bid = XCD && nb % 8 == 0 ? (blockIdx.x % 8) * (nb / 8) + blockIdx.x / 8 : blockIdx.x;
    const u64 wave = bid * (BLK / 64) + (threadIdx.x >> 6);
    const u64 step = (u64)gridDim.x * BLK * 2;
    for (u64 wb = wave * 128; wb < a.G; wb += step) {
        const u64 g = wb + 2 * (u64)lane;
        bool c0 = false, c1 = false;
        if (g + 2 <= a.G) {
            const u64x2 m0 = ld2(a.m + g), m1 = ld2(a.m + a.stride + g), m2 = ld2(a.m + 2 * a.stride + g);
            const u64x2 ci = ld2(a.cin + g), la = ld2(a.last + g), ts = ld2(a.ts + g);
            const u64 q0 = med3(m0.x, m1.x, m2.x), q1 = med3(m0.y, m1.y, m2.y);
            c0 = (q0 > ci.x) & (q0 >= ts.x) & (q0 <= la.x);
            c1 = (q1 > ci.y) & (q1 >= ts.y) & (q1 <= la.y);
            st2<ST>(a.cout + g, (u64x2){c0 ? q0 : ci.x, c1 ? q1 : ci.y});
        }
        const u64 b0 = __ballot(c0), b1 = __ballot(c1);
        if (lane < 2) {
            const u64 w = spread32((unsigned)(b0 >> (32 * lane))) | (spread32((unsigned)(b1 >> (32 * lane))) << 1);
            const u64 wi = (wb >> 6) + lane;
            if (wi < a.nwords) st1<ST>(a.chg + wi, w);
        }
    }
}

// the same bytes with no decision: 6 x 16-B loads per lane, one 16-B store (xor of the loads so
// nothing is dead) — the floor for one 1M-group launch of this footprint
template <int BLK>
__global__ __launch_bounds__(BLK) void copy_like(C2 a) {
    const u64 wave = (u64)blockIdx.x * (BLK / 64) + (threadIdx.x >> 6);
    const u64 step = (u64)gridDim.x * BLK * 2;
    for (u64 wb = wave * 128; wb < a.G; wb += step) {
        const u64 g = wb + 2 * (u64)(threadIdx.x & 63);
        if (g + 2 <= a.G) {
            const u64x2 m0 = ld2(a.m + g), m1 = ld2(a.m + a.stride + g), m2 = ld2(a.m + 2 * a.stride + g);
            const u64x2 ci = ld2(a.cin + g), la = ld2(a.last + g), ts = ld2(a.ts + g);
            *reinterpret_cast<u64x2 *>(a.cout + g) = m0 ^ m1 ^ m2 ^ ci ^ la ^ ts;
        }
    }
}

int main() {
    const u64 G = 1ull << 20, nw = G / 64;
    hq_ctx *ctx = nullptr;
    HQ(hq_open(0, 0, &ctx));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const int nsets = 24;
    std::vector<hq_commit_args> s2(nsets);
    for (int s = 0; s < nsets; ++s) {
        hq_commit_args &a = s2[s];
        memset(&a, 0, sizeof a);
        a.G = G; a.n_max = 3; a.form = HQ_FORM_TERM_START; a.ring_len = 16; a.match_stride = G;
        void *p;
        HQ(hq_malloc_dev(ctx, G * 24, &p)); a.match = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.committed_in = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.committed_out = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.last_index = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.term_start = (u64 *)p;
        HQ(hq_malloc_dev(ctx, nw * 8, &p)); a.changed = (u64 *)p;
        hq_synth_spec sp = {0x5EED0001ull + ((u64)s << 40), G, 1, 1, 3, 0, 16, 0};
        HQ(hq_synth_commit_dev(ctx, &sp, &a));
    }
    HQ(hq_sync(ctx));
    std::vector<u64> ref_out(G), ref_chg(nw), out(G), chg(nw);
    HQ(hq_commit_dev(ctx, &s2[0]));
    HQ(hq_sync(ctx));
    CK(hipMemcpy(ref_out.data(), s2[0].committed_out, G * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ref_chg.data(), s2[0].changed, nw * 8, hipMemcpyDeviceToHost));
    auto mk = [&](int s) {
        const hq_commit_args &a = s2[s];
        return C2{a.match, G, a.committed_in, a.last_index, a.term_start, a.committed_out, a.changed, G, nw};
    };
    typedef void (*KF)(C2);
    struct V { const char *name; KF k; int blk; unsigned grid; };
    const unsigned g512 = (unsigned)(G / 2 / 512);
    V vs[] = {{"copy-like b1024", copy_like<1024>, 1024, g512 / 2},
              {"copy-like b512", copy_like<512>, 512, g512},
              {"plain b1024", c2<ST_PLAIN, 1024>, 1024, g512 / 2},
              {"plain b1024 xcd", c2<ST_PLAIN, 1024, true>, 1024, g512 / 2},
              {"plain b512 xcd", c2<ST_PLAIN, 512, true>, 512, g512},
              {"plain b512", c2<ST_PLAIN, 512>, 512, g512},
              {"plain b256", c2<ST_PLAIN, 256>, 256, 2 * g512},
              {"plain b1024", c2<ST_PLAIN, 1024>, 1024, g512 / 2},
              {"plain b512 g768", c2<ST_PLAIN, 512>, 512, 768},
              {"plain b512 g512", c2<ST_PLAIN, 512>, 512, 512},
              {"plain b256 g1024", c2<ST_PLAIN, 256>, 256, 1024},
              {"plain b512 g2048", c2<ST_PLAIN, 512>, 512, 2048},
              {"sc0", c2<ST_SC0, 512>, 512, g512}};
    for (int rep = 0; rep < 2; ++rep) {
        // library kernel for reference
        {
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
            for (int i = 0; i < 40; ++i) HQ(hq_commit_dev(ctx, &s2[i % nsets]));
            HQ(hq_sync(ctx));
            double ms_tot; u64 launches;
            HQ(hq_timing_reset(ctx)); HQ(hq_timing_enable(ctx, 1));
            for (int i = 0; i < 400; ++i) HQ(hq_commit_dev(ctx, &s2[i % nsets]));
            HQ(hq_sync(ctx)); HQ(hq_timing_enable(ctx, 0));
            HQ(hq_timing_read(ctx, &ms_tot, &launches));
            printf("%-10s per launch %.2f us  (%.0f GB/s)\n", "library", ms_tot * 1e3 / launches, G * 56.0 / (ms_tot * 1e-3 / launches) / 1e9);
        }
        for (const V &v : vs) {
            CK(hipMemsetAsync((void *)s2[0].committed_out, 0, G * 8, st));
            CK(hipMemsetAsync((void *)s2[0].changed, 0, nw * 8, st));
            hipLaunchKernelGGL(v.k, v.grid, v.blk, 0, st, mk(0));
            CK(hipStreamSynchronize(st));
            CK(hipMemcpy(out.data(), s2[0].committed_out, G * 8, hipMemcpyDeviceToHost));
            CK(hipMemcpy(chg.data(), s2[0].changed, nw * 8, hipMemcpyDeviceToHost));
            const bool ok = out == ref_out && chg == ref_chg;
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
            for (int i = 0; i < 40; ++i) hipLaunchKernelGGL(v.k, v.grid, v.blk, 0, st, mk(i % nsets));
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < 400; ++i) hipLaunchKernelGGL(v.k, v.grid, v.blk, 0, st, mk(i % nsets));
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("%-10s per launch %.2f us  (%.0f GB/s)  %s\n", v.name, ms * 1e3 / 400, G * 56.0 / (ms * 1e-3 / 400) / 1e9, ok ? "exact" : (strncmp(v.name, "copy", 4) == 0 ? "(no decision)" : "MISMATCH"));
        }
    }
    hq_close(ctx);
    return 0;
}
