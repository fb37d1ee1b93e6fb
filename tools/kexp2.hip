// kexp2.hip — C2 (term-start, n = 3, 1M groups) kernel variants: block size x groups per lane x
// nontemporal. Each variant is checked bit-exact against hq_commit_dev, then launched 400 times
// back to back (rotating 24 input sets > 1 GiB); run under rocprofv3 --kernel-trace --stats for
// per-variant kernel durations. Not shipped.
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

template <bool NT> __device__ __forceinline__ u64x2 ld2(const u64 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(p));
    return *reinterpret_cast<const u64x2 *>(p);
}
template <bool NT> __device__ __forceinline__ void st2(u64 *p, u64x2 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u64x2 *>(p));
    else *reinterpret_cast<u64x2 *>(p) = v;
}
__device__ __forceinline__ u64 med3(u64 a, u64 b, u64 c) {
    u64 lo = a < b ? a : b, hi = a < b ? b : a;
    u64 m = hi < c ? hi : c;
    return lo > m ? lo : m;
}
// bit k of the 4-bit nibble of each lane -> bit 4*lane + k of the 256-bit result, word w
__device__ __forceinline__ u64 spread16x4(unsigned x) {  // bit i -> bit 4i (16 bits)
    u64 v = x & 0xFFFF;
    v = (v | (v << 24)) & 0x000000FF000000FFull;
    v = (v | (v << 12)) & 0x000F000F000F000Full;
    v = (v | (v << 6)) & 0x0303030303030303ull;
    v = (v | (v << 3)) & 0x1111111111111111ull;
    return v;
}

struct C2 { const u64 *m; u64 stride; const u64 *cin, *last, *ts; u64 *cout, *chg; u64 G, nwords; };

// VEC groups per lane (2 or 4), each 16-byte load covers 2 groups
template <int BLK, int VEC, bool NT>
__global__ __launch_bounds__(BLK) void c2(C2 a) {
    const int lane = threadIdx.x & 63;
    const u64 wave = (u64)blockIdx.x * (BLK / 64) + (threadIdx.x >> 6);
    const u64 step = (u64)gridDim.x * BLK * VEC;
    for (u64 wb = wave * 64 * VEC; wb < a.G; wb += step) {
        const u64 g = wb + (u64)VEC * lane;
        bool c[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) c[j] = false;
        if (g + VEC <= a.G) {
            u64x2 m0[VEC / 2], m1[VEC / 2], m2[VEC / 2], ci[VEC / 2], la[VEC / 2], ts[VEC / 2];
#pragma unroll
            for (int h = 0; h < VEC / 2; ++h) {
                m0[h] = ld2<NT>(a.m + g + 2 * h);
                m1[h] = ld2<NT>(a.m + a.stride + g + 2 * h);
                m2[h] = ld2<NT>(a.m + 2 * a.stride + g + 2 * h);
                ci[h] = ld2<NT>(a.cin + g + 2 * h);
                la[h] = ld2<NT>(a.last + g + 2 * h);
                ts[h] = ld2<NT>(a.ts + g + 2 * h);
            }
#pragma unroll
            for (int h = 0; h < VEC / 2; ++h) {
                const u64 q0 = med3(m0[h].x, m1[h].x, m2[h].x), q1 = med3(m0[h].y, m1[h].y, m2[h].y);
                c[2 * h] = (q0 > ci[h].x) & (q0 >= ts[h].x) & (q0 <= la[h].x);
                c[2 * h + 1] = (q1 > ci[h].y) & (q1 >= ts[h].y) & (q1 <= la[h].y);
                u64x2 co;
                co.x = c[2 * h] ? q0 : ci[h].x;
                co.y = c[2 * h + 1] ? q1 : ci[h].y;
                st2<NT>(a.cout + g + 2 * h, co);
            }
        }
        // changed bits: lane's VEC bits are consecutive groups
        u64 b[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) b[j] = __ballot(c[j]);
        if (VEC == 4) {
            // word k covers lanes 16k..16k+15
            if (lane < 4) {
                const int k = lane;
                u64 w = 0;
#pragma unroll
                for (int j = 0; j < VEC; ++j) w |= spread16x4((unsigned)(b[j] >> (16 * k))) << j;
                const u64 wi = (wb >> 6) + k;
                if (wi < a.nwords) a.chg[wi] = w;
            }
        } else {
            if (lane < 2) {
                const int k = lane;
                u64 w = 0;
                unsigned lo0 = (unsigned)(b[0] >> (32 * k)), lo1 = (unsigned)(b[1] >> (32 * k));
#pragma unroll
                for (int i = 0; i < 32; ++i) w |= (u64)((lo0 >> i) & 1) << (2 * i) | (u64)((lo1 >> i) & 1) << (2 * i + 1);
                const u64 wi = (wb >> 6) + k;
                if (wi < a.nwords) a.chg[wi] = w;
            }
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
    struct V { const char *name; KF k; int blk, vec; unsigned cap; };
    V vs[] = {
        {"b256 v2 nt", c2<256, 2, true>, 256, 2, 1u << 30},
        {"b512 v2 nt", c2<512, 2, true>, 512, 2, 1u << 30},
        {"b1024 v2 nt", c2<1024, 2, true>, 1024, 2, 1u << 30},
        {"b1024 v2 plain", c2<1024, 2, false>, 1024, 2, 1u << 30},
        {"b256 v4 nt", c2<256, 4, true>, 256, 4, 1u << 30},
        {"b1024 v4 nt", c2<1024, 4, true>, 1024, 4, 1u << 30},
        {"b1024 v2 nt cap256", c2<1024, 2, true>, 1024, 2, 256},
        {"b1024 v4 nt cap256", c2<1024, 4, true>, 1024, 4, 256},
        {"b512 v4 nt cap512", c2<512, 4, true>, 512, 4, 512},
    };
    for (const V &v : vs) {
        u64 lanes = G / v.vec;
        unsigned grid = (unsigned)((lanes + v.blk - 1) / v.blk);
        if (grid > v.cap) grid = v.cap;
        CK(hipMemsetAsync((void *)s2[0].committed_out, 0, G * 8, st));
        CK(hipMemsetAsync((void *)s2[0].changed, 0, nw * 8, st));
        hipLaunchKernelGGL(v.k, grid, v.blk, 0, st, mk(0));
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(out.data(), s2[0].committed_out, G * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(chg.data(), s2[0].changed, nw * 8, hipMemcpyDeviceToHost));
        printf("%-22s grid %6u  %s\n", v.name, grid, (out == ref_out && chg == ref_chg) ? "exact" : "MISMATCH");
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int i = 0; i < 40; ++i) hipLaunchKernelGGL(v.k, grid, v.blk, 0, st, mk(i % nsets));
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < 400; ++i) hipLaunchKernelGGL(v.k, grid, v.blk, 0, st, mk(i % nsets));
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("   per launch %.2f us  (%.0f GB/s)\n", ms * 1e3 / 400, G * 56.0 / (ms * 1e-3 / 400) / 1e9);
    }
    hq_close(ctx);
    return 0;
}
