// kexp.hip — kernel-variant experiments for the commit / bitmap streams (not shipped).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include tools/kexp.hip \
//        -L dragonboat_amd/lib -lhipquorum -Wl,-rpath,$PWD/dragonboat_amd/lib -o tools/kexp
// Every variant is checked bit-exact against hq_commit_dev before it is timed.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "hipquorum.h"

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)
#define HQ(x)                                                                              \
    do {                                                                                   \
        int r_ = (x);                                                                      \
        if (r_) {                                                                          \
            fprintf(stderr, "%s:%d hq rc %d %s\n", __FILE__, __LINE__, r_, hq_last_error(ctx)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef uint64_t u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ u64x2 ld2(const u64 *p) {
    if constexpr (NT) return __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(p));
    return *reinterpret_cast<const u64x2 *>(p);
}
template <bool NT>
__device__ __forceinline__ void st2(u64 *p, u64x2 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u64x2 *>(p));
    else *reinterpret_cast<u64x2 *>(p) = v;
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
__device__ __forceinline__ u64 med3(u64 a, u64 b, u64 c) {
    u64 lo = a < b ? a : b, hi = a < b ? b : a;
    u64 m = hi < c ? hi : c;
    return lo > m ? lo : m;
}

struct C2 {
    const u64 *m;
    u64 stride;
    const u64 *cin, *last, *ts;
    u64 *cout, *chg;
    u64 G, nwords;
};

// grid-stride C2 (term-start, n = 3), 2 groups per lane; BLK threads; NT loads/stores
template <int BLK, bool NT>
__global__ __launch_bounds__(BLK) void c2_v2(C2 a) {
    const int lane = threadIdx.x & 63;
    const u64 wave = (u64)blockIdx.x * (BLK / 64) + (threadIdx.x >> 6);
    const u64 step = (u64)gridDim.x * BLK * 2;
    for (u64 wb = wave * 128; wb < a.G; wb += step) {
        const u64 g = wb + 2 * lane;
        bool c0 = false, c1 = false;
        if (g + 1 < a.G) {
            u64x2 m0 = ld2<NT>(a.m + g), m1 = ld2<NT>(a.m + a.stride + g),
                  m2 = ld2<NT>(a.m + 2 * a.stride + g);
            u64x2 ci = ld2<NT>(a.cin + g), la = ld2<NT>(a.last + g), ts = ld2<NT>(a.ts + g);
            u64 q0 = med3(m0.x, m1.x, m2.x), q1 = med3(m0.y, m1.y, m2.y);
            c0 = (q0 > ci.x) & (q0 >= ts.x) & (q0 <= la.x);
            c1 = (q1 > ci.y) & (q1 >= ts.y) & (q1 <= la.y);
            u64x2 co;
            co.x = c0 ? q0 : ci.x;
            co.y = c1 ? q1 : ci.y;
            st2<NT>(a.cout + g, co);
        }
        u64 b0 = __ballot(c0), b1 = __ballot(c1);
        if (lane == 0) {
            u64 w = wb >> 6;
            a.chg[w] = spread32((unsigned)b0) | (spread32((unsigned)b1) << 1);
            if (w + 1 < a.nwords) a.chg[w + 1] = spread32((unsigned)(b0 >> 32)) | (spread32((unsigned)(b1 >> 32)) << 1);
        }
    }
}

// 1 group per lane, 8-byte loads
template <int BLK, bool NT>
__global__ __launch_bounds__(BLK) void c2_v1(C2 a) {
    const int lane = threadIdx.x & 63;
    const u64 wave = (u64)blockIdx.x * (BLK / 64) + (threadIdx.x >> 6);
    const u64 step = (u64)gridDim.x * BLK;
    for (u64 wb = wave * 64; wb < a.G; wb += step) {
        const u64 g = wb + lane;
        bool c0 = false;
        if (g < a.G) {
            u64 q = med3(a.m[g], a.m[a.stride + g], a.m[2 * a.stride + g]);
            u64 ci = a.cin[g];
            c0 = (q > ci) & (q >= a.ts[g]) & (q <= a.last[g]);
            a.cout[g] = c0 ? q : ci;
        }
        u64 b0 = __ballot(c0);
        if (lane == 0) a.chg[wb >> 6] = b0;
    }
}

// pure stream with the same bytes: read 6 u64 columns (16 B/lane), write 1 column
template <int BLK>
__global__ __launch_bounds__(BLK) void copy_like(C2 a) {
    const u64 step = (u64)gridDim.x * BLK * 2;
    for (u64 g = ((u64)blockIdx.x * BLK + threadIdx.x) * 2; g + 1 < a.G; g += step) {
        u64x2 s = ld2<false>(a.m + g) + ld2<false>(a.m + a.stride + g) +
                  ld2<false>(a.m + 2 * a.stride + g) + ld2<false>(a.cin + g) +
                  ld2<false>(a.last + g) + ld2<false>(a.ts + g);
        st2<false>(a.cout + g, s);
    }
}

__global__ void empty_kernel() {}

// ---- C3: ring form n = 5 -------------------------------------------------------------------
struct C3 {
    const u64 *m;
    u64 stride;
    const u64 *cin, *last, *term, *ring;
    u64 *cout, *chg, *fb;
    u64 G, nwords;
    unsigned R;
};

__device__ __forceinline__ void ce(u64 &a, u64 &b) {
    u64 lo = a < b ? a : b, hi = a < b ? b : a;
    a = lo;
    b = hi;
}
__device__ __forceinline__ u64 med5(u64 a, u64 b, u64 c, u64 d, u64 e) {
    // median of 5 via 7 compare-exchanges (selection network)
    ce(a, b); ce(c, d); ce(a, c); ce(b, d);  // a = min of 4 (discard), d = max of 4 (discard)
    ce(b, e); ce(b, c);                        // b = min(b, c, e) (discard)
    return c < e ? c : e;                      // median = min(c, e)
}

struct Prep {
    u64 q, cin;
    bool cand, fb;
    u64 term;
};

__device__ __forceinline__ Prep prep5(u64 m0, u64 m1, u64 m2, u64 m3, u64 m4, u64 cin, u64 last,
                                      u64 term, unsigned R) {
    Prep p;
    p.q = med5(m0, m1, m2, m3, m4);
    p.cin = cin;
    p.term = term;
    p.fb = (term == 0) | (cin > last) | (last - cin > R);
    p.cand = !p.fb && p.q > cin && p.q <= last;
    return p;
}

// persistent, software-pipelined: gather of chunk i overlaps the column loads of chunk i+1
template <int BLK>
__global__ __launch_bounds__(BLK) void c3_pipe(C3 a) {
    const int lane = threadIdx.x & 63;
    const u64 nw = (u64)gridDim.x * (BLK / 64);
    const u64 wave = (u64)blockIdx.x * (BLK / 64) + (threadIdx.x >> 6);
    const u64 nchunks = (a.G + 127) / 128;
    u64 c = wave;
    if (c >= nchunks) return;
    auto loadc = [&](u64 chunk, u64x2 (&mm)[5], u64x2 &ci, u64x2 &la, u64x2 &te) {
        const u64 g = chunk * 128 + 2 * lane;
        if (g + 1 < a.G) {
#pragma unroll
            for (int s = 0; s < 5; ++s) mm[s] = ld2<false>(a.m + s * a.stride + g);
            ci = ld2<false>(a.cin + g);
            la = ld2<false>(a.last + g);
            te = ld2<false>(a.term + g);
        } else {
#pragma unroll
            for (int s = 0; s < 5; ++s) mm[s] = (u64x2){0, 0};
            ci = (u64x2){0, 0};
            la = (u64x2){0, 0};
            te = (u64x2){1, 1};
        }
    };
    u64x2 mm[5], ci, la, te;
    loadc(c, mm, ci, la, te);
    for (;;) {
        const u64 g = c * 128 + 2 * lane;
        Prep p0 = prep5(mm[0].x, mm[1].x, mm[2].x, mm[3].x, mm[4].x, ci.x, la.x, te.x, a.R);
        Prep p1 = prep5(mm[0].y, mm[1].y, mm[2].y, mm[3].y, mm[4].y, ci.y, la.y, te.y, a.R);
        const bool valid = g + 1 < a.G;
        p0.cand &= valid;
        p1.cand &= valid;
        u64 lt0 = 0, lt1 = 0;
        if (p0.cand) lt0 = a.ring[g * a.R + (p0.q & (a.R - 1))];
        if (p1.cand) lt1 = a.ring[(g + 1) * a.R + (p1.q & (a.R - 1))];
        const u64 cn = c + nw;
        if (cn < nchunks) loadc(cn, mm, ci, la, te);
        const bool c0 = p0.cand && lt0 == p0.term, c1 = p1.cand && lt1 == p1.term;
        if (valid) {
            u64x2 co;
            co.x = c0 ? p0.q : p0.cin;
            co.y = c1 ? p1.q : p1.cin;
            st2<false>(a.cout + g, co);
        }
        const u64 b0 = __ballot(c0), b1 = __ballot(c1);
        const u64 f0 = __ballot(p0.fb && valid), f1 = __ballot(p1.fb && valid);
        if (lane == 0) {
            const u64 w = (c * 128) >> 6;
            a.chg[w] = spread32((unsigned)b0) | (spread32((unsigned)b1) << 1);
            a.fb[w] = spread32((unsigned)f0) | (spread32((unsigned)f1) << 1);
            if (w + 1 < a.nwords) {
                a.chg[w + 1] = spread32((unsigned)(b0 >> 32)) | (spread32((unsigned)(b1 >> 32)) << 1);
                a.fb[w + 1] = spread32((unsigned)(f0 >> 32)) | (spread32((unsigned)(f1 >> 32)) << 1);
            }
        }
        if (cn >= nchunks) break;
        c = cn;
    }
}

// non-pipelined grid-stride version of the same arithmetic (baseline for the pipe)
template <int BLK>
__global__ __launch_bounds__(BLK) void c3_flat(C3 a) {
    const int lane = threadIdx.x & 63;
    const u64 wave = (u64)blockIdx.x * (BLK / 64) + (threadIdx.x >> 6);
    const u64 step = (u64)gridDim.x * BLK * 2;
    for (u64 wb = wave * 128; wb < a.G; wb += step) {
        const u64 g = wb + 2 * lane;
        bool c0 = false, c1 = false, f0 = false, f1 = false;
        if (g + 1 < a.G) {
            u64x2 mm[5];
#pragma unroll
            for (int s = 0; s < 5; ++s) mm[s] = ld2<false>(a.m + s * a.stride + g);
            u64x2 ci = ld2<false>(a.cin + g), la = ld2<false>(a.last + g), te = ld2<false>(a.term + g);
            Prep p0 = prep5(mm[0].x, mm[1].x, mm[2].x, mm[3].x, mm[4].x, ci.x, la.x, te.x, a.R);
            Prep p1 = prep5(mm[0].y, mm[1].y, mm[2].y, mm[3].y, mm[4].y, ci.y, la.y, te.y, a.R);
            u64 lt0 = 0, lt1 = 0;
            if (p0.cand) lt0 = a.ring[g * a.R + (p0.q & (a.R - 1))];
            if (p1.cand) lt1 = a.ring[(g + 1) * a.R + (p1.q & (a.R - 1))];
            c0 = p0.cand && lt0 == p0.term;
            c1 = p1.cand && lt1 == p1.term;
            f0 = p0.fb;
            f1 = p1.fb;
            u64x2 co;
            co.x = c0 ? p0.q : p0.cin;
            co.y = c1 ? p1.q : p1.cin;
            st2<false>(a.cout + g, co);
        }
        const u64 b0 = __ballot(c0), b1 = __ballot(c1), x0 = __ballot(f0), x1 = __ballot(f1);
        if (lane == 0) {
            const u64 w = wb >> 6;
            a.chg[w] = spread32((unsigned)b0) | (spread32((unsigned)b1) << 1);
            a.fb[w] = spread32((unsigned)x0) | (spread32((unsigned)x1) << 1);
            if (w + 1 < a.nwords) {
                a.chg[w + 1] = spread32((unsigned)(b0 >> 32)) | (spread32((unsigned)(b1 >> 32)) << 1);
                a.fb[w + 1] = spread32((unsigned)(x0 >> 32)) | (spread32((unsigned)(x1 >> 32)) << 1);
            }
        }
    }
}

// ------------------------------------------------------------------------------ harness -----
struct Timer {
    std::vector<hipEvent_t> a, b;
    Timer(int n) : a(n), b(n) {
        for (int i = 0; i < n; ++i) { CK(hipEventCreate(&a[i])); CK(hipEventCreate(&b[i])); }
    }
};

static double time_variant(hipStream_t st, int nsets, int iters,
                           const std::function<void(int, hipStream_t)> &launch, double *wall_us) {
    Timer t(iters);
    hipEvent_t w0, w1;
    CK(hipEventCreate(&w0));
    CK(hipEventCreate(&w1));
    for (int i = 0; i < 20; ++i) launch(i % nsets, st);
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(w0, st));
    for (int i = 0; i < iters; ++i) {
        CK(hipEventRecord(t.a[i], st));
        launch(i % nsets, st);
        CK(hipEventRecord(t.b[i], st));
    }
    CK(hipEventRecord(w1, st));
    CK(hipStreamSynchronize(st));
    double sum = 0;
    std::vector<float> v(iters);
    for (int i = 0; i < iters; ++i) {
        CK(hipEventElapsedTime(&v[i], t.a[i], t.b[i]));
        sum += v[i];
    }
    float wall;
    CK(hipEventElapsedTime(&wall, w0, w1));
    *wall_us = wall * 1e3 / iters;
    std::sort(v.begin(), v.end());
    return v[iters / 2] * 1e3;  // median kernel us
}

int main(int argc, char **argv) {
    const u64 G = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 20);
    const int iters = 200;
    hq_ctx *ctx = nullptr;
    HQ(hq_open(0, 0, &ctx));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const u64 nw = (G + 63) / 64;

    // ---------------- C2 sets
    const int n2 = 3;
    const u64 set_bytes2 = G * 8 * (n2 + 3);
    const int nsets2 = std::max<u64>(4, (u64)(1.1 * (1ull << 30)) / set_bytes2 + 1);
    std::vector<hq_commit_args> s2(nsets2);
    for (int s = 0; s < nsets2; ++s) {
        hq_commit_args &a = s2[s];
        memset(&a, 0, sizeof a);
        a.G = G; a.n_max = n2; a.form = HQ_FORM_TERM_START; a.ring_len = 16; a.match_stride = G;
        void *p;
        HQ(hq_malloc_dev(ctx, G * 8 * n2, &p)); a.match = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.committed_in = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.committed_out = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.last_index = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.term_start = (u64 *)p;
        HQ(hq_malloc_dev(ctx, nw * 8, &p)); a.changed = (u64 *)p;
        HQ(hq_malloc_dev(ctx, nw * 8, &p)); a.fallback = (u64 *)p;
        hq_synth_spec sp = {0x5EED0001ull + ((u64)s << 40), G, 1, 1, (uint32_t)n2, 0, 16, 0};
        HQ(hq_synth_commit_dev(ctx, &sp, &a));
    }
    HQ(hq_sync(ctx));
    u64 *ref_out, *ref_chg;
    CK(hipMalloc(&ref_out, G * 8));
    CK(hipMalloc(&ref_chg, nw * 8));
    auto mk2 = [&](int s) {
        const hq_commit_args &a = s2[s];
        return C2{a.match, a.match_stride, a.committed_in, a.last_index, a.term_start,
                  a.committed_out, a.changed, G, nw};
    };
    auto check2 = [&](const char *name, const std::function<void(int, hipStream_t)> &launch) {
        // reference via the library, then the variant; compare out + changed
        hq_commit_args a = s2[0];
        HQ(hq_commit_dev(ctx, &a));
        HQ(hq_sync(ctx));
        CK(hipMemcpy(ref_out, a.committed_out, G * 8, hipMemcpyDeviceToDevice));
        CK(hipMemcpy(ref_chg, a.changed, nw * 8, hipMemcpyDeviceToDevice));
        CK(hipMemsetAsync((void *)a.committed_out, 0, G * 8, st));
        CK(hipMemsetAsync((void *)a.changed, 0, nw * 8, st));
        launch(0, st);
        CK(hipStreamSynchronize(st));
        std::vector<u64> x(G), y(G), cx(nw), cy(nw);
        CK(hipMemcpy(x.data(), ref_out, G * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(y.data(), a.committed_out, G * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(cx.data(), ref_chg, nw * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(cy.data(), a.changed, nw * 8, hipMemcpyDeviceToHost));
        bool ok = x == y && cx == cy;
        if (!ok) printf("  %-28s MISMATCH\n", name);
        return ok;
    };
    const double bytes2 = (double)G * (8 * n2 + 32);
    struct V { std::string name; std::function<void(int, hipStream_t)> fn; bool exact; };
    std::vector<V> v2;
    auto grid = [&](u64 lanes, int blk, int cap) {
        u64 b = (lanes + blk - 1) / blk;
        return (unsigned)std::min<u64>(b, cap);
    };
    v2.push_back({"lib hq_commit_dev", [&](int s, hipStream_t) { HQ(hq_commit_dev(ctx, &s2[s])); }, true});
    for (int cap : {1024, 2048, 4096}) {
        v2.push_back({"v2 blk256 cap" + std::to_string(cap), [&, cap](int s, hipStream_t t) {
                          hipLaunchKernelGGL((c2_v2<256, false>), grid(G / 2, 256, cap), 256, 0, t, mk2(s));
                      }, true});
    }
    v2.push_back({"v2 blk256 NT", [&](int s, hipStream_t t) {
                      hipLaunchKernelGGL((c2_v2<256, true>), grid(G / 2, 256, 4096), 256, 0, t, mk2(s));
                  }, true});
    v2.push_back({"v2 blk512", [&](int s, hipStream_t t) {
                      hipLaunchKernelGGL((c2_v2<512, false>), grid(G / 2, 512, 4096), 512, 0, t, mk2(s));
                  }, true});
    v2.push_back({"v2 blk1024", [&](int s, hipStream_t t) {
                      hipLaunchKernelGGL((c2_v2<1024, false>), grid(G / 2, 1024, 4096), 1024, 0, t, mk2(s));
                  }, true});
    v2.push_back({"v1 blk256", [&](int s, hipStream_t t) {
                      hipLaunchKernelGGL((c2_v1<256, false>), grid(G, 256, 8192), 256, 0, t, mk2(s));
                  }, true});
    v2.push_back({"v1 blk256 NT", [&](int s, hipStream_t t) {
                      hipLaunchKernelGGL((c2_v1<256, true>), grid(G, 256, 8192), 256, 0, t, mk2(s));
                  }, true});
    v2.push_back({"copy-like (same bytes)", [&](int s, hipStream_t t) {
                      hipLaunchKernelGGL((copy_like<256>), grid(G / 2, 256, 4096), 256, 0, t, mk2(s));
                  }, false});
    v2.push_back({"empty kernel", [&](int, hipStream_t t) {
                      hipLaunchKernelGGL(empty_kernel, 1, 64, 0, t);
                  }, false});
    printf("C2: G=%llu n=3 term-start, %d sets, algorithmic %.1f MB/launch\n", G, nsets2, bytes2 / 1e6);
    for (auto &v : v2)
        if (v.exact && v.name != "lib hq_commit_dev") check2(v.name.c_str(), v.fn);
    for (int round = 0; round < 2; ++round)
        for (auto &v : v2) {
            double wall;
            double k = time_variant(st, nsets2, iters, v.fn, &wall);
            printf("  %-28s kernel %7.2f us  (%6.0f GB/s)  wall/launch %7.2f us\n", v.name.c_str(), k,
                   bytes2 / k / 1e3, wall);
        }

    // ---------------- C3 sets (ring, n = 5)
    const int n3 = 5;
    const u64 set_bytes3 = G * 8 * (n3 + 4) + G * 128;
    const int nsets3 = std::max<u64>(4, (u64)(1.1 * (1ull << 30)) / set_bytes3 + 1);
    std::vector<hq_commit_args> s3(nsets3);
    for (int s = 0; s < nsets3; ++s) {
        hq_commit_args &a = s3[s];
        memset(&a, 0, sizeof a);
        a.G = G; a.n_max = n3; a.form = HQ_FORM_TERM_RING; a.ring_len = 16; a.match_stride = G;
        void *p;
        HQ(hq_malloc_dev(ctx, G * 8 * n3, &p)); a.match = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.committed_in = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.committed_out = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.last_index = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.term = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8 * 16, &p)); a.ring = (u64 *)p;
        HQ(hq_malloc_dev(ctx, nw * 8, &p)); a.changed = (u64 *)p;
        HQ(hq_malloc_dev(ctx, nw * 8, &p)); a.fallback = (u64 *)p;
        hq_synth_spec sp = {0x5EED0002ull + ((u64)s << 40), G, 1, 1, (uint32_t)n3, 0, 16, 0};
        HQ(hq_synth_commit_dev(ctx, &sp, &a));
    }
    HQ(hq_sync(ctx));
    auto mk3 = [&](int s) {
        const hq_commit_args &a = s3[s];
        return C3{a.match, a.match_stride, a.committed_in, a.last_index, a.term, a.ring,
                  a.committed_out, a.changed, a.fallback, G, nw, 16};
    };
    auto check3 = [&](const char *name, const std::function<void(int, hipStream_t)> &launch) {
        hq_commit_args a = s3[0];
        HQ(hq_commit_dev(ctx, &a));
        HQ(hq_sync(ctx));
        std::vector<u64> x(G), y(G), cx(nw), cy(nw);
        CK(hipMemcpy(x.data(), a.committed_out, G * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(cx.data(), a.changed, nw * 8, hipMemcpyDeviceToHost));
        CK(hipMemsetAsync((void *)a.committed_out, 0, G * 8, st));
        CK(hipMemsetAsync((void *)a.changed, 0, nw * 8, st));
        launch(0, st);
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(y.data(), a.committed_out, G * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(cy.data(), a.changed, nw * 8, hipMemcpyDeviceToHost));
        if (!(x == y && cx == cy)) printf("  %-28s MISMATCH\n", name);
    };
    const double bytes3 = (double)G * (8 * n3 + 40);
    std::vector<V> v3;
    v3.push_back({"lib hq_commit_dev", [&](int s, hipStream_t) { HQ(hq_commit_dev(ctx, &s3[s])); }, true});
    v3.push_back({"flat blk256", [&](int s, hipStream_t t) {
                      hipLaunchKernelGGL((c3_flat<256>), grid(G / 2, 256, 4096), 256, 0, t, mk3(s));
                  }, true});
    for (int per_cu : {2, 4, 8}) {
        v3.push_back({"pipe blk256 x" + std::to_string(per_cu) + "/CU", [&, per_cu](int s, hipStream_t t) {
                          hipLaunchKernelGGL((c3_pipe<256>), 256 * per_cu, 256, 0, t, mk3(s));
                      }, true});
    }
    v3.push_back({"pipe blk512 x4/CU", [&](int s, hipStream_t t) {
                      hipLaunchKernelGGL((c3_pipe<512>), 256 * 4, 512, 0, t, mk3(s));
                  }, true});
    printf("C3: G=%llu n=5 ring R=16, %d sets, algorithmic %.1f MB/launch\n", G, nsets3, bytes3 / 1e6);
    for (auto &v : v3)
        if (v.name != "lib hq_commit_dev") check3(v.name.c_str(), v.fn);
    for (int round = 0; round < 2; ++round)
        for (auto &v : v3) {
            double wall;
            double k = time_variant(st, nsets3, iters, v.fn, &wall);
            printf("  %-28s kernel %7.2f us  (%6.0f GB/s)  wall/launch %7.2f us\n", v.name.c_str(), k,
                   bytes3 / k / 1e3, wall);
        }
    hq_close(ctx);
    return 0;
}
