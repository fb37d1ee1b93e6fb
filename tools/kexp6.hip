// kexp6.hip — same-box A/B of the 1M x 3 commit launch (term-start): the library kernel over
// columns and over 128-group tiles (hq_commit_dev), against the no-decision floors of both
// layouts (kexp5) and a loop-free tiled decision kernel. Interleaved rounds, 400 launches each
// over 21 rotated input sets (> 1.1 GiB). Not shipped.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <chrono>
#include <vector>

#include "hipquorum.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
#define HQ(x) do { int r_ = (x); if (r_) { fprintf(stderr, "%s:%d hq %d %s\n", __FILE__, __LINE__, r_, hq_last_error(ctx)); exit(1); } } while (0)

typedef uint64_t u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u64x2 ld2(const u64 *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(p));
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

struct K {
    const u64 *tiles;
    const u64 *col[6];
    u64 *out, *chg, *fb;
    u64 G, tw;
};

// floors (no decision): six 16-B loads, one 16-B store per lane
__global__ __launch_bounds__(1024) void f_soa(K a) {
    const u64 g = ((u64)blockIdx.x * 1024 + threadIdx.x) * 2;
    u64x2 x = ld2(a.col[0] + g);
#pragma unroll
    for (int c = 1; c < 6; ++c) x ^= ld2(a.col[c] + g);
    *reinterpret_cast<u64x2 *>(a.out + g) = x;
}
__global__ __launch_bounds__(1024) void f_tile(K a) {
    const u64 wave = (u64)blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const u64 *t = a.tiles + wave * 768 + lane * 2;
    u64x2 x = ld2(t);
#pragma unroll
    for (int c = 1; c < 6; ++c) x ^= ld2(t + c * 128);
    *reinterpret_cast<u64x2 *>(a.out + wave * 128 + lane * 2) = x;
}
// loop-free tiled decision (G a multiple of 128): term-start rule, changed + fallback words
template <bool FB>
__global__ __launch_bounds__(1024, 8) void d_tile(K a) {
    const u64 wave = (u64)blockIdx.x * 16 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const u64 *t = a.tiles + wave * 768 + lane * 2;
    const u64x2 m0 = ld2(t), m1 = ld2(t + 128), m2 = ld2(t + 256), ci = ld2(t + 384),
                la = ld2(t + 512), ts = ld2(t + 640);
    const u64 q0 = med3(m0.x, m1.x, m2.x), q1 = med3(m0.y, m1.y, m2.y);
    const bool c0 = (q0 > ci.x) & (q0 >= ts.x) & (q0 <= la.x);
    const bool c1 = (q1 > ci.y) & (q1 >= ts.y) & (q1 <= la.y);
    *reinterpret_cast<u64x2 *>(a.out + wave * 128 + lane * 2) = (u64x2){c0 ? q0 : ci.x, c1 ? q1 : ci.y};
    const u64 b0 = __ballot(c0), b1 = __ballot(c1);
    if (lane < 2) {
        const u64 w = wave * 2 + lane;
        a.chg[w] = spread32((unsigned)(b0 >> (32 * lane))) | (spread32((unsigned)(b1 >> (32 * lane))) << 1);
        if (FB) a.fb[w] = 0;
    }
}

// d_tile walked towards the library's commit_blocks, one feature at a time:
//   RT: tile stride from the kernel argument; LOOP: grid-stride loop; LANE0: lane 0 writes the
//   bitmap words (2 changed + 2 fallback); TAIL: the odd-G scalar tail branch
template <bool RT, bool LOOP, bool LANE0, bool TAIL>
__global__ __launch_bounds__(1024, 8) void a_tile(K a) {
    const u64 lane = threadIdx.x & 63;
    const u64 wave0 = (u64)blockIdx.x * 16 + (threadIdx.x >> 6);
    const u64 tw = RT ? a.tw : 768;
    for (u64 wb = wave0 * 128; wb < a.G; wb += (u64)gridDim.x * 2048) {
        const u64 g0 = wb + lane * 2;
        const u64 *t = a.tiles + (wb / 128) * tw + lane * 2;
        bool c0 = false, c1 = false;
        if (!TAIL || g0 + 1 < a.G) {
            const u64x2 m0 = ld2(t), m1 = ld2(t + 128), m2 = ld2(t + 256), ci = ld2(t + 384),
                        la = ld2(t + 512), ts = ld2(t + 640);
            const u64 q0 = med3(m0.x, m1.x, m2.x), q1 = med3(m0.y, m1.y, m2.y);
            c0 = (q0 > ci.x) & (q0 >= ts.x) & (q0 <= la.x);
            c1 = (q1 > ci.y) & (q1 >= ts.y) & (q1 <= la.y);
            *reinterpret_cast<u64x2 *>(a.out + g0) = (u64x2){c0 ? q0 : ci.x, c1 ? q1 : ci.y};
        } else if (g0 < a.G) {
            const u64 q0 = med3(t[0], t[128], t[256]);
            c0 = (q0 > t[384]) & (q0 >= t[640]) & (q0 <= t[512]);
            a.out[g0] = c0 ? q0 : t[384];
        }
        const u64 b0 = __ballot(c0), b1 = __ballot(c1);
        if (LANE0) {
            if (lane == 0) {
                const u64 w = wb >> 6;
                a.chg[w] = spread32((unsigned)b0) | (spread32((unsigned)b1) << 1);
                a.chg[w + 1] = spread32((unsigned)(b0 >> 32)) | (spread32((unsigned)(b1 >> 32)) << 1);
                a.fb[w] = 0;
                a.fb[w + 1] = 0;
            }
        } else if (lane < 2) {
            const u64 w = (wb >> 6) + lane;
            a.chg[w] = spread32((unsigned)(b0 >> (32 * lane))) | (spread32((unsigned)(b1 >> (32 * lane))) << 1);
            a.fb[w] = 0;
        }
        if (!LOOP) break;
    }
}

// the library's features with a wave-uniform (scalar) wave index and full-tile fast path: the
// bounds test is an s_cbranch, not an exec mask, and full tiles carry no per-lane guard
template <int PAD> struct KP { K k; u64 pad[PAD]; };
template <bool LOOP, int PAD = 0>
__device__ __forceinline__ void b_tile_body(const K &a);
template <bool LOOP>
__global__ __launch_bounds__(1024, 8) void b_tile(K a) { b_tile_body<LOOP>(a); }
template <int PAD>
__global__ __launch_bounds__(1024, 8) void b_tile_pad(KP<PAD> a) { b_tile_body<true>(a.k); }
template <bool LOOP, int PAD>
__device__ __forceinline__ void b_tile_body(const K &a) {
    const u64 lane = threadIdx.x & 63;
    const u64 wave0 = (u64)blockIdx.x * 16 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const u64 tw = a.tw;
    for (u64 wb = wave0 * 128; wb < a.G; wb += (u64)gridDim.x * 2048) {
        const u64 g0 = wb + lane * 2;
        const u64 *t = a.tiles + (wb / 128) * tw + lane * 2;
        bool c0 = false, c1 = false;
        if (wb + 128 <= a.G) {
            const u64x2 m0 = ld2(t), m1 = ld2(t + 128), m2 = ld2(t + 256), ci = ld2(t + 384),
                        la = ld2(t + 512), ts = ld2(t + 640);
            const u64 q0 = med3(m0.x, m1.x, m2.x), q1 = med3(m0.y, m1.y, m2.y);
            c0 = (q0 > ci.x) & (q0 >= ts.x) & (q0 <= la.x);
            c1 = (q1 > ci.y) & (q1 >= ts.y) & (q1 <= la.y);
            *reinterpret_cast<u64x2 *>(a.out + g0) = (u64x2){c0 ? q0 : ci.x, c1 ? q1 : ci.y};
        } else {
            for (int j = 0; j < 2; ++j) {
                if (g0 + j < a.G) {
                    const u64 q = med3(t[j], t[128 + j], t[256 + j]);
                    const bool c = (q > t[384 + j]) & (q >= t[640 + j]) & (q <= t[512 + j]);
                    a.out[g0 + j] = c ? q : t[384 + j];
                    (j ? c1 : c0) = c;
                }
            }
        }
        const u64 b0 = __ballot(c0), b1 = __ballot(c1);
        if (lane < 2) {
            const u64 w = (wb >> 6) + lane;
            a.chg[w] = spread32((unsigned)(b0 >> (32 * lane))) | (spread32((unsigned)(b1 >> (32 * lane))) << 1);
            a.fb[w] = 0;
        }
        if (!LOOP) break;
    }
}

int main() {
    const u64 G = 1ull << 20, nw = G / 64;
    const int nsets = 21;
    hq_ctx *ctx = nullptr;
    HQ(hq_open(0, 0, &ctx));
    std::vector<hq_commit_args> cols(nsets), tl(nsets);
    std::vector<u64 *> tiles(nsets);
    for (int s = 0; s < nsets; ++s) {
        hq_commit_args &a = cols[s];
        memset(&a, 0, sizeof a);
        a.G = G; a.n_max = 3; a.form = HQ_FORM_TERM_START; a.ring_len = 16; a.match_stride = G;
        void *p;
        HQ(hq_malloc_dev(ctx, G * 24, &p)); a.match = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.committed_in = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.committed_out = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.last_index = (u64 *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.term_start = (u64 *)p;
        HQ(hq_malloc_dev(ctx, nw * 8, &p)); a.changed = (u64 *)p;
        HQ(hq_malloc_dev(ctx, nw * 8, &p)); a.fallback = (u64 *)p;
        hq_synth_spec sp = {0x5EED0001ull + ((u64)s << 40), G, 1, 1, 3, 0, 16, 0};
        HQ(hq_synth_commit_dev(ctx, &sp, &a));
        HQ(hq_malloc_dev(ctx, hq_commit_tiles(G) * hq_commit_tile_words(3, 0) * 8, &p));
        tiles[s] = (u64 *)p;
        HQ(hq_tile_commit_dev(ctx, &a, tiles[s]));
        tl[s] = a;
        tl[s].layout = HQ_LAYOUT_TILES;
        tl[s].match = tiles[s];
        tl[s].committed_in = tl[s].last_index = tl[s].term_start = nullptr;
    }
    HQ(hq_sync(ctx));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    auto mk = [&](int s) {
        K k{};
        k.tiles = tiles[s];
        k.col[0] = cols[s].match; k.col[1] = cols[s].match + G; k.col[2] = cols[s].match + 2 * G;
        k.col[3] = cols[s].committed_in; k.col[4] = cols[s].last_index; k.col[5] = cols[s].term_start;
        k.out = cols[s].committed_out; k.chg = cols[s].changed; k.fb = cols[s].fallback;
        k.G = G;
        k.tw = 768;
        return k;
    };
    // reference decisions of set 0 (columns) for the exactness check of d_tile
    std::vector<u64> ref(G), ref_chg(nw), out(G), chg(nw);
    HQ(hq_commit_dev(ctx, &cols[0]));
    HQ(hq_sync(ctx));
    CK(hipMemcpy(ref.data(), cols[0].committed_out, G * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ref_chg.data(), cols[0].changed, nw * 8, hipMemcpyDeviceToHost));
    for (auto kf : {d_tile<true>, d_tile<false>}) {
        CK(hipMemset((void *)cols[0].committed_out, 0, G * 8));
        hipLaunchKernelGGL(kf, G / 2048, 1024, 0, st, mk(0));
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(out.data(), cols[0].committed_out, G * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(chg.data(), cols[0].changed, nw * 8, hipMemcpyDeviceToHost));
        printf("d_tile exact: %s\n", out == ref && chg == ref_chg ? "yes" : "NO");
    }
    const int steps = 400, reps = 12;
    struct V { const char *name; void (*k)(K); int lib; };   // lib: 1 columns, 2 tiles
    V vs[] = {{"library columns", nullptr, 1}, {"library tiles", nullptr, 2},
              {"floor soa", f_soa, 0}, {"floor tile", f_tile, 0}, {"d_tile fb", d_tile<true>, 0},
              {"d_tile", d_tile<false>, 0},
              {"a ----", a_tile<false, false, false, false>, 0},
              {"a RT", a_tile<true, false, false, false>, 0},
              {"a LOOP", a_tile<false, true, false, false>, 0},
              {"a LANE0", a_tile<false, false, true, false>, 0},
              {"a TAIL", a_tile<false, false, false, true>, 0},
              {"a all", a_tile<true, true, true, true>, 0},
              {"b scalar", b_tile<false>, 0}, {"b scalar loop", b_tile<true>, 0},
              {"b pad 64B", nullptr, 3}, {"b pad 256B", nullptr, 4}};
    const int nv = sizeof(vs) / sizeof(vs[0]);
    std::vector<std::vector<double>> us(nv), cpu_us(nv);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int rep = 0; rep < reps; ++rep) {
        for (int k = 0; k < nv; ++k) {
            const V &v = vs[k];
            if (v.lib == 1 || v.lib == 2) {
                std::vector<hq_commit_args> &a = v.lib == 2 ? tl : cols;
                for (int i = 0; i < 40; ++i) HQ(hq_commit_dev(ctx, &a[i % nsets]));
                HQ(hq_sync(ctx));
                double ms; u64 launches;
                HQ(hq_timing_reset(ctx)); HQ(hq_timing_enable(ctx, 1));
                const auto c0 = std::chrono::steady_clock::now();
                for (int i = 0; i < steps; ++i) HQ(hq_commit_dev(ctx, &a[i % nsets]));
                const auto c1 = std::chrono::steady_clock::now();
                cpu_us[k].push_back(std::chrono::duration<double, std::micro>(c1 - c0).count() / steps);
                HQ(hq_sync(ctx)); HQ(hq_timing_enable(ctx, 0));
                HQ(hq_timing_read(ctx, &ms, &launches));
                us[k].push_back(ms * 1e3 / launches);
                continue;
            }
            auto launch = [&](int i) {
                if (v.lib == 3) hipLaunchKernelGGL(b_tile_pad<8>, G / 2048, 1024, 0, st, KP<8>{mk(i % nsets), {}});
                else if (v.lib == 4) hipLaunchKernelGGL(b_tile_pad<32>, G / 2048, 1024, 0, st, KP<32>{mk(i % nsets), {}});
                else hipLaunchKernelGGL(v.k, G / 2048, 1024, 0, st, mk(i % nsets));
            };
            for (int i = 0; i < 40; ++i) launch(i);
            CK(hipEventRecord(e0, st));
            const auto c0 = std::chrono::steady_clock::now();
            for (int i = 0; i < steps; ++i) launch(i);
            const auto c1 = std::chrono::steady_clock::now();
            cpu_us[k].push_back(std::chrono::duration<double, std::micro>(c1 - c0).count() / steps);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            us[k].push_back(ms * 1e3 / steps);
        }
    }
    printf("%-16s %8s %8s %8s   (us per launch over %d reps of %d launches)\n", "variant", "median",
           "min", "max", reps, steps);
    for (int k = 0; k < nv; ++k) {
        std::vector<double> x = us[k];
        std::sort(x.begin(), x.end());
        std::vector<double> c = cpu_us[k];
        std::sort(c.begin(), c.end());
        printf("%-16s %8.2f %8.2f %8.2f   median %6.0f GB/s   host issue %5.2f us/launch\n",
               vs[k].name, x[x.size() / 2], x[0], x.back(), G * 56.0 / (x[x.size() / 2] * 1e-6) / 1e9,
               c[c.size() / 2]);
    }
    hq_close(ctx);
    return 0;
}
