// kexp9.hip — the 0.3 us between kexp6's b_tile and the library's tiled kernel: is it the output
// pattern? b_tile (lane = groups 2i, 2i+1: one 16-B store, bit-interleaved ballots) against the
// same body with the library's row order (lane = groups i, i+64: two 8-B stores, ballots as
// they are). 1M x 3 term-start, 21 rotating sets. Not shipped.
#include "../dragonboat_amd/csrc/hq_kernels.hip"

#include <algorithm>
#include <cstring>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
#define HQ(x) do { int r_ = (x); if (r_) { fprintf(stderr, "%s:%d hq %d %s\n", __FILE__, __LINE__, r_, hq_last_error(ctx)); exit(1); } } while (0)

typedef uint64_t u64;
__device__ __forceinline__ u64x2 ld2(const u64 *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(p));
}
__device__ __forceinline__ u64 spread32_k6(unsigned x) {
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
        a.chg[w] = spread32_k6((unsigned)(b0 >> (32 * lane))) | (spread32_k6((unsigned)(b1 >> (32 * lane))) << 1);
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
                a.chg[w] = spread32_k6((unsigned)b0) | (spread32_k6((unsigned)b1) << 1);
                a.chg[w + 1] = spread32_k6((unsigned)(b0 >> 32)) | (spread32_k6((unsigned)(b1 >> 32)) << 1);
                a.fb[w] = 0;
                a.fb[w + 1] = 0;
            }
        } else if (lane < 2) {
            const u64 w = (wb >> 6) + lane;
            a.chg[w] = spread32_k6((unsigned)(b0 >> (32 * lane))) | (spread32_k6((unsigned)(b1 >> (32 * lane))) << 1);
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
            a.chg[w] = spread32_k6((unsigned)(b0 >> (32 * lane))) | (spread32_k6((unsigned)(b1 >> (32 * lane))) << 1);
            a.fb[w] = 0;
        }
        if (!LOOP) break;
    }
}


template <bool IL>
__global__ __launch_bounds__(1024, 8) void v_tile(K a) {
    const u64 lane = threadIdx.x & 63;
    const u64 wave0 = (u64)blockIdx.x * 16 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (u64 wb = wave0 * 128; wb < a.G; wb += (u64)gridDim.x * 2048) {
        const u64 *t = a.tiles + (wb / 128) * a.tw + lane * 2;
        const u64x2 m0 = ld2(t), m1 = ld2(t + 128), m2 = ld2(t + 256), ci = ld2(t + 384),
                    la = ld2(t + 512), ts = ld2(t + 640);
        const u64 q0 = med3(m0.x, m1.x, m2.x), q1 = med3(m0.y, m1.y, m2.y);
        const bool c0 = (q0 > ci.x) & (q0 >= ts.x) & (q0 <= la.x);
        const bool c1 = (q1 > ci.y) & (q1 >= ts.y) & (q1 <= la.y);
        const u64 r0 = c0 ? q0 : ci.x, r1 = c1 ? q1 : ci.y;
        const u64 b0 = __ballot(c0), b1 = __ballot(c1);
        if (IL) {
            a.out[wb + lane] = r0;
            a.out[wb + 64 + lane] = r1;
            if (lane < 2) { a.chg[(wb >> 6) + lane] = lane ? b1 : b0; a.fb[(wb >> 6) + lane] = 0; }
        } else {
            *reinterpret_cast<u64x2 *>(a.out + wb + lane * 2) = (u64x2){r0, r1};
            if (lane < 2) {
                const u64 w = (wb >> 6) + lane;
                a.chg[w] = spread32_k6((unsigned)(b0 >> (32 * lane))) | (spread32_k6((unsigned)(b1 >> (32 * lane))) << 1);
                a.fb[w] = 0;
            }
        }
    }
}

int main() {
    const uint64_t G = 1ull << 20, nw = G / 64;
    const int nsets = 21, steps = 400, reps = 12;
    hq_ctx *ctx = nullptr;
    HQ(hq_open(0, 0, &ctx));
    std::vector<hq_commit_args> tl(nsets);
    for (int s = 0; s < nsets; ++s) {
        hq_commit_args a;
        memset(&a, 0, sizeof a);
        a.G = G; a.n_max = 3; a.form = HQ_FORM_TERM_START; a.ring_len = 16; a.match_stride = G;
        void *p;
        HQ(hq_malloc_dev(ctx, G * 24, &p)); a.match = (uint64_t *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.committed_in = (uint64_t *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.committed_out = (uint64_t *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.last_index = (uint64_t *)p;
        HQ(hq_malloc_dev(ctx, G * 8, &p)); a.term_start = (uint64_t *)p;
        HQ(hq_malloc_dev(ctx, nw * 8, &p)); a.changed = (uint64_t *)p;
        HQ(hq_malloc_dev(ctx, nw * 8, &p)); a.fallback = (uint64_t *)p;
        hq_synth_spec sp = {0x5EED0001ull + ((uint64_t)s << 40), G, 1, 1, 3, 0, 16, 0};
        HQ(hq_synth_commit_dev(ctx, &sp, &a));
        HQ(hq_malloc_dev(ctx, hq_commit_tiles(G) * hq_commit_tile_words(3, 0) * 8, &p));
        HQ(hq_tile_commit_dev(ctx, &a, (uint64_t *)p));
        tl[s] = a;
        tl[s].layout = HQ_LAYOUT_TILES;
        tl[s].match = (uint64_t *)p;
        tl[s].committed_in = tl[s].last_index = tl[s].term_start = nullptr;
    }
    HQ(hq_sync(ctx));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    std::vector<CommitK> ks(nsets);
    for (int s = 0; s < nsets; ++s) ks[s] = commit_k(&tl[s]);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const char *names[] = {"library hq_commit_dev", "same kernel, direct launch",
                           "direct, 512-thread twin", "kexp6 b_tile, ctx stream",
                           "v_tile pairs (16-B store)", "v_tile i/i+64 (2 x 8-B)"};
    const int NV = 6;
    std::vector<double> us[NV];
    std::vector<K> kk(nsets);
    for (int s = 0; s < nsets; ++s) {
        K k{};
        k.tiles = tl[s].match; k.out = tl[s].committed_out; k.chg = tl[s].changed;
        k.fb = tl[s].fallback; k.G = G; k.tw = 768;
        kk[s] = k;
    }
    for (int rep = 0; rep < reps; ++rep) {
        for (int v = 0; v < NV; ++v) {
            hipStream_t sv = ctx->stream;
            auto launch = [&](int i) {
                if (v == 0) HQ(hq_commit_dev(ctx, &tl[i % nsets]));
                else if (v == 1)
                    hipLaunchKernelGGL((k_commit_big<3, 0, 2, false, true>), dim3(512), dim3(1024), 0,
                                       ctx->stream, ks[i % nsets]);
                else if (v == 2)
                    hipLaunchKernelGGL((k_commit<3, 0, 2, false, true>), dim3(1024), dim3(512), 0,
                                       ctx->stream, ks[i % nsets]);
                else if (v == 3)
                    hipLaunchKernelGGL(b_tile<true>, dim3(512), dim3(1024), 0, sv, kk[i % nsets]);
                else if (v == 4)
                    hipLaunchKernelGGL(v_tile<false>, dim3(512), dim3(1024), 0, sv, kk[i % nsets]);
                else
                    hipLaunchKernelGGL(v_tile<true>, dim3(512), dim3(1024), 0, sv, kk[i % nsets]);
            };
            for (int i = 0; i < 40; ++i) launch(i);
            CK(hipEventRecord(e0, sv));
            for (int i = 0; i < steps; ++i) launch(i);
            CK(hipEventRecord(e1, sv));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            us[v].push_back(ms * 1e3 / steps);
        }
    }
    for (int v = 0; v < NV; ++v) {
        std::sort(us[v].begin(), us[v].end());
        printf("%-28s median %6.2f us  min %6.2f\n", names[v], us[v][reps / 2], us[v][0]);
    }
    hq_close(ctx);
    return 0;
}
