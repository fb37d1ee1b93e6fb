// kexp10.hip — is the headline kernel (1 M x 3 over leader-row tiles, HQ_LAYOUT_TILES_LEADER)
// at the floor its launch size sets? Beside the library call, in the same process and on the
// same rotating inputs: a copy kernel with the same geometry (1024-thread blocks, one wave per
// 128-group tile, five 16-B loads + one 16-B store per lane, no decision), and the 56-B tiles.
// Not shipped.
#include "../dragonboat_amd/csrc/hq_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)
#define HQ(x) do { int r_ = (x); if (r_) { fprintf(stderr, "%s:%d hq %d %s\n", __FILE__, __LINE__, r_, hq_last_error(ctx)); exit(1); } } while (0)

typedef uint64_t u64;

// ROWS 16-B loads per lane from one tile of ROWS x 128 u64, one 16-B store: the bytes of the
// decision kernel without the decision (G a multiple of 128, grid = G / 2048 blocks)
template <int ROWS>
__global__ __launch_bounds__(1024, 8) void floor_tile(const u64 *tiles, u64 *out) {
    const u64 wave = (u64)blockIdx.x * 16 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const u64 lane = threadIdx.x & 63;
    const u64 *t = tiles + wave * (ROWS * 128) + lane * 2;
    u64x2 x = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(t));
#pragma unroll
    for (int r = 1; r < ROWS; ++r)
        x ^= __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(t + r * 128));
    *reinterpret_cast<u64x2 *>(out + wave * 128 + lane * 2) = x;
}

// the same loads, the output as the library writes it: two 8-B stores, groups i and i + 64
__global__ __launch_bounds__(1024, 8) void floor_tile_split(const u64 *tiles, u64 *out) {
    const u64 wave = (u64)blockIdx.x * 16 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const u64 lane = threadIdx.x & 63;
    const u64 *t = tiles + wave * (5 * 128) + lane * 2;
    u64x2 x = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(t));
#pragma unroll
    for (int r = 1; r < 5; ++r)
        x ^= __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(t + r * 128));
    out[wave * 128 + lane] = x.x;
    out[wave * 128 + lane + 64] = x.y;
}

int main() {
    const uint64_t G = 1ull << 20, nw = G / 64;
    const int nsets = 24, steps = 400, reps = 12;
    hq_ctx *ctx = nullptr;
    HQ(hq_open(0, 0, &ctx));
    std::vector<hq_commit_args> t1(nsets), t2(nsets);
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
        for (int lay = 1; lay <= 2; ++lay) {
            HQ(hq_malloc_dev(ctx, hq_commit_tiles(G) * hq_commit_tile_words_for(3, 0, lay) * 8, &p));
            HQ(hq_tile_commit_as_dev(ctx, &a, (uint64_t *)p, lay));
            hq_commit_args &t = lay == 1 ? t1[s] : t2[s];
            t = a;
            t.layout = lay;
            t.match = (uint64_t *)p;
            t.committed_in = t.last_index = t.term_start = nullptr;
        }
    }
    HQ(hq_sync(ctx));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[] = {"c2tl library (48 B)", "floor 5 rows + store (48 B)",
                           "c2t library (56 B)", "floor 6 rows + store (56 B)",
                           "c2tl 512-thread twin (48 B)", "c2tl 1024, 2 tiles/wave (48 B)",
                           "floor 5 rows, two 8-B stores", "c2tl, no changed/fallback",
                           "c2tl, changed only"};
    const int NV = 9;
    std::vector<CommitK> k2(nsets);
    for (int s = 0; s < nsets; ++s) k2[s] = commit_k(&t2[s]);
    std::vector<CommitK> k3 = k2, k4 = k2;
    for (int s = 0; s < nsets; ++s) {
        k3[s].changed = k3[s].fallback = nullptr;
        k4[s].fallback = nullptr;
    }
    std::vector<double> us[NV];
    for (int rep = 0; rep < reps; ++rep) {
        for (int v = 0; v < NV; ++v) {
            auto launch = [&](int i) {
                const int s = i % nsets;
                if (v == 0) HQ(hq_commit_dev(ctx, &t2[s]));
                else if (v == 2) HQ(hq_commit_dev(ctx, &t1[s]));
                else if (v == 1)
                    hipLaunchKernelGGL(floor_tile<5>, dim3(G / 2048), dim3(1024), 0, ctx->stream,
                                       t2[s].match, t2[s].committed_out);
                else if (v == 3)
                    hipLaunchKernelGGL(floor_tile<6>, dim3(G / 2048), dim3(1024), 0, ctx->stream,
                                       t1[s].match, t1[s].committed_out);
                else if (v == 4)
                    hipLaunchKernelGGL((k_commit<3, 0, 2, false, 2>), dim3(G / 1024), dim3(512), 0,
                                       ctx->stream, k2[s]);
                else if (v == 5)
                    hipLaunchKernelGGL((k_commit_big<3, 0, 2, false, 2>), dim3(G / 4096), dim3(1024),
                                       0, ctx->stream, k2[s]);
                else if (v == 7)
                    hipLaunchKernelGGL((k_commit_big<3, 0, 2, false, 2>), dim3(G / 2048), dim3(1024),
                                       0, ctx->stream, k3[s]);
                else if (v == 8)
                    hipLaunchKernelGGL((k_commit_big<3, 0, 2, false, 2>), dim3(G / 2048), dim3(1024),
                                       0, ctx->stream, k4[s]);
                else
                    hipLaunchKernelGGL(floor_tile_split, dim3(G / 2048), dim3(1024), 0, ctx->stream,
                                       t2[s].match, t2[s].committed_out);
            };
            for (int i = 0; i < 40; ++i) launch(i);
            CK(hipEventRecord(e0, ctx->stream));
            for (int i = 0; i < steps; ++i) launch(i);
            CK(hipEventRecord(e1, ctx->stream));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            us[v].push_back(ms * 1e3 / steps);
        }
    }
    for (int v = 0; v < NV; ++v) {
        std::sort(us[v].begin(), us[v].end());
        const double bytes = (v == 2 || v == 3 ? 56.0 : 48.0) * G;
        printf("%-30s median %6.2f us  min %6.2f  (%5.0f GB/s at the median)\n", names[v],
               us[v][reps / 2], us[v][0], bytes / (us[v][reps / 2] * 1e3));
    }
    hq_close(ctx);
    return 0;
}
