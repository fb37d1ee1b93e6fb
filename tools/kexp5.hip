// kexp5.hip — stream-layout floor for the commit launch: does reading the six input columns of
// a 3-voter group (3 match rows, committed, last, term_start; 48 B) as six separate column
// streams cost bandwidth against reading the same bytes as ONE contiguous stream of 128-group
// tiles (AoSoA: [m0 x128][m1 x128][m2 x128][cin x128][last x128][ts x128], 6 KB per tile)?
// No decision is taken: each lane xors its loads and stores 16 B (the committed column), so
// only the data movement is timed. 1M and 8M groups, inputs rotated past the Infinity Cache.
// Not shipped.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

typedef unsigned long long u64;
typedef u64 u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u64x2 ld2(const u64 *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(p));
}

struct Cols {
    const u64 *col[6];   // soa: six column bases; tile: col[0] = tile array
    u64 *out;
    u64 G;
};

// six column streams + one output stream (the library's layout)
__global__ __launch_bounds__(1024) void k_soa(Cols a) {
    const u64 g = ((u64)blockIdx.x * 1024 + threadIdx.x) * 2;
    if (g + 2 > a.G) return;
    u64x2 x = ld2(a.col[0] + g);
#pragma unroll
    for (int c = 1; c < 6; ++c) x ^= ld2(a.col[c] + g);
    *reinterpret_cast<u64x2 *>(a.out + g) = x;
}

// one contiguous stream of 128-group tiles; a wave owns one tile (64 lanes x 2 groups)
__global__ __launch_bounds__(1024) void k_tile(Cols a) {
    const u64 wave = (u64)blockIdx.x * 16 + (threadIdx.x >> 6);
    const u64 lane = threadIdx.x & 63;
    const u64 g = wave * 128 + lane * 2;
    if (g + 2 > a.G) return;
    const u64 *t = a.col[0] + wave * (128 * 6) + lane * 2;
    u64x2 x = ld2(t);
#pragma unroll
    for (int c = 1; c < 6; ++c) x ^= ld2(t + c * 128);
    *reinterpret_cast<u64x2 *>(a.out + g) = x;
}

// the tile stream, result written back into the tile's committed row (in place: one stream)
__global__ __launch_bounds__(1024) void k_tile_inplace(Cols a) {
    const u64 wave = (u64)blockIdx.x * 16 + (threadIdx.x >> 6);
    const u64 lane = threadIdx.x & 63;
    const u64 g = wave * 128 + lane * 2;
    if (g + 2 > a.G) return;
    u64 *t = const_cast<u64 *>(a.col[0]) + wave * (128 * 6) + lane * 2;
    u64x2 x = ld2(t);
#pragma unroll
    for (int c = 1; c < 6; ++c) x ^= ld2(t + c * 128);
    *reinterpret_cast<u64x2 *>(t + 3 * 128) = x;
}

// reference floors: read-only of the 48 B/group (one u64 per wave written) and a 1:1 copy
__global__ __launch_bounds__(1024) void k_read_only(Cols a) {
    const u64 wave = (u64)blockIdx.x * 16 + (threadIdx.x >> 6);
    const u64 lane = threadIdx.x & 63;
    const u64 g = wave * 128 + lane * 2;
    if (g + 2 > a.G) return;
    const u64 *t = a.col[0] + wave * (128 * 6) + lane * 2;
    u64x2 x = ld2(t);
#pragma unroll
    for (int c = 1; c < 6; ++c) x ^= ld2(t + c * 128);
    if ((x.x ^ x.y) == 0x123456789ull) a.out[g] = x.x;   // never true for the fill pattern
}

__global__ __launch_bounds__(1024) void k_copy(Cols a) {   // 28 B in + 28 B out per group
    const u64 i = ((u64)blockIdx.x * 1024 + threadIdx.x) * 2;
    const u64 n = a.G * 28 / 8;   // u64 words
    if (i + 2 > n) return;
    *reinterpret_cast<u64x2 *>(a.out + i) = ld2(a.col[0] + i);
}

__global__ void k_fill(u64 *p, u64 n, u64 seed) {
    for (u64 i = (u64)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x)
        p[i] = (i + seed) * 0x9E3779B97F4A7C15ull;
}

int main() {
    for (u64 G : {1ull << 20, 8ull << 20}) {
        const u64 per = G * 56;
        const int nsets = (int)std::max<u64>(4, (u64)(1.1 * (1ull << 30)) / per + 1);
        std::vector<u64 *> in(nsets), out(nsets);
        for (int s = 0; s < nsets; ++s) {
            CK(hipMalloc(&in[s], G * 48 + 4096));
            CK(hipMalloc(&out[s], G * 8 * 4 + 4096));
            k_fill<<<1024, 256>>>(in[s], G * 6, s);
        }
        CK(hipDeviceSynchronize());
        auto soa = [&](int s) {
            Cols c{};
            for (int k = 0; k < 6; ++k) c.col[k] = in[s] + k * G;
            c.out = out[s];
            c.G = G;
            return c;
        };
        auto tile = [&](int s) {
            Cols c{};
            c.col[0] = in[s];
            c.out = out[s];
            c.G = G;
            return c;
        };
        typedef void (*KF)(Cols);
        struct V {
            const char *name;
            KF k;
            bool tiled;
            unsigned grid;
            double bytes;   // bytes moved per launch
        };
        const unsigned grid = (unsigned)(G / 2 / 1024);
        V vs[] = {{"soa 6+1 streams", k_soa, false, grid, 56.0 * G},
                  {"tile 1+1 streams", k_tile, true, grid, 56.0 * G},
                  {"tile in place", k_tile_inplace, true, grid, 56.0 * G},
                  {"tile read-only 48B", k_read_only, true, grid, 48.0 * G},
                  {"copy 1:1 56B", k_copy, true, (unsigned)(G * 28 / 16 / 1024), 56.0 * G}};
        for (int rep = 0; rep < 3; ++rep) {
            for (const V &v : vs) {
                hipEvent_t e0, e1;
                CK(hipEventCreate(&e0));
                CK(hipEventCreate(&e1));
                const int steps = G > (1ull << 20) ? 60 : 400;
                for (int i = 0; i < 20; ++i)
                    hipLaunchKernelGGL(v.k, v.grid, 1024, 0, 0, v.tiled ? tile(i % nsets) : soa(i % nsets));
                CK(hipEventRecord(e0, 0));
                for (int i = 0; i < steps; ++i)
                    hipLaunchKernelGGL(v.k, v.grid, 1024, 0, 0, v.tiled ? tile(i % nsets) : soa(i % nsets));
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double us = ms * 1e3 / steps;
                printf("G=%lluM %-20s %8.2f us  %6.0f GB/s\n", G >> 20, v.name, us, v.bytes / us / 1e3);
                CK(hipEventDestroy(e0));
                CK(hipEventDestroy(e1));
            }
        }
        for (int s = 0; s < nsets; ++s) {
            CK(hipFree(in[s]));
            CK(hipFree(out[s]));
        }
    }
    return 0;
}
