// link_probe — what the host link moves for kernels that read or write pinned host memory in
// place (the device step's zero-copy pass A reads, k_step_lite's ReadyToRead writes): one
// direction at a time and both at once (two kernels on two streams). Build:
//   hipcc -O3 --offload-arch=gfx950 -o tools/link_probe tools/link_probe.cpp
// Run: tools/link_probe [MiB per direction, default 64] [device] [--json]
// --json: one line, the best of the grids per figure (bench.py's step legs read it)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>

#define CHECK(x)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
            std::exit(1);                                                                \
        }                                                                                \
    } while (0)

__global__ __launch_bounds__(256) void k_read(const uint4 *src, size_t n, unsigned *sink) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const uint4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;   // (keeps the loads)
}

__global__ __launch_bounds__(256) void k_write(uint4 *dst, size_t n, unsigned tag) {
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        dst[i] = make_uint4(tag, (unsigned)i, 0u, 0u);
}

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 64;
    const int device = argc > 2 ? std::atoi(argv[2]) : 0;
    const bool json = argc > 3 && std::string(argv[3]) == "--json";
    CHECK(hipSetDevice(device));
    double top[5] = {0, 0, 0, 0, 0};   // read, write, read and write together, their sum
    const size_t bytes = mib << 20, n = bytes / 16;
    void *hr = nullptr, *hw = nullptr;
    unsigned *sink = nullptr;
    CHECK(hipHostMalloc(&hr, bytes, hipHostMallocDefault));
    CHECK(hipHostMalloc(&hw, bytes, hipHostMallocDefault));
    CHECK(hipMalloc(&sink, 65536 * sizeof(unsigned)));
    for (size_t i = 0; i < bytes / 4; ++i) static_cast<unsigned *>(hr)[i] = (unsigned)i;
    hipStream_t s1, s2;
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t a0, a1, b0, b1;
    for (hipEvent_t *e : {&a0, &a1, &b0, &b1}) CHECK(hipEventCreate(e));
    const unsigned grids[] = {256, 1024, 4096};
    for (unsigned grid : grids) {
        float best_r = 1e9f, best_w = 1e9f, best_rb = 1e9f, best_wb = 1e9f;
        for (int rep = 0; rep < 6; ++rep) {
            float t;
            CHECK(hipEventRecord(a0, s1));
            hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, s1, (const uint4 *)hr, n, sink);
            CHECK(hipEventRecord(a1, s1));
            CHECK(hipEventSynchronize(a1));
            CHECK(hipEventElapsedTime(&t, a0, a1));
            if (rep) best_r = t < best_r ? t : best_r;
            CHECK(hipEventRecord(b0, s2));
            hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, s2, (uint4 *)hw, n, (unsigned)rep);
            CHECK(hipEventRecord(b1, s2));
            CHECK(hipEventSynchronize(b1));
            CHECK(hipEventElapsedTime(&t, b0, b1));
            if (rep) best_w = t < best_w ? t : best_w;
            // both directions at once: half the grid each, on two streams
            CHECK(hipEventRecord(a0, s1));
            CHECK(hipEventRecord(b0, s2));
            hipLaunchKernelGGL(k_read, dim3(grid / 2), dim3(256), 0, s1, (const uint4 *)hr, n, sink);
            hipLaunchKernelGGL(k_write, dim3(grid / 2), dim3(256), 0, s2, (uint4 *)hw, n, (unsigned)rep);
            CHECK(hipEventRecord(a1, s1));
            CHECK(hipEventRecord(b1, s2));
            CHECK(hipEventSynchronize(a1));
            CHECK(hipEventSynchronize(b1));
            float tr, tw;
            CHECK(hipEventElapsedTime(&tr, a0, a1));
            CHECK(hipEventElapsedTime(&tw, b0, b1));
            if (rep) {
                best_rb = tr < best_rb ? tr : best_rb;
                best_wb = tw < best_wb ? tw : best_wb;
            }
        }
        const double gb = bytes / 1e9;
        const double f[5] = {gb / (best_r * 1e-3), gb / (best_w * 1e-3), gb / (best_rb * 1e-3),
                             gb / (best_wb * 1e-3), gb / (best_rb * 1e-3) + gb / (best_wb * 1e-3)};
        for (int i = 0; i < 5; ++i) top[i] = f[i] > top[i] ? f[i] : top[i];
        if (!json) std::printf("grid %5u x 256: read %.1f GB/s, write %.1f GB/s; together read %.1f GB/s "
                    "+ write %.1f GB/s (%.0f / %.0f us for %zu MiB each)\n",
                    grid, gb / (best_r * 1e-3), gb / (best_w * 1e-3), gb / (best_rb * 1e-3),
                    gb / (best_wb * 1e-3), best_rb * 1e3, best_wb * 1e3, mib);
    }
    if (json)
        std::printf("{\"read_GBps\": %.2f, \"write_GBps\": %.2f, \"both_read_GBps\": %.2f, "
                    "\"both_write_GBps\": %.2f, \"both_GBps\": %.2f, \"MiB\": %zu}\n",
                    top[0], top[1], top[2], top[3], top[4], mib);
    CHECK(hipHostFree(hr));
    CHECK(hipHostFree(hw));
    CHECK(hipFree(sink));
    return 0;
}
