// hq_internal.h — shared between the runtime (hq_runtime.hip) and the kernels (hq_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/hipquorum.h"

struct hq_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    // kernel timing (hq_timing_*): one event pair on the stream brackets a timed region; every
    // launch inside it is counted. Per-launch event pairs are avoided on purpose: on gfx950 an
    // event pair around a ~10 us kernel adds 3-6 us to the measured time and to the wall clock.
    bool timing = false;      // a region is open (begin recorded, end not yet)
    bool region_done = false; // a closed region awaits hq_timing_read
    hipEvent_t ev_begin = nullptr, ev_end = nullptr;
    uint64_t region_launches = 0;
    // hq_timing_begin_after: launches still to go before the begin event is recorded
    uint64_t begin_after = 0;
    double timed_ms = 0.0;
    uint64_t timed_launches = 0;
    // launch geometry of the bitmap kernels (256; HQ_BITS_BLOCK=512|1024 at hq_open)
    int bits_block = 256;
    // multi-ctx ReadIndex two groups per lane when the batch allows it (HQ_RI_PAIRS=0: off, A/B)
    bool ri_pairs = true;
    // uniform multi-ctx tiles (K_max in {2, 4, 8}, n = n_max) on k_ri_tiles_u (HQ_RI_UNIFORM=0:
    // on the general k_ri_multi2, A/B)
    bool ri_uniform = true;
    // hq_wait_for: recorded on this context's stream when another context orders after it
    hipEvent_t ev_order = nullptr;
    // device workspace for the host-pointer entry points
    void *ws = nullptr;
    size_t ws_bytes = 0;
    // device workspace of the binned table ingest (hq_table.hip): the chunks' binned records
    // and their per-bucket offsets; chunks per launch (HQ_BIN_LAUNCH_CHUNKS at hq_open: tests)
    void *bin_ws = nullptr;
    size_t bin_ws_bytes = 0;
    uint32_t bin_launch_chunks = 4096;
    uint32_t bin_grid = 256;      // persistent workgroups of the binned ingest (HQ_BIN_GRID)
    uint32_t bin_tpb_shift = 6;   // its largest region, 2^shift tiles (HQ_BIN_TPB: A/B)
    // k_apply's workgroup: 1024 threads with up to 128 KB of rows (one per CU), or 512 with up to
    // 64 KB (two per CU, HQ_BIN_APPLY_T=512: A/B)
    uint32_t bin_apply_threads = 1024;
    // host readback of the fallback count (hq_commit etc.)
};

namespace hq {

int fail(hq_ctx *ctx, int code, const std::string &msg);
int check_hip(hq_ctx *ctx, hipError_t e, const char *what);
// bracket a launch with timing events when enabled
int pre_launch(hq_ctx *ctx);
int post_launch(hq_ctx *ctx, const char *what);
int ensure_workspace(hq_ctx *ctx, size_t bytes);

inline bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
inline uint64_t words64(uint64_t G) { return (G + 63) / 64; }
inline uint64_t words32(uint64_t G) { return (G + 31) / 32; }  // 2-bit outcome words

}  // namespace hq
