// engine_exp.hip — tuning experiments beside the persistent commit engine (tools/ab_engine.py):
// K headline batches (c3mtl: 1M groups x 5 voters, leader-row tiles, mask form) decided by ONE
// launch in several ownership schemes. Built only as tools/lib_engexp/libengexp.so (Makefile),
// linked against the product library for its context and launch bookkeeping; never part of the
// product. Findings: DESIGN.md §3 (k_commit_engine) and profiles/r04a/README.md.
//   variant 1  every wave loops over the K batches (tiles w, w + W, ...)
//   variant 2  one wave per (batch, tile), batch-major: the launches' waves in one grid
//   variant 3/4/5  each workgroup owns a contiguous range of every batch's tiles, its waves claim
//              them from an LDS counter per batch (256 / 512 / 1024 workgroups)
//   variant 6  device claim counters shared by workgroup pairs
//   variant 7  claim512 plus a shared pool of each batch's last tiles on one device counter
#include <cstdlib>

#include "../dragonboat_amd/csrc/hq_commit_body.h"

namespace {
constexpr int kExpMax = 32;
struct MultiK {
    uint64_t stride, G;
    uint32_t R, count, waves, ntiles;
    const uint64_t *tiles[kExpMax];
    uint64_t *cout[kExpMax];
    uint64_t *chg[kExpMax];
    uint64_t *fb[kExpMax];
};
// V1: each wave loops over the `count` batches (the engine's ownership, no doorbell)
template <int N, int FORM, int LEAD, int BLK>
__global__ __launch_bounds__(BLK, BLK >= 1024 ? 8 : 1) void k_exp_loop(const MultiK m) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (BLK / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t c = 0; c < m.count; ++c) {
        CommitK k{};
        k.G = m.G;
        k.stride = m.stride;
        k.match = m.tiles[c];
        k.cout = m.cout[c];
        k.changed = m.chg[c];
        k.fallback = m.fb[c];
        k.R = m.R;
        for (uint64_t t = wave; t < m.ntiles; t += m.waves)
            commit_tile<N, FORM, false, LEAD, false>(k, t * HQ_TILE_GROUPS, lane);
    }
}
// V2: one wave per (batch, tile), batch-major: the launches' waves in one grid
template <int N, int FORM, int LEAD, int BLK>
__global__ __launch_bounds__(BLK, BLK >= 1024 ? 8 : 1) void k_exp_flat(const MultiK m) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (BLK / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t c = (uint32_t)(wave / m.ntiles);
    const uint64_t t = wave % m.ntiles;
    if (c >= m.count) return;
    CommitK k{};
    k.G = m.G;
    k.stride = m.stride;
    k.match = m.tiles[c];
    k.cout = m.cout[c];
    k.changed = m.chg[c];
    k.fallback = m.fb[c];
    k.R = m.R;
    commit_tile<N, FORM, false, LEAD, false>(k, t * HQ_TILE_GROUPS, lane);
}
// V3: each workgroup owns a contiguous range of every batch's tiles; its waves claim them one by
// one from an LDS counter per batch (the waves of one workgroup balance each other)
template <int N, int FORM, int LEAD, int BLK, int OCC>
__global__ __launch_bounds__(BLK, OCC) void k_exp_claim(const MultiK m) {
    __shared__ uint32_t claim[kExpMax];
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i = threadIdx.x; i < (uint32_t)kExpMax; i += BLK) claim[i] = 0;
    __syncthreads();
    const uint64_t per = (m.ntiles + gridDim.x - 1) / gridDim.x;
    const uint64_t base = blockIdx.x * per;
    const uint64_t end = base + per < m.ntiles ? base + per : m.ntiles;
    for (uint32_t c = 0; c < m.count; ++c) {
        CommitK k{};
        k.G = m.G;
        k.stride = m.stride;
        k.match = m.tiles[c];
        k.cout = m.cout[c];
        k.changed = m.chg[c];
        k.fallback = m.fb[c];
        k.R = m.R;
        for (;;) {
            uint32_t t = 0;
            if (lane == 0) t = __hip_atomic_fetch_add(&claim[c], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            t = __builtin_amdgcn_readfirstlane(t);
            if (base + t >= end) break;
            commit_tile<N, FORM, false, LEAD, false>(k, (base + t) * HQ_TILE_GROUPS, lane);
        }
    }
}
// V6: every wave claims tiles one at a time from a device counter shared by the waves of
// workgroups b and b + grid/2 (per batch), the next claim issued before the current tile is
// decided: balance across the two workgroups of a CU, no LDS
template <int N, int FORM, int LEAD, int BLK>
__global__ __launch_bounds__(BLK, 8) void k_exp_gclaim(const MultiK m, uint32_t *ctr) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t half = gridDim.x / 2;
    const uint32_t pair = blockIdx.x % half;
    const uint64_t per = (m.ntiles + half - 1) / half;
    const uint64_t b0 = pair * per;
    const uint32_t len = (uint32_t)(b0 >= m.ntiles ? 0 : m.ntiles - b0 < per ? m.ntiles - b0 : per);
    uint32_t c = 0;
    uint32_t nxt = 0;
    if (lane == 0) nxt = __hip_atomic_fetch_add(ctr + c * half + pair, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while (c < m.count) {
        const uint32_t i = __builtin_amdgcn_readfirstlane(nxt);
        if (i >= len) {
            ++c;
            if (c < m.count && lane == 0)
                nxt = __hip_atomic_fetch_add(ctr + c * half + pair, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            continue;
        }
        if (lane == 0) nxt = __hip_atomic_fetch_add(ctr + c * half + pair, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        CommitK k{};
        k.G = m.G;
        k.stride = m.stride;
        k.match = m.tiles[c];
        k.cout = m.cout[c];
        k.changed = m.chg[c];
        k.fallback = m.fb[c];
        k.R = m.R;
        commit_tile<N, FORM, false, LEAD, false>(k, (b0 + i) * HQ_TILE_GROUPS, lane);
    }
}
}  // namespace

// V7: the claim512 shape plus a shared pool: per batch, the last `pool` tiles are claimed by
// any wave of the grid from one device counter (the next claim issued before the current tile
// is decided) once its workgroup's own range of the batch is exhausted; fast workgroups take
// more of the pool, so the slowest one no longer sets the window
template <int N, int FORM, int LEAD, int BLK>
__global__ __launch_bounds__(BLK, 8) void k_exp_pool(const MultiK m, uint32_t *ctr, uint32_t pool) {
    __shared__ uint32_t claim[kExpMax];
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i = threadIdx.x; i < (uint32_t)kExpMax; i += BLK) claim[i] = 0;
    __syncthreads();
    const uint64_t S = m.ntiles - pool;   // the static part
    const uint64_t per = (S + gridDim.x - 1) / gridDim.x;
    const uint64_t base = blockIdx.x * per;
    const uint64_t end = base + per < S ? base + per : S;
    for (uint32_t c = 0; c < m.count; ++c) {
        CommitK k{};
        k.G = m.G;
        k.stride = m.stride;
        k.match = m.tiles[c];
        k.cout = m.cout[c];
        k.changed = m.chg[c];
        k.fallback = m.fb[c];
        k.R = m.R;
        for (;;) {
            uint32_t t = 0;
            if (lane == 0) t = __hip_atomic_fetch_add(&claim[c], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            t = __builtin_amdgcn_readfirstlane(t);
            if (base + t >= end) break;
            commit_tile<N, FORM, false, LEAD, false>(k, (base + t) * HQ_TILE_GROUPS, lane);
        }
        uint32_t nxt = 0;
        if (lane == 0) nxt = __hip_atomic_fetch_add(ctr + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (;;) {
            const uint32_t i = __builtin_amdgcn_readfirstlane(nxt);
            if (i >= pool) break;
            if (lane == 0) nxt = __hip_atomic_fetch_add(ctr + c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            commit_tile<N, FORM, false, LEAD, false>(k, (S + i) * HQ_TILE_GROUPS, lane);
        }
    }
}

extern "C" int hq_exp_multi(hq_ctx *ctx, const hq_commit_args *a, uint32_t count, int variant,
                            uint32_t grid) {
    if (!ctx) return HQ_E_INVAL;
    if (!a || count == 0 || count > (uint32_t)kExpMax)
        return hq::fail(ctx, HQ_E_INVAL, "hq_exp_multi: 1..32 batches");
    if (a[0].n_max != 5 || a[0].form != HQ_FORM_TERM_MASK || a[0].layout != HQ_LAYOUT_TILES_LEADER)
        return hq::fail(ctx, HQ_E_INVAL, "hq_exp_multi: serves the headline shape only (n 5, mask, "
                                         "leader-row tiles)");
    MultiK m{};
    m.stride = hq_commit_tile_words_for(5, HQ_FORM_TERM_MASK, HQ_LAYOUT_TILES_LEADER);
    m.G = a[0].G;
    m.R = a[0].ring_len;
    m.count = count;
    m.ntiles = (uint32_t)((m.G + HQ_TILE_GROUPS - 1) / HQ_TILE_GROUPS);
    for (uint32_t i = 0; i < count; ++i) {
        if (a[i].G != m.G) return hq::fail(ctx, HQ_E_INVAL, "hq_exp_multi: batches of one G");
        m.tiles[i] = a[i].match;
        m.cout[i] = a[i].committed_out;
        m.chg[i] = a[i].changed;
        m.fb[i] = a[i].fallback;
    }
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    if (variant == 1) {
        if (!grid) grid = 512;
        m.waves = grid * 16;
        hipLaunchKernelGGL((k_exp_loop<5, HQ_FORM_TERM_MASK, 1, 1024>), dim3(grid), dim3(1024), 0,
                           ctx->stream, m);
    } else if (variant == 7) {
        static uint32_t *ctr = nullptr;
        if (!ctr && hipMalloc(&ctr, 4 * kExpMax) != hipSuccess) return hq::fail(ctx, HQ_E_NOMEM, "hq_exp_multi: hipMalloc");
        (void)hipMemsetAsync(ctr, 0, 4 * kExpMax, ctx->stream);
        const char *pv = std::getenv("AB_POOL");   // permille of a batch's tiles in the pool
        const uint32_t pool = (uint32_t)((uint64_t)m.ntiles * (pv ? std::atoi(pv) : 250) / 1000);
        hipLaunchKernelGGL((k_exp_pool<5, HQ_FORM_TERM_MASK, 1, 1024>), dim3(grid ? grid : 512),
                           dim3(1024), 0, ctx->stream, m, ctr, pool);
    } else if (variant == 6) {
        static uint32_t *ctr = nullptr;
        if (!ctr && hipMalloc(&ctr, 4 * kExpMax * 1024) != hipSuccess) return hq::fail(ctx, HQ_E_NOMEM, "hq_exp_multi: hipMalloc");
        (void)hipMemsetAsync(ctr, 0, 4 * kExpMax * 1024, ctx->stream);
        hipLaunchKernelGGL((k_exp_gclaim<5, HQ_FORM_TERM_MASK, 1, 1024>), dim3(grid ? grid : 512),
                           dim3(1024), 0, ctx->stream, m, ctr);
    } else if (variant == 3) {
        hipLaunchKernelGGL((k_exp_claim<5, HQ_FORM_TERM_MASK, 1, 1024, 4>), dim3(grid ? grid : 256),
                           dim3(1024), 0, ctx->stream, m);
    } else if (variant == 4) {
        hipLaunchKernelGGL((k_exp_claim<5, HQ_FORM_TERM_MASK, 1, 1024, 8>), dim3(grid ? grid : 512),
                           dim3(1024), 0, ctx->stream, m);
    } else if (variant == 5) {
        hipLaunchKernelGGL((k_exp_claim<5, HQ_FORM_TERM_MASK, 1, 512, 8>), dim3(grid ? grid : 1024),
                           dim3(512), 0, ctx->stream, m);
    } else {
        const uint64_t waves = (uint64_t)m.ntiles * count;
        m.waves = 0;
        hipLaunchKernelGGL((k_exp_flat<5, HQ_FORM_TERM_MASK, 1, 1024>), dim3((waves + 15) / 16),
                           dim3(1024), 0, ctx->stream, m);
    }
    return hq::post_launch(ctx, "k_exp");
}
