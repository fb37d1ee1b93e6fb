// hq_engine.hip — the persistent commit engine (hq_engine_*, include/hipquorum.h).
//
// One resident launch decides a stream of posted commit batches (raft.tryCommit over a step's
// leader groups, raft.go:888-909 + logentry.go:378-393). The host side mirrors the reference's
// step-worker wake-up: execEngine's workReady.clusterReady (execengine.go:115-123) posts a
// cluster on the worker's channel and stepWorkerMain (execengine.go:860-882) loops on it; here a
// step worker posts a batch descriptor into a pinned ring and the resident kernel loops on the
// ring. What it removes is the dependent-launch boundary every step pays when each batch is its
// own launch (MI355X_MICROARCH.md "boundary": 1.7-1.9 us between streaming kernels, ~18 % of a
// 1M-group step; DESIGN.md §7 size sweep).
//
// Ownership: workgroup b owns tiles [b * per, b * per + per) of every posted batch (per =
// ceil(tiles / grid), computed by the host). Its waves take those tiles through ONE monotone LDS
// ticket counter: ticket t is tile t - end(s - 1) of the first step s with t < end(s), where
// end(s) is the workgroup's cumulative tile count through step s. The waves balance each other
// inside the workgroup, a wave moves from step s to s + 1 with no barrier, re-arm or failing claim
// (a ticket is always a tile of some step), and a step transition costs a few LDS reads.
// A group's step s + 1 depends only on its own step s (the in-place table's committed row,
// raft.go:888-909 run per ReplicateResp on that group's state); with HQ_LAYOUT_IN_PLACE the
// posted steps keep one G, so a tile stays with its workgroup and a wave starts step s + 1 only
// when the workgroup has decided all of step s.
//
// Doorbell: the host writes a 64-byte descriptor into the pinned ring and then bumps `posted`
// (both fine-grained host memory). The poller of workgroup 0 relays new descriptors into a
// device copy of the ring and publishes the relayed count in 16 device copies; a workgroup whose
// waves have run out of known steps polls one copy (relaxed agent-scope load + s_sleep,
// MI355X_MICROARCH.md "polling-cost"). Completion (HQ_ENGINE_SIGNAL): a workgroup counts its
// arrival on one of 8 shard counters, the last workgroup of a shard on the step's top counter,
// and the last of those writes the step's sequence number into the pinned done array (one PCIe
// write per step).
//
// Every spin is bounded: workgroup 0 ends the launch after idle_us without a post by publishing
// the launch's epoch in `d_exit` (after relaying everything it saw); every workgroup leaves once
// its waves have caught up with the relayed steps, so the grid exits as a whole and the next post
// or wait relaunches it (each workgroup resumes at its cursor). A host that dies never leaves
// waves spinning on the GPU.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>

#include "hq_commit_body.h"

namespace {

constexpr uint32_t kEngineMaxDepth = 64;   // posted steps in flight
constexpr uint64_t kDescStop = 1;          // EngineDesc.flags: the workgroups exit at this step
constexpr int kShards = 8;                 // workgroup arrival counters per step (blockIdx % 8:
                                           // one per XCD under round-robin dispatch)
constexpr int kPollCopies = 16;            // copies of the relayed count, 256 B apart: 512
                                           // workgroups polling ONE word queue on its channel
                                           // (the first descriptors reached the last sampled
                                           // workgroup 97 us after the launch, round-4 probes)
constexpr int kPollStride = 32;            // u64 between copies
constexpr int kInit = 32;                  // descriptors handed over in the kernel arguments
constexpr int kPools = 8;                  // balanced mode: one tile pool per XCD (blockIdx % 8)
constexpr int kPoolStride = 16;            // u64 between pool counters (one 128-B line each)
constexpr int kChunkQ = 32;                // balanced mode: claimed chunks a workgroup keeps

struct EngineDesc {   // one posted step, 64 bytes = 8 u64 words (one per relay lane)
    uint64_t G;
    const uint64_t *tiles;
    uint64_t *cout;
    uint64_t *changed;
    uint64_t *fallback;
    uint64_t seq;
    uint64_t flags;
    uint64_t per;       // tiles per workgroup: ceil(ceil(G / 128) / grid), set by the host
};
static_assert(sizeof(EngineDesc) == 64, "a descriptor is 8 relay lanes of u64");

struct EngineK {
    uint64_t stride;        // u64 words per tile
    uint64_t idle_ticks;    // s_memrealtime ticks (100 MHz) of polling without news before exit
    uint32_t R;             // term-mask window
    uint32_t depth;         // ring slots (power of two <= kEngineMaxDepth)
    uint32_t signal;        // per-step completion into the pinned done array
    uint32_t epoch;         // this launch's number (d_exit == epoch: the grid ends)
    const uint64_t *h_posted;      // pinned: descriptors written by the host
    uint64_t *h_done;              // pinned [depth]: seq + 1 of the last step completed per slot
    uint64_t *h_clock;             // pinned [depth]: s_memrealtime at that completion
    const EngineDesc *h_ring;      // pinned [depth]
    uint64_t *d_posted;            // device: descriptors relayed into d_ring
    uint64_t *d_arrive;            // device [depth][kShards]
    uint64_t *d_top;               // device [depth]
    uint64_t *d_cursor;            // device [grid]: the next step of each workgroup
    EngineDesc *d_ring;            // device [depth]
    uint64_t *d_polled;            // device [kPollCopies * kPollStride]: copies of d_posted
    uint64_t *d_exit;              // device: the epoch of the launch that is ending
    // balanced mode (BAL): each step's tiles split into `pools` contiguous pools, pool x taken
    // by the workgroups with blockIdx % pools == x (one XCD under round-robin dispatch) in chunks
    // of `chunk` tiles through a device ticket counter per pool
    uint64_t *d_claim;             // device [kPools * kPoolStride]: tickets taken this launch
    uint64_t *d_pdone;             // device [depth][kPools * kPoolStride]: tiles decided per pool
    uint32_t chunk, pools;
    // the descriptors of steps [init_base, init_base + init_count), known when the grid was
    // launched: every workgroup starts with them in LDS (no relay, no poll at the start)
    uint64_t init_base;
    uint32_t init_count, pad;
    EngineDesc init[kInit];
};

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

// A pointer read from memory (a posted descriptor) is generic to the compiler, and generic
// pointers compile to FLAT loads and stores (counted in both vmcnt and lgkmcnt: every wait drains
// everything; 13.1 vs 10.2 us per 1M-group step, round-4 probes). Descriptors hold device
// (global) addresses by contract, so the value is cast into the global address space and back:
// the compiler then infers global for every access through it.
template <class T>
__device__ __forceinline__ T *as_global(uint64_t v) {
    typedef __attribute__((address_space(1))) T GT;
    return (T *)(GT *)v;
}

// The kernel's argument as the rare paths (poll, relay, arrival) read it: volatile loads from the
// kernarg segment at each use, so the compiler keeps none of those fields live across the tile
// loop (held in SGPRs, they pushed the loop's own values into VGPR lanes and scratch)
typedef __attribute__((address_space(1))) const volatile EngineK GlobalEngineK;
__device__ __forceinline__ GlobalEngineK &kargs() {
    return *(GlobalEngineK *)reinterpret_cast<uintptr_t>(__builtin_amdgcn_kernarg_segment_ptr());
}

// a pointer field of the engine's argument as a global-address-space pointer (no FLAT access)
template <class T>
__device__ __forceinline__ T *gp(T *p) { return as_global<T>(reinterpret_cast<uint64_t>(p)); }

// Workgroup 0's poller: copy the descriptors the host has posted since the last relay into the
// device ring and publish their count. Lane l moves u64 word l & 7 of descriptor l >> 3 (+8i).
// The host never posts more than `depth` steps beyond the last completed one, so the slots
// written here are no longer read by any workgroup.
__device__ void relay(GlobalEngineK &e, uint32_t lane) {
    const uint64_t have = __hip_atomic_load(gp(e.d_posted), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t hp = __hip_atomic_load(gp(e.h_posted), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (hp <= have) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // system scope: the ring entries behind posted
    const uint64_t n = hp - have < e.depth ? hp - have : e.depth;
    const uint64_t dmask = e.depth - 1;
    // up to 32 descriptors per round, every load issued before the first store (one PCIe round
    // trip per round instead of one per 8 descriptors)
    for (uint64_t base = 0; base < n; base += 32) {
        uint64_t v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t i = base + (lane >> 3) + 8 * j;
            v[j] = i < n ? __hip_atomic_load(
                               reinterpret_cast<const uint64_t *>(gp(e.h_ring) + ((have + i) & dmask)) +
                                   (lane & 7),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                         : 0;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t i = base + (lane >> 3) + 8 * j;
            if (i < n)
                __hip_atomic_store(reinterpret_cast<uint64_t *>(gp(e.d_ring) + ((have + i) & dmask)) +
                                       (lane & 7),
                                   v[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (lane == 0)
        __hip_atomic_store(gp(e.d_posted), have + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane < (uint32_t)kPollCopies)
        __hip_atomic_store(gp(e.d_polled) + lane * kPollStride, have + n, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// The workgroup is done with step s (called once per workgroup and step). In signal mode the
// tiles' stores were write-through (WT) and every deciding wave drained them before counting its
// tile, so they are visible device-wide with no release fence (Guideline 16 R1; a release fence
// per workgroup and step, an L2 write-back each, took 26 us per step). The workgroup counts on
// the step's shard counter (blockIdx % 8), the last workgroup of a shard on the step's top
// counter, and the last of those publishes the step to the host. The last arriver of a counter
// resets it for the slot's next step: the host posts that step only after it has seen this one's
// done flag, which is written after the resets.
__device__ void publish(GlobalEngineK &e, uint64_t s) {
    const uint64_t slot = s & (e.depth - 1);
    __hip_atomic_store(gp(e.h_clock) + slot, now_ticks(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(gp(e.h_done) + slot, s + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ void arrive(GlobalEngineK &e, uint64_t s) {
    const uint64_t slot = s & (e.depth - 1);
    const uint32_t shard = blockIdx.x % kShards;
    const uint32_t nshard = gridDim.x < (uint32_t)kShards ? gridDim.x : (uint32_t)kShards;
    const uint64_t per = (gridDim.x - shard + kShards - 1) / kShards;   // workgroups in the shard
    uint64_t *ctr = gp(e.d_arrive) + slot * kShards + shard;
    if (__hip_atomic_fetch_add(ctr, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 !=
        per)
        return;
    __hip_atomic_store(ctr, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__hip_atomic_fetch_add(gp(e.d_top) + slot, (uint64_t)1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT) + 1 != nshard)
        return;
    __hip_atomic_store(gp(e.d_top) + slot, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    publish(e, s);
}

// Balanced mode: tiles [*b, *b + *n) of a step of G groups form pool x
__device__ __forceinline__ void pool_range(uint64_t G, uint32_t pools, uint32_t x, uint64_t *b,
                                           uint64_t *n) {
    const uint64_t tiles = (G + HQ_TILE_GROUPS - 1) / HQ_TILE_GROUPS;
    *b = tiles * x / pools;
    *n = tiles * (x + 1) / pools - *b;
}

// Balanced mode, one lane: `n` tiles of pool x of step s decided (their stores complete) — the
// add, issued (pool_add) one chunk before its returned value is looked at (pool_settle), so no
// wave waits for an atomic's round trip. The adder that completes the pool counts it on the
// step's top counter, and the one that completes the last non-empty pool publishes the step (the
// counters reset by their last adder, as in arrive)
__device__ __forceinline__ uint64_t *pool_ctr(GlobalEngineK &e, uint64_t s, uint32_t x) {
    return gp(e.d_pdone) + ((s & (e.depth - 1)) * kPools + x) * kPoolStride;
}

__device__ __forceinline__ uint64_t pool_add(GlobalEngineK &e, uint64_t s, uint32_t x, uint32_t n) {
    return __hip_atomic_fetch_add(pool_ctr(e, s, x), (uint64_t)n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ void pool_settle(GlobalEngineK &e, uint64_t s, uint64_t G, uint32_t x, uint32_t n,
                            uint64_t before_add) {
    const uint64_t slot = s & (e.depth - 1);
    uint64_t b, len;
    pool_range(G, e.pools, x, &b, &len);
    if (before_add + n != len) return;
    __hip_atomic_store(pool_ctr(e, s, x), (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t tiles = (G + HQ_TILE_GROUPS - 1) / HQ_TILE_GROUPS;
    const uint64_t busy = tiles < e.pools ? tiles : e.pools;     // the pools with a tile
    if (__hip_atomic_fetch_add(gp(e.d_top) + slot, (uint64_t)1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT) + 1 != busy)
        return;
    __hip_atomic_store(gp(e.d_top) + slot, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    publish(e, s);
}

// Per-workgroup state in LDS. The descriptors of steps [.., known) sit in `ring` (slot = step &
// (depth - 1)) with `end` (the workgroup's cumulative tile count through the slot's step, counted
// from this launch's cursor, mod 2^32) and `tgt` (the value of the slot's `fin` counter at which
// the workgroup has decided the slot's step: signal mode). `ticket` hands out the workgroup's
// tiles of all its steps in order; `done` counts decided tiles (in-place mode). Tickets, ends and
// counters are u32 compared by differences: only values within a few ring lengths of steps are
// ever compared. A wave whose ticket is beyond the known steps waits for `known` to grow: the
// first such wave takes `lock` and becomes the workgroup's poller (workgroup 0's poller relays
// from the host ring first), copies the new descriptors into LDS, extends `end` / `tgt` and
// publishes `known`. `waiting` counts the waves at the end of what they know; the workgroup
// exits only when all of them are (at one step).
struct EngineLds {
    EngineDesc ring[kEngineMaxDepth];
    uint32_t end[kEngineMaxDepth];
    uint32_t fin[kEngineMaxDepth];
    uint32_t tgt[kEngineMaxDepth];
    uint64_t known;
    uint32_t ticket;
    uint32_t top_end;     // end of the last installed step
    uint32_t done;
    uint32_t waiting, lock, exit;
    uint32_t stopc;       // balanced mode: waves at the STOP
    // balanced mode: the workgroup's claimed chunks (pool tickets), chunk q at q % kChunkQ;
    // cq_have = chunks published; cq_done = tiles of the chunk counted
    uint32_t cq_have;
    uint32_t cq_T[kChunkQ];
    uint32_t cq_done[kChunkQ];
};

__device__ __forceinline__ bool before(uint32_t a, uint32_t b) { return (int32_t)(a - b) < 0; }

// the workgroup's tiles of a step
__device__ __forceinline__ uint64_t wg_len(uint64_t G, uint64_t per) {
    const uint64_t tiles = (G + HQ_TILE_GROUPS - 1) / HQ_TILE_GROUPS;
    const uint64_t b0 = (uint64_t)blockIdx.x * per;
    return b0 >= tiles ? 0 : (tiles - b0 < per ? tiles - b0 : per);
}

// One thread: extend end / tgt over the descriptors of steps [from, to) now in the LDS ring. A
// step in which the workgroup owns no tile is complete for it at once (signal: arrive now).
__device__ void install(GlobalEngineK &e, EngineLds &l, uint64_t from, uint64_t to) {
    const uint64_t dmask = e.depth - 1;
    uint32_t top = l.top_end;
    if (e.chunk) {
        // balanced: `end` counts the tickets (chunks) of this workgroup's pool; a step with no
        // tile at all is published by workgroup 0 at once
        const uint32_t pools = e.pools, x = blockIdx.x % pools, chunk = e.chunk;
        for (uint64_t s = from; s < to; ++s) {
            const EngineDesc &d = l.ring[s & dmask];
            uint32_t len = 0;
            if (!(d.flags & kDescStop)) {
                uint64_t b, n;
                pool_range(d.G, pools, x, &b, &n);
                len = (uint32_t)((n + chunk - 1) / chunk);
                if (d.G == 0 && e.signal && blockIdx.x == 0) publish(e, s);
            }
            top += len;
            l.end[s & dmask] = top;
        }
        l.top_end = top;
        return;
    }
    for (uint64_t s = from; s < to; ++s) {
        const EngineDesc &d = l.ring[s & dmask];
        const uint32_t len = (d.flags & kDescStop) ? 0u : (uint32_t)wg_len(d.G, d.per);
        top += len;
        l.end[s & dmask] = top;
        l.tgt[s & dmask] += len;
        if (len == 0 && e.signal && !(d.flags & kDescStop)) arrive(e, s);
    }
    l.top_end = top;
}

__device__ __forceinline__ uint64_t lds_known(EngineLds &l) {
    return __hip_atomic_load(&l.known, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// lane 0's value of a 32-bit LDS atomic, for the whole wave
__device__ __forceinline__ uint32_t wave_u32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// A wave at step s with no descriptor beyond it (s == the workgroup's known count): returns the
// new known count, or s when the workgroup exits (the wave then exits at s).
template <int WPW>
__device__ uint64_t frontier(GlobalEngineK &e, EngineLds &l, uint64_t s, uint32_t lane) {
    uint64_t k = lds_known(l);
    if (k > s) return k;
    const bool relayer = blockIdx.x == 0;
    if (lane == 0) __hip_atomic_fetch_add(&l.waiting, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (;;) {
        k = uniform64(lds_known(l));
        if (k > s) break;
        if (wave_u32(__hip_atomic_load(&l.exit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)))
            return s;
        uint32_t got = 0;
        if (lane == 0)
            got = __hip_atomic_exchange(&l.lock, 1u, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0;
        if (wave_u32(got)) {
            // the workgroup's poller. Another poller may have published news between this
            // wave's look at `known` and its lock: look again under the lock, or the steps it
            // installed would be installed twice (their ends counted twice)
            k = uniform64(lds_known(l));
            if (k > s) {
                if (lane == 0) __hip_atomic_store(&l.lock, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                break;
            }
            const uint64_t t0 = now_ticks();
            uint32_t backoff = 1;
            bool leave = false;
            for (;;) {
                if (relayer) relay(e, lane);
                const uint64_t p = uniform64(
                    __hip_atomic_load(gp(e.d_polled) + (blockIdx.x % kPollCopies) * kPollStride,
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                if (p > s) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    const uint64_t dmask = e.depth - 1;
                    for (uint64_t i = lane >> 3; i < p - s; i += 8) {
                        const uint64_t slot = (s + i) & dmask;
                        reinterpret_cast<uint64_t *>(l.ring + slot)[lane & 7] = __hip_atomic_load(
                            reinterpret_cast<const uint64_t *>(gp(e.d_ring) + slot) + (lane & 7),
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    if (lane == 0) {
                        install(e, l, s, p);
                        __hip_atomic_store(&l.known, p, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    k = p;
                    break;
                }
                const bool all_waiting =
                    wave_u32(__hip_atomic_load(&l.waiting, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP)) == (uint32_t)WPW;
                if (relayer) {
                    // the grid's exit: after idle_ticks without news, once every relayed step is
                    // this workgroup's too (p == s) and its waves all wait
                    if (all_waiting && now_ticks() - t0 > e.idle_ticks) {
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                        if (lane == 0)
                            __hip_atomic_store(gp(e.d_exit), (uint64_t)e.epoch, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                        leave = true;
                    }
                } else if (all_waiting) {
                    // workgroup 0 has ended the launch and every step it relayed is here
                    // (re-read after the exit word: nothing relayed is left behind); or, as a
                    // backstop, 64 idle limits without news
                    const bool ended = uniform64(__hip_atomic_load(gp(e.d_exit), __ATOMIC_RELAXED,
                                                                   __HIP_MEMORY_SCOPE_AGENT)) == e.epoch;
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    const uint64_t p2 = uniform64(
                        __hip_atomic_load(gp(e.d_polled) + (blockIdx.x % kPollCopies) * kPollStride,
                                          __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                    if ((ended && p2 <= s) || now_ticks() - t0 > 64 * e.idle_ticks) leave = true;
                }
                if (leave) {
                    if (lane == 0)
                        __hip_atomic_store(&l.exit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    k = s;
                    break;
                }
                for (uint32_t i = 0; i < backoff; ++i) __builtin_amdgcn_s_sleep(16);
                backoff = backoff < 4 ? 2 * backoff : 4;
            }
            if (lane == 0) __hip_atomic_store(&l.lock, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (k == s) return s;   // exit
            break;
        }
        __builtin_amdgcn_s_sleep(4);
    }
    if (lane == 0) __hip_atomic_fetch_sub(&l.waiting, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return k;
}

// The workgroup's look-ahead (one wave, at its step transition to step s): when no step beyond s
// is known, workgroup 0 relays what the host has posted, and the workgroup installs what has been
// relayed — the frontier's work, done while the other waves still decide tiles. Skipped while the
// workgroup's poller holds the lock (it is doing the same).
__device__ void refresh(GlobalEngineK &e, EngineLds &l, uint64_t s, uint32_t lane) {
    if (uniform64(lds_known(l)) > s + 1) return;
    uint32_t got = 0;
    if (lane == 0)
        got = __hip_atomic_exchange(&l.lock, 1u, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0;
    if (!wave_u32(got)) return;
    const uint64_t k = uniform64(lds_known(l));
    if (blockIdx.x == 0) relay(e, lane);
    const uint64_t p = uniform64(__hip_atomic_load(gp(e.d_polled) + (blockIdx.x % kPollCopies) * kPollStride,
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    if (p > k) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const uint64_t dmask = e.depth - 1;
        for (uint64_t i = lane >> 3; i < p - k; i += 8) {
            const uint64_t slot = (k + i) & dmask;
            reinterpret_cast<uint64_t *>(l.ring + slot)[lane & 7] = __hip_atomic_load(
                reinterpret_cast<const uint64_t *>(gp(e.d_ring) + slot) + (lane & 7),
                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) {
            install(e, l, k, p);
            __hip_atomic_store(&l.known, p, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    if (lane == 0) __hip_atomic_store(&l.lock, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// the next ticket of the workgroup, for the whole wave
__device__ __forceinline__ uint32_t claim(EngineLds &l, uint32_t lane) {
    uint32_t t = 0;
    if (lane == 0) t = __hip_atomic_fetch_add(&l.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return wave_u32(t);
}

#ifdef HQ_ENGINE_WGPROF
// probe builds only (-DHQ_ENGINE_WGPROF, tools/engine_wgprof.py): per workgroup of the static
// path, 8 words — the device clock at its start, its XCC id, its HW_ID register, the ticks its
// waves spent in their tile loops (summed), the tiles it decided, the clock when its last wave
// left, the ticks its waves spent at the frontier (bits 0-39) and their entries there (40-63),
// and the ticks its first wave spent in the look-ahead — read and reset by hq_engine_wgprof
constexpr uint32_t kWgProfMax = 2048;
__device__ uint64_t g_wgprof[kWgProfMax * 8];
#endif

// SIG: per-step completion signals (write-through stores, drained before a tile is counted).
// INPLACE: the device-resident table decided in place (committed' into the tile's row).
// BAL: balanced mode (tiles taken from per-XCD pools through device tickets; not with INPLACE).
template <int N, int FORM, int LEAD, bool INPLACE, int BLK, bool SIG, bool BAL>
__global__ __launch_bounds__(BLK) __attribute__((amdgpu_waves_per_eu(BLK >= 1024 ? 8 : 1, 8)))
void k_commit_engine(const EngineK e) {
    static_assert(!(BAL && INPLACE), "an in-place table keeps each tile with one workgroup");
    constexpr int WPW = BLK / 64;   // waves per workgroup
    __shared__ EngineLds l;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t dmask = e.depth - 1;
    // written by the previous launch (balanced: every workgroup resumes where workgroup 0 did,
    // so that all map the pools' tickets to the same steps)
    const uint64_t s0 = uniform64(gp(e.d_cursor)[BAL ? 0 : blockIdx.x]);
    // the descriptors handed over at launch (the host's oldest incomplete step <= the cursor)
    for (uint32_t i = threadIdx.x; i < kEngineMaxDepth; i += BLK) {
        l.fin[i] = 0;
        l.tgt[i] = 0;
    }
    for (uint32_t i = threadIdx.x; i < e.init_count * 8; i += BLK)
        reinterpret_cast<uint64_t *>(l.ring + ((e.init_base + (i >> 3)) & dmask))[i & 7] =
            reinterpret_cast<const uint64_t *>(e.init)[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint64_t top = e.init_base + e.init_count;
        l.ticket = 0;
        l.done = 0;
        l.top_end = 0;
        l.waiting = l.lock = l.exit = l.stopc = 0;
        if constexpr (BAL) {
            // the workgroup's first chunk
            l.cq_T[0] = (uint32_t)__hip_atomic_fetch_add(gp(e.d_claim) + (blockIdx.x % e.pools) * kPoolStride,
                                                        (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            l.cq_have = 1;
            for (int i = 0; i < kChunkQ; ++i) l.cq_done[i] = 0;
        }
        if (top > s0) install(kargs(), l, s0, top);
        l.known = top > s0 ? top : s0;
    }
    __syncthreads();
    // (workgroup 0 relays once at the start: steps posted one call each right after the launch
    // are then in the device ring when the other workgroups first look ahead)
    if (blockIdx.x == 0 && wv == 0) refresh(kargs(), l, s0, lane);
    uint64_t s = s0;          // the step of the wave's ticket (or the first it may be in)
    uint64_t known = s0;      // descriptors the wave has seen as known
    uint32_t e_prev = 0;      // the workgroup's tickets before step s
    if constexpr (BAL) {
        // Balanced: the workgroup takes the tiles of its pool (x = blockIdx % pools) a chunk of
        // `chunk` tiles at a time through the pool's device ticket counter (zeroed before the
        // launch): pool ticket T is chunk T - end(s - 1) of the pool's tiles of the first step s
        // with T < end(s), and every workgroup of the pool computes the same ends from the same
        // descriptors. Inside the workgroup the waves share the claimed chunks through the LDS
        // ticket: LDS ticket u is tile u % chunk of the workgroup's chunk u / chunk. The wave
        // holding the first ticket of chunk q claims chunk q + 1 and publishes it (no wait in
        // between, so a wave waiting for a chunk never waits on a frontier), while the other
        // waves decide chunk q. A chunk is counted on its pool's step counter when its last tile
        // is counted (a tile once its stores are complete: after the wave's next tile's loads
        // have returned, or at a drain).
        const uint32_t x = blockIdx.x % e.pools, K = e.chunk;
        uint64_t *const tickets = gp(e.d_claim) + x * kPoolStride;
        uint32_t u = claim(l, lane);
        bool pend = false;
        uint64_t p_s = 0, p_G = 0;
        uint32_t p_q = 0, p_n = 0;
        // the pool count in flight (its add issued, its return not yet looked at)
        bool c_fly = false;
        uint64_t c_s = 0, c_G = 0, c_ret = 0;
        uint32_t c_n = 0;
        auto settle = [&]() {
            if (c_fly && lane == 0) pool_settle(kargs(), c_s, c_G, x, c_n, c_ret);
            c_fly = false;
        };
        auto count = [&]() {
            uint32_t f = 0;
            if (lane == 0)
                f = __hip_atomic_fetch_add(&l.cq_done[p_q % kChunkQ], 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP) + 1;
            if (wave_u32(f) == p_n) {           // the chunk's last tile
                settle();
                if (lane == 0) {
                    __hip_atomic_store(&l.cq_done[p_q % kChunkQ], 0u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                    c_ret = pool_add(kargs(), p_s, x, p_n);
                }
                c_fly = true;
                c_s = p_s;
                c_G = p_G;
                c_n = p_n;
            }
            pend = false;
        };
        auto drain = [&]() {
            if constexpr (SIG) {
                if (pend) {
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    count();
                }
                settle();
            }
        };
        for (;;) {
            const uint32_t q = u / K, i = u % K;
            // chunk q is published by the wave holding the first ticket of chunk q - 1
            while (before(wave_u32(__hip_atomic_load(&l.cq_have, __ATOMIC_ACQUIRE,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP)), q + 1))
                __builtin_amdgcn_s_sleep(1);
            const uint32_t T = wave_u32(l.cq_T[q % kChunkQ]);
            if (i == 0) {
                uint32_t tn = 0;
                if (lane == 0) {
                    tn = (uint32_t)__hip_atomic_fetch_add(tickets, (uint64_t)1, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT);
                    l.cq_T[(q + 1) % kChunkQ] = tn;
                    __hip_atomic_store(&l.cq_have, q + 2, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
            // the step of pool ticket T
            bool out = false;
            for (;;) {
                if (s >= known) {
                    drain();
                    known = frontier<WPW>(kargs(), l, s, lane);
                    if (known <= s) {        // idle: the next launch resumes at workgroup 0's step
                        out = true;
                        break;
                    }
                }
                const uint64_t *d = reinterpret_cast<const uint64_t *>(l.ring + (s & dmask));
                if (uniform64(d[6]) & kDescStop) {
                    // the workgroup arrives at the STOP when its last wave does
                    drain();
                    if (lane == 0 && __hip_atomic_fetch_add(&l.stopc, 1u, __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_WORKGROUP) + 1 == (uint32_t)WPW)
                        arrive(kargs(), s);
                    ++s;
                    out = true;
                    break;
                }
                const uint32_t e_cur = wave_u32(l.end[s & dmask]);
                if (before(T, e_cur)) break;
                e_prev = e_cur;
                ++s;
                if (wv == 0) refresh(kargs(), l, s, lane);
            }
            if (out) break;
            const uint64_t *d = reinterpret_cast<const uint64_t *>(l.ring + (s & dmask));
            CommitK k{};
            k.stride = e.stride;
            k.R = e.R;
            k.G = uniform64(d[0]);
            k.match = as_global<const uint64_t>(uniform64(d[1]));
            k.cout = as_global<uint64_t>(uniform64(d[2]));
            k.changed = as_global<uint64_t>(uniform64(d[3]));
            k.fallback = as_global<uint64_t>(uniform64(d[4]));
            uint64_t pb, pn;
            pool_range(k.G, e.pools, x, &pb, &pn);
            const uint64_t tile0 = pb + (uint64_t)(T - e_prev) * K;
            const uint32_t n = (uint32_t)(tile0 + K < pb + pn ? K : pb + pn - tile0);
            if (i < n) {
                const uint64_t wbase = uniform64((tile0 + i) * HQ_TILE_GROUPS);
                uint32_t ln;
                asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
                commit_tile<N, FORM, false, LEAD, false, SIG, true>(k, wbase, ln);
                if constexpr (SIG) {
                    asm volatile("" ::: "memory");
                    if (pend) count();
                    pend = true;
                    p_s = s;
                    p_G = k.G;
                    p_q = q;
                    p_n = n;
                }
            }
            u = claim(l, lane);
        }
        drain();
        if (lane == 0 && wv == 0) gp(e.d_cursor)[blockIdx.x] = s;
        return;
    }
#ifdef HQ_ENGINE_WGPROF
    uint64_t *const prof = blockIdx.x < kWgProfMax ? g_wgprof + (size_t)blockIdx.x * 8 : nullptr;
    uint64_t p_busy = 0, p_tiles = 0, p_front = 0, p_nfront = 0, p_refr = 0;
    if (prof && threadIdx.x == 0) {
        __hip_atomic_store(prof + 0, now_ticks(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(prof + 1, (uint64_t)__builtin_amdgcn_s_getreg((3 << 11) | 20),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // HW_REG_XCC_ID [3:0]
        __hip_atomic_store(prof + 2, (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // HW_REG_HW_ID
    }
#endif
    uint32_t t = claim(l, lane);
    // SIG / INPLACE: a decided tile is counted (fin / done) only once its stores are complete.
    // The count of tile k is taken after tile k + 1's loads have returned (vector memory
    // operations complete in issue order on the VM counter, so tile k's stores are done by then):
    // the wave issues the next tile's loads without waiting for its stores' acknowledgements.
    // Before the wave waits (a step barrier, the frontier) or leaves, it drains and counts.
    bool pend = false;        // a decided tile not yet counted
    uint64_t p_s = 0;         // its step
    uint32_t p_tgt = 0;       // SIG: fin value at which its step is decided
    auto count = [&]() {
        if constexpr (INPLACE) {
            if (lane == 0)
                __hip_atomic_fetch_add(&l.done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if constexpr (SIG) {
            uint32_t f = 0;
            if (lane == 0)
                f = __hip_atomic_fetch_add(&l.fin[p_s & dmask], 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP) + 1;
            if (wave_u32(f) == p_tgt && lane == 0) arrive(kargs(), p_s);
        }
        pend = false;
    };
    auto drain = [&]() {
        if constexpr (SIG || INPLACE) {
            if (pend) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                count();
            }
        }
    };
    for (;;) {
        // the step of ticket t
        if (s >= known) {
            drain();
            #ifdef HQ_ENGINE_WGPROF
            const uint64_t p_f0 = now_ticks();
            #endif
            known = frontier<WPW>(kargs(), l, s, lane);
            #ifdef HQ_ENGINE_WGPROF
            p_front += now_ticks() - p_f0;
            ++p_nfront;
            #endif
            if (known <= s) break;   // idle: resume here at the next launch
        }
        const uint64_t slot = s & dmask;
        const uint64_t *d = reinterpret_cast<const uint64_t *>(l.ring + slot);
        if (uniform64(d[6]) & kDescStop) {
            // the wave holding the first ticket past the workgroup's last tile counts the
            // workgroup's arrival at the STOP (every step before it is complete once the grid
            // has exited)
            drain();
            if (t == e_prev && lane == 0) arrive(kargs(), s);
            ++s;
            break;
        }
        const uint32_t e_cur = wave_u32(l.end[slot]);
        if (before(t, e_cur)) {
            CommitK k{};
            k.stride = e.stride;
            k.R = e.R;
            k.G = uniform64(d[0]);
            k.match = as_global<const uint64_t>(uniform64(d[1]));
            k.cout = as_global<uint64_t>(uniform64(d[2]));
            k.changed = as_global<uint64_t>(uniform64(d[3]));
            k.fallback = as_global<uint64_t>(uniform64(d[4]));
            const uint64_t b0 = (uint64_t)blockIdx.x * uniform64(d[7]);
            uint32_t tgt = 0;
            if constexpr (SIG) tgt = wave_u32(l.tgt[slot]);
            if constexpr (INPLACE) {
                // the table's tiles of step s are those of step s - 1: wait until the workgroup
                // has decided every tile before this step (no tile of step s is decided before)
                drain();
                while (before(wave_u32(__hip_atomic_load(&l.done, __ATOMIC_ACQUIRE,
                                                         __HIP_MEMORY_SCOPE_WORKGROUP)),
                              e_prev))
                    __builtin_amdgcn_s_sleep(2);
            }
            // the workgroup's tiles of step s, one ticket at a time
#ifdef HQ_ENGINE_WGPROF
            const uint64_t p_t0 = now_ticks();
#endif
            do {
                const uint64_t wbase = uniform64((b0 + (uint32_t)(t - e_prev)) * HQ_TILE_GROUPS);
                // the lane index laundered per tile: nothing derived from it is loop-invariant, so
                // no per-lane 64-bit address is hoisted and kept (spilled) across the loop
                uint32_t ln;
                asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
                commit_tile<N, FORM, false, LEAD, INPLACE, SIG, true>(k, wbase, ln);
                if constexpr (SIG || INPLACE) {
                    // this tile's loads have returned (its decision used them; the compiler
                    // barrier keeps the count below that wait): the previous tile's stores are
                    // complete
                    asm volatile("" ::: "memory");
                    if (pend) count();
                    pend = true;
                    p_s = s;
                    p_tgt = tgt;
                }
#ifdef HQ_ENGINE_WGPROF
                ++p_tiles;
#endif
                t = claim(l, lane);
            } while (before(t, e_cur));
#ifdef HQ_ENGINE_WGPROF
            p_busy += now_ticks() - p_t0;
#endif
        }
        e_prev = e_cur;
        ++s;
        // Steps posted one at a time reach a working grid one relay at a time: the first wave
        // of each workgroup looks ahead at its step transitions, while its other waves work on
        // (refresh), so that the workgroup seldom runs out of known steps and stalls at its
        // frontier for a relay round trip and a polling sleep (post-as-ready windows)
        #ifdef HQ_ENGINE_WGPROF
        const uint64_t p_r0 = now_ticks();
        #endif
        if (wv == 0) refresh(kargs(), l, s, lane);
        #ifdef HQ_ENGINE_WGPROF
        if (wv == 0) p_refr += now_ticks() - p_r0;
        #endif
    }
    drain();
    if (lane == 0 && wv == 0) gp(e.d_cursor)[blockIdx.x] = s;
#ifdef HQ_ENGINE_WGPROF
    if (prof && lane == 0) {
        __hip_atomic_fetch_add(prof + 3, p_busy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(prof + 4, p_tiles, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_max(prof + 5, now_ticks(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(prof + 6, p_front | (p_nfront << 40), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);   // frontier ticks | entries << 40
        __hip_atomic_fetch_add(prof + 7, p_refr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#endif
}

typedef void (*EngineKernel)(const EngineK);

// 1024-thread workgroups (two per CU) where the tile loop fits 64 VGPRs with no scratch (n <= 5;
// some n = 7, 8 bodies spill at that size), 512 otherwise
template <int N, int FORM, int LEAD, bool INPLACE>
void engine_kernel_for(bool sig, bool bal, EngineKernel *fn, int *blk) {
    constexpr int B = N <= 5 ? 1024 : 512;
    if constexpr (!INPLACE) {
        if (bal) {
            *fn = sig ? k_commit_engine<N, FORM, LEAD, false, B, true, true>
                      : k_commit_engine<N, FORM, LEAD, false, B, false, true>;
            *blk = B;
            return;
        }
    }
    *fn = sig ? k_commit_engine<N, FORM, LEAD, INPLACE, B, true, false>
              : k_commit_engine<N, FORM, LEAD, INPLACE, B, false, false>;
    *blk = B;
}

template <int N>
int engine_kernel_n(uint32_t form, uint32_t layout, bool sig, bool bal, EngineKernel *fn, int *blk) {
    const bool lead = (layout & 0xFFu) == HQ_LAYOUT_TILES_LEADER;
    const bool inplace = (layout & HQ_LAYOUT_IN_PLACE) != 0;
#define HQ_ENGINE_PICK(F)                                                                        \
    if (inplace) engine_kernel_for<N, F, 1, true>(sig, false, fn, blk);                          \
    else if (lead) engine_kernel_for<N, F, 1, false>(sig, bal, fn, blk);                         \
    else engine_kernel_for<N, F, 0, false>(sig, bal, fn, blk);
    if (form == HQ_FORM_TERM_MASK) {
        HQ_ENGINE_PICK(HQ_FORM_TERM_MASK)
    } else {
        HQ_ENGINE_PICK(HQ_FORM_TERM_START)
    }
#undef HQ_ENGINE_PICK
    return HQ_OK;
}

// sig: per-step completion signals (write-through stores: a step's outputs are visible once its
// waves' stores have drained)
int engine_kernel(uint32_t n, uint32_t form, uint32_t layout, bool sig, bool bal, EngineKernel *fn,
                  int *blk) {
    switch (n) {
    case 1: return engine_kernel_n<1>(form, layout, sig, bal, fn, blk);
    case 2: return engine_kernel_n<2>(form, layout, sig, bal, fn, blk);
    case 3: return engine_kernel_n<3>(form, layout, sig, bal, fn, blk);
    case 4: return engine_kernel_n<4>(form, layout, sig, bal, fn, blk);
    case 5: return engine_kernel_n<5>(form, layout, sig, bal, fn, blk);
    case 6: return engine_kernel_n<6>(form, layout, sig, bal, fn, blk);
    case 7: return engine_kernel_n<7>(form, layout, sig, bal, fn, blk);
    default: return engine_kernel_n<8>(form, layout, sig, bal, fn, blk);
    }
}

}  // namespace

struct hq_engine {
    hq_ctx *ctx = nullptr;
    std::mutex mu;               // step workers post from their own threads
    std::string err;
    hq_engine_config cfg{};
    hipStream_t stream = nullptr;   // the resident launch never blocks the context's stream
    hipEvent_t ev_start = nullptr, ev_end = nullptr;
    EngineKernel fn = nullptr;
    int block = 0;
    uint32_t grid = 0;
    EngineK k{};
    char *host = nullptr;        // pinned, coherent: posted | done | clock | ring
    char *dev = nullptr;         // device: posted | arrive | top | cursor | ring
    uint64_t posted = 0;         // descriptors written to the host ring
    uint64_t completed = 0;      // every step below it is known complete
    bool running = false;        // a launch is on the stream (maybe exiting)
    uint64_t launches = 0;       // finished launches since the last timing reset
    double launch_ms = 0.0;
    uint64_t relaunches = 0;
    uint32_t epoch = 0;          // launches so far (the kernel's exit word names its launch)
    uint64_t wait_limit_ms = 60000;   // a wait that sees no completion this long fails (HQ_ENGINE_WAIT_MS)
    size_t cur_off = 0, exit_off = 0, polled_off = 0;   // device state (hq_engine_dump)
    uint64_t inplace_G = 0;      // HQ_LAYOUT_IN_PLACE: the table's G (every post keeps it)
    bool balanced = false;       // per-XCD tile pools (not with HQ_LAYOUT_IN_PLACE)
    size_t claim_off = 0;        // the pools' ticket counters (zeroed before each launch)
};

namespace {

int efail(hq_engine *e, int code, const std::string &msg) {
    e->err = msg;
    return code;
}

int echeck(hq_engine *e, hipError_t r, const char *what) {
    if (r == hipSuccess) return HQ_OK;
    return efail(e, r == hipErrorOutOfMemory ? HQ_E_NOMEM : HQ_E_DEVICE,
                 std::string(what) + ": " + hipGetErrorString(r));
}

uint64_t host_load(const uint64_t *p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }

// the launch on the stream has ended (its events complete): fold its time
int fold_if_ended(hq_engine *e, bool *ended) {
    *ended = !e->running;
    if (!e->running) return HQ_OK;
    const hipError_t q = hipEventQuery(e->ev_end);
    if (q == hipErrorNotReady) return HQ_OK;
    int rc = echeck(e, q, "hipEventQuery(engine)");
    if (rc) return rc;
    float ms = 0.f;
    rc = echeck(e, hipEventElapsedTime(&ms, e->ev_start, e->ev_end), "hipEventElapsedTime");
    if (rc) return rc;
    e->launches++;
    e->launch_ms += ms;
    e->running = false;
    *ended = true;
    return HQ_OK;
}

int launch(hq_engine *e) {
    // hand over the descriptors of the oldest incomplete steps (every wave's cursor is at or
    // beyond e->completed): the grid starts on them without waiting for the relay
    const EngineDesc *ring = reinterpret_cast<const EngineDesc *>(e->host + 128 + 16 * (size_t)e->cfg.depth);
    const uint64_t n = std::min<uint64_t>(e->posted - e->completed, kInit);
    e->k.init_base = e->completed;
    e->k.init_count = (uint32_t)n;
    for (uint64_t i = 0; i < n; ++i) e->k.init[i] = ring[(e->completed + i) & (e->cfg.depth - 1)];
    e->k.epoch = ++e->epoch;
    int rc = echeck(e, hipSetDevice(e->ctx->device), "hipSetDevice");
    // (balanced: the pools' tickets restart with the launch; the previous launch has ended)
    if (!rc && e->balanced)
        rc = echeck(e, hipMemsetAsync(e->dev + e->claim_off, 0, 8 * kPools * kPoolStride, e->stream),
                    "hipMemsetAsync(engine tickets)");
    if (!rc) rc = echeck(e, hipEventRecord(e->ev_start, e->stream), "hipEventRecord");
    if (rc) return rc;
    hipLaunchKernelGGL(e->fn, dim3(e->grid), dim3(e->block), 0, e->stream, e->k);
    rc = echeck(e, hipGetLastError(), "k_commit_engine");
    if (!rc) rc = echeck(e, hipEventRecord(e->ev_end, e->stream), "hipEventRecord");
    if (rc) return rc;
    e->running = true;
    return HQ_OK;
}

int ensure_running(hq_engine *e) {
    bool ended = false;
    int rc = fold_if_ended(e, &ended);
    if (rc || !ended) return rc;
    return launch(e);
}

uint64_t *done_arr(hq_engine *e) { return reinterpret_cast<uint64_t *>(e->host + 128); }

bool step_done(hq_engine *e, uint64_t seq) {
    return host_load(done_arr(e) + (seq & (e->cfg.depth - 1))) >= seq + 1;
}

// Wait until step `seq` (posted) is complete; relaunch the grid if it exited idle meanwhile
// (a post can land just after the workgroups gave up polling).
int wait_step(hq_engine *e, uint64_t seq) {
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t spins = 0;
    for (;;) {
        if (step_done(e, seq)) break;
        bool ended = false;
        int rc = fold_if_ended(e, &ended);
        if (rc) return rc;
        if (ended) {
            if (step_done(e, seq)) break;
            e->relaunches++;
            rc = launch(e);
            if (rc) return rc;
        }
        if (++spins > 256) {
            std::this_thread::yield();
            spins = 0;
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(e->wait_limit_ms))
                return efail(e, HQ_E_DEVICE, "hq_engine: step " + std::to_string(seq) +
                                                 " not completed within the wait limit (" +
                                                 std::to_string(e->wait_limit_ms) + " ms)");
        }
    }
    while (e->completed < e->posted && step_done(e, e->completed)) e->completed++;
    return HQ_OK;
}

int write_desc(hq_engine *e, const EngineDesc &d) {
    EngineDesc *ring = reinterpret_cast<EngineDesc *>(e->host + 128 + 16 * (size_t)e->cfg.depth);
    std::memcpy(ring + (e->posted & (e->cfg.depth - 1)), &d, sizeof d);
    e->posted++;
    __atomic_store_n(reinterpret_cast<uint64_t *>(e->host), e->posted, __ATOMIC_RELEASE);
    return HQ_OK;
}

int drain_locked(hq_engine *e);

// room for one more descriptor: at most `depth` posted steps beyond the last completed one
int make_room(hq_engine *e) {
    if (e->posted - e->completed < e->cfg.depth) return HQ_OK;
    if (e->cfg.flags & HQ_ENGINE_SIGNAL) {
        int rc = ensure_running(e);
        if (!rc) rc = wait_step(e, e->completed);
        return rc;
    }
    return drain_locked(e);
}

int drain_locked(hq_engine *e) {
    bool ended = false;
    int rc = fold_if_ended(e, &ended);
    if (rc) return rc;
    if (!ended) {
        // a grid is (or may still be) resident: a STOP step ends every workgroup after the
        // steps before it (STOP always signals, whatever the flags)
        if (e->posted - e->completed >= e->cfg.depth) {
            // no room for the STOP: wait for the oldest posted step (STOP-less drain impossible)
            if (!(e->cfg.flags & HQ_ENGINE_SIGNAL)) {
                // without per-step signals the steps complete only as a whole: the ring was
                // sized so this cannot happen (post keeps one slot for the STOP)
                return efail(e, HQ_E_STATE, "hq_engine: ring full without a STOP slot");
            }
            rc = wait_step(e, e->completed);
            if (rc) return rc;
        }
        EngineDesc d{};
        d.flags = kDescStop;
        d.seq = e->posted;
        const uint64_t seq = e->posted;
        write_desc(e, d);
        rc = wait_step(e, seq);
        if (rc) return rc;
        rc = echeck(e, hipEventSynchronize(e->ev_end), "hipEventSynchronize(engine)");
        if (rc) return rc;
        rc = fold_if_ended(e, &ended);
        if (rc) return rc;
    } else if (e->posted != e->completed) {
        // the grid exited idle with steps posted after it gave up: run them, then stop
        EngineDesc d{};
        d.flags = kDescStop;
        d.seq = e->posted;
        const uint64_t seq = e->posted;
        write_desc(e, d);
        rc = launch(e);
        if (!rc) rc = wait_step(e, seq);
        if (!rc) rc = echeck(e, hipEventSynchronize(e->ev_end), "hipEventSynchronize(engine)");
        if (!rc) rc = fold_if_ended(e, &ended);
        if (rc) return rc;
    }
    e->completed = e->posted;
    return HQ_OK;
}

int validate_post(hq_engine *e, const hq_commit_args *a) {
    const hq_engine_config &c = e->cfg;
    if (a->n_max != c.n_max || a->form != c.form || a->layout != c.layout)
        return efail(e, HQ_E_INVAL, "hq_engine_post: n_max / form / layout differ from the engine's");
    if (a->n_voting)
        return efail(e, HQ_E_INVAL, "hq_engine_post: per-group n is not served (bucket by n)");
    if (c.form == HQ_FORM_TERM_MASK && a->ring_len != c.ring_len)
        return efail(e, HQ_E_INVAL, "hq_engine_post: ring_len differs from the engine's");
    if (a->G == 0) return HQ_OK;
    const bool in_place = (c.layout & HQ_LAYOUT_IN_PLACE) != 0;
    if (!a->match || (!in_place && !a->committed_out))
        return efail(e, HQ_E_INVAL, "hq_engine_post: NULL tiles (match) / committed_out");
    if (!hq::aligned16(a->match) || (!in_place && !hq::aligned16(a->committed_out)))
        return efail(e, HQ_E_INVAL, "hq_engine_post: tiles and committed_out must be 16-byte aligned");
    // an in-place table keeps its G: a tile then belongs to the same workgroup at every step,
    // which is what orders a group's steps (the kernel orders steps inside a workgroup only)
    if (in_place && e->inplace_G && a->G != e->inplace_G)
        return efail(e, HQ_E_INVAL, "hq_engine_post: an in-place table's steps must keep one G (the "
                                    "engine's first in-place post set it)");
    return HQ_OK;
}

}  // namespace

extern "C" {

int hq_engine_open(hq_ctx *ctx, const hq_engine_config *cfg, hq_engine **out) {
    if (!ctx || !cfg || !out) return HQ_E_INVAL;
    *out = nullptr;
    hq_engine_config c = *cfg;
    if (c.depth == 0) c.depth = kEngineMaxDepth;
    if (c.idle_us == 0) c.idle_us = 1000;     // (the sharing policy)
    if (c.n_max < 1 || c.n_max > HQ_MAX_VOTERS)
        return hq::fail(ctx, HQ_E_INVAL, "hq_engine_open: n_max must be 1..8");
    if (c.form != HQ_FORM_TERM_START && c.form != HQ_FORM_TERM_MASK)
        return hq::fail(ctx, HQ_E_INVAL, "hq_engine_open: the engine serves the term-start and "
                                         "term-mask forms");
    if (c.layout != HQ_LAYOUT_TILES && c.layout != HQ_LAYOUT_TILES_LEADER &&
        c.layout != (HQ_LAYOUT_TILES_LEADER | HQ_LAYOUT_IN_PLACE))
        return hq::fail(ctx, HQ_E_INVAL, "hq_engine_open: layout must be HQ_LAYOUT_TILES, "
                                         "_TILES_LEADER or _TILES_LEADER | HQ_LAYOUT_IN_PLACE");
    if (c.layout == HQ_LAYOUT_TILES_LEADER && c.n_max < 1)
        return hq::fail(ctx, HQ_E_INVAL, "hq_engine_open: bad n_max");
    if (c.form == HQ_FORM_TERM_MASK &&
        (c.ring_len < 1 || c.ring_len > 16 || (c.ring_len & (c.ring_len - 1))))
        return hq::fail(ctx, HQ_E_INVAL, "hq_engine_open: mask form needs ring_len <= 16 (power of two)");
    if (c.depth < 2 || c.depth > kEngineMaxDepth || (c.depth & (c.depth - 1)))
        return hq::fail(ctx, HQ_E_INVAL, "hq_engine_open: depth must be a power of two in 2..64");
    if (c.flags & ~(uint32_t)HQ_ENGINE_SIGNAL)
        return hq::fail(ctx, HQ_E_INVAL, "hq_engine_open: unknown flags");
    hq_engine *e = new (std::nothrow) hq_engine();
    if (!e) return hq::fail(ctx, HQ_E_NOMEM, "hq_engine_open: out of host memory");
    e->ctx = ctx;
    e->cfg = c;
    // balanced mode (per-XCD pools of each step's tiles, HQ_ENGINE_BALANCE=1; not with an
    // in-place table): measured slower than the static ownership on the headline windows at every
    // chunk size, so it is off unless asked for
    e->balanced = false;
    if (const char *b = std::getenv("HQ_ENGINE_BALANCE"))
        e->balanced = !(c.layout & HQ_LAYOUT_IN_PLACE) && std::atoi(b) != 0;
    engine_kernel(c.n_max, c.form, c.layout, (c.flags & HQ_ENGINE_SIGNAL) != 0, e->balanced, &e->fn,
                  &e->block);
    // tiles per claimed chunk: one per wave of the workgroup unless HQ_ENGINE_CHUNK says
    uint32_t chunk = (uint32_t)e->block / 64;
    if (const char *ch = std::getenv("HQ_ENGINE_CHUNK")) chunk = (uint32_t)std::max(1, std::atoi(ch));
    int rc = hq::check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    int cus = 0, per_cu = 0;
    if (!rc) rc = hq::check_hip(ctx, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount,
                                                           ctx->device), "hipDeviceGetAttribute");
    if (!rc) rc = hq::check_hip(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(
                                         &per_cu, reinterpret_cast<const void *>(e->fn), e->block, 0),
                                "hipOccupancyMaxActiveBlocksPerMultiprocessor");
    if (!rc && (cus < 1 || per_cu < 1))
        rc = hq::fail(ctx, HQ_E_DEVICE, "hq_engine_open: the engine kernel does not fit a CU");
    if (rc) {
        delete e;
        return rc;
    }
    e->grid = (uint32_t)(cus * per_cu);
    if (c.max_workgroups && c.max_workgroups < e->grid) e->grid = c.max_workgroups;
    const size_t D = c.depth;
    const size_t host_bytes = 128 + 16 * D + sizeof(EngineDesc) * D;
    if (const char *w = std::getenv("HQ_ENGINE_WAIT_MS")) e->wait_limit_ms = std::max(1, std::atoi(w));
    const size_t arrive_off = 128, top_off = arrive_off + 8 * kShards * D, cur_off = top_off + 8 * D;
    const size_t ring_off = (cur_off + 8 * (size_t)e->grid + 127) & ~(size_t)127;
    const size_t exit_off = ring_off + sizeof(EngineDesc) * D;
    const size_t polled_off = exit_off + 256;
    const size_t claim_off = polled_off + 8 * kPollCopies * kPollStride;
    const size_t pdone_off = claim_off + 8 * kPools * kPoolStride;
    const size_t dev_bytes = pdone_off + 8 * kPools * kPoolStride * D;
    e->claim_off = claim_off;
    e->cur_off = cur_off;
    e->exit_off = exit_off;
    e->polled_off = polled_off;
    void *hp = nullptr, *dp = nullptr;
    rc = hq::check_hip(ctx, hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking),
                       "hipStreamCreateWithFlags");
    if (!rc) rc = hq::check_hip(ctx, hipEventCreate(&e->ev_start), "hipEventCreate");
    if (!rc) rc = hq::check_hip(ctx, hipEventCreate(&e->ev_end), "hipEventCreate");
    if (!rc) rc = hq::check_hip(ctx, hipHostMalloc(&hp, host_bytes, hipHostMallocCoherent),
                                "hipHostMalloc(engine ring)");
    if (!rc) rc = hq::check_hip(ctx, hipMalloc(&dp, dev_bytes), "hipMalloc(engine)");
    if (!rc) rc = hq::check_hip(ctx, hipMemset(dp, 0, dev_bytes), "hipMemset(engine)");
    e->host = static_cast<char *>(hp);
    e->dev = static_cast<char *>(dp);
    if (rc) {
        hq_engine_close(e);
        return rc;
    }
    std::memset(hp, 0, host_bytes);
    EngineK &k = e->k;
    k.stride = hq_commit_tile_words_for(c.n_max, c.form, c.layout);
    k.idle_ticks = (uint64_t)c.idle_us * 100;   // s_memrealtime runs at 100 MHz
    k.R = c.form == HQ_FORM_TERM_MASK ? c.ring_len : 16;
    k.depth = c.depth;
    k.signal = (c.flags & HQ_ENGINE_SIGNAL) ? 1u : 0u;
    k.h_posted = reinterpret_cast<const uint64_t *>(e->host);
    k.h_done = reinterpret_cast<uint64_t *>(e->host + 128);
    k.h_clock = reinterpret_cast<uint64_t *>(e->host + 128 + 8 * D);
    k.h_ring = reinterpret_cast<const EngineDesc *>(e->host + 128 + 16 * D);
    k.d_posted = reinterpret_cast<uint64_t *>(e->dev);
    k.d_arrive = reinterpret_cast<uint64_t *>(e->dev + arrive_off);
    k.d_top = reinterpret_cast<uint64_t *>(e->dev + top_off);
    k.d_cursor = reinterpret_cast<uint64_t *>(e->dev + cur_off);
    k.d_ring = reinterpret_cast<EngineDesc *>(e->dev + ring_off);
    k.d_polled = reinterpret_cast<uint64_t *>(e->dev + polled_off);
    k.d_exit = reinterpret_cast<uint64_t *>(e->dev + exit_off);
    k.d_claim = reinterpret_cast<uint64_t *>(e->dev + claim_off);
    k.d_pdone = reinterpret_cast<uint64_t *>(e->dev + pdone_off);
    k.chunk = e->balanced ? chunk : 0;
    k.pools = std::min<uint32_t>(e->grid, kPools);
    *out = e;
    return HQ_OK;
}

namespace {

// hq_engine_post under the lock; start: launch the grid if none is resident (hq_engine_run
// leaves that to its drain, so that the launch carries the STOP too)
int post_locked(hq_engine *e, const hq_commit_args *args, uint32_t count, uint64_t *first_seq,
                bool start) {
    if (count && !args) return efail(e, HQ_E_INVAL, "hq_engine_post: args is NULL");
    const uint64_t keep_G = e->inplace_G;
    for (uint32_t i = 0; i < count; ++i) {
        int rc = validate_post(e, args + i);
        if (!rc && (e->cfg.layout & HQ_LAYOUT_IN_PLACE) && args[i].G) e->inplace_G = args[i].G;
        if (rc) {
            e->inplace_G = keep_G;
            return rc;
        }
    }
    e->inplace_G = keep_G;
    if (first_seq) *first_seq = e->posted;
    int rc = echeck(e, hipSetDevice(e->ctx->device), "hipSetDevice");
    for (uint32_t i = 0; i < count && !rc; ++i) {
        // keep one slot free for the STOP of a drain when there are no per-step signals
        const bool signal = (e->cfg.flags & HQ_ENGINE_SIGNAL) != 0;
        if (!signal && e->posted - e->completed >= e->cfg.depth - 1) rc = drain_locked(e);
        else rc = make_room(e);
        if (rc) break;
        EngineDesc d{};
        d.G = args[i].G;
        d.tiles = args[i].match;
        d.cout = args[i].committed_out;
        d.changed = args[i].changed;
        d.fallback = args[i].fallback;
        d.seq = e->posted;
        const uint64_t tiles = (d.G + HQ_TILE_GROUPS - 1) / HQ_TILE_GROUPS;
        d.per = (tiles + e->grid - 1) / e->grid;
        if ((e->cfg.layout & HQ_LAYOUT_IN_PLACE) && d.G) e->inplace_G = d.G;
        rc = write_desc(e, d);
    }
    if (!rc && count && start) rc = ensure_running(e);
    return rc;
}

}  // namespace

int hq_engine_post(hq_engine *e, const hq_commit_args *args, uint32_t count, uint64_t *first_seq) {
    if (!e) return HQ_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    return post_locked(e, args, count, first_seq, true);
}

int hq_engine_run(hq_engine *e, const hq_commit_args *args, uint32_t count, uint64_t *first_seq) {
    if (!e) return HQ_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    int rc = post_locked(e, args, count, first_seq, false);
    // no grid resident: the drain launches one whose arguments carry the steps and the STOP (no
    // relay: the grid ends as soon as its last step is decided); a resident grid gets the STOP
    // through the ring as in hq_engine_drain
    if (!rc) rc = echeck(e, hipSetDevice(e->ctx->device), "hipSetDevice");
    return rc ? rc : drain_locked(e);
}

int hq_engine_wait(hq_engine *e, uint64_t seq) {
    if (!e) return HQ_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    if (seq >= e->posted) return efail(e, HQ_E_INVAL, "hq_engine_wait: step not posted");
    if (seq < e->completed) return HQ_OK;
    if (!(e->cfg.flags & HQ_ENGINE_SIGNAL)) return drain_locked(e);
    int rc = echeck(e, hipSetDevice(e->ctx->device), "hipSetDevice");
    if (!rc) rc = ensure_running(e);
    if (!rc) rc = wait_step(e, seq);
    return rc;
}

int hq_engine_drain(hq_engine *e) {
    if (!e) return HQ_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    int rc = echeck(e, hipSetDevice(e->ctx->device), "hipSetDevice");
    return rc ? rc : drain_locked(e);
}

int hq_engine_timing(hq_engine *e, uint64_t *launches, double *total_ms, int reset) {
    if (!e) return HQ_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    bool ended = false;
    int rc = fold_if_ended(e, &ended);
    if (rc) return rc;
    if (launches) *launches = e->launches;
    if (total_ms) *total_ms = e->launch_ms;
    if (reset) {
        e->launches = 0;
        e->launch_ms = 0.0;
    }
    return HQ_OK;
}

int hq_engine_info(hq_engine *e, hq_engine_stats *out) {
    if (!e || !out) return HQ_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    out->grid = e->grid;
    out->block = (uint32_t)e->block;
    out->posted = e->posted;
    out->completed = e->completed;
    out->relaunches = e->relaunches;
    out->running = e->running ? 1u : 0u;
    out->depth = e->cfg.depth;
    return HQ_OK;
}

int hq_engine_done_clock(hq_engine *e, uint64_t seq, uint64_t *ticks) {
    if (!e || !ticks) return HQ_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    if (!(e->cfg.flags & HQ_ENGINE_SIGNAL))
        return efail(e, HQ_E_STATE, "hq_engine_done_clock: needs HQ_ENGINE_SIGNAL");
    if (seq >= e->posted || !step_done(e, seq) ||
        host_load(done_arr(e) + (seq & (e->cfg.depth - 1))) != seq + 1)
        return efail(e, HQ_E_STATE, "hq_engine_done_clock: step not complete or slot reused");
    *ticks = host_load(done_arr(e) + e->cfg.depth + (seq & (e->cfg.depth - 1)));
    return HQ_OK;
}

int hq_engine_dump(hq_engine *e, uint64_t *out, uint32_t n_words) {
    if (!e || !out) return HQ_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    const uint32_t head = 8;
    const size_t D = e->cfg.depth;
    if (n_words < head + e->grid + (kShards + 1) * D)
        return efail(e, HQ_E_INVAL, "hq_engine_dump: needs 8 + grid + 9 * depth words");
    hipStream_t st = nullptr;
    int rc = echeck(e, hipSetDevice(e->ctx->device), "hipSetDevice");
    if (!rc) rc = echeck(e, hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
    uint64_t dp = 0, polled = 0, ex = 0;
    if (!rc) rc = echeck(e, hipMemcpyAsync(&dp, e->dev, 8, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
    if (!rc) rc = echeck(e, hipMemcpyAsync(&polled, e->dev + e->polled_off, 8, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
    if (!rc) rc = echeck(e, hipMemcpyAsync(&ex, e->dev + e->exit_off, 8, hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
    if (!rc) rc = echeck(e, hipMemcpyAsync(out + head, e->dev + e->cur_off, 8 * (size_t)e->grid,
                                           hipMemcpyDeviceToHost, st), "hipMemcpyAsync");
    // the arrival counters: [depth][kShards] then the top counters [depth]
    if (!rc) rc = echeck(e, hipMemcpyAsync(out + head + e->grid, e->dev + 128,
                                           8 * (kShards + 1) * D, hipMemcpyDeviceToHost, st),
                         "hipMemcpyAsync");
    if (!rc) rc = echeck(e, hipStreamSynchronize(st), "hipStreamSynchronize");
    if (st) (void)hipStreamDestroy(st);
    if (rc) return rc;
    out[0] = host_load(reinterpret_cast<const uint64_t *>(e->host));   // posted (host ring)
    out[1] = dp;                                                      // relayed
    out[2] = polled;                                                  // relayed count, copy 0
    out[3] = ex;                                                      // exit epoch
    out[4] = e->epoch;
    out[5] = e->grid;
    out[6] = e->completed;
    out[7] = e->running ? 1 : 0;
    return HQ_OK;
}

const char *hq_engine_last_error(const hq_engine *e) { return e ? e->err.c_str() : ""; }

#ifdef HQ_ENGINE_WGPROF
// probe builds only: the per-workgroup words of the launches since the last reset (8 per
// workgroup, kWgProfMax workgroups), then zeroed when reset is set. Call with no grid resident.
int hq_engine_wgprof(uint64_t *out, uint32_t n_words, int reset) {
    const size_t bytes = sizeof(uint64_t) * 8 * kWgProfMax;
    if (out && n_words < 8 * kWgProfMax) return HQ_E_INVAL;
    if (hipDeviceSynchronize() != hipSuccess) return HQ_E_DEVICE;
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wgprof), bytes) != hipSuccess) return HQ_E_DEVICE;
    if (reset) {
        void *z = nullptr;
        if (hipGetSymbolAddress(&z, HIP_SYMBOL(g_wgprof)) != hipSuccess ||
            hipMemset(z, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
            return HQ_E_DEVICE;
    }
    return HQ_OK;
}
#endif

void hq_engine_close(hq_engine *e) {
    if (!e) return;
    (void)hipSetDevice(e->ctx->device);
    if (e->host && e->dev && e->stream) {
        std::lock_guard<std::mutex> g(e->mu);
        (void)drain_locked(e);
    }
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    if (e->ev_start) (void)hipEventDestroy(e->ev_start);
    if (e->ev_end) (void)hipEventDestroy(e->ev_end);
    if (e->host) (void)hipHostFree(e->host);
    if (e->dev) (void)hipFree(e->dev);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
}

}  // extern "C"

