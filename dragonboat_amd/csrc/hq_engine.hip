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
// Ownership: wave w of the grid decides tiles w, w + W, w + 2W, ... of EVERY posted batch, in
// post order. A group's step s + 1 depends only on its own step s (the in-place table's
// committed row, raft.go:888-909 run per ReplicateResp on that group's state), so the waves need
// no grid barrier between steps: a wave that finishes its tiles of step s starts step s + 1 while
// the others still stream step s (every wave runs its own step sequence: no barrier, no LDS).
//
// Doorbell: the host writes a 64-byte descriptor into the pinned ring and then bumps `posted`
// (both fine-grained host memory). The first wave of workgroup 0 relays new descriptors into a
// device copy of the ring and publishes the relayed count in device memory; a wave at the end of
// what it knows polls that count (relaxed agent-scope load + s_sleep, MI355X_MICROARCH.md
// "polling-cost") and reads each step's descriptor one step ahead. Completion
// (HQ_ENGINE_SIGNAL): a wave counts its arrival on one of 64 shard counters, the last wave of a
// shard on the step's top counter, and the last of those writes the step's sequence number into
// the pinned done array (one PCIe write per step).
//
// Every spin is bounded: a wave that polls without news for idle_us exits (its next step is kept
// in a device cursor, and the next post or wait relaunches the grid, which resumes every wave at
// its cursor), so a host that dies never leaves waves spinning on the GPU.
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
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
                                           // workgroup 97 us after the launch, tools/ab_engine.py)
constexpr int kPollStride = 32;            // u64 between copies
constexpr int kInit = 32;                  // descriptors handed over in the kernel arguments

// A descriptor as the kernel arguments carry it (EngineDesc without seq / reserved).
struct InitDesc {
    uint64_t G;
    const uint64_t *tiles;
    uint64_t *cout, *changed, *fallback;
    uint64_t flags;
};

struct EngineDesc {   // one posted step, 64 bytes = 8 u64 words (one per relay lane)
    uint64_t G;
    const uint64_t *tiles;
    uint64_t *cout;
    uint64_t *changed;
    uint64_t *fallback;
    uint64_t seq;
    uint64_t flags;
    uint64_t reserved;
};
static_assert(sizeof(EngineDesc) == 64, "a descriptor is 8 relay lanes of u64");

struct EngineK {
    uint64_t stride;        // u64 words per tile
    uint64_t idle_ticks;    // s_memrealtime ticks (100 MHz) of polling without news before exit
    uint32_t R;             // term-mask window
    uint32_t depth;         // ring slots (power of two <= kEngineMaxDepth)
    uint32_t waves;         // worker waves in the grid
    uint32_t signal;        // per-step completion into the pinned done array
    const uint64_t *h_posted;      // pinned: descriptors written by the host
    uint64_t *h_done;              // pinned [depth]: seq + 1 of the last step completed per slot
    uint64_t *h_clock;             // pinned [depth]: s_memrealtime at that completion
    const EngineDesc *h_ring;      // pinned [depth]
    uint64_t *d_posted;            // device: descriptors relayed into d_ring
    uint64_t *d_arrive;            // device [depth][kShards]
    uint64_t *d_top;               // device [depth]
    uint64_t *d_cursor;            // device [grid]: the next step of each workgroup
    EngineDesc *d_ring;            // device [depth]
    uint64_t *dbg;                 // HQ_ENGINE_EXP phase clocks (tools/ab_engine.py), else NULL
    uint64_t *d_polled;            // device [kPollCopies * kPollStride]: copies of d_posted
    // the descriptors of steps [init_base, init_base + init_count), known when the grid was
    // launched: every workgroup starts with them in LDS (no relay, no poll at the start)
    uint64_t init_base;
    uint32_t init_count, exp;   // exp: HQ_ENGINE_EXP variant bits (0 in the product)
    InitDesc init[kInit];
};

#ifdef HQ_ENGINE_EXP
// phase clocks of the experiment build: min (i even) / max (i odd) or plain store
#define HQ_EPROBE_MIN(e, i) __hip_atomic_fetch_min((e).dbg + (i), now_ticks(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#define HQ_EPROBE_MAX(e, i) __hip_atomic_fetch_max((e).dbg + (i), now_ticks(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#else
#define HQ_EPROBE_MIN(e, i) ((void)0)
#define HQ_EPROBE_MAX(e, i) ((void)0)
#endif

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

// A pointer read from memory (a posted descriptor) is generic to the compiler, and generic
// pointers compile to FLAT loads and stores (counted in both vmcnt and lgkmcnt: every wait drains
// everything; 13.1 vs 10.2 us per 1M-group step, tools/ab_engine.py). Descriptors hold device
// (global) addresses by contract, so the value is cast into the global address space and back:
// the compiler then infers global for every access through it.
template <class T>
__device__ __forceinline__ T *as_global(uint64_t v) {
    typedef __attribute__((address_space(1))) T GT;
    return (T *)(GT *)v;
}

// Workgroup 0, first wave: copy the descriptors the host has posted since the last relay into
// the device ring and publish their count. Lane l moves u64 word l & 7 of descriptor l >> 3 (+8i).
// The host never posts more than `depth` steps beyond the last completed one, so the slots
// written here are no longer read by any workgroup.
__device__ void relay(const EngineK &e, uint32_t lane) {
    const uint64_t have = __hip_atomic_load(e.d_posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t hp = __hip_atomic_load(e.h_posted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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
                               reinterpret_cast<const uint64_t *>(e.h_ring + ((have + i) & dmask)) +
                                   (lane & 7),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                         : 0;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t i = base + (lane >> 3) + 8 * j;
            if (i < n)
                __hip_atomic_store(reinterpret_cast<uint64_t *>(e.d_ring + ((have + i) & dmask)) +
                                       (lane & 7),
                                   v[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (lane == 0)
        __hip_atomic_store(e.d_posted, have + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane < (uint32_t)kPollCopies)
        __hip_atomic_store(e.d_polled + lane * kPollStride, have + n, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (lane == 0) {
        HQ_EPROBE_MIN(e, 2);   // first relay published
        HQ_EPROBE_MAX(e, 3);   // last relay published
    }
}

// Per-workgroup state in LDS. The descriptors of steps [.., known) sit in `ring` (slot = step &
// (depth - 1)); a wave that has run out of them waits for `known` to grow. The first such wave
// takes `lock` and becomes the workgroup's poller: it polls the relayed count in device memory
// (workgroup 0's poller relays from the host ring first), copies the new descriptors into LDS and
// publishes `known`. `waiting` counts the waves at the end of what they know; the workgroup exits
// idle only when all of them are (so they leave at one step). Per ring slot, `claim` hands out
// the workgroup's tiles of the slot's step one by one (a fetch-add per tile) and `fin` counts
// those decided; `tag` is the step they serve. The first wave to reach a step re-arms its
// slot's counters, once no wave of the workgroup is still on the slot's previous step
// (`cur[w]`: the step wave w claims in).
struct EngineLds {
    EngineDesc ring[kEngineMaxDepth];
    uint64_t tag[kEngineMaxDepth];
    uint32_t claim[kEngineMaxDepth];
    uint32_t fin[kEngineMaxDepth];
    uint64_t cur[16];
    uint64_t known;
    uint32_t waiting, lock, exit, pad;
};

constexpr uint64_t kTagBusy = ~0ull;   // a wave is re-arming the slot

// lane 0: make slot `slot` serve step s (no-op when it does): the winner of the tag waits until
// every wave of the workgroup has left the slot's previous step (s - depth), zeroes the
// counters and publishes the tag; the others wait for it.
template <int WPW>
__device__ void arm_slot(EngineLds &l, uint64_t slot, uint64_t s, uint64_t depth) {
    for (;;) {
        uint64_t t = __hip_atomic_load(&l.tag[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (t == s) return;
        if (t != kTagBusy && __hip_atomic_compare_exchange_strong(
                                 &l.tag[slot], &t, kTagBusy, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP)) {
#pragma unroll 1
            for (int w = 0; w < WPW; ++w)
                while (__hip_atomic_load(&l.cur[w], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) +
                           depth <= s)
                    __builtin_amdgcn_s_sleep(1);
            __hip_atomic_store(&l.claim[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_store(&l.fin[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_store(&l.tag[slot], s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            return;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

__device__ __forceinline__ uint64_t lds_known(EngineLds &l) {
    return __hip_atomic_load(&l.known, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// lane 0's value of a 32-bit LDS atomic, for the whole wave
__device__ __forceinline__ uint32_t wave_u32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// A wave at step s with no descriptor beyond it (s == the workgroup's known count): returns the
// new known count, or s when the workgroup exits idle (the wave then exits at s).
template <int WPW>
__device__ uint64_t frontier(const EngineK &e, EngineLds &l, uint64_t s, uint32_t lane,
                             bool relayer) {
    uint64_t k = lds_known(l);
    if (k > s) return k;
    if (lane == 0) __hip_atomic_fetch_add(&l.waiting, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (;;) {
        k = lds_known(l);
        if (k > s) break;
        if (__hip_atomic_load(&l.exit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return s;
        uint32_t got = 0;
        if (lane == 0)
            got = __hip_atomic_exchange(&l.lock, 1u, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0;
        if (wave_u32(got)) {
            // the workgroup's poller
            const uint64_t t0 = now_ticks();
            uint32_t backoff = 1;
            for (;;) {
                if (relayer) relay(e, lane);
                const uint64_t p =
                    __hip_atomic_load(e.d_polled + (blockIdx.x % kPollCopies) * kPollStride,
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (p > s) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    const uint64_t dmask = e.depth - 1;
                    for (uint64_t i = lane >> 3; i < p - s; i += 8) {
                        const uint64_t slot = (s + i) & dmask;
                        reinterpret_cast<uint64_t *>(l.ring + slot)[lane & 7] = __hip_atomic_load(
                            reinterpret_cast<const uint64_t *>(e.d_ring + slot) + (lane & 7),
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                    if (lane == 0) {
                        __hip_atomic_store(&l.known, p, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                        if (blockIdx.x % 64 == 0) {
                            HQ_EPROBE_MIN(e, 4);   // a sampled workgroup's first descriptors
                            HQ_EPROBE_MAX(e, 5);   // a sampled workgroup's last descriptors
                        }
                    }
                    k = p;
                    break;
                }
                if (now_ticks() - t0 > e.idle_ticks &&
                    __hip_atomic_load(&l.waiting, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) ==
                        (uint32_t)WPW) {
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

// The workgroup is done with step s (called once per workgroup and step, by lane 0 of the wave
// that decided its last tile). The tiles' stores were write-through (WT) and every deciding wave
// drained them before counting its tile, so they are visible device-wide with no release fence
// (Guideline 16 R1; a release fence per workgroup and step, an L2 write-back each, took 26 us per
// step). The workgroup counts on the step's shard counter (blockIdx % 8), the last workgroup of
// a shard on the step's top counter, and the last of those publishes the step to the host. The
// last arriver of a counter resets it for the slot's next step: the host posts that step only
// after it has seen this one's done flag, which is written after the resets.
__device__ void arrive(const EngineK &e, uint64_t s) {
    const uint64_t slot = s & (e.depth - 1);
    const uint32_t shard = blockIdx.x % kShards;
    const uint32_t nshard = gridDim.x < (uint32_t)kShards ? gridDim.x : (uint32_t)kShards;
    const uint64_t per = (gridDim.x - shard + kShards - 1) / kShards;   // workgroups in the shard
    uint64_t *ctr = e.d_arrive + slot * kShards + shard;
    if (__hip_atomic_fetch_add(ctr, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1 !=
        per)
        return;
    __hip_atomic_store(ctr, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__hip_atomic_fetch_add(e.d_top + slot, (uint64_t)1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT) + 1 != nshard)
        return;
    __hip_atomic_store(e.d_top + slot, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(e.h_clock + slot, now_ticks(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(e.h_done + slot, s + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    HQ_EPROBE_MAX(e, 11);   // a step (or STOP) published to the host
}

// Workgroup b owns tiles [b * per, b * per + per) of every step (per = ceil(tiles / grid)); its
// waves take them one at a time from the slot's LDS claim counter, so the waves of a workgroup
// balance each other (older waves are served first by the memory pipeline: with a fixed tile
// per wave the youngest finished a 20-step window 2.8 x later than the oldest, 236 vs 83 us,
// tools/ab_engine.py). A wave that finds the workgroup's tiles of step s all taken moves on to
// step s + 1 while the others finish theirs: no barrier between steps. In-place tables
// (INPLACE) are the exception: a wave takes tiles of step s + 1 only when the workgroup has
// decided all of step s, since the same table tiles come back at every step.
template <int N, int FORM, int LEAD, bool INPLACE, int BLK, bool WT>
__global__ __launch_bounds__(BLK, BLK >= 1024 ? 8 : 1) void k_commit_engine(const EngineK e) {
    constexpr int WPW = BLK / 64;   // waves per workgroup
    __shared__ EngineLds l;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool relayer = blockIdx.x == 0;
    const uint64_t dmask = e.depth - 1;
    uint64_t s = uniform64(e.d_cursor[blockIdx.x]);   // written by the previous launch
    for (uint32_t i = threadIdx.x; i < kEngineMaxDepth; i += BLK) l.tag[i] = kTagBusy - 1;
    if (lane == 0) l.cur[wv] = s;
    // the descriptors handed over at launch (the host's oldest incomplete step <= the cursor)
    if (wv == 0 && lane < 6) {
#pragma unroll
        for (int i = 0; i < kInit; ++i) {
            if ((uint32_t)i < e.init_count) {
                const InitDesc &x = e.init[i];
                const uint64_t v = lane == 0 ? x.G
                                 : lane == 1 ? reinterpret_cast<uint64_t>(x.tiles)
                                 : lane == 2 ? reinterpret_cast<uint64_t>(x.cout)
                                 : lane == 3 ? reinterpret_cast<uint64_t>(x.changed)
                                 : lane == 4 ? reinterpret_cast<uint64_t>(x.fallback)
                                             : x.flags;
                reinterpret_cast<uint64_t *>(l.ring + ((e.init_base + i) & dmask))[lane < 5 ? lane : 6] = v;
            }
        }
    }
    if (threadIdx.x == 0) {
        const uint64_t top = e.init_base + e.init_count;
        l.known = top > s ? top : s;
        l.waiting = l.lock = l.exit = 0;
    }
    if (threadIdx.x == 0 && blockIdx.x % 64 == 0) {
        HQ_EPROBE_MIN(e, 0);   // kernel start (sampled)
        HQ_EPROBE_MAX(e, 1);
    }
    __syncthreads();
    uint64_t known = s;
    for (;;) {
        if (s >= known) {
            known = frontier<WPW>(e, l, s, lane, relayer);
            if (known <= s) break;   // idle: resume here at the next launch
        }
        const uint64_t slot = s & dmask;
        const uint64_t *d = reinterpret_cast<const uint64_t *>(l.ring + slot);
        if (uniform64(d[6]) & kDescStop) {
            // the first wave here counts the workgroup's arrival at the STOP (every step before
            // it is complete once the grid has exited)
            uint32_t i = 0;
            if (lane == 0) {
                arm_slot<WPW>(l, slot, s, e.depth);
                i = __hip_atomic_fetch_add(&l.claim[slot], 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (wave_u32(i) == 0 && lane == 0) {
                if (blockIdx.x % 64 == 0) HQ_EPROBE_MAX(e, 10);   // workgroups at the STOP
                arrive(e, s);
            }
            ++s;
            break;
        }
        CommitK k{};
        k.G = uniform64(d[0]);
        k.stride = e.stride;
        k.match = as_global<const uint64_t>(uniform64(d[1]));
        k.cout = as_global<uint64_t>(uniform64(d[2]));
        k.changed = as_global<uint64_t>(uniform64(d[3]));
        k.fallback = as_global<uint64_t>(uniform64(d[4]));
        k.R = e.R;
        const uint64_t tiles = (k.G + HQ_TILE_GROUPS - 1) / HQ_TILE_GROUPS;
        const uint64_t per = (tiles + gridDim.x - 1) / gridDim.x;
        const uint64_t b0 = (uint64_t)blockIdx.x * per;
        const uint32_t len = (uint32_t)(b0 >= tiles ? 0 : tiles - b0 < per ? tiles - b0 : per);
        if (lane == 0) arm_slot<WPW>(l, slot, s, e.depth);
        for (;;) {
            uint32_t i = 0;
            if (lane == 0)
                i = __hip_atomic_fetch_add(&l.claim[slot], 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
            i = wave_u32(i);
            if (i >= len) {
                // the first claim past the end of an empty range stands in for its last tile
                if (i == len && len == 0 && e.signal && lane == 0) arrive(e, s);
                break;
            }
            commit_tile<N, FORM, false, LEAD, INPLACE, WT>(k, (b0 + i) * HQ_TILE_GROUPS, lane);
            if (e.signal || INPLACE) {
                if (e.signal) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // WT drained
                uint32_t f = 0;
                if (lane == 0)
                    f = __hip_atomic_fetch_add(&l.fin[slot], 1u, __ATOMIC_RELEASE,
                                               __HIP_MEMORY_SCOPE_WORKGROUP) + 1;
                if (wave_u32(f) == len && e.signal && lane == 0) arrive(e, s);
            }
        }
#ifdef HQ_ENGINE_EXP
        if (lane == 0 && blockIdx.x % 64 == 0) {
            HQ_EPROBE_MIN(e, 6);   // first step done (sampled)
            HQ_EPROBE_MAX(e, 7);   // last step done (sampled)
        }
        if (lane == 0 && s + 1 == e.init_base + e.init_count && wave_u32(wv) < 16 &&
            (uint64_t)blockIdx.x * 16 + wv < 16384)
            e.dbg[64 + (uint64_t)blockIdx.x * 16 + wv] = now_ticks();   // every wave's finish
#endif
        if constexpr (INPLACE) {
            // the table's tiles of step s + 1 are those of step s: wait until they are decided
            while (__hip_atomic_load(&l.fin[slot], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <
                   len)
                __builtin_amdgcn_s_sleep(2);
        }
        ++s;
        if (lane == 0) __hip_atomic_store(&l.cur[wv], s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    if (lane == 0 && wv == 0) e.d_cursor[blockIdx.x] = s;
}

typedef void (*EngineKernel)(const EngineK);

template <int N, int FORM, int LEAD, bool INPLACE>
void engine_kernel_for(bool wt, EngineKernel *fn, int *blk) {
#ifdef HQ_ENGINE_EXP   // A/B: HQ_ENGINE_BLOCK=512 takes 512-thread workgroups at any N
    const char *eb = std::getenv("HQ_ENGINE_BLOCK");
    if (N <= 5 && eb && std::atoi(eb) == 512) {
        *fn = wt ? k_commit_engine<N, FORM, LEAD, INPLACE, 512, true>
                 : k_commit_engine<N, FORM, LEAD, INPLACE, 512, false>;
        *blk = 512;
        return;
    }
#endif
    if constexpr (N <= 5) {
        *fn = wt ? k_commit_engine<N, FORM, LEAD, INPLACE, 1024, true>
                 : k_commit_engine<N, FORM, LEAD, INPLACE, 1024, false>;
        *blk = 1024;
    } else {
        *fn = wt ? k_commit_engine<N, FORM, LEAD, INPLACE, 512, true>
                 : k_commit_engine<N, FORM, LEAD, INPLACE, 512, false>;
        *blk = 512;
    }
}

template <int N>
int engine_kernel_n(uint32_t form, uint32_t layout, bool wt, EngineKernel *fn, int *blk) {
    const bool lead = (layout & 0xFFu) == HQ_LAYOUT_TILES_LEADER;
    const bool inplace = (layout & HQ_LAYOUT_IN_PLACE) != 0;
#define HQ_ENGINE_PICK(F)                                                                        \
    if (inplace) engine_kernel_for<N, F, 1, true>(wt, fn, blk);                                  \
    else if (lead) engine_kernel_for<N, F, 1, false>(wt, fn, blk);                               \
    else engine_kernel_for<N, F, 0, false>(wt, fn, blk);
    if (form == HQ_FORM_TERM_MASK) {
        HQ_ENGINE_PICK(HQ_FORM_TERM_MASK)
    } else {
        HQ_ENGINE_PICK(HQ_FORM_TERM_START)
    }
#undef HQ_ENGINE_PICK
    return HQ_OK;
}

// WT (write-through stores) for the per-step completion signals: a step's outputs are visible
// once its waves' stores have drained
int engine_kernel(uint32_t n, uint32_t form, uint32_t layout, bool wt, EngineKernel *fn, int *blk) {
    switch (n) {
    case 1: return engine_kernel_n<1>(form, layout, wt, fn, blk);
    case 2: return engine_kernel_n<2>(form, layout, wt, fn, blk);
    case 3: return engine_kernel_n<3>(form, layout, wt, fn, blk);
    case 4: return engine_kernel_n<4>(form, layout, wt, fn, blk);
    case 5: return engine_kernel_n<5>(form, layout, wt, fn, blk);
    case 6: return engine_kernel_n<6>(form, layout, wt, fn, blk);
    case 7: return engine_kernel_n<7>(form, layout, wt, fn, blk);
    default: return engine_kernel_n<8>(form, layout, wt, fn, blk);
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
    for (uint64_t i = 0; i < n; ++i) {
        const EngineDesc &d = ring[(e->completed + i) & (e->cfg.depth - 1)];
        e->k.init[i] = InitDesc{d.G, d.tiles, d.cout, d.changed, d.fallback, d.flags};
    }
    int rc = echeck(e, hipSetDevice(e->ctx->device), "hipSetDevice");
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
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60))
                return efail(e, HQ_E_DEVICE, "hq_engine: step not completed within 60 s");
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
    return HQ_OK;
}

}  // namespace

extern "C" {

int hq_engine_open(hq_ctx *ctx, const hq_engine_config *cfg, hq_engine **out) {
    if (!ctx || !cfg || !out) return HQ_E_INVAL;
    *out = nullptr;
    hq_engine_config c = *cfg;
    if (c.depth == 0) c.depth = kEngineMaxDepth;
    if (c.idle_us == 0) c.idle_us = 20000;
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
    engine_kernel(c.n_max, c.form, c.layout, (c.flags & HQ_ENGINE_SIGNAL) != 0, &e->fn, &e->block);
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
    const size_t arrive_off = 128, top_off = arrive_off + 8 * kShards * D, cur_off = top_off + 8 * D;
    const size_t ring_off = (cur_off + 8 * (size_t)e->grid + 127) & ~(size_t)127;
    const size_t dbg_off = ring_off + sizeof(EngineDesc) * D;
    const size_t polled_off = dbg_off + 8 * (64 + 16384);
    const size_t dev_bytes = polled_off + 8 * kPollCopies * kPollStride;
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
    k.waves = e->grid * (uint32_t)(e->block / 64);
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
#ifdef HQ_ENGINE_EXP
    k.dbg = reinterpret_cast<uint64_t *>(e->dev + dbg_off);
#endif
    *out = e;
    return HQ_OK;
}

int hq_engine_post(hq_engine *e, const hq_commit_args *args, uint32_t count, uint64_t *first_seq) {
    if (!e) return HQ_E_INVAL;
    std::lock_guard<std::mutex> g(e->mu);
    if (count && !args) return efail(e, HQ_E_INVAL, "hq_engine_post: args is NULL");
    for (uint32_t i = 0; i < count; ++i) {
        int rc = validate_post(e, args + i);
        if (rc) return rc;
    }
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
        rc = write_desc(e, d);
    }
    if (!rc && count) rc = ensure_running(e);
    return rc;
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

const char *hq_engine_last_error(const hq_engine *e) { return e ? e->err.c_str() : ""; }

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

#ifdef HQ_ENGINE_EXP
// ---- tuning experiments (tools/lib_engexp, tools/ab_engine.py): never in the product build ----
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

extern "C" int hq_exp_engine_set(hq_engine *e, uint32_t bits) {
    e->k.exp = bits;
    return HQ_OK;
}

extern "C" int hq_exp_engine_probe(hq_engine *e, uint64_t *out) {
    // read and re-arm the phase clocks (even slots min, odd max)
    if (hipMemcpy(out, e->k.dbg, (64 + 16384) * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return HQ_E_DEVICE;
    uint64_t init[32];
    for (int i = 0; i < 32; ++i) init[i] = (i & 1) ? 0 : ~0ull;
    return hipMemcpy(e->k.dbg, init, sizeof init, hipMemcpyHostToDevice) == hipSuccess ? HQ_OK
                                                                                         : HQ_E_DEVICE;
}

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
    if (!ctx || !a || count == 0 || count > (uint32_t)kExpMax) return HQ_E_INVAL;
    if (a[0].n_max != 5 || a[0].form != HQ_FORM_TERM_MASK || a[0].layout != HQ_LAYOUT_TILES_LEADER)
        return HQ_E_INVAL;
    MultiK m{};
    m.stride = hq_commit_tile_words_for(5, HQ_FORM_TERM_MASK, HQ_LAYOUT_TILES_LEADER);
    m.G = a[0].G;
    m.R = a[0].ring_len;
    m.count = count;
    m.ntiles = (uint32_t)((m.G + HQ_TILE_GROUPS - 1) / HQ_TILE_GROUPS);
    for (uint32_t i = 0; i < count; ++i) {
        if (a[i].G != m.G) return HQ_E_INVAL;
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
        if (!ctr && hipMalloc(&ctr, 4 * kExpMax) != hipSuccess) return HQ_E_NOMEM;
        (void)hipMemsetAsync(ctr, 0, 4 * kExpMax, ctx->stream);
        const char *pv = std::getenv("AB_POOL");   // permille of a batch's tiles in the pool
        const uint32_t pool = (uint32_t)((uint64_t)m.ntiles * (pv ? std::atoi(pv) : 250) / 1000);
        hipLaunchKernelGGL((k_exp_pool<5, HQ_FORM_TERM_MASK, 1, 1024>), dim3(grid ? grid : 512),
                           dim3(1024), 0, ctx->stream, m, ctr, pool);
    } else if (variant == 6) {
        static uint32_t *ctr = nullptr;
        if (!ctr && hipMalloc(&ctr, 4 * kExpMax * 1024) != hipSuccess) return HQ_E_NOMEM;
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
#endif
