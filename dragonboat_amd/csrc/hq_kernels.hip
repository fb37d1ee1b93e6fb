// hq_kernels.hip — CDNA4 (gfx950) kernels of the batched quorum engine and their _dev launchers.
//
// Every kernel is an HBM stream over structure-of-arrays group state: one lane owns one or more
// whole groups, loads are coalesced (consecutive lanes -> consecutive groups), decisions are
// integer min/max networks and popcounts in registers, and bitmap outputs are assembled with
// wave-wide __ballot (64-bit on wave64). No LDS and no MFMA: nothing here is reused or a
// contraction (DESIGN.md "Kernels").
#include <cstdlib>

#include "hq_internal.h"
#include "hq_commit_body.h"

namespace {

constexpr int kBlock = 256;           // 4 waves of 64
// The commit stream runs 512-thread blocks: ~5 % shorter than 256 on the 1M x 3 launch under
// rocprofv3 (11.7 vs 12.4 us, tools/kexp2.hip, git history); 4 groups per lane was slower.
constexpr int kCommitBlock = 512;
// Kernels that fit 64 VGPRs (occupancy 8) run 1024-thread blocks: 10.57 vs 11.1 us per 1M x 3
// launch (tools/kexp3.hip, git history: fewer workgroups to dispatch for the same waves); the others keep
// 512 so that two or more blocks still fit a CU. HQ_COMMIT_BLOCK_BIG=512 restores one size.
#ifndef HQ_COMMIT_BLOCK_BIG
#define HQ_COMMIT_BLOCK_BIG 1024
#endif
template <int N, int FORM, bool PERN>
constexpr int commit_blk() {
    return !PERN && N <= 5 ? HQ_COMMIT_BLOCK_BIG : kCommitBlock;
}
template <int N, bool PERN>
constexpr int lag_blk() {
    return !PERN && N <= 4 ? HQ_COMMIT_BLOCK_BIG : kCommitBlock;
}
// Grid cap in 256-thread units (64 per CU), grid-stride beyond. An 8M-group x 5 launch then runs
// one tile per wave: 92-94 vs 96-98 us with the earlier cap of 16 per CU, neutral at 1M groups
// (profiles/r01e/ab_maxblocks.log).
#ifndef HQ_MAX_BLOCKS
#define HQ_MAX_BLOCKS (256 * 64)
#endif
constexpr int kMaxBlocks = HQ_MAX_BLOCKS;

// Every field of a column batch (the generator and the tile packer write / read them all).
struct CommitCols {
    uint64_t G, stride, nwords;
    uint32_t n_max, R;
    const uint64_t *match;
    const uint8_t *nv;
    const uint64_t *cin;
    uint64_t *cout;
    const uint64_t *last;
    const uint64_t *tstart;
    const uint64_t *term;
    const uint64_t *ring;
    uint64_t *changed;
    uint64_t *fallback;
    const uint16_t *mask;
    const uint32_t *ring32;
    uint64_t tile_words;   // HQ_LAYOUT_TILES: u64 words per tile
};

// VEC = groups per lane (2: 16-byte loads of every SoA column; 1: 8-byte loads). The body of
// one workgroup `blk` of `nblk` working on batch `a` (k_commit: the grid; k_commit_fused: the
// workgroups one batch of the launch owns). TILED (HQ_LAYOUT_TILES, VEC = 2 only): a wave's 128
// groups are one tile, so its loads walk one contiguous 128·(n+3)·8-byte block instead of n + 3
// column streams. TILED = 2 (HQ_LAYOUT_TILES_LEADER): the same tiles without the leader's match
// row; slot 0 is last_index (the leader's own match, raft.go:918, 1031).
template <int N, int FORM, bool PERN, int BLK, int LEAD, bool INPLACE = false>
__device__ __forceinline__ void tile_blocks(const CommitK &a, uint64_t blk, uint64_t nblk);

template <int N, int FORM, int VEC, bool PERN, int BLK>
__device__ __forceinline__ void column_blocks(const CommitK &a, uint64_t blk, uint64_t nblk) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = blk * (BLK / 64) + (threadIdx.x >> 6);
    const uint64_t step = nblk * BLK * VEC;
    for (uint64_t wbase = wave * 64 * VEC; wbase < a.G; wbase += step) {
        const uint64_t g0 = wbase + (uint64_t)lane * VEC;
        // every input field as a base + this lane's element offset: slot s of match at
        // bm[s * ms + off], then committed_in, last_index and aux (term_start / term as u64, or
        // the u16 mask)
        const uint64_t *bm = a.match, *bcin = a.cin, *blast = a.last;
        const uint64_t *baux = static_cast<const uint64_t *>(a.aux);
        const uint16_t *bmask = static_cast<const uint16_t *>(a.aux);
        const uint64_t ms = a.stride, off = g0;
        auto aux1 = [&]() -> uint64_t {
            if constexpr (FORM == HQ_FORM_TERM_MASK) return bmask[off];
            return baux[off];
        };
        bool chg[VEC], fb[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) chg[j] = fb[j] = false;
        if constexpr (VEC == 2) {
            // both groups of the lane: 16-byte loads of every field
            auto pair = [&]() {
                uint64_t m0[N], m1[N];
#pragma unroll
                for (int s = 0; s < N; ++s) {
                    const u64x2 v = ld_stream2(bm + s * ms + off);
                    m0[s] = v.x;
                    m1[s] = v.y;
                }
                const u64x2 ci = ld_stream2(bcin + off);
                const u64x2 la = ld_stream2(blast + off);
                u64x2 ax;
                if constexpr (FORM == HQ_FORM_TERM_MASK) {
                    const uint32_t mm = __builtin_nontemporal_load(
                        reinterpret_cast<const uint32_t *>(bmask + off));
                    ax = (u64x2){mm & 0xFFFFu, mm >> 16};
                } else {
                    ax = ld_stream2(baux + off);
                }
                int n0 = N, n1 = N;
                if constexpr (PERN) {
                    const uint16_t nn = *reinterpret_cast<const uint16_t *>(a.nv + g0);
                    n0 = nn & 0xFF;
                    n1 = nn >> 8;
                }
                uint64_t co0, co1;
                decide<N, FORM, PERN>(a, g0, m0, n0, ci.x, la.x, ax.x, co0, chg[0], fb[0]);
                decide<N, FORM, PERN>(a, g0 + 1, m1, n1, ci.y, la.y, ax.y, co1, chg[1], fb[1]);
                st_stream2(a.cout + g0, (u64x2){co0, co1});
            };
            // one group (the other of the lane's pair is outside the batch)
            auto single = [&](int j) {
                uint64_t m0[N];
#pragma unroll
                for (int s = 0; s < N; ++s) m0[s] = bm[s * ms + off + j];
                const int n0 = PERN ? (int)a.nv[g0 + j] : N;
                const uint64_t ax = FORM == HQ_FORM_TERM_MASK ? (uint64_t)bmask[off + j]
                                                              : baux[off + j];
                uint64_t co;
                decide<N, FORM, PERN>(a, g0 + j, m0, n0, bcin[off + j], blast[off + j], ax, co,
                                      chg[j], fb[j]);
                a.cout[g0 + j] = co;
            };
            if (g0 + 1 < a.G) pair();
            else if (g0 < a.G) single(0);
            // the wave's 128 groups are two bitmap words: lane k < 2 writes word k (lane i's
            // groups are bits 2i, 2i+1: the two ballots interleaved)
            const uint64_t b0 = __ballot(chg[0]), b1 = __ballot(chg[1]);
            const uint64_t f0 = __ballot(fb[0]), f1 = __ballot(fb[1]);
            const uint64_t w = (wbase >> 6) + lane;
            if (lane < 2 && w < ((a.G + 63) >> 6)) {
                const int sh = 32 * lane;
                if (a.changed)
                    a.changed[w] = spread32((uint32_t)(b0 >> sh)) |
                                   (spread32((uint32_t)(b1 >> sh)) << 1);
                if (a.fallback)
                    a.fallback[w] = spread32((uint32_t)(f0 >> sh)) |
                                    (spread32((uint32_t)(f1 >> sh)) << 1);
            }
        } else {
            auto one = [&]() {
                uint64_t m0[N];
#pragma unroll
                for (int s = 0; s < N; ++s) m0[s] = bm[s * ms + off];
                const int n0 = PERN ? (int)a.nv[g0] : N;
                uint64_t co;
                decide<N, FORM, PERN>(a, g0, m0, n0, bcin[off], blast[off], aux1(), co, chg[0],
                                      fb[0]);
                a.cout[g0] = co;
            };
            if (g0 < a.G) one();
            const uint64_t b0 = __ballot(chg[0]);
            const uint64_t f0 = __ballot(fb[0]);
            if (lane == 0) {
                if (a.changed) a.changed[wbase >> 6] = b0;
                if (a.fallback) a.fallback[wbase >> 6] = f0;
            }
        }
    }
}

// HQ_LAYOUT_TILES: one wave per 128-group tile. Row position 2i holds group i of the tile and
// position 2i + 1 group i + 64, so lane i's 16-byte load of a row brings groups i and i + 64:
// every field of the wave is ONE contiguous block of (n + 3) KiB, and the two ballots are the
// tile's two bitmap words as they are (no bit interleave). The full-tile test is scalar (the
// wave index is read into an SGPR), so full tiles carry no per-lane guard.
// TILED = 3: HQ_LAYOUT_TILES_LEADER | HQ_LAYOUT_IN_PLACE, the device-resident table decided in
// place (committed' written into the tile's committed row)
template <int N, int FORM, int VEC, bool PERN, int BLK, int TILED = 0>
__device__ __forceinline__ void commit_blocks(const CommitK &a, uint64_t blk, uint64_t nblk) {
    static_assert(!TILED || VEC == 2, "tiles are read two groups per lane");
    if constexpr (TILED) tile_blocks<N, FORM, PERN, BLK, TILED >= 2 ? 1 : 0, TILED == 3>(a, blk, nblk);
    else column_blocks<N, FORM, VEC, PERN, BLK>(a, blk, nblk);
}

// LEAD = 1: rows start at slot 1 (row s - 1 holds slot s) and m[0] = last_index, so the wave's
// block is (n + 2) KiB: 8 bytes less per group.
template <int N, int FORM, bool PERN, int BLK, int LEAD, bool INPLACE>
__device__ __forceinline__ void tile_blocks(const CommitK &a, uint64_t blk, uint64_t nblk) {
    constexpr uint64_t T = HQ_TILE_GROUPS;
    const uint64_t lane = threadIdx.x & 63;
    const uint64_t wave = blk * (BLK / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t step = nblk * BLK * 2;
    for (uint64_t wbase = wave * T; wbase < a.G; wbase += step)
        commit_tile<N, FORM, PERN, LEAD, INPLACE>(a, wbase, lane);
}

template <int N, int FORM, int VEC, bool PERN, int TILED>
__global__ __launch_bounds__(kCommitBlock) void k_commit(const CommitK a) {
    commit_blocks<N, FORM, VEC, PERN, kCommitBlock, TILED>(a, blockIdx.x, gridDim.x);
}
// the 1024-thread twin: two blocks per CU need occupancy 8 (<= 64 VGPRs), so it is asked for
template <int N, int FORM, int VEC, bool PERN, int TILED>
__global__ __launch_bounds__(HQ_COMMIT_BLOCK_BIG, 8) void k_commit_big(const CommitK a) {
    commit_blocks<N, FORM, VEC, PERN, HQ_COMMIT_BLOCK_BIG, TILED>(a, blockIdx.x, gridDim.x);
}

// Several uniform-n batches of one step in ONE launch (a step worker's voter-count buckets):
// batch i owns workgroups [first[i], first[i+1]); the batch index and its n are uniform per
// workgroup, so the switch costs no divergence. Saves the dependent-launch boundary and the
// grid fill / drain between buckets (MI355X_MICROARCH.md "boundary": 1.7-1.9 us each).
constexpr int kMaxFused = 8;        // lag batches per fused launch
// commit batches per fused launch: a step worker's voter-count buckets, or the independent
// batches of several steps / step workers posted together (32 x 1M-group batches in one launch:
// no boundary, fill or drain between them; 3.3 KB of kernel arguments)
constexpr int kMaxFusedCommit = 32;
struct FusedK {
    CommitK b[kMaxFusedCommit];
    uint32_t first[kMaxFusedCommit + 1];
    uint32_t n[kMaxFusedCommit];   // dwords: a scalar load (a byte array is read with a vector load + wait)
    uint32_t count;
};

template <int FORM, int BLK, int TILED>
__global__ __launch_bounds__(BLK, BLK > kCommitBlock ? 8 : 1) void k_commit_fused(const FusedK f) {
    const uint32_t blk = blockIdx.x;
    uint32_t i = 0;
#pragma unroll
    for (int k = 1; k < kMaxFusedCommit; ++k) i += (k < (int)f.count && blk >= f.first[k]) ? 1u : 0u;
    const uint64_t b = blk - f.first[i], nb = f.first[i + 1] - f.first[i];
    switch (f.n[i]) {
    case 1: commit_blocks<1, FORM, 2, false, BLK, TILED>(f.b[i], b, nb); break;
    case 2: commit_blocks<2, FORM, 2, false, BLK, TILED>(f.b[i], b, nb); break;
    case 3: commit_blocks<3, FORM, 2, false, BLK, TILED>(f.b[i], b, nb); break;
    case 4: commit_blocks<4, FORM, 2, false, BLK, TILED>(f.b[i], b, nb); break;
    case 5: commit_blocks<5, FORM, 2, false, BLK, TILED>(f.b[i], b, nb); break;
    case 6: commit_blocks<6, FORM, 2, false, BLK, TILED>(f.b[i], b, nb); break;
    case 7: commit_blocks<7, FORM, 2, false, BLK, TILED>(f.b[i], b, nb); break;
    default: commit_blocks<8, FORM, 2, false, BLK, TILED>(f.b[i], b, nb); break;
    }
}

// ---- commit over lags (hq_commit_lag_dev): int32 distances below lastIndex -------------------
// Four groups per lane: every column is read with 16-byte loads of four int32 (consecutive
// lanes -> consecutive groups). The quorum-th largest match is the quorum-th SMALLEST lag.
struct LagK {
    uint64_t G, stride, nwords;
    uint32_t n_max, R;
    const int32_t *lag;
    const uint8_t *nv;
    const int32_t *cin;
    int32_t *cout;
    const int32_t *ts;
    const uint16_t *mask;
    uint64_t *changed, *fallback;
};

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

// groups per lane of the lag kernels (4: 16-byte loads, 2: 8-byte loads); HQ_LAG_VEC at build
#ifndef HQ_LAG_VEC
#define HQ_LAG_VEC 4
#endif
constexpr int kLagVec = HQ_LAG_VEC;

__device__ __forceinline__ void ce_i32(int32_t &a, int32_t &b) {
    const int32_t lo = a < b ? a : b, hi = a < b ? b : a;
    a = lo;
    b = hi;
}

// the (n/2+1)-th smallest of v[0..n); slots >= n are padded with INT32_MAX (the maximum), so
// with a runtime n the (n/2+1)-th smallest of the padded N values is the same element
template <int N, bool PERN>
__device__ __forceinline__ int32_t lag_select(int32_t (&v)[N], int n) {
    if constexpr (!PERN && N == 1) {
        return v[0];
    } else if constexpr (!PERN && N == 2) {
        return v[0] > v[1] ? v[0] : v[1];   // quorum 2 of 2: the larger lag
    } else if constexpr (!PERN && N == 3) {  // median of 3
        ce_i32(v[0], v[1]);
        ce_i32(v[1], v[2]);
        return v[0] > v[1] ? v[0] : v[1];
    } else {
#pragma unroll
        for (int r = 0; r < N; ++r) {
#pragma unroll
            for (int i = r & 1; i + 1 < N; i += 2) ce_i32(v[i], v[i + 1]);
        }
        if constexpr (!PERN) return v[N / 2];   // index quorum - 1 = N/2
        const int idx = n / 2;
        int32_t r = 0;
#pragma unroll
        for (int k = 0; k < N; ++k) r = (k == idx) ? v[k] : r;
        return r;
    }
}

template <int N, int FORM, bool PERN>
__device__ __forceinline__ void decide_lag(const LagK &a, int32_t (&l)[N], int n, int32_t c,
                                           int32_t aux, int32_t &co, bool &chg, bool &fb) {
    co = c;
    chg = false;
    if constexpr (PERN) {
        fb = n < 1 || n > N;
#pragma unroll
        for (int s = 0; s < N; ++s) l[s] = (s < n) ? l[s] : INT32_MAX;
    } else {
        fb = false;
    }
    if constexpr (FORM == HQ_FORM_TERM_START) {
        fb |= c == INT32_MAX || c == INT32_MIN;   // committed not representable as a lag
    } else {
        fb |= c < 0 || c > (int32_t)a.R;
    }
    const int32_t d = lag_select<N, PERN>(l, n);
    if constexpr (FORM == HQ_FORM_TERM_START) {
        // q > committed, q <= last, q >= term_start (aux = ts_lag)
        chg = !fb & (d < c) & (d >= 0) & (d <= aux);
    } else {
        // bit d of the lag-indexed mask: term(last - d) == term (d < c <= R <= 16)
        chg = !fb & (d < c) & (d >= 0) && ((aux >> (d & 31)) & 1);
    }
    co = chg ? d : c;
}

// bit i of x (16 bits) -> bit 4i
__device__ __forceinline__ uint64_t spread16x4(uint32_t x) {
    uint64_t v = x & 0xFFFFu;
    v = (v | (v << 24)) & 0x000000FF000000FFull;
    v = (v | (v << 12)) & 0x000F000F000F000Full;
    v = (v | (v << 6)) & 0x0303030303030303ull;
    v = (v | (v << 3)) & 0x1111111111111111ull;
    return v;
}

template <int V> struct LagVec;   // VEC int32 lanes of one load
template <> struct LagVec<4> { typedef i32x4 T; typedef uint64_t M; typedef uint32_t NV; };
template <> struct LagVec<2> {
    typedef int32_t T __attribute__((ext_vector_type(2)));
    typedef uint32_t M;
    typedef uint16_t NV;
};

// bit i of the V ballots' 64/V-bit slice -> bit V*i + j of a bitmap word
template <int V>
__device__ __forceinline__ uint64_t spread_v(uint32_t x) {
    if constexpr (V == 4) return spread16x4(x);
    else if constexpr (V == 2) return spread32(x);
    else return x;
}

// VEC = 4 / 2: lane owns groups g0..g0+VEC-1 (16- / 8-byte loads of every column); VEC = 1: one
// group, 4-byte loads. The body of workgroup `blk` of `nblk` on batch `a`.
// LEAD = 1 (HQ_LAG_LEADER_IMPLICIT): lag row s - 1 holds slot s, slot 0's lag is 0 (the
// leader's own match is lastIndex, raft.go:918, 1031): 4 bytes less per group.
template <int N, int FORM, int VEC, bool PERN, int BLK, int LEAD = 0>
__device__ __forceinline__ void lag_blocks(const LagK &a, uint64_t blk, uint64_t nblk) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = blk * (BLK / 64) + (threadIdx.x >> 6);
    const uint64_t step = nblk * BLK * VEC;
    for (uint64_t wbase = wave * 64 * VEC; wbase < a.G; wbase += step) {
        const uint64_t g0 = wbase + (uint64_t)lane * VEC;
        bool chg[VEC], fb[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) chg[j] = fb[j] = false;
        bool done = false;
        if constexpr (VEC > 1) {
            if (g0 + VEC <= a.G) {
                done = true;
                typedef typename LagVec<VEC>::T VT;
                int32_t l[VEC][N];
#pragma unroll
                for (int s = LEAD; s < N; ++s) {
                    const VT v = __builtin_nontemporal_load(
                        reinterpret_cast<const VT *>(a.lag + (s - LEAD) * a.stride + g0));
#pragma unroll
                    for (int j = 0; j < VEC; ++j) l[j][s] = v[j];
                }
                if constexpr (LEAD) {
#pragma unroll
                    for (int j = 0; j < VEC; ++j) l[j][0] = 0;
                }
                const VT ci = __builtin_nontemporal_load(reinterpret_cast<const VT *>(a.cin + g0));
                int32_t av[VEC];
                if constexpr (FORM == HQ_FORM_TERM_START) {
                    const VT t = __builtin_nontemporal_load(reinterpret_cast<const VT *>(a.ts + g0));
#pragma unroll
                    for (int j = 0; j < VEC; ++j) av[j] = t[j];
                } else {
                    // the lane's VEC u16 masks in one aligned load
                    typedef typename LagVec<VEC>::M MT;
                    const MT m = __builtin_nontemporal_load(reinterpret_cast<const MT *>(a.mask + g0));
#pragma unroll
                    for (int j = 0; j < VEC; ++j) av[j] = (int32_t)((m >> (16 * j)) & 0xFFFF);
                }
                int nn[VEC];
#pragma unroll
                for (int j = 0; j < VEC; ++j) nn[j] = N;
                if constexpr (PERN) {
                    typedef typename LagVec<VEC>::NV NT;
                    const NT x = *reinterpret_cast<const NT *>(a.nv + g0);
#pragma unroll
                    for (int j = 0; j < VEC; ++j) nn[j] = (x >> (8 * j)) & 0xFF;
                }
                VT co;
#pragma unroll
                for (int j = 0; j < VEC; ++j) {
                    int32_t c;
                    decide_lag<N, FORM, PERN>(a, l[j], nn[j], ci[j], av[j], c, chg[j], fb[j]);
                    co[j] = c;
                }
                *reinterpret_cast<VT *>(a.cout + g0) = co;
            }
        }
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            const uint64_t g = g0 + j;
            if (!done && g < a.G) {
                int32_t l[N];
#pragma unroll
                for (int s = LEAD; s < N; ++s) l[s] = a.lag[(s - LEAD) * a.stride + g];
                if constexpr (LEAD) l[0] = 0;
                const int n = PERN ? (int)a.nv[g] : N;
                const int32_t aux = FORM == HQ_FORM_TERM_START ? a.ts[g] : (int32_t)a.mask[g];
                int32_t co;
                decide_lag<N, FORM, PERN>(a, l, n, a.cin[g], aux, co, chg[j], fb[j]);
                a.cout[g] = co;
            }
        }
        {
        // lane l owns groups VEC*l .. VEC*l+VEC-1 of the wave's 64*VEC: bitmap word k covers
        // lanes (64/VEC)*k .. (64/VEC)*(k+1)-1
        uint64_t bc[VEC], bf[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
            bc[j] = __ballot(chg[j]);
            bf[j] = __ballot(fb[j]);
        }
        if (lane < VEC) {
            const int sh = (64 / VEC) * lane;
            const uint64_t w = (wbase >> 6) + lane;
            uint64_t wc = 0, wf = 0;
#pragma unroll
            for (int j = 0; j < VEC; ++j) {
                wc |= spread_v<VEC>((uint32_t)(bc[j] >> sh)) << j;
                wf |= spread_v<VEC>((uint32_t)(bf[j] >> sh)) << j;
            }
            if (VEC == 1) {
                wc = bc[0];
                wf = bf[0];
            }
            if (w < a.nwords) {
                if (a.changed) a.changed[w] = wc;
                if (a.fallback) a.fallback[w] = wf;
            }
        }
    }
    }
}

template <int N, int FORM, int VEC, bool PERN, int LEAD>
__global__ __launch_bounds__(kCommitBlock) void k_commit_lag(const LagK a) {
    lag_blocks<N, FORM, VEC, PERN, kCommitBlock, LEAD>(a, blockIdx.x, gridDim.x);
}
template <int N, int FORM, int VEC, bool PERN, int LEAD>
__global__ __launch_bounds__(HQ_COMMIT_BLOCK_BIG, 8) void k_commit_lag_big(const LagK a) {
    lag_blocks<N, FORM, VEC, PERN, HQ_COMMIT_BLOCK_BIG, LEAD>(a, blockIdx.x, gridDim.x);
}

// the lag twin of k_commit_fused: uniform-n lag batches of one step in one launch
struct FusedLagK {
    LagK b[kMaxFused];
    uint32_t first[kMaxFused + 1];
    uint32_t n[kMaxFused];   // dwords: a scalar load (a byte array is read with a vector load + wait)
    uint32_t count;
};

template <int FORM, int BLK, int LEAD>
__global__ __launch_bounds__(BLK, BLK > kCommitBlock ? 8 : 1) void k_commit_lag_fused(const FusedLagK f) {
    const uint32_t blk = blockIdx.x;
    uint32_t i = 0;
#pragma unroll
    for (int k = 1; k < kMaxFusedCommit; ++k) i += (k < (int)f.count && blk >= f.first[k]) ? 1u : 0u;
    const uint64_t b = blk - f.first[i], nb = f.first[i + 1] - f.first[i];
    switch (f.n[i]) {
    case 1: lag_blocks<1, FORM, kLagVec, false, BLK, LEAD>(f.b[i], b, nb); break;
    case 2: lag_blocks<2, FORM, kLagVec, false, BLK, LEAD>(f.b[i], b, nb); break;
    case 3: lag_blocks<3, FORM, kLagVec, false, BLK, LEAD>(f.b[i], b, nb); break;
    case 4: lag_blocks<4, FORM, kLagVec, false, BLK, LEAD>(f.b[i], b, nb); break;
    case 5: lag_blocks<5, FORM, kLagVec, false, BLK, LEAD>(f.b[i], b, nb); break;
    case 6: lag_blocks<6, FORM, kLagVec, false, BLK, LEAD>(f.b[i], b, nb); break;
    case 7: lag_blocks<7, FORM, kLagVec, false, BLK, LEAD>(f.b[i], b, nb); break;
    default: lag_blocks<8, FORM, kLagVec, false, BLK, LEAD>(f.b[i], b, nb); break;
    }
}

// ---- ReadIndex / vote / CheckQuorum over u8 bitmaps: 16 groups per lane ---------------------
struct BitsK {
    uint64_t G;
    uint32_t n_uniform, self_slot;
    const uint8_t *ack, *granted, *rejected;
    uint8_t *active;
    const uint8_t *nv;
    uint64_t *confirmed, *outcome, *has_quorum, *fallback;
    uint64_t n16;   // number of 16-group slots covered by the 64-group bitmap words
    uint64_t n16o;  // number of 16-group slots covered by the 32-group outcome words
    const uint8_t *tiles;  // HQ_LAYOUT_TILES: 1024-group tiles of rows [n] ack granted rejected
    uint32_t tile_rows;    // 4 with the per-group n row, else 3
};

constexpr int kRI = 1, kVOTE = 2, kCHECKQ = 4;

union V16 {
    uint4 v;
    u32x4 w;
    uint8_t b[16];
};

__device__ __forceinline__ V16 load16(const uint8_t *p, uint64_t g, uint64_t G) {
    V16 r;
    if (g + 16 <= G) {
        r.w = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p + g));
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) r.b[k] = (g + k < G) ? p[g + k] : 0;
    }
    return r;
}

// ---- SWAR helpers: four groups per 32-bit word, one byte each -------------------------------
constexpr uint32_t kB80 = 0x80808080u, kB01 = 0x01010101u;

// per-byte popcount (each result byte 0..8)
__device__ __forceinline__ uint32_t popc_bytes(uint32_t x) {
    x = x - ((x >> 1) & 0x55555555u);
    x = (x & 0x33333333u) + ((x >> 2) & 0x33333333u);
    return (x + (x >> 4)) & 0x0F0F0F0Fu;
}
// bit 7 of each byte: a_byte >= b_byte, for bytes a, b < 128
__device__ __forceinline__ uint32_t ge_bytes(uint32_t a, uint32_t b) {
    return ((a | kB80) - b) & kB80;
}
// 4 flag bytes (0x80 / 0x00) -> 4 consecutive bits (group k -> bit k): a byte dot product with
// weights 1, 2, 4, 8 (v_dot4_u32_u8, full rate; the multiply it replaces is quarter rate)
__device__ __forceinline__ uint32_t pack4(uint32_t f) {
    return __builtin_amdgcn_udot4(f, 0x08040201u, 0u, false) >> 7;
}
// 4 flag bytes -> bits 0, 2, 4, 6 (the low bit of 2-bit fields); `hi` flags -> bits 1, 3, 5, 7
__device__ __forceinline__ uint32_t pack4x2(uint32_t f, uint32_t hi = 0) {
    return __builtin_amdgcn_udot4(f, 0x40100401u, __builtin_amdgcn_udot4(hi, 0x80200802u, 0u, false),
                                  false) >> 7;
}
// per-byte valid n in [1, 8] -> 0x80
__device__ __forceinline__ uint32_t valid_n(uint32_t n) {
    const uint32_t lo = n & 0x0F0F0F0Fu, hi = (n >> 4) & 0x0F0F0F0Fu;
    return (lo + 0x7F7F7F7Fu) & ~(lo + 0x77777777u) & ~(hi + 0x7F7F7F7Fu) & kB80;
}
// per-byte (1 << n) - 1 for n in [0, 8] with v_perm_b32 as a byte lookup table: selectors 0..7
// pick masks 0x00..0x7F from {0x7F3F1F0F, 0x07030100}; selector 13 (n = 8) yields 0xFF
__device__ __forceinline__ uint32_t mask_n(uint32_t n) {
    const uint32_t b3 = n & 0x08080808u;   // n = 8 -> selector 8 | 4 | 1 = 13 (no multiply)
    const uint32_t sel = n | (b3 >> 1) | (b3 >> 3);
    return __builtin_amdgcn_perm(0x7F3F1F0Fu, 0x07030100u, sel);
}

// One 16-group slot starting at group g. FULL: all 16 groups exist (g + 16 <= G), so every load
// is one unconditional 16-byte nontemporal load and no byte needs masking (the common case; the
// ragged tail slot takes the guarded path).
// TILED: the inputs are the slot's tile rows, loaded by the caller before it branches on the full
// tile test (so the four loads issue together); every tile is padded to 1024 groups, so even the
// ragged last slot holds 16 loaded bytes (the padding bytes are masked by `inr` like any byte
// beyond G).
template <int MODE, bool PERN, bool FULL, bool TILED = false, bool FB = true>
__device__ __forceinline__ void bits_slot(const BitsK &a, uint64_t g, uint32_t nu,
                                          const V16 *trow = nullptr) {
    const uint64_t slot = g >> 4;
    V16 nv = {}, ack = {}, gr = {}, rj = {}, ac = {};
    auto ld = [&](const uint8_t *p, uint32_t row = 0) -> V16 {
        if constexpr (TILED) {
            return trow[row];
        } else if constexpr (FULL) {
            V16 r;
            r.w = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p + g));
            return r;
        }
        return g < a.G ? load16(p, g, a.G) : V16{};
    };
    constexpr uint32_t r0 = PERN ? 1 : 0;   // tile rows: [n] ack granted rejected
    if constexpr (PERN) nv = ld(a.nv, 0);
    if constexpr (MODE & kRI) ack = ld(a.ack, r0);
    if constexpr (MODE & kVOTE) {
        gr = ld(a.granted, r0 + 1);
        rj = ld(a.rejected, r0 + 2);
    }
    if constexpr (MODE & kCHECKQ) ac = ld(a.active);
    uint32_t conf = 0, outc = 0, hq = 0, fb = 0;
    V16 keep;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        // bytes of groups >= G are excluded (their output bits stay 0)
        uint32_t inr = kB80;
        if constexpr (!FULL) {
            const uint64_t left = g < a.G ? a.G - g : 0;
            inr = left >= (uint64_t)(4 * w + 4) ? kB80
                  : left <= (uint64_t)(4 * w)   ? 0u
                                                : (kB80 >> (8 * (4 - (uint32_t)(left - 4 * w))));
        }
        const uint32_t n = PERN ? nv.w[w] : nu;
        const uint32_t ok = valid_n(n) & inr;
        const uint32_t mask = mask_n(n);
        const uint32_t quorum = ((n >> 1) & 0x7F7F7F7Fu) + kB01;  // n/2 + 1 (valid bytes)
        uint32_t bad = ~ok & inr;
        if constexpr (MODE & kRI) {
            // readindex.go:84: len(confirmed) + 1 >= quorum  <=>  acks >= quorum - 1
            const uint32_t c = popc_bytes(ack.w[w] & mask);
            conf |= pack4(ge_bytes(c, quorum - kB01) & ok) << (4 * w);
        }
        if constexpr (MODE & kVOTE) {
            const uint32_t gm = gr.w[w] & mask;
            const uint32_t rm = rj.w[w] & mask & ~gm;  // first response wins
            const uint32_t lead = ge_bytes(popc_bytes(gm), quorum) & ok;
            const uint32_t foll = ge_bytes(popc_bytes(rm), quorum) & ok & ~lead;
            const uint32_t cand = inr & ~lead & ~foll;
            // 2-bit codes: leader 2 (bit 1), candidate 1 (bit 0), follower 0
            outc |= pack4x2(cand, lead) << (8 * w);
        }
        if constexpr (MODE & kCHECKQ) {
            const uint32_t self = kB01 << a.self_slot;
            const uint32_t selfok = ge_bytes(n, (a.self_slot + 1) * kB01) & ok;
            bad = ~selfok & inr;
            const uint32_t c = popc_bytes((ac.w[w] | self) & mask);
            hq |= pack4(ge_bytes(c, quorum) & selfok) << (4 * w);
            // setNotActive for every voting member (raft.go:385, remote.go:196-198);
            // groups left to the CPU path keep their flags
            keep.w[w] = ac.w[w] & ((bad >> 7) * 0xFFu);
        }
        if constexpr (FB) fb |= pack4(bad) << (4 * w);
    }
    // 64-group bitmap words viewed as 16-bit slots, 32-group outcome words as 32-bit slots
    // (a full slot lies below G / 16 <= n16, n16o)
    if (FULL || slot < a.n16) {
        if constexpr (MODE & kRI) reinterpret_cast<uint16_t *>(a.confirmed)[slot] = conf;
        if constexpr (MODE & kCHECKQ) reinterpret_cast<uint16_t *>(a.has_quorum)[slot] = hq;
        if (FB && a.fallback) reinterpret_cast<uint16_t *>(a.fallback)[slot] = fb;
    }
    if constexpr (MODE & kVOTE) {
        if (FULL || slot < a.n16o) reinterpret_cast<uint32_t *>(a.outcome)[slot] = outc;
    }
    if constexpr (MODE & kCHECKQ) {
        if constexpr (FULL) {
            *reinterpret_cast<uint4 *>(a.active + g) = keep.v;
        } else {
            for (int k = 0; k < 16; ++k)
                if (g + k < a.G) a.active[g + k] = keep.b[k];
        }
    }
}

// FB = false (no fallback bitmap requested) drops the fallback bits' arithmetic (tiles only)
template <int MODE, bool PERN, int BLK, bool TILED = false, bool FB = true>
__global__ __launch_bounds__(BLK) void k_bits(const BitsK a) {
    const uint64_t tid = (uint64_t)blockIdx.x * BLK + threadIdx.x;
    const uint64_t step = (uint64_t)gridDim.x * BLK * 16;
    const uint32_t nu = a.n_uniform * kB01;  // n_uniform <= 8: no byte overflow
    if constexpr (TILED) {
        // one wave per 1024-group tile: the tile base is wave-uniform (scalar), lane i reads
        // bytes [16 i, 16 i + 16) of every row
        constexpr uint64_t R = PERN ? 4 : 3;
        const uint64_t lane = threadIdx.x & 63;
        const uint64_t wave = (uint64_t)blockIdx.x * (BLK / 64) +
                              __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        const uint64_t nw = (uint64_t)gridDim.x * (BLK / 64);
        const uint64_t slots = a.n16o > a.n16 ? a.n16o : a.n16;
        const uint64_t ntiles = (slots * 16 + 1023) >> 10;
        for (uint64_t t = wave; t < ntiles; t += nw) {
            const uint8_t *base = a.tiles + t * (R << 10) + lane * 16;
            V16 rows[R];
#pragma unroll
            for (uint64_t r = 0; r < R; ++r)
                rows[r].w = __builtin_nontemporal_load(
                    reinterpret_cast<const u32x4 *>(base + (r << 10)));
            const uint64_t g = (t << 10) + lane * 16;
            if ((t << 10) + 1024 <= a.G)
                bits_slot<MODE, PERN, true, true, FB>(a, g, nu, rows);
            else
                bits_slot<MODE, PERN, false, true, FB>(a, g, nu, rows);
        }
        return;
    }
    for (uint64_t g = tid * 16; g < a.n16o * 16 || g < a.n16 * 16; g += step) {
        if (g + 16 <= a.G)
            bits_slot<MODE, PERN, true, TILED>(a, g, nu);
        else
            bits_slot<MODE, PERN, false, TILED>(a, g, nu);
    }
}

// ---- 3-byte bitmap tiles (hq_readindex_vote_tiles3_dev) -------------------------------------
// The leader's / candidate's own slot 0 carries no information: it never acks its own ReadIndex
// ctx (readindex.go:84 counts it as the +1), always grants its own vote (campaign, raft.go:1093)
// and never rejects it. So each of the three rows keeps the 7 bits of slots 1..7 (bit k = slot
// k + 1) and its bit 7 holds one bit of n - 1: ack row bit 0 of n - 1, granted row bit 1,
// rejected row bit 2. 3 bytes per group instead of 4 (rows [n] ack granted rejected), n always
// in [1, 8]: nothing to fall back on.
template <bool FULL>
__device__ __forceinline__ void bits3_slot(const BitsK &a, uint64_t g, const V16 *rows) {
    const uint64_t slot = g >> 4;
    uint32_t conf = 0, outc = 0;
#ifdef HQ_BITS3_COPY   // tuning floor: the same loads and stores, no decision (wrong results)
    for (int w = 0; w < 4; ++w) {
        conf ^= rows[0].w[w] ^ rows[1].w[w];
        outc += rows[2].w[w];
    }
    if (FULL || slot < a.n16) reinterpret_cast<uint16_t *>(a.confirmed)[slot] = conf ^ (conf >> 16);
    if (FULL || slot < a.n16o) reinterpret_cast<uint32_t *>(a.outcome)[slot] = outc;
    return;
#endif
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        uint32_t inr = kB80;
        if constexpr (!FULL) {
            const uint64_t left = g < a.G ? a.G - g : 0;
            inr = left >= (uint64_t)(4 * w + 4) ? kB80
                  : left <= (uint64_t)(4 * w)   ? 0u
                                                : (kB80 >> (8 * (4 - (uint32_t)(left - 4 * w))));
        }
        const uint32_t A = rows[0].w[w], Gr = rows[1].w[w], Rj = rows[2].w[w];
        const uint32_t nm1 = ((A >> 7) & kB01) | ((Gr >> 6) & 0x02020202u) | ((Rj >> 5) & 0x04040404u);
        const uint32_t mask = mask_n(nm1);                 // the other voters' bits 0 .. n-2
        const uint32_t half = ((nm1 + kB01) >> 1) & 0x7F7F7F7Fu;   // n/2 = quorum - 1
        // readindex.go:84: acks + 1 >= quorum <=> acks >= n/2
        conf |= pack4(ge_bytes(popc_bytes(A & mask), half) & inr) << (4 * w);
        // handleVoteResp: granted (self included) / rejected (first response wins) >= quorum
        const uint32_t gm = Gr & mask, rm = Rj & mask & ~gm;
        const uint32_t lead = ge_bytes(popc_bytes(gm), half) & inr;          // gm + 1 >= n/2 + 1
        const uint32_t foll = ge_bytes(popc_bytes(rm), half + kB01) & inr & ~lead;
        outc |= pack4x2(inr & ~lead & ~foll, lead) << (8 * w);
    }
    if (FULL || slot < a.n16) reinterpret_cast<uint16_t *>(a.confirmed)[slot] = conf;
    if (FULL || slot < a.n16o) reinterpret_cast<uint32_t *>(a.outcome)[slot] = outc;
}

// TPW tiles per wave and iteration, every row load of them issued before the first decision
// (HQ_BITS3_TPW: 2 took 12.6-12.7 vs 13.4-13.6 us per 16M-group launch on one box, 4 no
// better than 1; tools/ab_libs.sh with tools/lib_b3tpw{2,4})
#ifndef HQ_BITS3_TPW
#define HQ_BITS3_TPW 2
#endif
constexpr int kB3TPW = HQ_BITS3_TPW;

template <int BLK>
__global__ __launch_bounds__(BLK) void k_bits3(const BitsK a) {
    const uint64_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (BLK / 64) +
                          __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * (BLK / 64);
    const uint64_t slots = a.n16o > a.n16 ? a.n16o : a.n16;
    const uint64_t ntiles = (slots * 16 + 1023) >> 10;
    for (uint64_t t0 = wave * kB3TPW; t0 < ntiles; t0 += nw * kB3TPW) {
        V16 rows[kB3TPW][3];
#pragma unroll
        for (int j = 0; j < kB3TPW; ++j) {
            const uint64_t t = t0 + j < ntiles ? t0 + j : t0;   // wave-uniform
            const uint8_t *base = a.tiles + t * (3 << 10) + lane * 16;
#pragma unroll
            for (uint64_t r = 0; r < 3; ++r)
                rows[j][r].w = __builtin_nontemporal_load(
                    reinterpret_cast<const u32x4 *>(base + (r << 10)));
        }
#pragma unroll
        for (int j = 0; j < kB3TPW; ++j) {
            const uint64_t t = t0 + j;
            if (t >= ntiles) break;
            const uint64_t g = (t << 10) + lane * 16;
            if ((t << 10) + 1024 <= a.G) bits3_slot<true>(a, g, rows[j]);
            else bits3_slot<false>(a, g, rows[j]);
        }
    }
}

// columns -> 3-byte tiles: one thread per group; a group outside the contract (n not in
// [1, 8], its own slot acked / not granted / rejected) gets a fallback bit and zero bytes
__global__ __launch_bounds__(kBlock) void k_tile_bits3(uint64_t G, const uint8_t *nv, uint32_t nu,
                                                       const uint8_t *ack, const uint8_t *gr,
                                                       const uint8_t *rj, uint8_t *tiles,
                                                       uint64_t *fallback) {
    const uint64_t total = (G + 1023) / 1024 * 1024;
    for (uint64_t g0 = (uint64_t)blockIdx.x * kBlock; g0 < total; g0 += (uint64_t)gridDim.x * kBlock) {
        const uint64_t g = g0 + threadIdx.x;
        uint32_t A = 0, Gr = 0, Rj = 0;
        bool bad = false;
        if (g < G) {
            const uint32_t n = nv ? nv[g] : nu;
            const uint32_t a = ack[g], x = gr[g], r = rj[g];
            bad = n < 1 || n > 8 || (a & 1) || !(x & 1) || (r & 1);
            if (!bad) {
                const uint32_t keep = (1u << n) - 2u, m = n - 1;   // slots 1 .. n-1
                A = ((a & keep) >> 1) | ((m & 1) << 7);
                Gr = ((x & keep) >> 1) | (((m >> 1) & 1) << 7);
                Rj = ((r & keep) >> 1) | (((m >> 2) & 1) << 7);
            }
        }
        if (g < total) {
            uint8_t *row = tiles + (g >> 10) * (3 << 10) + (g & 1023);
            row[0] = (uint8_t)A;
            row[1024] = (uint8_t)Gr;
            row[2048] = (uint8_t)Rj;
        }
        const uint64_t b = __ballot(bad);
        if (fallback && (threadIdx.x & 63) == 0 && g < ((G + 63) & ~63ull)) fallback[g >> 6] = b;
    }
}

// ---- bit-plane tiles (hq_readindex_vote_planes_dev) -----------------------------------------
// The 3-byte tiles transposed: a 2048-group tile holds 24 planes of 256 bytes, plane 8r + b =
// bit b of row r's byte (rows ack, granted, rejected) for the tile's groups, bit j of dword k =
// group 32k + j. A lane takes 32 groups: one dword of every plane, and decides them with
// bitwise full adders and comparators over the planes (bit-sliced: ~6 instructions per group
// for both decisions, against ~15 for the byte-SWAR form of k_bits3). The confirmed plane is
// the confirmed bitmap word as it is; the outcome codes interleave the candidate and leader
// planes.
constexpr uint32_t kPlaneTile = HQ_PLANE_TILE_GROUPS;   // 2048
// HQ_PLANES_TPW tiles per wave and iteration (1: 10.3 us per 16M-group launch, 2: 10.7 us — 103
// VGPRs, half the occupancy — tools/ab_libs.sh), HQ_PLANES_BLK threads per block
#ifndef HQ_PLANES_TPW
#define HQ_PLANES_TPW 1
#endif
#ifndef HQ_PLANES_BLK
#define HQ_PLANES_BLK 256
#endif
constexpr int kPlTPW = HQ_PLANES_TPW;
// tiles per wave of the fused ReadIndex + vote + CheckQuorum pass (one after the other)
#ifndef HQ_PLCQ_TPW
#define HQ_PLCQ_TPW 1
#endif
// the fused pass zeroes the active planes right behind their loads (1: 15.5-15.7 us per 16 M x 7
// launch, 70-71 % of peak) or after the decision (0: 15.7-15.9 us; profiles/r03c/ab_c4pq_zero_early.log)
#ifndef HQ_PLCQ_ZERO_EARLY
#define HQ_PLCQ_ZERO_EARLY 1
#endif

__device__ __forceinline__ void full_add(uint32_t a, uint32_t b, uint32_t c, uint32_t &s,
                                         uint32_t &co) {
    const uint32_t t = a ^ b;
    s = t ^ c;
    co = (a & b) | (c & t);
}

// popcount of 7 planes as a 3-bit bit-sliced number (c0 + 2 c1 + 4 c2)
__device__ __forceinline__ void count7(const uint32_t *x, uint32_t &c0, uint32_t &c1,
                                       uint32_t &c2) {
    uint32_t s1, k1, s2, k2, k3;
    full_add(x[0], x[1], x[2], s1, k1);
    full_add(x[3], x[4], x[5], s2, k2);
    full_add(s1, s2, x[6], c0, k3);
    full_add(k1, k2, k3, c1, c2);
}

// (a2 a1 a0) >= (b2 b1 b0), bit-sliced
__device__ __forceinline__ uint32_t ge3(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t b0,
                                        uint32_t b1, uint32_t b2) {
    const uint32_t lt = (~a2 & b2) | (~(a2 ^ b2) & ((~a1 & b1) | (~(a1 ^ b1) & (~a0 & b0))));
    return ~lt;
}

// 2-bit codes of 32 groups: bit 2j = lo_j, bit 2j + 1 = hi_j (byte zip, then a perfect shuffle
// of each 16-bit unit)
__device__ __forceinline__ uint32_t shuffle16(uint32_t x) {
    x = (x & 0xF00FF00Fu) | ((x & 0x00F000F0u) << 4) | ((x >> 4) & 0x00F000F0u);
    x = (x & 0xC3C3C3C3u) | ((x & 0x0C0C0C0Cu) << 2) | ((x >> 2) & 0x0C0C0C0Cu);
    x = (x & 0x99999999u) | ((x & 0x22222222u) << 1) | ((x >> 1) & 0x22222222u);
    return x;
}

// CQ: also decide CheckQuorum for the same 32 groups from `act`, this lane's dword of the tile's
// 7 active-flag planes (plane k = the active flag of voting slot k + 1; the leader's slot 0
// counts implicitly, raft.go:384), masked to the group's voting slots by the n planes of `p`.
template <bool FULL, bool CQ = false>
__device__ __forceinline__ void planes_slot(const BitsK &a, uint64_t g, const uint32_t *p,
                                            const uint32_t *act = nullptr) {
#ifdef HQ_PLANES_COPY   // tuning floor: the same loads and stores, no decision (wrong results)
    uint32_t x0 = 0, x1 = 0, x2 = 0;
    for (int q = 0; q < 8; ++q) {
        x0 ^= p[q];
        x1 += p[8 + q];
        x2 |= p[16 + q];
    }
    reinterpret_cast<uint32_t *>(a.confirmed)[g >> 5] = x0;
    *reinterpret_cast<uint2 *>(reinterpret_cast<uint32_t *>(a.outcome) + (g >> 4)) =
        make_uint2(x1, x2);
    return;
#endif
    const uint32_t n0 = p[7], n1 = p[15], n2 = p[23];     // n - 1
    uint32_t m[7];                                        // slot k + 1 votes: n - 1 > k
    m[0] = n0 | n1 | n2;
    m[1] = n1 | n2;
    m[2] = n2 | (n1 & n0);
    m[3] = n2;
    m[4] = n2 & (n1 | n0);
    m[5] = n2 & n1;
    m[6] = n2 & n1 & n0;
    const uint32_t c = n1 & n0;                           // n / 2 = (n - 1 + 1) >> 1
    const uint32_t h0 = n1 ^ n0, h1 = n2 ^ c, h2 = n2 & c;
    uint32_t x[7], y[7], z[7];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        x[k] = p[k] & m[k];
        y[k] = p[8 + k] & m[k];
        z[k] = p[16 + k] & m[k] & ~y[k];                  // first response wins
    }
    uint32_t a0, a1, a2, g0, g1, g2, r0, r1, r2;
    count7(x, a0, a1, a2);
    count7(y, g0, g1, g2);
    count7(z, r0, r1, r2);
    uint32_t inr = ~0u;
    if constexpr (!FULL) {
        const uint64_t left = a.G - g;                    // g < G
        inr = left >= 32 ? ~0u : (1u << left) - 1u;
    }
    // readindex.go:84: acks + 1 >= quorum <=> acks >= n/2; handleVoteResp: granted + 1 >=
    // quorum, rejected >= quorum <=> rejected > n/2
    const uint32_t conf = ge3(a0, a1, a2, h0, h1, h2) & inr;
    const uint32_t lead = ge3(g0, g1, g2, h0, h1, h2) & inr;
    const uint32_t foll = ~ge3(h0, h1, h2, r0, r1, r2) & inr & ~lead;
    const uint32_t cand = inr & ~lead & ~foll;
    reinterpret_cast<uint32_t *>(a.confirmed)[g >> 5] = conf;
    if constexpr (CQ) {
        // leaderHasQuorum (raft.go:380-390): 1 + active voting slots >= n/2 + 1, the same
        // threshold as the ReadIndex acks
        uint32_t v[7], c0, c1, c2;
#pragma unroll
        for (int k = 0; k < 7; ++k) v[k] = act[k] & m[k];
        count7(v, c0, c1, c2);
        reinterpret_cast<uint32_t *>(a.has_quorum)[g >> 5] = ge3(c0, c1, c2, h0, h1, h2) & inr;
    }
    const uint32_t w0 = shuffle16(__builtin_amdgcn_perm(lead, cand, 0x05010400u));
    const uint32_t w1 = shuffle16(__builtin_amdgcn_perm(lead, cand, 0x07030602u));
    *reinterpret_cast<uint2 *>(reinterpret_cast<uint32_t *>(a.outcome) + (g >> 4)) =
        make_uint2(w0, w1);
}

template <int BLK>
__global__ __launch_bounds__(BLK) void k_planes(const BitsK a) {
    const uint64_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (BLK / 64) +
                          __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * (BLK / 64);
    const uint64_t ntiles = (a.G + kPlaneTile - 1) / kPlaneTile;
    for (uint64_t t0 = wave * kPlTPW; t0 < ntiles; t0 += nw * kPlTPW) {
        uint32_t p[kPlTPW][24];
#pragma unroll
        for (int j = 0; j < kPlTPW; ++j) {
            const uint64_t t = t0 + j < ntiles ? t0 + j : t0;   // wave-uniform
            const uint32_t *base =
                reinterpret_cast<const uint32_t *>(a.tiles + t * (kPlaneTile * 3)) + lane;
#pragma unroll
            for (int q = 0; q < 24; ++q) {
#ifdef HQ_PLANES_PLAIN
                p[j][q] = base[q * 64];
#else
                p[j][q] = __builtin_nontemporal_load(base + q * 64);
#endif
            }
        }
#pragma unroll
        for (int j = 0; j < kPlTPW; ++j) {
            const uint64_t t = t0 + j;
            if (t >= ntiles) break;
            const uint64_t g = t * kPlaneTile + lane * 32;
            if (t * kPlaneTile + kPlaneTile <= a.G) planes_slot<true>(a, g, p[j]);
            else if (g < a.G) planes_slot<false>(a, g, p[j]);
            else if (g < ((a.G + 63) & ~63ull))           // the rest of the last bitmap word
                reinterpret_cast<uint32_t *>(a.confirmed)[g >> 5] = 0;
        }
    }
}

// ReadIndex + vote + CheckQuorum in one pass (hq_readindex_vote_cq_planes_dev): a step worker
// decides all three for the same leader groups (readindex.go:77-116, raft.go:1968-1985,
// raft.go:380-390), so one launch reads a tile's 24 vote / ack planes and its 7 active-flag
// planes (a separate 1792-byte tile per 2048 groups, the layout hq_tile_cq_planes_dev builds with
// n_uniform 8 and self slot 0), writes the confirmed, outcome and has-quorum words and zeroes
// the active planes it read (setNotActive of every voting member, remote.go:196-198): one
// launch boundary instead of two.
template <int BLK>
__global__ __launch_bounds__(BLK) void k_planes_cq(const BitsK a, uint8_t *active_planes) {
    const uint64_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (BLK / 64) +
                          __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * (BLK / 64);
    const uint64_t ntiles = (a.G + kPlaneTile - 1) / kPlaneTile;
    for (uint64_t t = wave; t < ntiles; t += nw) {
        const uint32_t *base = reinterpret_cast<const uint32_t *>(a.tiles + t * (kPlaneTile * 3)) + lane;
        uint32_t *abase = reinterpret_cast<uint32_t *>(active_planes + t * (7 * (kPlaneTile / 8))) + lane;
        uint32_t p[24], q[7];
#pragma unroll
        for (int k = 0; k < 24; ++k) p[k] = __builtin_nontemporal_load(base + k * 64);
#pragma unroll
        for (int k = 0; k < 7; ++k) q[k] = __builtin_nontemporal_load(abase + k * 64);
#if HQ_PLCQ_ZERO_EARLY
        // the zeroes go out right behind the loads of the same words (in order per wave)
#pragma unroll
        for (int k = 0; k < 7; ++k) __builtin_nontemporal_store(0u, abase + k * 64);
#endif
        const uint64_t g = t * kPlaneTile + lane * 32;
        if (t * kPlaneTile + kPlaneTile <= a.G) {
            planes_slot<true, true>(a, g, p, q);
        } else if (g < a.G) {
            planes_slot<false, true>(a, g, p, q);
        } else if (g < ((a.G + 63) & ~63ull)) {           // the rest of the last bitmap words
            reinterpret_cast<uint32_t *>(a.confirmed)[g >> 5] = 0;
            reinterpret_cast<uint32_t *>(a.has_quorum)[g >> 5] = 0;
        }
#if !HQ_PLCQ_ZERO_EARLY
#pragma unroll
        for (int k = 0; k < 7; ++k) __builtin_nontemporal_store(0u, abase + k * 64);
#endif
    }
}

// columns -> bit-plane tiles: one thread per group computes its 3 bytes (as k_tile_bits3), the
// wave's 64 groups become 24 ballots, lane q < 24 stores plane q's 8 bytes
__global__ __launch_bounds__(kBlock) void k_tile_planes(uint64_t G, const uint8_t *nv,
                                                        uint32_t nu, const uint8_t *ack,
                                                        const uint8_t *gr, const uint8_t *rj,
                                                        uint8_t *planes, uint64_t *fallback) {
    const uint64_t total = (G + kPlaneTile - 1) / kPlaneTile * kPlaneTile;
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t g0 = (uint64_t)blockIdx.x * kBlock; g0 < total;
         g0 += (uint64_t)gridDim.x * kBlock) {
        const uint64_t g = g0 + threadIdx.x;
        uint32_t bytes = 0;
        bool bad = false;
        if (g < G) {
            const uint32_t n = nv ? nv[g] : nu;
            const uint32_t av = ack[g], x = gr[g], r = rj[g];
            bad = n < 1 || n > 8 || (av & 1) || !(x & 1) || (r & 1);
            if (!bad) {
                const uint32_t keep = (1u << n) - 2u, m = n - 1;
                bytes = (((av & keep) >> 1) | ((m & 1) << 7)) |
                        ((((x & keep) >> 1) | (((m >> 1) & 1) << 7)) << 8) |
                        ((((r & keep) >> 1) | (((m >> 2) & 1) << 7)) << 16);
            }
        }
        uint64_t mine = 0;
#pragma unroll
        for (int q = 0; q < 24; ++q) {
            const uint64_t b = __ballot((bytes >> q) & 1);
            if (lane == (uint32_t)q) mine = b;
        }
        const uint64_t gw = g - lane;                     // the wave's first group
        if (gw < total && lane < 24)
            *reinterpret_cast<uint64_t *>(planes + (gw / kPlaneTile) * (kPlaneTile * 3) +
                                          lane * (kPlaneTile / 8) + (gw % kPlaneTile) / 8) = mine;
        const uint64_t b = __ballot(bad);
        if (fallback && lane == 0 && gw < ((G + 63) & ~63ull)) fallback[gw >> 6] = b;
    }
}

// ---- CheckQuorum over active-flag planes (hq_check_quorum_planes_dev) -----------------------
// The leader's own slot always counts (`nid == r.nodeID`, raft.go:384), so a group's CheckQuorum
// state is the active flags of its other voting slots plus its voter count. Plane k < 7 holds the
// active flag of the group's (k + 1)-th voting slot other than the leader, planes 7..9 the bits of
// n - 1 (per-group n); a uniform-n batch keeps only its n - 1 active planes. 2048-group tiles as
// the vote / ReadIndex planes, bit j of dword k of a plane = the tile's group 32 k + j. A lane
// decides 32 groups: 1 + popcount(the active planes masked to the group's slots) >= n/2 + 1,
// then zeroes the active planes it read (setNotActive of every voting member, raft.go:385,
// remote.go:196-198).
template <int P, bool PERN, int BLK>
__global__ __launch_bounds__(BLK) void k_cq_planes(uint64_t G, uint8_t *planes,
                                                   uint64_t *has_quorum) {
    constexpr int NP = PERN ? 10 : P;   // planes per tile
    constexpr int NA = PERN ? 7 : P;    // of which active planes
    const uint64_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (BLK / 64) +
                          __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * (BLK / 64);
    const uint64_t ntiles = (G + kPlaneTile - 1) / kPlaneTile;
    uint32_t *out = reinterpret_cast<uint32_t *>(has_quorum);
    for (uint64_t t = wave; t < ntiles; t += nw) {
        uint32_t *base = reinterpret_cast<uint32_t *>(planes + t * (uint64_t)NP * (kPlaneTile / 8)) + lane;
        uint32_t p[NP > 0 ? NP : 1];
#pragma unroll
        for (int q = 0; q < NP; ++q) p[q] = __builtin_nontemporal_load(base + q * 64);
        uint32_t x[7] = {0, 0, 0, 0, 0, 0, 0};
        uint32_t h0, h1, h2;                              // n / 2, bit-sliced
        if constexpr (PERN) {
            const uint32_t n0 = p[7], n1 = p[8], n2 = p[9];
            const uint32_t m[7] = {n0 | n1 | n2, n1 | n2, n2 | (n1 & n0), n2, n2 & (n1 | n0),
                                   n2 & n1, n2 & n1 & n0};   // slot k + 1 votes: n - 1 > k
#pragma unroll
            for (int k = 0; k < 7; ++k) x[k] = p[k] & m[k];
            const uint32_t c = n1 & n0;
            h0 = n1 ^ n0;
            h1 = n2 ^ c;
            h2 = n2 & c;
        } else {
#pragma unroll
            for (int k = 0; k < NP; ++k) x[k] = p[k];
            constexpr int h = (P + 1) / 2;
            h0 = (h & 1) ? ~0u : 0u;
            h1 = (h & 2) ? ~0u : 0u;
            h2 = (h & 4) ? ~0u : 0u;
        }
        uint32_t c0, c1, c2;
        count7(x, c0, c1, c2);
        const uint32_t hq = ge3(c0, c1, c2, h0, h1, h2);
        const uint64_t g = t * kPlaneTile + lane * 32;
        if (g < G) {
            const uint64_t left = G - g;
            out[g >> 5] = left >= 32 ? hq : hq & ((1u << left) - 1u);
        } else if (g < ((G + 63) & ~63ull)) {             // the rest of the last bitmap word
            out[g >> 5] = 0;
        }
#pragma unroll
        for (int q = 0; q < NA; ++q) __builtin_nontemporal_store(0u, base + q * 64);
    }
}

// columns -> CheckQuorum planes: one thread per group packs the active flags of its voting slots
// other than self_slot (in slot order) and n - 1, the wave's 64 groups become one ballot per
// plane, lane q < NP stores plane q's 8 bytes
__global__ __launch_bounds__(kBlock) void k_tile_cq_planes(uint64_t G, const uint8_t *active,
                                                           const uint8_t *nv, uint32_t nu,
                                                           uint32_t self_slot, uint8_t *planes,
                                                           uint64_t *fallback) {
    const uint64_t total = (G + kPlaneTile - 1) / kPlaneTile * kPlaneTile;
    const uint32_t NP = nv ? 10u : nu - 1u;
    const uint32_t lane = threadIdx.x & 63;
    for (uint64_t g0 = (uint64_t)blockIdx.x * kBlock; g0 < total;
         g0 += (uint64_t)gridDim.x * kBlock) {
        const uint64_t g = g0 + threadIdx.x;
        uint32_t bits = 0;
        bool bad = false;
        if (g < G) {
            const uint32_t n = nv ? nv[g] : nu;
            bad = n < 1 || n > 8 || self_slot >= n;
            if (!bad) {
                const uint32_t a = active[g] & ((1u << n) - 1u);
                bits = (a & ((1u << self_slot) - 1u)) | ((a >> (self_slot + 1)) << self_slot);
                if (nv) bits |= (n - 1) << 7;
            }
        }
        uint64_t mine = 0;
#pragma unroll
        for (uint32_t q = 0; q < 10; ++q) {
            const uint64_t b = __ballot((bits >> q) & 1);
            if (lane == q) mine = b;
        }
        const uint64_t gw = g - lane;
        if (gw < total && lane < NP)
            *reinterpret_cast<uint64_t *>(planes + (gw / kPlaneTile) * (NP * (kPlaneTile / 8)) +
                                          lane * (kPlaneTile / 8) + (gw % kPlaneTile) / 8) = mine;
        const uint64_t b = __ballot(bad);
        if (fallback && lane == 0 && gw < ((G + 63) & ~63ull)) fallback[gw >> 6] = b;
    }
}

// ---- synthetic inputs (recipe: DESIGN.md "Synthetic inputs"; CPU twin oracle/qgen.c) --------
__device__ __forceinline__ uint64_t splitmix64(uint64_t &s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ int synth_n(const hq_synth_spec &s, uint64_t cid) {
    const uint32_t r = (uint32_t)(cid % 3);
    return s.mixed_n ? (r == 0 ? 3 : r == 1 ? 5 : 7) : (int)s.n_max;
}

// lag-layout outputs of the generator (hq_synth_commit_lag_dev); all NULL for the u64 layout
struct LagOut {
    int32_t *lag;
    uint64_t stride;
    int32_t *cin, *ts;
    uint16_t *mask;
    uint64_t *last;
};

__device__ __forceinline__ int32_t lag_of(uint64_t last, uint64_t x) {  // clamp(last - x)
    if (x <= last) {
        const uint64_t d = last - x;
        return d >= (uint64_t)INT32_MAX ? INT32_MAX : (int32_t)d;
    }
    const uint64_t d = x - last;
    return d >= (uint64_t)INT32_MAX + 1 ? INT32_MIN : -(int32_t)d;
}

__global__ __launch_bounds__(kBlock) void k_synth_commit(const hq_synth_spec s, CommitCols o,
                                                         LagOut lo) {
    const uint64_t R = s.ring_len;
    for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < s.G;
         j += (uint64_t)gridDim.x * kBlock) {
        const uint64_t cid = s.cid_base + j * s.cid_stride;
        uint64_t st = s.seed ^ cid;
        const int n = synth_n(s, cid);
        const uint64_t term = 2 + splitmix64(st) % ((1ull << 20) - 2);
        const uint64_t last = (1ull << 20) + splitmix64(st) % (1ull << 40);
        uint64_t committed = last - splitmix64(st) % R;
        const uint64_t term_start = last - splitmix64(st) % R + 1;
        if (s.parity_extras) {
            const uint64_t x = splitmix64(st);
            if (x % 100 == 0) committed = last;
        }
        for (int k = 0; k < (int)s.n_max; ++k) {
            uint64_t m;
            if (k >= n) {
                m = 0;
            } else if (k == 0) {
                m = last;
            } else {
                const uint64_t x = splitmix64(st);
                const uint64_t y = splitmix64(st);
                m = committed - x % 4 + y % (last - committed + 4);
                if (m > last) m = last;
                if (s.parity_extras) {
                    const uint64_t c = splitmix64(st);
                    if (c % 100 == 0) m = last + 1 + (c / 100) % 3;
                }
            }
            if (o.match) const_cast<uint64_t *>(o.match)[(uint64_t)k * o.stride + j] = m;
            if (lo.lag) lo.lag[(uint64_t)k * lo.stride + j] = k < n ? lag_of(last, m) : 0;
        }
        if (lo.cin) lo.cin[j] = lag_of(last, committed);
        if (lo.ts) lo.ts[j] = lag_of(last, term_start);
        if (lo.last) lo.last[j] = last;
        if (o.nv) const_cast<uint8_t *>(o.nv)[j] = (uint8_t)n;
        if (o.cin) const_cast<uint64_t *>(o.cin)[j] = committed;
        if (o.last) const_cast<uint64_t *>(o.last)[j] = last;
        if (o.tstart) const_cast<uint64_t *>(o.tstart)[j] = term_start;
        if (o.term) const_cast<uint64_t *>(o.term)[j] = term;
        if (o.ring || o.mask || o.ring32 || lo.mask) {
            uint64_t cur = term;
            uint32_t mask = 0, lmask = 0;
            for (uint64_t k = 0; k < R; ++k) {
                const uint64_t i = last - k;
                uint64_t t;
                if (i >= term_start) {
                    t = term;
                } else {
                    const uint64_t x = splitmix64(st);
                    const uint64_t dec = (i + 1 == term_start) ? 1 + (x & 1) : (x & 1);
                    cur = cur > dec ? cur - dec : 1;
                    t = cur;
                }
                if (o.ring) const_cast<uint64_t *>(o.ring)[j * R + (i & (R - 1))] = t;
                if (o.ring32)
                    const_cast<uint32_t *>(o.ring32)[j * R + (i & (R - 1))] =
                        t < 0xFFFFFFFFull ? (uint32_t)t : 0xFFFFFFFFu;
                mask |= (uint32_t)(t == term) << (i & (R - 1));
                lmask |= (uint32_t)(t == term) << k;   // indexed by lag k = last - i
            }
            if (o.mask) const_cast<uint16_t *>(o.mask)[j] = (uint16_t)mask;
            if (lo.mask) lo.mask[j] = (uint16_t)lmask;
        }
    }
}

struct Bern {
    uint64_t st, buf;
    int avail;
    __device__ __forceinline__ bool operator()(uint32_t thr16) {
        if (avail == 0) {
            buf = splitmix64(st);
            avail = 4;
        }
        const uint32_t v = (uint32_t)(buf & 0xFFFF);
        buf >>= 16;
        --avail;
        return v < thr16;
    }
};

__global__ __launch_bounds__(kBlock) void k_synth_bits(const hq_synth_spec s, uint8_t *ack,
                                                       uint8_t *granted, uint8_t *rejected,
                                                       uint8_t *nv) {
    constexpr uint32_t P60 = 39322u, P30 = 19661u;
    for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < s.G;
         j += (uint64_t)gridDim.x * kBlock) {
        const uint64_t cid = s.cid_base + j * s.cid_stride;
        Bern b{s.seed ^ cid, 0, 0};
        const int n = synth_n(s, cid);
        uint32_t a = 0, g = 1, r = 0;
        for (int k = 1; k < n; ++k)
            if (b(P60)) a |= 1u << k;
        for (int k = 1; k < n; ++k)
            if (b(P60)) g |= 1u << k;
        for (int k = 1; k < n; ++k)
            if (!((g >> k) & 1) && b(P30)) r |= 1u << k;
        if (s.parity_extras) {
            const uint64_t x = splitmix64(b.st);
            if (x % 50 == 0) r |= g & ~1u;
            if (x % 50 == 1) a |= 1u;
            if (x % 50 == 2) a |= 0xFFu & ~((1u << n) - 1);
        }
        if (ack) ack[j] = (uint8_t)a;
        if (granted) granted[j] = (uint8_t)g;
        if (rejected) rejected[j] = (uint8_t)r;
        if (nv) nv[j] = (uint8_t)n;
    }
}

unsigned grid_for(uint64_t lanes_needed, int block = kBlock, uint64_t max_blocks = kMaxBlocks) {
    uint64_t b = (lanes_needed + block - 1) / block;
    if (b < 1) b = 1;
    if (b > max_blocks) b = max_blocks;
    return (unsigned)b;
}

template <int N, int FORM, int VEC, bool PERN, int TILED = 0>
int launch_commit_t(hq_ctx *ctx, const CommitK &k) {
    constexpr int B = commit_blk<N, FORM, PERN>();
    const unsigned grid = grid_for((k.G + VEC - 1) / VEC, B, kMaxBlocks * 256 / B);
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    if constexpr (B == kCommitBlock)
        hipLaunchKernelGGL((k_commit<N, FORM, VEC, PERN, TILED>), dim3(grid), dim3(B), 0,
                           ctx->stream, k);
    else
        hipLaunchKernelGGL((k_commit_big<N, FORM, VEC, PERN, TILED>), dim3(grid), dim3(B), 0,
                           ctx->stream, k);
    return hq::post_launch(ctx, "k_commit");
}

// tiles are always read two groups per lane (the validation requires a 16-byte aligned base);
// tiled: 0 columns, 1 HQ_LAYOUT_TILES, 2 HQ_LAYOUT_TILES_LEADER
template <int N>
int launch_commit_n(hq_ctx *ctx, const CommitK &k, int form, bool vec2, bool pern, int tiled) {
#define HQ_DISPATCH(F)                                                                   \
    if (tiled == 3) return pern ? launch_commit_t<N, F, 2, true, 3>(ctx, k)              \
                                : launch_commit_t<N, F, 2, false, 3>(ctx, k);            \
    if (tiled == 2) return pern ? launch_commit_t<N, F, 2, true, 2>(ctx, k)              \
                                : launch_commit_t<N, F, 2, false, 2>(ctx, k);            \
    if (tiled) return pern ? launch_commit_t<N, F, 2, true, 1>(ctx, k)                   \
                           : launch_commit_t<N, F, 2, false, 1>(ctx, k);                 \
    if (vec2) return pern ? launch_commit_t<N, F, 2, true>(ctx, k)                       \
                          : launch_commit_t<N, F, 2, false>(ctx, k);                     \
    return pern ? launch_commit_t<N, F, 1, true>(ctx, k) : launch_commit_t<N, F, 1, false>(ctx, k);
    if (form == HQ_FORM_TERM_START) {
        HQ_DISPATCH(HQ_FORM_TERM_START)
    } else if (form == HQ_FORM_TERM_MASK) {
        HQ_DISPATCH(HQ_FORM_TERM_MASK)
    } else if (form == HQ_FORM_TERM_RING32) {
        HQ_DISPATCH(HQ_FORM_TERM_RING32)
    } else {
        HQ_DISPATCH(HQ_FORM_TERM_RING)
    }
#undef HQ_DISPATCH
}

int validate_commit(hq_ctx *ctx, const hq_commit_args *a) {
    if (!ctx) return HQ_E_INVAL;
    if (!a) return hq::fail(ctx, HQ_E_INVAL, "hq_commit: args is NULL");
    if (a->n_max < 1 || a->n_max > HQ_MAX_VOTERS)
        return hq::fail(ctx, HQ_E_INVAL, "hq_commit: n_max must be 1..8");
    const bool in_place = a->layout == (HQ_LAYOUT_TILES_LEADER | HQ_LAYOUT_IN_PLACE);
    if (a->layout != HQ_LAYOUT_COLUMNS && a->layout != HQ_LAYOUT_TILES &&
        a->layout != HQ_LAYOUT_TILES_LEADER && !in_place)
        return hq::fail(ctx, HQ_E_INVAL, "hq_commit: unknown layout");
    if (in_place && a->form != HQ_FORM_TERM_START && a->form != HQ_FORM_TERM_MASK)
        return hq::fail(ctx, HQ_E_INVAL,
                        "hq_commit: an in-place table holds the term-start or term-mask form");
    if (a->G == 0) return HQ_OK;
    const bool tiles = a->layout != HQ_LAYOUT_COLUMNS;
    if (tiles) {
        if (!a->match || (!a->committed_out && !in_place))
            return hq::fail(ctx, HQ_E_INVAL, "hq_commit: NULL tiles (match) / committed_out");
        if (!hq::aligned16(a->match) || (!in_place && !hq::aligned16(a->committed_out)) ||
            (a->n_voting && (reinterpret_cast<uintptr_t>(a->n_voting) & 1)))
            return hq::fail(ctx, HQ_E_INVAL,
                            "hq_commit: tiles and committed_out must be 16-byte aligned, "
                            "n_voting 2-byte aligned");
    } else {
        if (!a->match || !a->committed_in || !a->committed_out || !a->last_index)
            return hq::fail(ctx, HQ_E_INVAL, "hq_commit: NULL match/committed/last_index");
        if (a->match_stride < a->G)
            return hq::fail(ctx, HQ_E_INVAL, "hq_commit: match_stride < G");
    }
    if (a->form == HQ_FORM_TERM_START) {
        if (!tiles && !a->term_start)
            return hq::fail(ctx, HQ_E_INVAL, "hq_commit: term_start is NULL");
    } else if (a->form == HQ_FORM_TERM_RING || a->form == HQ_FORM_TERM_RING32) {
        if ((!tiles && !a->term) || (a->form == HQ_FORM_TERM_RING ? !a->ring : !a->ring32))
            return hq::fail(ctx, HQ_E_INVAL, "hq_commit: term/ring NULL");
        if (a->ring_len < 1 || a->ring_len > 1024 || (a->ring_len & (a->ring_len - 1)))
            return hq::fail(ctx, HQ_E_INVAL, "hq_commit: ring_len must be a power of two <= 1024");
    } else if (a->form == HQ_FORM_TERM_MASK) {
        if (!tiles && !a->term_mask)
            return hq::fail(ctx, HQ_E_INVAL, "hq_commit: term_mask is NULL");
        if (a->ring_len < 1 || a->ring_len > 16 || (a->ring_len & (a->ring_len - 1)))
            return hq::fail(ctx, HQ_E_INVAL, "hq_commit: mask form needs ring_len <= 16 (power of two)");
    } else {
        return hq::fail(ctx, HQ_E_INVAL, "hq_commit: unknown form");
    }
    return HQ_OK;
}

}  // namespace

namespace {

CommitK commit_k(const hq_commit_args *a) {
    CommitK k{};
    const bool tiles = a->layout != HQ_LAYOUT_COLUMNS;
    k.G = a->G;
    k.stride = tiles ? hq_commit_tile_words_for(a->n_max, a->form, a->layout) : a->match_stride;
    k.R = a->ring_len;
    k.match = a->match;
    k.nv = a->n_voting;
    k.cin = a->committed_in;
    k.cout = a->committed_out;
    k.last = a->last_index;
    k.aux = a->form == HQ_FORM_TERM_START ? static_cast<const void *>(a->term_start)
          : a->form == HQ_FORM_TERM_MASK  ? static_cast<const void *>(a->term_mask)
                                          : static_cast<const void *>(a->term);
    k.ring = a->form == HQ_FORM_TERM_RING32 ? static_cast<const void *>(a->ring32)
                                            : static_cast<const void *>(a->ring);
    k.changed = a->changed;
    k.fallback = a->fallback;
    return k;
}

// every field of a column batch (generator, tile packer)
CommitCols commit_cols(const hq_commit_args *a) {
    CommitCols k{};
    k.G = a->G;
    k.stride = a->match_stride;
    k.nwords = hq::words64(a->G);
    k.n_max = a->n_max;
    k.R = a->ring_len;
    k.match = a->match;
    k.nv = a->n_voting;
    k.cin = a->committed_in;
    k.cout = a->committed_out;
    k.last = a->last_index;
    k.tstart = a->term_start;
    k.term = a->term;
    k.ring = a->ring;
    k.changed = a->changed;
    k.fallback = a->fallback;
    k.mask = a->term_mask;
    k.ring32 = a->ring32;
    k.tile_words = hq_commit_tile_words(a->n_max, a->form);
    return k;
}

// every column of the batch can be read two groups per lane with 16-byte loads
bool commit_vec2(const hq_commit_args *a) {
    if (a->layout != HQ_LAYOUT_COLUMNS) return true;   // alignment checked by validate_commit
    const bool aux_ok = a->form == HQ_FORM_TERM_START ? hq::aligned16(a->term_start)
                      : a->form == HQ_FORM_TERM_MASK
                          ? (reinterpret_cast<uintptr_t>(a->term_mask) & 3) == 0
                          : hq::aligned16(a->term);
    return hq::aligned16(a->match) && (a->match_stride % 2 == 0) &&
           hq::aligned16(a->committed_in) && hq::aligned16(a->committed_out) &&
           hq::aligned16(a->last_index) && aux_ok &&
           (!a->n_voting || (reinterpret_cast<uintptr_t>(a->n_voting) & 1) == 0);
}

}  // namespace

extern "C" int hq_commit_dev(hq_ctx *ctx, const hq_commit_args *a) {
    int rc = validate_commit(ctx, a);
    if (rc || a->G == 0) return rc;
    const CommitK k = commit_k(a);
    const bool vec2 = commit_vec2(a);
    const bool pern = a->n_voting != nullptr;
    const int tiled = a->layout == (HQ_LAYOUT_TILES_LEADER | HQ_LAYOUT_IN_PLACE) ? 3
                    : a->layout == HQ_LAYOUT_TILES_LEADER                       ? 2
                    : a->layout == HQ_LAYOUT_TILES                              ? 1
                                                                                : 0;
    switch (a->n_max) {
    case 1: return launch_commit_n<1>(ctx, k, a->form, vec2, pern, tiled);
    case 2: return launch_commit_n<2>(ctx, k, a->form, vec2, pern, tiled);
    case 3: return launch_commit_n<3>(ctx, k, a->form, vec2, pern, tiled);
    case 4: return launch_commit_n<4>(ctx, k, a->form, vec2, pern, tiled);
    case 5: return launch_commit_n<5>(ctx, k, a->form, vec2, pern, tiled);
    case 6: return launch_commit_n<6>(ctx, k, a->form, vec2, pern, tiled);
    case 7: return launch_commit_n<7>(ctx, k, a->form, vec2, pern, tiled);
    default: return launch_commit_n<8>(ctx, k, a->form, vec2, pern, tiled);
    }
}

#ifndef HQ_LAG_HEAVY_FIRST
#define HQ_LAG_HEAVY_FIRST 1
#endif
#ifndef HQ_FUSED_HEAVY_FIRST
#define HQ_FUSED_HEAVY_FIRST 1
#endif
#ifndef HQ_FUSED_BIG_NMAX
#define HQ_FUSED_BIG_NMAX 5
#endif
extern "C" int hq_commit_fused_dev(hq_ctx *ctx, const hq_commit_args *args, uint32_t count) {
    if (!ctx) return HQ_E_INVAL;
    if (count && !args) return hq::fail(ctx, HQ_E_INVAL, "hq_commit_fused_dev: args is NULL");
    for (uint32_t i = 0; i < count; ++i) {
        int rc = validate_commit(ctx, args + i);
        if (rc) return rc;
    }
    // batches that can share the launch: uniform n, 16-byte aligned columns, one form
    bool fusable = count >= 2 && count <= (uint32_t)kMaxFusedCommit;
    for (uint32_t i = 0; fusable && i < count; ++i)
        fusable = args[i].G > 0 && !args[i].n_voting && commit_vec2(args + i) &&
                  args[i].form == args[0].form && args[i].layout == args[0].layout &&
                  !(args[i].layout & HQ_LAYOUT_IN_PLACE);
    if (!fusable) return hq_commit_many_dev(ctx, args, count);
    FusedK f{};
    f.count = count;
    // one block size for the launch: the big one only if every batch's kernel body fits it
    bool big = true;
    // (the fused kernel's bodies fit 64 VGPRs without spilling for these two forms only)
    for (uint32_t i = 0; i < count; ++i)
        big &= args[i].n_max <= HQ_FUSED_BIG_NMAX &&
               (args[i].form == HQ_FORM_TERM_START || args[i].form == HQ_FORM_TERM_MASK);
    const int B = big ? HQ_COMMIT_BLOCK_BIG : kCommitBlock;
    uint64_t blocks = 0;
    // workgroup ranges in launch order, the widest batches first (their waves are dispatched
    // first, so the tail is made of the light ones: c5t 96-97 -> 93-94 us,
    // profiles/r01f/ab_heavy_first.log; HQ_FUSED_HEAVY_FIRST=0 keeps the argument order)
    uint32_t order[kMaxFusedCommit];
    for (uint32_t i = 0; i < count; ++i) order[i] = i;
#if HQ_FUSED_HEAVY_FIRST
    for (uint32_t i = 1; i < count; ++i)
        for (uint32_t j = i; j > 0 && args[order[j]].n_max > args[order[j - 1]].n_max; --j) {
            const uint32_t t = order[j];
            order[j] = order[j - 1];
            order[j - 1] = t;
        }
#endif
    for (uint32_t k = 0; k < count; ++k) {
        const uint32_t i = k;
        f.b[i] = commit_k(args + order[k]);
        f.n[i] = args[order[k]].n_max;
        f.first[i] = (uint32_t)blocks;
        // the same lanes per batch as its own launch would get (grid-stride beyond that)
        blocks += grid_for((args[order[k]].G + 1) / 2, B, (uint64_t)kMaxBlocks * 256 / B);
    }
    for (uint32_t i = count; i <= (uint32_t)kMaxFusedCommit; ++i) f.first[i] = (uint32_t)blocks;
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
#define HQ_FUSED(F, BLK)                                                                       \
    if (args[0].layout == HQ_LAYOUT_TILES_LEADER)                                              \
        hipLaunchKernelGGL((k_commit_fused<F, BLK, 2>), dim3(blocks), dim3(BLK), 0,            \
                           ctx->stream, f);                                                    \
    else if (args[0].layout == HQ_LAYOUT_TILES)                                                \
        hipLaunchKernelGGL((k_commit_fused<F, BLK, 1>), dim3(blocks), dim3(BLK), 0,            \
                           ctx->stream, f);                                                    \
    else                                                                                       \
        hipLaunchKernelGGL((k_commit_fused<F, BLK, 0>), dim3(blocks), dim3(BLK), 0,            \
                           ctx->stream, f);
    switch (args[0].form) {
    case HQ_FORM_TERM_START:
        if (big) {
            HQ_FUSED(HQ_FORM_TERM_START, HQ_COMMIT_BLOCK_BIG)
        } else {
            HQ_FUSED(HQ_FORM_TERM_START, kCommitBlock)
        }
        break;
    case HQ_FORM_TERM_MASK:
        if (big) {
            HQ_FUSED(HQ_FORM_TERM_MASK, HQ_COMMIT_BLOCK_BIG)
        } else {
            HQ_FUSED(HQ_FORM_TERM_MASK, kCommitBlock)
        }
        break;
    case HQ_FORM_TERM_RING32: HQ_FUSED(HQ_FORM_TERM_RING32, kCommitBlock) break;
    default: HQ_FUSED(HQ_FORM_TERM_RING, kCommitBlock) break;
    }
#undef HQ_FUSED
    return hq::post_launch(ctx, "k_commit_fused");
}

namespace {

template <int N, int FORM, int VEC, bool PERN, int LEAD>
int launch_lag_t(hq_ctx *ctx, const LagK &k) {
    constexpr int B = lag_blk<N, PERN>();
    const unsigned grid = grid_for((k.G + VEC - 1) / VEC, B, kMaxBlocks * 256 / B);
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    if constexpr (B == kCommitBlock)
        hipLaunchKernelGGL((k_commit_lag<N, FORM, VEC, PERN, LEAD>), dim3(grid), dim3(B), 0,
                           ctx->stream, k);
    else
        hipLaunchKernelGGL((k_commit_lag_big<N, FORM, VEC, PERN, LEAD>), dim3(grid), dim3(B), 0,
                           ctx->stream, k);
    return hq::post_launch(ctx, "k_commit_lag");
}

template <int N, int LEAD>
int launch_lag_nl(hq_ctx *ctx, const LagK &k, int form, bool vec, bool pern) {
#define HQ_LAG_DISPATCH(F)                                                                   \
    if (vec) return pern ? launch_lag_t<N, F, kLagVec, true, LEAD>(ctx, k)                    \
                         : launch_lag_t<N, F, kLagVec, false, LEAD>(ctx, k);                  \
    return pern ? launch_lag_t<N, F, 1, true, LEAD>(ctx, k)                                   \
                : launch_lag_t<N, F, 1, false, LEAD>(ctx, k);
    if (form == HQ_FORM_TERM_START) {
        HQ_LAG_DISPATCH(HQ_FORM_TERM_START)
    } else {
        HQ_LAG_DISPATCH(HQ_FORM_TERM_MASK)
    }
#undef HQ_LAG_DISPATCH
}
template <int N>
int launch_lag_n(hq_ctx *ctx, const LagK &k, int form, bool vec, bool pern, bool lead) {
    return lead ? launch_lag_nl<N, 1>(ctx, k, form, vec, pern)
                : launch_lag_nl<N, 0>(ctx, k, form, vec, pern);
}

int validate_lag(hq_ctx *ctx, const hq_commit_lag_args *a) {
    if (!ctx) return HQ_E_INVAL;
    if (!a) return hq::fail(ctx, HQ_E_INVAL, "hq_commit_lag: args is NULL");
    if (a->n_max < 1 || a->n_max > HQ_MAX_VOTERS)
        return hq::fail(ctx, HQ_E_INVAL, "hq_commit_lag: n_max must be 1..8");
    if (a->G == 0) return HQ_OK;
    if (!a->lag || !a->cin_lag || !a->cout_lag)
        return hq::fail(ctx, HQ_E_INVAL, "hq_commit_lag: NULL lag/cin_lag/cout_lag");
    if (a->lag_stride < a->G) return hq::fail(ctx, HQ_E_INVAL, "hq_commit_lag: lag_stride < G");
    if (a->flags & ~(uint32_t)HQ_LAG_LEADER_IMPLICIT)
        return hq::fail(ctx, HQ_E_INVAL, "hq_commit_lag: unknown flags");
    if (a->form == HQ_FORM_TERM_START) {
        if (!a->ts_lag) return hq::fail(ctx, HQ_E_INVAL, "hq_commit_lag: ts_lag is NULL");
    } else if (a->form == HQ_FORM_TERM_MASK) {
        if (!a->lag_mask) return hq::fail(ctx, HQ_E_INVAL, "hq_commit_lag: lag_mask is NULL");
        if (a->ring_len < 1 || a->ring_len > 16 || (a->ring_len & (a->ring_len - 1)))
            return hq::fail(ctx, HQ_E_INVAL, "hq_commit_lag: mask form needs ring_len <= 16 (power of two)");
    } else {
        return hq::fail(ctx, HQ_E_INVAL, "hq_commit_lag: form must be TERM_START or TERM_MASK");
    }
    return HQ_OK;
}

LagK lag_k(const hq_commit_lag_args *a) {
    LagK k;
    k.G = a->G;
    k.stride = a->lag_stride;
    k.nwords = hq::words64(a->G);
    k.n_max = a->n_max;
    k.R = a->ring_len;
    k.lag = a->lag;
    k.nv = a->n_voting;
    k.cin = a->cin_lag;
    k.cout = a->cout_lag;
    k.ts = a->ts_lag;
    k.mask = a->lag_mask;
    k.changed = a->changed;
    k.fallback = a->fallback;
    return k;
}

// every column can be read kLagVec groups per lane with aligned vector loads
bool lag_vec(const hq_commit_lag_args *a) {
    const uintptr_t al = 4 * kLagVec;   // bytes of one lane's int32 load
    auto ok = [&](const void *p, uintptr_t b) { return (reinterpret_cast<uintptr_t>(p) % b) == 0; };
    const bool aux_ok = a->form == HQ_FORM_TERM_START ? ok(a->ts_lag, al) : ok(a->lag_mask, al / 2);
    return ok(a->lag, al) && (a->lag_stride % kLagVec == 0) && ok(a->cin_lag, al) &&
           ok(a->cout_lag, al) && aux_ok && (!a->n_voting || ok(a->n_voting, al / 4));
}

}  // namespace

extern "C" int hq_commit_lag_dev(hq_ctx *ctx, const hq_commit_lag_args *a) {
    int rc = validate_lag(ctx, a);
    if (rc || a->G == 0) return rc;
    const LagK k = lag_k(a);
    const bool vec4 = lag_vec(a);
    const bool pern = a->n_voting != nullptr;
    const bool lead = (a->flags & HQ_LAG_LEADER_IMPLICIT) != 0;
    switch (a->n_max) {
    case 1: return launch_lag_n<1>(ctx, k, a->form, vec4, pern, lead);
    case 2: return launch_lag_n<2>(ctx, k, a->form, vec4, pern, lead);
    case 3: return launch_lag_n<3>(ctx, k, a->form, vec4, pern, lead);
    case 4: return launch_lag_n<4>(ctx, k, a->form, vec4, pern, lead);
    case 5: return launch_lag_n<5>(ctx, k, a->form, vec4, pern, lead);
    case 6: return launch_lag_n<6>(ctx, k, a->form, vec4, pern, lead);
    case 7: return launch_lag_n<7>(ctx, k, a->form, vec4, pern, lead);
    default: return launch_lag_n<8>(ctx, k, a->form, vec4, pern, lead);
    }
}

extern "C" int hq_commit_lag_fused_dev(hq_ctx *ctx, const hq_commit_lag_args *args,
                                       uint32_t count) {
    if (!ctx) return HQ_E_INVAL;
    if (count && !args) return hq::fail(ctx, HQ_E_INVAL, "hq_commit_lag_fused_dev: args is NULL");
    for (uint32_t i = 0; i < count; ++i) {
        int rc = validate_lag(ctx, args + i);
        if (rc) return rc;
    }
    bool fusable = count >= 2 && count <= (uint32_t)kMaxFusedCommit;
    for (uint32_t i = 0; fusable && i < count; ++i)
        fusable = args[i].G > 0 && !args[i].n_voting && lag_vec(args + i) &&
                  args[i].form == args[0].form && args[i].flags == args[0].flags;
    if (!fusable) {
        for (uint32_t i = 0; i < count; ++i) {
            int rc = hq_commit_lag_dev(ctx, args + i);
            if (rc) return rc;
        }
        return HQ_OK;
    }
    FusedLagK f{};
    f.count = count;
    bool big = true;
    for (uint32_t i = 0; i < count; ++i) big &= args[i].n_max <= 4;
    const int B = big ? HQ_COMMIT_BLOCK_BIG : kCommitBlock;
    uint64_t blocks = 0;
    uint32_t order[kMaxFused];
    for (uint32_t i = 0; i < count; ++i) order[i] = i;
#if HQ_LAG_HEAVY_FIRST
    for (uint32_t i = 1; i < count; ++i)   // the widest batches first, as in hq_commit_fused_dev
        for (uint32_t j = i; j > 0 && args[order[j]].n_max > args[order[j - 1]].n_max; --j) {
            const uint32_t t = order[j];
            order[j] = order[j - 1];
            order[j - 1] = t;
        }
#endif
    for (uint32_t i = 0; i < count; ++i) {
        const hq_commit_lag_args *b = args + order[i];
        f.b[i] = lag_k(b);
        f.n[i] = b->n_max;
        f.first[i] = (uint32_t)blocks;
        blocks += grid_for((b->G + kLagVec - 1) / kLagVec, B, (uint64_t)kMaxBlocks * 256 / B);
    }
    for (uint32_t i = count; i <= (uint32_t)kMaxFused; ++i) f.first[i] = (uint32_t)blocks;
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
#define HQ_LAG_FUSED(F, L)                                                                     \
    if (big)                                                                                   \
        hipLaunchKernelGGL((k_commit_lag_fused<F, HQ_COMMIT_BLOCK_BIG, L>), dim3(blocks),      \
                           dim3(HQ_COMMIT_BLOCK_BIG), 0, ctx->stream, f);                      \
    else                                                                                       \
        hipLaunchKernelGGL((k_commit_lag_fused<F, kCommitBlock, L>), dim3(blocks),             \
                           dim3(kCommitBlock), 0, ctx->stream, f);
    const bool lead = (args[0].flags & HQ_LAG_LEADER_IMPLICIT) != 0;
    if (args[0].form == HQ_FORM_TERM_START) {
        if (lead) {
            HQ_LAG_FUSED(HQ_FORM_TERM_START, 1)
        } else {
            HQ_LAG_FUSED(HQ_FORM_TERM_START, 0)
        }
    } else {
        if (lead) {
            HQ_LAG_FUSED(HQ_FORM_TERM_MASK, 1)
        } else {
            HQ_LAG_FUSED(HQ_FORM_TERM_MASK, 0)
        }
    }
#undef HQ_LAG_FUSED
    return hq::post_launch(ctx, "k_commit_lag_fused");
}

extern "C" int hq_commit_many_dev(hq_ctx *ctx, const hq_commit_args *args, uint32_t count) {
    if (!ctx) return HQ_E_INVAL;
    if (count && !args) return hq::fail(ctx, HQ_E_INVAL, "hq_commit_many_dev: args is NULL");
    for (uint32_t i = 0; i < count; ++i) {
        int rc = hq_commit_dev(ctx, args + i);
        if (rc) return rc;
    }
    return HQ_OK;
}

namespace {

template <int MODE>
int launch_bits(hq_ctx *ctx, BitsK &k, const char *what) {
    if (!ctx) return HQ_E_INVAL;
    if (k.G == 0) return HQ_OK;
    if (!k.nv && !(k.tiles && k.tile_rows == 4) && (k.n_uniform < 1 || k.n_uniform > 8))
        return hq::fail(ctx, HQ_E_INVAL, std::string(what) + ": n_uniform must be 1..8");
    if (k.tiles && (k.nv || !hq::aligned16(k.tiles) || (k.tile_rows != 3 && k.tile_rows != 4)))
        return hq::fail(ctx, HQ_E_INVAL, std::string(what) + ": bad tiles");
    const uint8_t *ins[5] = {k.nv, k.ack, k.granted, k.rejected, k.active};
    for (const uint8_t *p : ins)
        if (p && !hq::aligned16(p))
            return hq::fail(ctx, HQ_E_INVAL, std::string(what) + ": byte arrays must be 16-byte aligned");
    k.n16 = hq::words64(k.G) * 4;
    k.n16o = (MODE & kVOTE) ? hq::words32(k.G) * 2 : 0;
    const uint64_t slots = k.n16 > k.n16o ? k.n16 : k.n16o;
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    // block size: ctx->bits_block (256 default; HQ_BITS_BLOCK at hq_open, a tuning knob)
#define HQ_BITS_LAUNCH(B)                                                                      \
    {                                                                                          \
        const unsigned grid = grid_for(slots, B, (uint64_t)kMaxBlocks * 256 / B);              \
        if constexpr (MODE == (kRI | kVOTE)) {                                                 \
            if (k.tiles && k.tile_rows == 4 && k.fallback)                                     \
                hipLaunchKernelGGL((k_bits<MODE, true, B, true>), dim3(grid), dim3(B), 0,      \
                                   ctx->stream, k);                                            \
            else if (k.tiles && k.tile_rows == 4)                                              \
                hipLaunchKernelGGL((k_bits<MODE, true, B, true, false>), dim3(grid), dim3(B),  \
                                   0, ctx->stream, k);                                         \
            else if (k.tiles && k.fallback)                                                    \
                hipLaunchKernelGGL((k_bits<MODE, false, B, true>), dim3(grid), dim3(B), 0,     \
                                   ctx->stream, k);                                            \
            else if (k.tiles)                                                                  \
                hipLaunchKernelGGL((k_bits<MODE, false, B, true, false>), dim3(grid), dim3(B), \
                                   0, ctx->stream, k);                                         \
        }                                                                                      \
        if (k.tiles) {                                                                         \
        } else if (k.nv)                                                                       \
            hipLaunchKernelGGL((k_bits<MODE, true, B>), dim3(grid), dim3(B), 0, ctx->stream, k); \
        else                                                                                   \
            hipLaunchKernelGGL((k_bits<MODE, false, B>), dim3(grid), dim3(B), 0, ctx->stream, k); \
    }
    if (ctx->bits_block == 512) HQ_BITS_LAUNCH(512)
    else if (ctx->bits_block == 1024) HQ_BITS_LAUNCH(1024)
    else HQ_BITS_LAUNCH(256)
#undef HQ_BITS_LAUNCH
    return hq::post_launch(ctx, what);
}

BitsK bits_args(uint64_t G, const uint8_t *nv, uint32_t nu, uint64_t *fallback) {
    BitsK k{};
    k.G = G;
    k.nv = nv;
    k.n_uniform = nu;
    k.fallback = fallback;
    return k;
}

}  // namespace

extern "C" int hq_readindex_dev(hq_ctx *ctx, uint64_t G, const uint8_t *ack,
                                const uint8_t *n_voting, uint32_t n_uniform, uint64_t *confirmed,
                                uint64_t *fallback) {
    if (ctx && G && (!ack || !confirmed))
        return hq::fail(ctx, HQ_E_INVAL, "hq_readindex: NULL ack/confirmed");
    BitsK k = bits_args(G, n_voting, n_uniform, fallback);
    k.ack = ack;
    k.confirmed = confirmed;
    return launch_bits<kRI>(ctx, k, "hq_readindex");
}

extern "C" int hq_vote_dev(hq_ctx *ctx, uint64_t G, const uint8_t *granted,
                           const uint8_t *rejected, const uint8_t *n_voting, uint32_t n_uniform,
                           uint64_t *outcome, uint64_t *fallback) {
    if (ctx && G && (!granted || !rejected || !outcome))
        return hq::fail(ctx, HQ_E_INVAL, "hq_vote: NULL granted/rejected/outcome");
    BitsK k = bits_args(G, n_voting, n_uniform, fallback);
    k.granted = granted;
    k.rejected = rejected;
    k.outcome = outcome;
    return launch_bits<kVOTE>(ctx, k, "hq_vote");
}

extern "C" int hq_readindex_vote_dev(hq_ctx *ctx, uint64_t G, const uint8_t *ack,
                                     const uint8_t *granted, const uint8_t *rejected,
                                     const uint8_t *n_voting, uint32_t n_uniform,
                                     uint64_t *confirmed, uint64_t *outcome, uint64_t *fallback) {
    if (ctx && G && (!ack || !granted || !rejected || !confirmed || !outcome))
        return hq::fail(ctx, HQ_E_INVAL, "hq_readindex_vote: NULL argument");
    BitsK k = bits_args(G, n_voting, n_uniform, fallback);
    k.ack = ack;
    k.granted = granted;
    k.rejected = rejected;
    k.confirmed = confirmed;
    k.outcome = outcome;
    return launch_bits<kRI | kVOTE>(ctx, k, "hq_readindex_vote");
}

extern "C" int hq_readindex_vote_tiles_dev(hq_ctx *ctx, uint64_t G, const uint8_t *tiles,
                                           uint32_t per_group_n, uint32_t n_uniform,
                                           uint64_t *confirmed, uint64_t *outcome,
                                           uint64_t *fallback) {
    if (ctx && G && (!tiles || !confirmed || !outcome))
        return hq::fail(ctx, HQ_E_INVAL, "hq_readindex_vote_tiles: NULL argument");
    BitsK k = bits_args(G, nullptr, n_uniform, fallback);
    k.tiles = tiles;
    k.tile_rows = per_group_n ? 4 : 3;
    k.confirmed = confirmed;
    k.outcome = outcome;
    return launch_bits<kRI | kVOTE>(ctx, k, "hq_readindex_vote_tiles");
}

extern "C" int hq_readindex_vote_tiles3_dev(hq_ctx *ctx, uint64_t G, const uint8_t *tiles,
                                            uint64_t *confirmed, uint64_t *outcome) {
    if (!ctx) return HQ_E_INVAL;
    if (G == 0) return HQ_OK;
    if (!tiles || !confirmed || !outcome || !hq::aligned16(tiles))
        return hq::fail(ctx, HQ_E_INVAL,
                        "hq_readindex_vote_tiles3: NULL argument or tiles not 16-byte aligned");
    BitsK k = bits_args(G, nullptr, 0, nullptr);
    k.tiles = tiles;
    k.tile_rows = 3;
    k.confirmed = confirmed;
    k.outcome = outcome;
    k.n16 = hq::words64(G) * 4;
    k.n16o = hq::words32(G) * 2;
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    const uint64_t ntiles = (G + 1023) / 1024;
    hipLaunchKernelGGL(k_bits3<256>, dim3(grid_for((ntiles + kB3TPW - 1) / kB3TPW * 64, 256)),
                       dim3(256), 0, ctx->stream, k);
    return hq::post_launch(ctx, "hq_readindex_vote_tiles3");
}

extern "C" int hq_readindex_vote_planes_dev(hq_ctx *ctx, uint64_t G, const uint8_t *planes,
                                            uint64_t *confirmed, uint64_t *outcome) {
    if (!ctx) return HQ_E_INVAL;
    if (G == 0) return HQ_OK;
    if (!planes || !confirmed || !outcome || !hq::aligned16(planes))
        return hq::fail(ctx, HQ_E_INVAL,
                        "hq_readindex_vote_planes: NULL argument or planes not 16-byte aligned");
    BitsK k = bits_args(G, nullptr, 0, nullptr);
    k.tiles = planes;
    k.confirmed = confirmed;
    k.outcome = outcome;
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    const uint64_t ntiles = (G + kPlaneTile - 1) / kPlaneTile;
    hipLaunchKernelGGL(k_planes<HQ_PLANES_BLK>,
                       dim3(grid_for((ntiles + kPlTPW - 1) / kPlTPW * 64, HQ_PLANES_BLK)),
                       dim3(HQ_PLANES_BLK), 0, ctx->stream, k);
    return hq::post_launch(ctx, "hq_readindex_vote_planes");
}

extern "C" int hq_readindex_vote_cq_planes_dev(hq_ctx *ctx, uint64_t G, const uint8_t *planes,
                                               uint8_t *active_planes, uint64_t *confirmed,
                                               uint64_t *outcome, uint64_t *has_quorum) {
    if (!ctx) return HQ_E_INVAL;
    if (G == 0) return HQ_OK;
    if (!planes || !active_planes || !confirmed || !outcome || !has_quorum ||
        !hq::aligned16(planes) || !hq::aligned16(active_planes))
        return hq::fail(ctx, HQ_E_INVAL,
                        "hq_readindex_vote_cq_planes: NULL argument or planes not 16-byte aligned");
    BitsK k = bits_args(G, nullptr, 0, nullptr);
    k.tiles = planes;
    k.confirmed = confirmed;
    k.outcome = outcome;
    k.has_quorum = has_quorum;
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    const uint64_t ntiles = (G + kPlaneTile - 1) / kPlaneTile;
    hipLaunchKernelGGL(k_planes_cq<HQ_PLANES_BLK>,
                       dim3(grid_for((ntiles + HQ_PLCQ_TPW - 1) / HQ_PLCQ_TPW * 64, HQ_PLANES_BLK)),
                       dim3(HQ_PLANES_BLK), 0, ctx->stream, k, active_planes);
    return hq::post_launch(ctx, "hq_readindex_vote_cq_planes");
}

extern "C" int hq_tile_planes_dev(hq_ctx *ctx, uint64_t G, const uint8_t *ack,
                                  const uint8_t *granted, const uint8_t *rejected,
                                  const uint8_t *n_voting, uint32_t n_uniform, uint8_t *planes,
                                  uint64_t *fallback) {
    if (!ctx) return HQ_E_INVAL;
    if (G == 0) return HQ_OK;
    if (!ack || !granted || !rejected || !planes || (reinterpret_cast<uintptr_t>(planes) & 7))
        return hq::fail(ctx, HQ_E_INVAL, "hq_tile_planes: NULL argument or planes misaligned");
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    hipLaunchKernelGGL(k_tile_planes, dim3(grid_for((G + kPlaneTile - 1) / kPlaneTile * kPlaneTile)),
                       dim3(kBlock), 0, ctx->stream, G, n_voting, n_uniform, ack, granted,
                       rejected, planes, fallback);
    return hq::post_launch(ctx, "k_tile_planes");
}

extern "C" int hq_tile_bits3_dev(hq_ctx *ctx, uint64_t G, const uint8_t *ack,
                                 const uint8_t *granted, const uint8_t *rejected,
                                 const uint8_t *n_voting, uint32_t n_uniform, uint8_t *tiles,
                                 uint64_t *fallback) {
    if (!ctx) return HQ_E_INVAL;
    if (G == 0) return HQ_OK;
    if (!ack || !granted || !rejected || !tiles)
        return hq::fail(ctx, HQ_E_INVAL, "hq_tile_bits3: NULL argument");
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    hipLaunchKernelGGL(k_tile_bits3, dim3(grid_for((G + 1023) / 1024 * 1024)), dim3(kBlock), 0,
                       ctx->stream, G, n_voting, n_uniform, ack, granted, rejected, tiles,
                       fallback);
    return hq::post_launch(ctx, "k_tile_bits3");
}

namespace {
// one lane per 16 groups: 16-byte column loads (guarded at G) into the tile rows (padding zeroed)
__global__ __launch_bounds__(kBlock) void k_tile_bits(uint64_t G, const uint8_t *nv,
                                                      const uint8_t *ack, const uint8_t *gr,
                                                      const uint8_t *rj, uint8_t *tiles,
                                                      uint32_t rows) {
    const uint64_t slots = (G + HQ_BITS_TILE_GROUPS - 1) / HQ_BITS_TILE_GROUPS * (HQ_BITS_TILE_GROUPS / 16);
    for (uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x; t < slots;
         t += (uint64_t)gridDim.x * kBlock) {
        const uint64_t g = t * 16;
        uint8_t *row = tiles + (g >> 10) * ((uint64_t)rows << 10) + (g & 1023);
        const uint8_t *cols[4] = {nv, ack, gr, rj};
        for (uint32_t r = 0; r < rows; ++r) {
            const uint8_t *c = cols[r + 4 - rows];
            *reinterpret_cast<uint4 *>(row + (r << 10)) = load16(c, g, G).v;
        }
    }
}
}  // namespace

extern "C" int hq_tile_bits_dev(hq_ctx *ctx, uint64_t G, const uint8_t *ack,
                                const uint8_t *granted, const uint8_t *rejected,
                                const uint8_t *n_voting, uint8_t *tiles) {
    if (!ctx) return HQ_E_INVAL;
    if (G == 0) return HQ_OK;
    if (!ack || !granted || !rejected || !tiles || !hq::aligned16(tiles) || !hq::aligned16(ack) ||
        !hq::aligned16(granted) || !hq::aligned16(rejected) ||
        (n_voting && !hq::aligned16(n_voting)))
        return hq::fail(ctx, HQ_E_INVAL, "hq_tile_bits_dev: NULL or misaligned argument");
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    hipLaunchKernelGGL(k_tile_bits, dim3(grid_for(hq_bits_tiles(G) * (HQ_BITS_TILE_GROUPS / 16))),
                       dim3(kBlock), 0, ctx->stream, G, n_voting, ack, granted, rejected, tiles,
                       n_voting ? 4u : 3u);
    return hq::post_launch(ctx, "k_tile_bits");
}

extern "C" int hq_check_quorum_dev(hq_ctx *ctx, uint64_t G, uint8_t *active,
                                   const uint8_t *n_voting, uint32_t n_uniform,
                                   uint32_t self_slot, uint64_t *has_quorum, uint64_t *fallback) {
    if (ctx && G && (!active || !has_quorum))
        return hq::fail(ctx, HQ_E_INVAL, "hq_check_quorum: NULL active/has_quorum");
    if (ctx && self_slot >= HQ_MAX_VOTERS)
        return hq::fail(ctx, HQ_E_INVAL, "hq_check_quorum: self_slot must be < 8");
    BitsK k = bits_args(G, n_voting, n_uniform, fallback);
    k.active = active;
    k.self_slot = self_slot;
    k.has_quorum = has_quorum;
    return launch_bits<kCHECKQ>(ctx, k, "hq_check_quorum");
}

extern "C" int hq_check_quorum_planes_dev(hq_ctx *ctx, uint64_t G, uint8_t *planes,
                                          uint32_t n_uniform, uint64_t *has_quorum) {
    if (!ctx) return HQ_E_INVAL;
    if (n_uniform > HQ_MAX_VOTERS)
        return hq::fail(ctx, HQ_E_INVAL, "hq_check_quorum_planes: n_uniform must be 0 or 1..8");
    if (G == 0) return HQ_OK;
    if (!has_quorum || (n_uniform != 1 && (!planes || !hq::aligned16(planes))))
        return hq::fail(ctx, HQ_E_INVAL,
                        "hq_check_quorum_planes: NULL argument or planes not 16-byte aligned");
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    constexpr int B = HQ_PLANES_BLK;
    const dim3 grid(grid_for((G + kPlaneTile - 1) / kPlaneTile * 64, B));
    switch (n_uniform) {
    case 0: hipLaunchKernelGGL((k_cq_planes<0, true, B>), grid, dim3(B), 0, ctx->stream, G, planes, has_quorum); break;
    case 1: hipLaunchKernelGGL((k_cq_planes<0, false, B>), grid, dim3(B), 0, ctx->stream, G, planes, has_quorum); break;
    case 2: hipLaunchKernelGGL((k_cq_planes<1, false, B>), grid, dim3(B), 0, ctx->stream, G, planes, has_quorum); break;
    case 3: hipLaunchKernelGGL((k_cq_planes<2, false, B>), grid, dim3(B), 0, ctx->stream, G, planes, has_quorum); break;
    case 4: hipLaunchKernelGGL((k_cq_planes<3, false, B>), grid, dim3(B), 0, ctx->stream, G, planes, has_quorum); break;
    case 5: hipLaunchKernelGGL((k_cq_planes<4, false, B>), grid, dim3(B), 0, ctx->stream, G, planes, has_quorum); break;
    case 6: hipLaunchKernelGGL((k_cq_planes<5, false, B>), grid, dim3(B), 0, ctx->stream, G, planes, has_quorum); break;
    case 7: hipLaunchKernelGGL((k_cq_planes<6, false, B>), grid, dim3(B), 0, ctx->stream, G, planes, has_quorum); break;
    default: hipLaunchKernelGGL((k_cq_planes<7, false, B>), grid, dim3(B), 0, ctx->stream, G, planes, has_quorum); break;
    }
    return hq::post_launch(ctx, "hq_check_quorum_planes");
}

extern "C" int hq_tile_cq_planes_dev(hq_ctx *ctx, uint64_t G, const uint8_t *active,
                                     const uint8_t *n_voting, uint32_t n_uniform,
                                     uint32_t self_slot, uint8_t *planes, uint64_t *fallback) {
    if (!ctx) return HQ_E_INVAL;
    if (n_voting ? n_uniform != 0 : (n_uniform < 1 || n_uniform > HQ_MAX_VOTERS))
        return hq::fail(ctx, HQ_E_INVAL,
                        "hq_tile_cq_planes: per-group n_voting with n_uniform 0, or n_uniform 1..8");
    if (!n_voting && self_slot >= n_uniform)
        return hq::fail(ctx, HQ_E_INVAL, "hq_tile_cq_planes: self_slot >= n_uniform");
    if (G == 0) return HQ_OK;
    const bool no_planes = !n_voting && n_uniform == 1;   // a single-node batch has none
    if (!active || (!no_planes && (!planes || (reinterpret_cast<uintptr_t>(planes) & 7))))
        return hq::fail(ctx, HQ_E_INVAL, "hq_tile_cq_planes: NULL argument or planes misaligned");
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    hipLaunchKernelGGL(k_tile_cq_planes,
                       dim3(grid_for((G + kPlaneTile - 1) / kPlaneTile * kPlaneTile)),
                       dim3(kBlock), 0, ctx->stream, G, active, n_voting, n_uniform, self_slot,
                       planes, fallback);
    return hq::post_launch(ctx, "k_tile_cq_planes");
}

extern "C" int hq_synth_commit_dev(hq_ctx *ctx, const hq_synth_spec *s,
                                   const hq_commit_args *a) {
    if (!ctx) return HQ_E_INVAL;
    if (!s || !a) return hq::fail(ctx, HQ_E_INVAL, "hq_synth_commit: NULL argument");
    if (s->ring_len < 1 || (s->ring_len & (s->ring_len - 1)) || s->n_max < 1 || s->n_max > 8 ||
        s->cid_stride < 1 || (s->mixed_n && s->n_max < 7) || (a->match && a->match_stride < s->G))
        return hq::fail(ctx, HQ_E_INVAL, "hq_synth_commit: bad spec");
    if (s->G == 0) return HQ_OK;
    CommitCols o{};
    o.G = s->G;
    o.stride = a->match_stride;
    o.match = a->match;
    o.nv = a->n_voting;
    o.cin = a->committed_in;
    o.last = a->last_index;
    o.tstart = a->term_start;
    o.term = a->term;
    o.ring = a->ring;
    o.mask = a->term_mask;
    o.ring32 = a->ring32;
    if (o.mask && s->ring_len > 16)
        return hq::fail(ctx, HQ_E_INVAL, "hq_synth_commit: term_mask needs ring_len <= 16");
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    hipLaunchKernelGGL(k_synth_commit, dim3(grid_for(s->G)), dim3(kBlock), 0, ctx->stream, *s, o,
                       LagOut{});
    return hq::post_launch(ctx, "k_synth_commit");
}

// Columns -> HQ_LAYOUT_TILES(_LEADER) tiles, one thread per tile word (include/hipquorum.h).
// Builds tiled inputs from column batches on the device (benchmark inputs, device-side packers).
// lead = 1 drops slot 0's row: tile row r < n holds match slot r + 1.
__global__ __launch_bounds__(kBlock) void k_tile_commit(const CommitCols c, uint64_t *tiles,
                                                        uint64_t ntiles, uint32_t n, int form,
                                                        int lead) {
    const uint64_t tw = c.tile_words, total = ntiles * tw;
    for (uint64_t w = (uint64_t)blockIdx.x * kBlock + threadIdx.x; w < total;
         w += (uint64_t)gridDim.x * kBlock) {
        const uint64_t t = w / tw, r = w % tw, row = r / HQ_TILE_GROUPS;
        uint64_t v = 0;
        // row position p holds group (p >> 1) + 64 * (p & 1) of the tile (include/hipquorum.h)
        auto group = [&](uint64_t p) { return t * HQ_TILE_GROUPS + (p >> 1) + (HQ_TILE_GROUPS / 2) * (p & 1); };
        if (form == HQ_FORM_TERM_MASK && row >= n + 2) {   // 4 u16 masks per word
            const uint64_t p0 = 4 * (r - (uint64_t)(n + 2) * HQ_TILE_GROUPS);
            for (int k = 3; k >= 0; --k) {
                const uint64_t g = group(p0 + k);
                v = (v << 16) | (g < c.G ? c.mask[g] : 0);
            }
        } else {
            const uint64_t g = group(r % HQ_TILE_GROUPS);
            if (g < c.G) {
                v = row < n       ? c.match[(row + lead) * c.stride + g]
                  : row == n      ? c.cin[g]
                  : row == n + 1  ? c.last[g]
                  : form == HQ_FORM_TERM_START ? c.tstart[g] : c.term[g];
            }
        }
        tiles[w] = v;
    }
}

extern "C" int hq_tile_commit_dev(hq_ctx *ctx, const hq_commit_args *a, uint64_t *tiles) {
    return hq_tile_commit_as_dev(ctx, a, tiles, HQ_LAYOUT_TILES);
}

extern "C" int hq_tile_commit_as_dev(hq_ctx *ctx, const hq_commit_args *a, uint64_t *tiles,
                                     uint32_t layout) {
    if (!ctx) return HQ_E_INVAL;
    if (!a || !tiles) return hq::fail(ctx, HQ_E_INVAL, "hq_tile_commit: NULL argument");
    if (a->layout != HQ_LAYOUT_COLUMNS)
        return hq::fail(ctx, HQ_E_INVAL, "hq_tile_commit: input must be the column layout");
    if (layout != HQ_LAYOUT_TILES && layout != HQ_LAYOUT_TILES_LEADER)
        return hq::fail(ctx, HQ_E_INVAL, "hq_tile_commit: target must be a tile layout");
    hq_commit_args chk = *a;
    chk.committed_out = chk.committed_out ? chk.committed_out : tiles;  // not written here
    int rc = validate_commit(ctx, &chk);
    if (rc || a->G == 0) return rc;
    const int lead = layout == HQ_LAYOUT_TILES_LEADER ? 1 : 0;
    CommitCols k = commit_cols(a);
    k.tile_words = hq_commit_tile_words_for(a->n_max, a->form, layout);
    const uint64_t ntiles = hq_commit_tiles(a->G);
    rc = hq::pre_launch(ctx);
    if (rc) return rc;
    hipLaunchKernelGGL(k_tile_commit, dim3(grid_for(ntiles * k.tile_words)), dim3(kBlock), 0,
                       ctx->stream, k, tiles, ntiles, a->n_max - lead, (int)a->form, lead);
    return hq::post_launch(ctx, "k_tile_commit");
}

extern "C" int hq_synth_commit_lag_dev(hq_ctx *ctx, const hq_synth_spec *s,
                                       const hq_commit_lag_args *a, uint64_t *last_index) {
    if (!ctx) return HQ_E_INVAL;
    if (!s || !a) return hq::fail(ctx, HQ_E_INVAL, "hq_synth_commit_lag: NULL argument");
    if (s->ring_len < 1 || (s->ring_len & (s->ring_len - 1)) || s->n_max < 1 || s->n_max > 8 ||
        s->cid_stride < 1 || (s->mixed_n && s->n_max < 7) || (a->lag && a->lag_stride < s->G) ||
        (a->lag_mask && s->ring_len > 16))
        return hq::fail(ctx, HQ_E_INVAL, "hq_synth_commit_lag: bad spec");
    if (a->flags)   // the generator writes every slot's row; view rows 1.. with lag + lag_stride
        return hq::fail(ctx, HQ_E_INVAL, "hq_synth_commit_lag: generate with flags = 0");
    if (s->G == 0) return HQ_OK;
    CommitCols o{};
    o.G = s->G;
    o.nv = a->n_voting;
    LagOut lo{const_cast<int32_t *>(a->lag), a->lag_stride, const_cast<int32_t *>(a->cin_lag),
              const_cast<int32_t *>(a->ts_lag), const_cast<uint16_t *>(a->lag_mask), last_index};
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    hipLaunchKernelGGL(k_synth_commit, dim3(grid_for(s->G)), dim3(kBlock), 0, ctx->stream, *s, o,
                       lo);
    return hq::post_launch(ctx, "k_synth_commit");
}

extern "C" int hq_synth_bitmaps_dev(hq_ctx *ctx, const hq_synth_spec *s, uint8_t *ack,
                                    uint8_t *granted, uint8_t *rejected, uint8_t *n_voting) {
    if (!ctx) return HQ_E_INVAL;
    if (!s || s->n_max < 1 || s->n_max > 8 || s->cid_stride < 1 || (s->mixed_n && s->n_max < 7))
        return hq::fail(ctx, HQ_E_INVAL, "hq_synth_bitmaps: bad spec");
    if (s->G == 0) return HQ_OK;
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    hipLaunchKernelGGL(k_synth_bits, dim3(grid_for(s->G)), dim3(kBlock), 0, ctx->stream, *s, ack,
                       granted, rejected, n_voting);
    return hq::post_launch(ctx, "k_synth_bits");
}

// ---- general multi-ctx ReadIndex ------------------------------------------
namespace {

struct RiMultiK {
    uint64_t G;
    uint32_t K_max, n_max, n_uniform;
    const uint8_t *tiles;         // tiled layout (hq_readindex_multi_tiles_dev), else columns
    uint64_t tile_bytes;
    const uint16_t *ord;
    const uint64_t *idx;
    const uint8_t *np, *nv;
    uint64_t *rel;
    uint8_t *cnt;
    uint8_t *bend;
    uint64_t *fallback;
};

__device__ __forceinline__ void ce32(uint32_t &a, uint32_t &b) {
    const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
    a = lo;
    b = hi;
}

// HQ_RI_NET 0: the transposition sort (A/B baseline, tools/ab_libs.sh)
#ifndef HQ_RI_NET
#define HQ_RI_NET 1
#endif
// Batcher's odd-even merge sort of 8 keys: 19 compare-exchanges in 6 layers (the transposition
// sort it replaces takes 28); only the selected rank is read, so the compiler keeps just the
// min / max halves on its path
#if HQ_RI_NET
constexpr int kNet8[19][2] = {{0, 1}, {2, 3}, {4, 5}, {6, 7}, {0, 2}, {1, 3}, {4, 6},
                              {5, 7}, {1, 2}, {5, 6}, {0, 4}, {1, 5}, {2, 6}, {3, 7},
                              {2, 4}, {3, 5}, {1, 2}, {3, 4}, {5, 6}};
#endif

template <typename CE>
__device__ __forceinline__ void sort8(uint32_t (&v)[8], CE ce) {
#if HQ_RI_NET
#pragma unroll
    for (int c = 0; c < 19; ++c) ce(v[kNet8[c][0]], v[kNet8[c][1]]);
#else
#pragma unroll
    for (int r = 0; r < 8; ++r) {
#pragma unroll
        for (int i = r & 1; i + 1 < 8; i += 2) ce(v[i], v[i + 1]);
    }
#endif
}

__device__ __forceinline__ void sort_net_u32(uint32_t (&v)[8]) {
    sort8(v, [](uint32_t &a, uint32_t &b) { ce32(a, b); });
}

template <bool PERK, bool PERN>
__global__ __launch_bounds__(kBlock) void k_ri_multi(const RiMultiK a) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const uint64_t step = (uint64_t)gridDim.x * kBlock;
    for (uint64_t wbase = wave * 64; wbase < a.G; wbase += step) {
        const uint64_t g = wbase + lane;
        bool fb = false;
        if (g < a.G) {
            const uint32_t K = PERK ? a.np[g] : a.K_max;
            const uint32_t n = PERN ? a.nv[g] : a.n_uniform;
            fb = n < 1 || n > a.n_max || K > a.K_max;
            uint64_t idx[8];
            uint32_t t[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                idx[k] = 0;
                t[k] = 0xFFFFu;
                if (!fb && k < (int)K) {
                    idx[k] = a.idx[(uint64_t)k * a.G + g];
                    fb |= k > 0 && idx[k] < idx[k - 1];   // addRequest: index moved backward
                    // reach time: the max(q-1, 1)-th smallest first-ack ordinal (readindex.go:84)
                    uint32_t v[8];
#pragma unroll
                    for (int s = 0; s < 8; ++s)
                        v[s] = (s < (int)n) ? a.ord[((uint64_t)k * a.n_max + s) * a.G + g] : 0xFFFFu;
                    sort_net_u32(v);
                    const int r = (int)(n / 2 + 1) - 1 > 1 ? (int)(n / 2 + 1) - 1 : 1;
                    uint32_t tk = 0xFFFFu;
#pragma unroll
                    for (int s = 0; s < 8; ++s) tk = (s == r - 1) ? v[s] : tk;
                    t[k] = tk;
                }
            }
            // suffix-min scan: entry i goes with the first ctx k >= i to reach quorum
            // (ties at equal reach times go to the earlier ctx: the replay's queue order)
            uint32_t best_t = 0xFFFFu;
            uint64_t best_idx = 0;
            uint32_t released = 0, bend = 0;
#pragma unroll
            for (int k = 7; k >= 0; --k) {
                bool own = false;
                if (!fb && k < (int)K && t[k] != 0xFFFFu && t[k] <= best_t) {
                    best_t = t[k];
                    best_idx = idx[k];
                    own = true;
                }
                const bool rel = !fb && k < (int)K && best_t != 0xFFFFu;
                released += rel;
                // entry k closes its release batch: it is the ctx whose confirm() released
                // the batch (readindex.go:96), whose ctx the ReadIndexResp hints carry
                bend |= (uint32_t)(rel && own) << k;
                if (a.rel && k < (int)a.K_max) a.rel[(uint64_t)k * a.G + g] = rel ? best_idx : ~0ull;
            }
            a.cnt[g] = (uint8_t)released;
            if (a.bend) a.bend[g] = (uint8_t)bend;
        }
        const uint64_t fw = __ballot(fb);
        if (a.fallback && lane == 0) a.fallback[wbase >> 6] = fw;
    }
}


// Two adjacent groups per lane (even G, aligned columns): the u16 first-ack ordinals of both
// groups travel packed in one 32-bit register, so one 4-byte load reads a (ctx, voter) pair and
// the sorting network runs on both groups at once with packed u16 min / max (v_pk_min_u16 /
// v_pk_max_u16); the ctx indexes and released indexes move as 16-byte pairs. Same decisions as
// k_ri_multi (the suffix-min release of readindex.go:77-116).
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void ce_pk(uint32_t &a, uint32_t &b) {
    const u16x2 x = __builtin_bit_cast(u16x2, a), y = __builtin_bit_cast(u16x2, b);
    a = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(x, y));
    b = __builtin_bit_cast(uint32_t, __builtin_elementwise_max(x, y));
}

// KM >= K_max ctx slots in registers: every (ctx, voter) load of the lane is issued before the
// first sorting network (K_max and n_max are uniform, so the guards are scalar branches; with the
// loads inside the per-ctx branches each ctx waited for its own round trip). The lane's two
// groups' loads (ri_load) and their decision (ri_decide) are written apart; a software-pipelined
// form that issued the next tile's loads before deciding the current one (2, 4 or 8 tiles per
// wave at 3 waves per SIMD) was no faster: 50.6-53.3 vs 50.3-51.5 us, profiles/r04b/ab_rimt.log.
template <bool PERK, bool PERN, int KM>
struct RiIn {
    u64x2 idx[KM];
    uint32_t ov[KM][8];
    uint32_t kk, nn;              // PERK / PERN: the two groups' K / n bytes
};

// TILED: the voter-major tile (include/hipquorum.h): voter s's block of K_max * 256 bytes holds,
// for lane l, the K_max ctx ordinal dwords of groups 2 l, 2 l + 1 back to back; EXACT (K_max ==
// KM) reads them as vectors (one 16-byte load per voter at K_max = 4), otherwise dword by dword.
template <bool PERK, bool PERN, int KM, bool TILED, bool EXACT = false>
__device__ __forceinline__ void ri_load(const RiMultiK &a, uint64_t wbase, int lane,
                                        RiIn<PERK, PERN, KM> &in) {
    const uint64_t g = wbase + 2 * (uint64_t)lane;
    // TILED: the wave's 128 groups are one tile (wbase is a multiple of 128)
    const uint8_t *tb = TILED ? a.tiles + (wbase >> 7) * a.tile_bytes : nullptr;
    const uint64_t ord_bytes = (uint64_t)a.K_max * a.n_max * 256;
    in.kk = in.nn = 0;
    if (g >= a.G) return;         // columns: G is even, g + 1 < G too; tiles: padded rows
    if constexpr (PERK)
        in.kk = TILED ? *reinterpret_cast<const uint16_t *>(tb + ord_bytes + a.K_max * 1024ull +
                                                           2 * lane)
                      : *reinterpret_cast<const uint16_t *>(a.np + g);
    if constexpr (PERN)
        in.nn = TILED ? *reinterpret_cast<const uint16_t *>(tb + ord_bytes + a.K_max * 1024ull +
                                                           (PERK ? 128 : 0) + 2 * lane)
                      : *reinterpret_cast<const uint16_t *>(a.nv + g);
#pragma unroll
    for (int k = 0; k < KM; ++k) {
        in.idx[k] = (u64x2){0, 0};
        if (k < (int)a.K_max)
            in.idx[k] = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(
                TILED ? tb + ord_bytes + k * 1024ull + 16 * lane
                      : reinterpret_cast<const uint8_t *>(a.idx + (uint64_t)k * a.G + g)));
    }
#pragma unroll
    for (int sl = 0; sl < 8; ++sl) {
#pragma unroll
        for (int k = 0; k < KM; ++k) in.ov[k][sl] = 0xFFFFFFFFu;
        if (sl >= (int)a.n_max) continue;
        if constexpr (TILED) {
            const uint8_t *p = tb + (uint64_t)sl * a.K_max * 256 + (uint64_t)lane * 4 * a.K_max;
            if constexpr (EXACT && KM == 2) {
                const u32x2 w = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(p));
                in.ov[0][sl] = w.x;
                in.ov[1][sl] = w.y;
            } else if constexpr (EXACT) {
#pragma unroll
                for (int q = 0; q < KM / 4; ++q) {
                    const u32x4 w = __builtin_nontemporal_load(
                        reinterpret_cast<const u32x4 *>(p + 16 * q));
                    in.ov[4 * q + 0][sl] = w.x;
                    in.ov[4 * q + 1][sl] = w.y;
                    in.ov[4 * q + 2][sl] = w.z;
                    in.ov[4 * q + 3][sl] = w.w;
                }
            } else {
#pragma unroll
                for (int k = 0; k < KM; ++k)
                    if (k < (int)a.K_max)
                        in.ov[k][sl] = __builtin_nontemporal_load(
                            reinterpret_cast<const uint32_t *>(p + 4 * k));
            }
        } else {
#pragma unroll
            for (int k = 0; k < KM; ++k)
                if (k < (int)a.K_max)
                    in.ov[k][sl] = __builtin_nontemporal_load(reinterpret_cast<const uint32_t *>(
                        a.ord + ((uint64_t)k * a.n_max + sl) * a.G + g));
        }
    }
}

template <bool PERK, bool PERN, int KM, bool TILED>
__device__ __forceinline__ void ri_decide(const RiMultiK &a, uint64_t wbase, int lane,
                                          const RiIn<PERK, PERN, KM> &in) {
    const uint64_t g = wbase + 2 * (uint64_t)lane;
    bool fb0 = false, fb1 = false;
    if (g < a.G) {
        uint32_t K0 = a.K_max, K1 = a.K_max, n0 = a.n_uniform, n1 = a.n_uniform;
        if constexpr (PERK) {
            K0 = in.kk & 0xFF;
            K1 = in.kk >> 8;
        }
        if constexpr (PERN) {
            n0 = in.nn & 0xFF;
            n1 = in.nn >> 8;
        }
        fb0 = n0 < 1 || n0 > a.n_max || K0 > a.K_max;
        fb1 = n1 < 1 || n1 > a.n_max || K1 > a.K_max;
        // padding of the voters >= n, per half (0xFFFF = never acked)
        const int r0 = n0 / 2 > 1 ? (int)(n0 / 2) : 1, r1 = n1 / 2 > 1 ? (int)(n1 / 2) : 1;
        const uint32_t kmax = K0 > K1 ? K0 : K1;
        uint32_t t[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            t[k] = 0xFFFFFFFFu;
            if (k < KM && k < (int)kmax && k < (int)a.K_max) {
                uint32_t v[8];
#pragma unroll
                for (int sl = 0; sl < 8; ++sl)
                    v[sl] = in.ov[k < KM ? k : 0][sl] | (sl < (int)n0 ? 0u : 0xFFFFu) |
                            (sl < (int)n1 ? 0u : 0xFFFF0000u);
                sort8(v, [](uint32_t &x, uint32_t &y) { ce_pk(x, y); });
                // reach time: the max(q-1, 1)-th smallest first-ack ordinal (readindex.go:84)
                uint32_t tk = 0;
#pragma unroll
                for (int sl = 0; sl < 8; ++sl) {
                    const uint32_t m = (sl == r0 - 1 ? 0xFFFFu : 0u) |
                                       (sl == r1 - 1 ? 0xFFFF0000u : 0u);
                    tk |= v[sl] & m;
                }
                t[k] = tk;
            }
        }
        u64x2 idx[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) idx[k] = k < KM ? in.idx[k < KM ? k : 0] : (u64x2){0, 0};
#pragma unroll
        for (int k = 1; k < 8; ++k) {   // addRequest: index moved backward
            if (k < KM && k < (int)kmax && k < (int)a.K_max) {
                fb0 |= k < (int)K0 && idx[k].x < idx[k - 1].x;
                fb1 |= k < (int)K1 && idx[k].y < idx[k - 1].y;
            }
        }
        // suffix-min scan per group (ties go to the earlier ctx, as in k_ri_multi)
        uint32_t bt0 = 0xFFFFu, bt1 = 0xFFFFu, rel0 = 0, rel1 = 0, be0 = 0, be1 = 0;
        uint64_t bi0 = 0, bi1 = 0;
#pragma unroll
        for (int k = 7; k >= 0; --k) {
            const uint32_t t0 = t[k] & 0xFFFFu, t1 = t[k] >> 16;
            const bool in0 = !fb0 && k < (int)K0, in1 = !fb1 && k < (int)K1;
            bool own0 = false, own1 = false;
            if (in0 && t0 != 0xFFFFu && t0 <= bt0) { bt0 = t0; bi0 = idx[k].x; own0 = true; }
            if (in1 && t1 != 0xFFFFu && t1 <= bt1) { bt1 = t1; bi1 = idx[k].y; own1 = true; }
            const bool rl0 = in0 && bt0 != 0xFFFFu, rl1 = in1 && bt1 != 0xFFFFu;
            rel0 += rl0;
            rel1 += rl1;
            be0 |= (uint32_t)(rl0 && own0) << k;
            be1 |= (uint32_t)(rl1 && own1) << k;
            if (a.rel && k < (int)a.K_max) {
                uint64_t *r = a.rel + (uint64_t)k * a.G + g;
                if (!TILED || g + 1 < a.G) {
                    *reinterpret_cast<u64x2 *>(r) = (u64x2){rl0 ? bi0 : ~0ull, rl1 ? bi1 : ~0ull};
                } else {
                    r[0] = rl0 ? bi0 : ~0ull;   // odd G: the tile's padding group has no slot
                }
            }
        }
        if (!TILED || g + 1 < a.G) {
            *reinterpret_cast<uint16_t *>(a.cnt + g) = (uint16_t)(rel0 | (rel1 << 8));
            if (a.bend) *reinterpret_cast<uint16_t *>(a.bend + g) = (uint16_t)(be0 | (be1 << 8));
        } else {
            a.cnt[g] = (uint8_t)rel0;
            if (a.bend) a.bend[g] = (uint8_t)be0;
            fb1 = false;
        }
    }
    const uint64_t f0 = __ballot(fb0), f1 = __ballot(fb1);
    if (a.fallback && lane < 2) {
        const uint32_t sh = 32 * lane;
        const uint64_t w = (wbase >> 6) + lane;
        if (w < (a.G + 63) >> 6)
            a.fallback[w] = spread32((uint32_t)(f0 >> sh)) | (spread32((uint32_t)(f1 >> sh)) << 1);
    }
}

template <bool PERK, bool PERN, int KM, bool TILED = false, bool EXACT = false>
__global__ __launch_bounds__(kBlock) void k_ri_multi2(const RiMultiK a) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const uint64_t step = (uint64_t)gridDim.x * kBlock * 2;
    for (uint64_t wbase = wave * 128; wbase < a.G; wbase += step) {
        RiIn<PERK, PERN, KM> in;
        ri_load<PERK, PERN, KM, TILED, EXACT>(a, wbase, lane, in);
        ri_decide<PERK, PERN, KM, TILED>(a, wbase, lane, in);
    }
}

// Uniform wide tiles (K_max == KM ctx slots and n_uniform == n_max == N voters in every group,
// the voter-major ordinal layout): every bound is a constant, so the loads are N 16-byte reads
// (KM = 4) plus KM ctx-index reads with no guards, the rank max(q - 1, 1) = max(N / 2, 1) is a
// constant that prunes the network to the comparators that reach it, and no per-half masks or
// SGPR-held exec masks remain. Same decisions as ri_decide (readindex.go:77-116).
template <int KM, int N>
__global__ __launch_bounds__(kBlock) void k_ri_tiles_u(const RiMultiK a) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
    const uint64_t step = (uint64_t)gridDim.x * kBlock * 2;
    constexpr int R = N / 2 > 1 ? N / 2 : 1;
    for (uint64_t wbase = wave * 128; wbase < a.G; wbase += step) {
        const uint64_t g = wbase + 2 * (uint64_t)lane;   // G even: g < G implies g + 1 < G
        bool fb0 = false, fb1 = false;
        if (g < a.G) {
            const uint8_t *tb = a.tiles + (wbase >> 7) * a.tile_bytes;
            uint32_t ov[KM][N];
#pragma unroll
            for (int sl = 0; sl < N; ++sl) {
                const uint8_t *p = tb + sl * KM * 256 + lane * 4 * KM;
                if constexpr (KM == 2) {
                    const u32x2 w = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(p));
                    ov[0][sl] = w.x;
                    ov[1][sl] = w.y;
                } else {
#pragma unroll
                    for (int q = 0; q < KM / 4; ++q) {
                        const u32x4 w = __builtin_nontemporal_load(
                            reinterpret_cast<const u32x4 *>(p + 16 * q));
                        ov[4 * q + 0][sl] = w.x;
                        ov[4 * q + 1][sl] = w.y;
                        ov[4 * q + 2][sl] = w.z;
                        ov[4 * q + 3][sl] = w.w;
                    }
                }
            }
            u64x2 idx[KM];
#pragma unroll
            for (int k = 0; k < KM; ++k)
                idx[k] = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(
                    tb + N * KM * 256 + k * 1024 + 16 * lane));
            uint32_t t[KM];
#pragma unroll
            for (int k = 0; k < KM; ++k) {
                uint32_t v[8];
#pragma unroll
                for (int sl = 0; sl < 8; ++sl) v[sl] = sl < N ? ov[k][sl < N ? sl : 0] : 0xFFFFFFFFu;
                sort8(v, [](uint32_t &x, uint32_t &y) { ce_pk(x, y); });
                t[k] = v[R - 1];       // the R-th smallest first-ack ordinal of both groups
            }
#pragma unroll
            for (int k = 1; k < KM; ++k) {   // addRequest: index moved backward
                fb0 |= idx[k].x < idx[k - 1].x;
                fb1 |= idx[k].y < idx[k - 1].y;
            }
            uint32_t bt0 = 0xFFFFu, bt1 = 0xFFFFu, rel0 = 0, rel1 = 0, be0 = 0, be1 = 0;
            uint64_t bi0 = 0, bi1 = 0;
#pragma unroll
            for (int k = KM - 1; k >= 0; --k) {
                const uint32_t t0 = t[k] & 0xFFFFu, t1 = t[k] >> 16;
                bool own0 = false, own1 = false;
                if (t0 != 0xFFFFu && t0 <= bt0) { bt0 = t0; bi0 = idx[k].x; own0 = true; }
                if (t1 != 0xFFFFu && t1 <= bt1) { bt1 = t1; bi1 = idx[k].y; own1 = true; }
                const bool rl0 = !fb0 && bt0 != 0xFFFFu, rl1 = !fb1 && bt1 != 0xFFFFu;
                rel0 += rl0;
                rel1 += rl1;
                be0 |= (uint32_t)(rl0 && own0) << k;
                be1 |= (uint32_t)(rl1 && own1) << k;
                if (a.rel)
                    *reinterpret_cast<u64x2 *>(a.rel + (uint64_t)k * a.G + g) =
                        (u64x2){rl0 ? bi0 : ~0ull, rl1 ? bi1 : ~0ull};
            }
            *reinterpret_cast<uint16_t *>(a.cnt + g) = (uint16_t)(rel0 | (rel1 << 8));
            if (a.bend) *reinterpret_cast<uint16_t *>(a.bend + g) = (uint16_t)(be0 | (be1 << 8));
        }
        const uint64_t f0 = __ballot(fb0), f1 = __ballot(fb1);
        if (a.fallback && lane < 2) {
            const uint32_t sh = 32 * lane;
            const uint64_t w = (wbase >> 6) + lane;
            if (w < (a.G + 63) >> 6)
                a.fallback[w] = spread32((uint32_t)(f0 >> sh)) | (spread32((uint32_t)(f1 >> sh)) << 1);
        }
    }
}

}  // namespace

extern "C" int hq_readindex_multi_dev(hq_ctx *ctx, uint64_t G, uint32_t K_max, uint32_t n_max,
                                      const uint16_t *ack_ordinal, const uint64_t *ctx_index,
                                      const uint8_t *n_pending, const uint8_t *n_voting,
                                      uint32_t n_uniform, uint64_t *released_index,
                                      uint8_t *released_count, uint8_t *batch_end,
                                      uint64_t *fallback) {
    if (!ctx) return HQ_E_INVAL;
    if (G == 0) return HQ_OK;
    // released_index may be NULL when batch_end is given (the caller derives it from ctx_index)
    if (!ack_ordinal || !ctx_index || (!released_index && !batch_end) || !released_count ||
        K_max < 1 || K_max > 8 || n_max < 1 || n_max > 8 ||
        (!n_voting && (n_uniform < 1 || n_uniform > 8)))
        return hq::fail(ctx, HQ_E_INVAL, "hq_readindex_multi_dev: bad arguments");
    RiMultiK k{G, K_max, n_max, n_uniform, nullptr, 0, ack_ordinal, ctx_index, n_pending,
               n_voting, released_index, released_count, batch_end, fallback};
    auto al = [](const void *p, uintptr_t m) { return ((uintptr_t)p & (m - 1)) == 0; };
    const bool pairs = ctx->ri_pairs && G % 2 == 0 && al(ack_ordinal, 4) && al(ctx_index, 16) &&
                       al(released_index, 16) && al(released_count, 2) && al(batch_end, 2) &&
                       al(n_pending, 2) && al(n_voting, 2);
    const unsigned grid = pairs ? grid_for(G / 2) : grid_for(G);
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    if (pairs) {
        const int km = K_max <= 2 ? 2 : K_max <= 4 ? 4 : 8;
#define HQ_RIM2(PK, PN)                                                                         \
        do {                                                                                    \
            if (km == 2)                                                                        \
                hipLaunchKernelGGL((k_ri_multi2<PK, PN, 2>), dim3(grid), dim3(kBlock), 0,       \
                                   ctx->stream, k);                                             \
            else if (km == 4)                                                                   \
                hipLaunchKernelGGL((k_ri_multi2<PK, PN, 4>), dim3(grid), dim3(kBlock), 0,       \
                                   ctx->stream, k);                                             \
            else                                                                                \
                hipLaunchKernelGGL((k_ri_multi2<PK, PN, 8>), dim3(grid), dim3(kBlock), 0,       \
                                   ctx->stream, k);                                             \
        } while (0)
        if (n_pending && n_voting) HQ_RIM2(true, true);
        else if (n_pending) HQ_RIM2(true, false);
        else if (n_voting) HQ_RIM2(false, true);
        else HQ_RIM2(false, false);
#undef HQ_RIM2
        return hq::post_launch(ctx, "k_ri_multi2");
    }
    if (n_pending && n_voting)
        hipLaunchKernelGGL((k_ri_multi<true, true>), dim3(grid), dim3(kBlock), 0, ctx->stream, k);
    else if (n_pending)
        hipLaunchKernelGGL((k_ri_multi<true, false>), dim3(grid), dim3(kBlock), 0, ctx->stream, k);
    else if (n_voting)
        hipLaunchKernelGGL((k_ri_multi<false, true>), dim3(grid), dim3(kBlock), 0, ctx->stream, k);
    else
        hipLaunchKernelGGL((k_ri_multi<false, false>), dim3(grid), dim3(kBlock), 0, ctx->stream, k);
    return hq::post_launch(ctx, "k_ri_multi");
}

namespace {

// columns -> multi-ctx ReadIndex tiles: one thread per (tile, row, 16-byte chunk)
__global__ __launch_bounds__(kBlock) void k_tile_ri_multi(uint64_t G, uint32_t K_max,
                                                          uint32_t n_max, const uint16_t *ord,
                                                          const uint64_t *idx, const uint8_t *np,
                                                          const uint8_t *nv, uint8_t *tiles,
                                                          uint64_t tile_bytes) {
    const uint64_t ntiles = (G + HQ_RI_TILE_GROUPS - 1) / HQ_RI_TILE_GROUPS;
    const uint64_t chunks = tile_bytes / 16;
    const uint64_t ord_rows = (uint64_t)K_max * n_max, ord_bytes = ord_rows * 256;
    for (uint64_t q = (uint64_t)blockIdx.x * kBlock + threadIdx.x; q < ntiles * chunks;
         q += (uint64_t)gridDim.x * kBlock) {
        const uint64_t t = q / chunks, off = (q % chunks) * 16;
        const uint64_t g0 = t * HQ_RI_TILE_GROUPS;
        uint8_t v[16];
        if (off < ord_bytes) {                           // 8 u16 ordinal entries
            for (int e = 0; e < 8; ++e) {
                // voter sl's block of K_max * 256 bytes: pair l's K_max dwords (groups 2 l and
                // 2 l + 1 of ctx k at dword k)
                const uint64_t b = off + 2 * e;
                const uint64_t sl = b / (K_max * 256ull), r = b % (K_max * 256ull);
                const uint64_t l = r / (4ull * K_max), w = r % (4ull * K_max);
                const uint64_t row = (w / 4) * n_max + sl, j = 2 * l + (w % 4) / 2;
                const uint64_t g = g0 + j;
                const uint16_t x = g < G ? ord[row * G + g] : 0xFFFFu;
                v[2 * e] = (uint8_t)x;
                v[2 * e + 1] = (uint8_t)(x >> 8);
            }
        } else if (off < ord_bytes + K_max * 1024ull) {  // 2 u64 entries of ctx row
            const uint64_t o = off - ord_bytes, k = o / 1024, j = (o % 1024) / 8;
            for (int e = 0; e < 2; ++e) {
                const uint64_t g = g0 + j + e;
                const uint64_t x = g < G ? idx[k * G + g] : 0;
                for (int b = 0; b < 8; ++b) v[8 * e + b] = (uint8_t)(x >> (8 * b));
            }
        } else {                                         // the u8 rows: n_pending, n_voting
            const uint64_t o = off - ord_bytes - K_max * 1024ull;
            const uint8_t *src = (np && o < 128) ? np : nv;
            const uint64_t j = o % 128;
            for (int e = 0; e < 16; ++e) {
                const uint64_t g = g0 + j + e;
                v[e] = g < G && src ? src[g] : 0;
            }
        }
        uint4 w;
        memcpy(&w, v, 16);
        *reinterpret_cast<uint4 *>(tiles + t * tile_bytes + off) = w;
    }
}

}  // namespace

extern "C" int hq_readindex_multi_tiles_dev(hq_ctx *ctx, uint64_t G, uint32_t K_max,
                                            uint32_t n_max, const uint8_t *tiles, uint32_t flags,
                                            uint32_t n_uniform, uint64_t *released_index,
                                            uint8_t *released_count, uint8_t *batch_end,
                                            uint64_t *fallback) {
    if (!ctx) return HQ_E_INVAL;
    if (G == 0) return HQ_OK;
    const bool perk = flags & HQ_RI_TILE_PER_K, pern = flags & HQ_RI_TILE_PER_N;
    if (!tiles || (!released_index && !batch_end) || !released_count || K_max < 1 || K_max > 8 ||
        n_max < 1 || n_max > 8 || (flags & ~(HQ_RI_TILE_PER_K | HQ_RI_TILE_PER_N)) ||
        (!pern && (n_uniform < 1 || n_uniform > 8)) || !hq::aligned16(tiles) ||
        (reinterpret_cast<uintptr_t>(released_index) & 15) ||
        (reinterpret_cast<uintptr_t>(released_count) & 1) ||
        (batch_end && (reinterpret_cast<uintptr_t>(batch_end) & 1)))
        return hq::fail(ctx, HQ_E_INVAL, "hq_readindex_multi_tiles_dev: bad arguments");
    RiMultiK k{G, K_max, n_max, n_uniform, tiles, hq_ri_tile_bytes(K_max, n_max, flags),
               nullptr, nullptr, nullptr, nullptr, released_index, released_count, batch_end,
               fallback};
    // the pair kernel's column stores need 16-byte rows: G even keeps k * G + g aligned
    if (G % 2)
        return hq::fail(ctx, HQ_E_INVAL, "hq_readindex_multi_tiles_dev: G must be even");
    const unsigned grid = grid_for(G / 2);
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    const int km = K_max <= 2 ? 2 : K_max <= 4 ? 4 : 8;
    const bool exact = (uint32_t)km == K_max;
    if (exact && ctx->ri_uniform && !perk && !pern && n_uniform == n_max) {
#define HQ_RITU(KMV)                                                                            \
        do {                                                                                    \
            switch (n_max) {                                                                    \
            case 1: hipLaunchKernelGGL((k_ri_tiles_u<KMV, 1>), dim3(grid), dim3(kBlock), 0, ctx->stream, k); break; \
            case 2: hipLaunchKernelGGL((k_ri_tiles_u<KMV, 2>), dim3(grid), dim3(kBlock), 0, ctx->stream, k); break; \
            case 3: hipLaunchKernelGGL((k_ri_tiles_u<KMV, 3>), dim3(grid), dim3(kBlock), 0, ctx->stream, k); break; \
            case 4: hipLaunchKernelGGL((k_ri_tiles_u<KMV, 4>), dim3(grid), dim3(kBlock), 0, ctx->stream, k); break; \
            case 5: hipLaunchKernelGGL((k_ri_tiles_u<KMV, 5>), dim3(grid), dim3(kBlock), 0, ctx->stream, k); break; \
            case 6: hipLaunchKernelGGL((k_ri_tiles_u<KMV, 6>), dim3(grid), dim3(kBlock), 0, ctx->stream, k); break; \
            case 7: hipLaunchKernelGGL((k_ri_tiles_u<KMV, 7>), dim3(grid), dim3(kBlock), 0, ctx->stream, k); break; \
            default: hipLaunchKernelGGL((k_ri_tiles_u<KMV, 8>), dim3(grid), dim3(kBlock), 0, ctx->stream, k); break; \
            }                                                                                   \
        } while (0)
        if (K_max == 2) HQ_RITU(2);
        else if (K_max == 4) HQ_RITU(4);
        else HQ_RITU(8);
#undef HQ_RITU
        return hq::post_launch(ctx, "k_ri_tiles_u");
    }
#define HQ_RIM2TK(PK, PN, KMV)                                                                  \
    do {                                                                                        \
        if (exact)                                                                              \
            hipLaunchKernelGGL((k_ri_multi2<PK, PN, KMV, true, true>), dim3(grid),              \
                               dim3(kBlock), 0, ctx->stream, k);                                \
        else                                                                                    \
            hipLaunchKernelGGL((k_ri_multi2<PK, PN, KMV, true, false>), dim3(grid),             \
                               dim3(kBlock), 0, ctx->stream, k);                                \
    } while (0)
#define HQ_RIM2T(PK, PN)                                                                        \
    do {                                                                                        \
        if (km == 2) HQ_RIM2TK(PK, PN, 2);                                                      \
        else if (km == 4) HQ_RIM2TK(PK, PN, 4);                                                 \
        else HQ_RIM2TK(PK, PN, 8);                                                              \
    } while (0)
    if (perk && pern) HQ_RIM2T(true, true);
    else if (perk) HQ_RIM2T(true, false);
    else if (pern) HQ_RIM2T(false, true);
    else HQ_RIM2T(false, false);
#undef HQ_RIM2T
#undef HQ_RIM2TK
    return hq::post_launch(ctx, "k_ri_multi2<tiles>");
}

extern "C" int hq_tile_ri_multi_dev(hq_ctx *ctx, uint64_t G, uint32_t K_max, uint32_t n_max,
                                    const uint16_t *ack_ordinal, const uint64_t *ctx_index,
                                    const uint8_t *n_pending, const uint8_t *n_voting,
                                    uint8_t *tiles) {
    if (!ctx) return HQ_E_INVAL;
    if (G == 0) return HQ_OK;
    if (!ack_ordinal || !ctx_index || !tiles || K_max < 1 || K_max > 8 || n_max < 1 ||
        n_max > 8 || !hq::aligned16(tiles))
        return hq::fail(ctx, HQ_E_INVAL, "hq_tile_ri_multi_dev: bad arguments");
    const uint32_t flags = (n_pending ? HQ_RI_TILE_PER_K : 0) | (n_voting ? HQ_RI_TILE_PER_N : 0);
    const uint64_t tb = hq_ri_tile_bytes(K_max, n_max, flags);
    const uint64_t ntiles = (G + HQ_RI_TILE_GROUPS - 1) / HQ_RI_TILE_GROUPS;
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    hipLaunchKernelGGL(k_tile_ri_multi, dim3(grid_for(ntiles * (tb / 16))), dim3(kBlock), 0,
                       ctx->stream, G, K_max, n_max, ack_ordinal, ctx_index, n_pending, n_voting,
                       tiles, tb);
    return hq::post_launch(ctx, "k_tile_ri_multi");
}

// ---- device-resident progress table: delta ingest ------------------------
namespace {

__device__ __forceinline__ void count_skip(uint64_t *n_skipped, bool skip) {
    // one atomic per wave: the ballot's popcount of skipped lanes
    const uint64_t m = __ballot(skip);
    if (n_skipped && m && (threadIdx.x & 63) == (uint32_t)(__ffsll((long long)m) - 1))
        atomicAdd(reinterpret_cast<unsigned long long *>(n_skipped),
                  (unsigned long long)__popcll(m));
}

__global__ __launch_bounds__(kBlock) void k_ingest_match(const hq_match_update *u, uint64_t count,
                                                         uint64_t *match, uint64_t stride,
                                                         uint64_t G, uint32_t n_max,
                                                         uint64_t *n_skipped) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i - threadIdx.x < count;
         i += (uint64_t)gridDim.x * kBlock) {
        bool skip = false;
        if (i < count) {
            const hq_match_update x = u[i];
            const uint64_t g = x.group_slot >> 8;
            const uint32_t s = (uint32_t)(x.group_slot & 0xFF);
            skip = g >= G || s >= n_max;
            // remote.tryUpdate (remote.go:127-131): match only rises
            if (!skip)
                atomicMax(reinterpret_cast<unsigned long long *>(match + s * stride + g),
                          (unsigned long long)x.index);
        }
        count_skip(n_skipped, skip);
    }
}

__global__ __launch_bounds__(kBlock) void k_ingest_ack(const uint64_t *gs, uint64_t count,
                                                       uint8_t *ack, uint64_t G, uint32_t n_max,
                                                       uint64_t *n_skipped) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i - threadIdx.x < count;
         i += (uint64_t)gridDim.x * kBlock) {
        bool skip = false;
        if (i < count) {
            const uint64_t x = gs[i];
            const uint64_t g = x >> 8;
            const uint32_t s = (uint32_t)(x & 0xFF);
            skip = g >= G || s >= n_max || s >= 8;
            // readIndex.confirm: p.confirmed[from] = struct{}{} (readindex.go:83)
            if (!skip)
                atomicOr(reinterpret_cast<unsigned int *>(ack + (g & ~3ull)),
                         1u << (s + 8 * (uint32_t)(g & 3)));
        }
        count_skip(n_skipped, skip);
    }
}

__global__ __launch_bounds__(kBlock) void k_append(const hq_append_update *u, uint64_t count,
                                                   uint64_t *last, uint64_t *match0,
                                                   uint16_t *mask, uint32_t R, uint64_t G,
                                                   uint64_t *n_skipped) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i - threadIdx.x < count;
         i += (uint64_t)gridDim.x * kBlock) {
        bool skip = false;
        if (i < count) {
            const hq_append_update x = u[i];
            skip = x.group >= G;
            if (!skip) {
                const uint64_t g = x.group;
                const uint64_t prev = atomicMax(reinterpret_cast<unsigned long long *>(last + g),
                                                (unsigned long long)x.new_last);
                if (x.new_last > prev) {
                    // the leader's own remote follows its log (raft.go:918)
                    atomicMax(reinterpret_cast<unsigned long long *>(match0 + g),
                              (unsigned long long)x.new_last);
                    if (mask) {
                        // entries (prev, new_last] carry the leader's term (raft.go:913-916)
                        const uint64_t n = x.new_last - prev;
                        uint32_t bits = 0;
                        if (n >= R) {
                            bits = R >= 32 ? 0xFFFFFFFFu : ((1u << R) - 1u);
                        } else {
                            for (uint64_t k = 1; k <= n; ++k) bits |= 1u << ((prev + k) & (R - 1));
                        }
                        atomicOr(reinterpret_cast<unsigned int *>(mask + (g & ~1ull)),
                                 (bits & 0xFFFFu) << (16 * (uint32_t)(g & 1)));
                    }
                }
            }
        }
        count_skip(n_skipped, skip);
    }
}

}  // namespace

// ---- compact 8-byte deltas (hq_ingest_lag_dev / hq_append_count_dev) ------------------------
namespace {

// the term-mask bits of the entries (prev, prev + n] (appendEntries at the leader's term)
__device__ __forceinline__ uint32_t append_bits(uint64_t prev, uint64_t n, uint32_t R) {
    if (n >= R) return R >= 32 ? 0xFFFFFFFFu : ((1u << R) - 1u);
    uint32_t bits = 0;
    for (uint64_t k = 1; k <= n; ++k) bits |= 1u << ((prev + k) & (R - 1));
    return bits;
}

__global__ __launch_bounds__(kBlock) void k_ingest_lag(const uint64_t *u, uint64_t count,
                                                       uint64_t *match, uint64_t stride,
                                                       const uint64_t *last, uint64_t G,
                                                       uint32_t n_max, uint64_t *n_skipped) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i - threadIdx.x < count;
         i += (uint64_t)gridDim.x * kBlock) {
        bool skip = false;
        if (i < count) {
            const uint64_t x = __builtin_nontemporal_load(u + i);
            const uint64_t g = x >> 32;
            const uint32_t s = (uint32_t)(x >> 28) & 0xFu;
            const uint64_t lag = x & 0x0FFFFFFFull;
            skip = g >= G || s >= n_max;
            if (!skip) {
                const uint64_t l = last[g];
                skip = lag > l;
                // remote.tryUpdate (remote.go:127-131) of the acknowledged index lastIndex - lag
                if (!skip)
                    atomicMax(reinterpret_cast<unsigned long long *>(match + s * stride + g),
                              (unsigned long long)(l - lag));
            }
        }
        count_skip(n_skipped, skip);
    }
}

__global__ __launch_bounds__(kBlock) void k_append_count(const uint64_t *u, uint64_t count,
                                                         uint64_t *last, uint64_t *match0,
                                                         uint16_t *mask, uint32_t R, uint64_t G,
                                                         uint64_t *n_skipped) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i - threadIdx.x < count;
         i += (uint64_t)gridDim.x * kBlock) {
        bool skip = false;
        if (i < count) {
            const uint64_t x = __builtin_nontemporal_load(u + i);
            const uint64_t g = x >> 32, n = x & 0xFFFFFFFFull;
            skip = g >= G || n == 0;
            if (!skip) {
                // appendEntries (raft.go:911-922): lastIndex += len(entries); additions commute,
                // so several appends of one group in a batch land in any order
                const uint64_t prev = atomicAdd(reinterpret_cast<unsigned long long *>(last + g),
                                                (unsigned long long)n);
                atomicMax(reinterpret_cast<unsigned long long *>(match0 + g),
                          (unsigned long long)(prev + n));          // raft.go:918
                if (mask)
                    atomicOr(reinterpret_cast<unsigned int *>(mask + (g & ~1ull)),
                             (append_bits(prev, n, R) & 0xFFFFu) << (16 * (uint32_t)(g & 1)));
            }
        }
        count_skip(n_skipped, skip);
    }
}

}  // namespace

extern "C" int hq_ingest_lag_dev(hq_ctx *ctx, const uint64_t *updates, uint64_t count,
                                 uint64_t *match, uint64_t match_stride,
                                 const uint64_t *last_index, uint64_t G, uint32_t n_max,
                                 uint64_t *n_skipped) {
    if (!ctx) return HQ_E_INVAL;
    if (count == 0) return HQ_OK;
    if (!updates || !match || !last_index || match_stride < G || n_max < 1 ||
        n_max > HQ_MAX_VOTERS)
        return hq::fail(ctx, HQ_E_INVAL, "hq_ingest_lag_dev: bad arguments");
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    hipLaunchKernelGGL(k_ingest_lag, dim3(grid_for(count)), dim3(kBlock), 0, ctx->stream,
                       updates, count, match, match_stride, last_index, G, n_max, n_skipped);
    return hq::post_launch(ctx, "k_ingest_lag");
}

extern "C" int hq_append_count_dev(hq_ctx *ctx, const uint64_t *updates, uint64_t count,
                                   uint64_t *last_index, uint64_t *match_slot0,
                                   uint16_t *term_mask, uint32_t ring_len, uint64_t G,
                                   uint64_t *n_skipped) {
    if (!ctx) return HQ_E_INVAL;
    if (count == 0) return HQ_OK;
    if (!updates || !last_index || !match_slot0 ||
        (term_mask && ((reinterpret_cast<uintptr_t>(term_mask) & 3) || ring_len < 1 ||
                       ring_len > 16 || (ring_len & (ring_len - 1)))))
        return hq::fail(ctx, HQ_E_INVAL, "hq_append_count_dev: bad arguments");
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    hipLaunchKernelGGL(k_append_count, dim3(grid_for(count)), dim3(kBlock), 0, ctx->stream,
                       updates, count, last_index, match_slot0, term_mask,
                       ring_len ? ring_len : 16u, G, n_skipped);
    return hq::post_launch(ctx, "k_append_count");
}

extern "C" int hq_ingest_match_dev(hq_ctx *ctx, const hq_match_update *updates, uint64_t count,
                                   uint64_t *match, uint64_t match_stride, uint64_t G,
                                   uint32_t n_max, uint64_t *n_skipped) {
    if (!ctx) return HQ_E_INVAL;
    if (count == 0) return HQ_OK;
    if (!updates || !match || match_stride < G || n_max < 1 || n_max > HQ_MAX_VOTERS)
        return hq::fail(ctx, HQ_E_INVAL, "hq_ingest_match_dev: bad arguments");
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    hipLaunchKernelGGL(k_ingest_match, dim3(grid_for(count)), dim3(kBlock), 0, ctx->stream,
                       updates, count, match, match_stride, G, n_max, n_skipped);
    return hq::post_launch(ctx, "k_ingest_match");
}

extern "C" int hq_ingest_ack_dev(hq_ctx *ctx, const uint64_t *group_slot, uint64_t count,
                                 uint8_t *ack, uint64_t G, uint32_t n_max, uint64_t *n_skipped) {
    if (!ctx) return HQ_E_INVAL;
    if (count == 0) return HQ_OK;
    if (!group_slot || !ack || (reinterpret_cast<uintptr_t>(ack) & 3) || n_max < 1 ||
        n_max > HQ_MAX_VOTERS)
        return hq::fail(ctx, HQ_E_INVAL, "hq_ingest_ack_dev: bad arguments (ack must be 4-byte aligned)");
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    hipLaunchKernelGGL(k_ingest_ack, dim3(grid_for(count)), dim3(kBlock), 0, ctx->stream,
                       group_slot, count, ack, G, n_max, n_skipped);
    return hq::post_launch(ctx, "k_ingest_ack");
}

extern "C" int hq_append_dev(hq_ctx *ctx, const hq_append_update *updates, uint64_t count,
                             uint64_t *last_index, uint64_t *match_slot0, uint16_t *term_mask,
                             uint32_t ring_len, uint64_t G, uint64_t *n_skipped) {
    if (!ctx) return HQ_E_INVAL;
    if (count == 0) return HQ_OK;
    if (!updates || !last_index || !match_slot0 ||
        (term_mask && ((reinterpret_cast<uintptr_t>(term_mask) & 3) || ring_len < 1 ||
                       ring_len > 16 || (ring_len & (ring_len - 1)))))
        return hq::fail(ctx, HQ_E_INVAL, "hq_append_dev: bad arguments");
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    hipLaunchKernelGGL(k_append, dim3(grid_for(count)), dim3(kBlock), 0, ctx->stream, updates,
                       count, last_index, match_slot0, term_mask, ring_len ? ring_len : 16u, G,
                       n_skipped);
    return hq::post_launch(ctx, "k_append");
}
