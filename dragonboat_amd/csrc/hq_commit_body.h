// hq_commit_body.h — the commit decision shared by the launch-per-step kernels (hq_kernels.hip)
// and the persistent commit engine (hq_engine.hip): the u64 selection networks, the term-check
// forms and the body that decides one 128-group tile (HQ_LAYOUT_TILES / _TILES_LEADER).
#pragma once

#include <type_traits>

#include "hq_internal.h"

namespace {

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Streaming columns are read once: nontemporal loads (measured ~6 % faster than plain ones on
// the 1M x 3 commit stream, tools/kexp.hip, git history). The committed column is stored with plain stores:
// 11.10 vs 11.45 us per 1M x 3 launch against nontemporal ones (tools/kexp3.hip, git history; sc1
// write-through 11.19, nt sc1 12.36).
__device__ __forceinline__ u64x2 ld_stream2(const uint64_t *p) {
    return __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(p));
}
__device__ __forceinline__ void st_stream2(uint64_t *p, u64x2 v) {
    *reinterpret_cast<u64x2 *>(p) = v;
}

// The decision kernels' argument: only what one form reads, 96 bytes. Kernel arguments past
// that cost the 1M-group launch 0.25 us (a 160-byte twin of the same kernel: 10.55 vs 10.30 us,
// tools/kexp6.hip, git history), so the form-specific columns share the `aux` and `ring` slots.
struct CommitK {
    uint64_t G;
    uint64_t stride;        // columns: elements between match rows; tiles: u64 words per tile
    const uint64_t *match;  // columns: slot 0's row; tiles: tile 0
    const uint64_t *cin;    // columns only (tiles carry it)
    uint64_t *cout;
    const uint64_t *last;   // columns only
    const void *aux;        // term_start (TERM_START) | term (RING, RING32) | u16 mask (MASK)
    const void *ring;       // u64 ring (RING) | u32 ring (RING32)
    uint64_t *changed, *fallback;
    const uint8_t *nv;
    uint32_t R, reserved;
};
static_assert(sizeof(CommitK) == 96, "keep the decision kernels' argument at 96 bytes");

// ---- compare-exchange networks over u64 held in registers --------------------------------
__device__ __forceinline__ void ce(uint64_t &a, uint64_t &b) {
    const uint64_t lo = a < b ? a : b;
    const uint64_t hi = a < b ? b : a;
    a = lo;
    b = hi;
}

// Ascending odd-even transposition network, fully unrolled; the compiler drops the
// compare-exchanges that do not reach the selected element.
template <int N>
__device__ __forceinline__ void sort_net(uint64_t (&v)[N]) {
#pragma unroll
    for (int r = 0; r < N; ++r) {
#pragma unroll
        for (int i = r & 1; i + 1 < N; i += 2) ce(v[i], v[i + 1]);
    }
}

// The quorum-th largest match = matched[n - quorum] after an ascending sort (raft.go:902-903).
template <int N>
__device__ __forceinline__ uint64_t quorum_match_uniform(uint64_t (&v)[N]) {
    if constexpr (N == 1) {
        return v[0];
    } else if constexpr (N == 2) {
        return v[0] < v[1] ? v[0] : v[1];
    } else if constexpr (N == 3) {  // median of 3: 3 compare-exchanges
        ce(v[0], v[1]);
        ce(v[1], v[2]);
        return v[0] > v[1] ? v[0] : v[1];
    } else {
        sort_net<N>(v);
        return v[N - (N / 2 + 1)];
    }
}

// Runtime n <= N: slots >= n are padded with 0 (the minimum), so the (n/2+1)-th largest of the
// padded N values is the (n/2+1)-th largest of the n real ones.
template <int N>
__device__ __forceinline__ uint64_t quorum_match_pern(uint64_t (&v)[N], int n) {
    sort_net<N>(v);
    const int idx = N - (n / 2 + 1);
    uint64_t r = 0;
#pragma unroll
    for (int k = 0; k < N; ++k) r = (k == idx) ? v[k] : r;
    return r;
}

__device__ __forceinline__ uint64_t spread32(uint32_t x) {  // bit i -> bit 2i
    uint64_t v = x;
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;
    v = (v | (v << 1)) & 0x5555555555555555ull;
    return v;
}

// One group's decision given its packed matches. FORM 0 = term-start, 1 = ring gather,
// 2 = current-term mask, 3 = u32 ring gather. aux = term_start (0), the leader's term (1, 3) or
// the mask (2).
template <int N, int FORM, bool PERN>
__device__ __forceinline__ void decide(const CommitK &a, uint64_t g, uint64_t (&m)[N], int n,
                                       uint64_t cin, uint64_t last, uint64_t aux,
                                       uint64_t &cout, bool &chg, bool &fb) {
    cout = cin;
    chg = false;
    fb = false;
    if constexpr (PERN) {
        if (n < 1 || n > N) {
            fb = true;
            return;
        }
#pragma unroll
        for (int s = 0; s < N; ++s) m[s] = (s < n) ? m[s] : 0;
    }
    uint64_t q;
    if constexpr (PERN) {
        q = quorum_match_pern<N>(m, n);
    } else {
        q = quorum_match_uniform<N>(m);
    }
    if constexpr (FORM == HQ_FORM_TERM_START) {
        // term(q) == term  <=>  term_start <= q <= last   (aux = term_start)
        chg = (q > cin) & (q >= aux) & (q <= last);
    } else if constexpr (FORM == HQ_FORM_TERM_MASK) {
        // bit (i mod R) of the mask = term(i) == term for i in (last - R, last]
        fb = (cin > last) || (last - cin > a.R);
        chg = !fb && q > cin && q <= last && ((aux >> (q & (uint64_t)(a.R - 1))) & 1);
    } else if constexpr (FORM == HQ_FORM_TERM_RING32) {
        // the same gather from a u32 ring (entries saturated at 0xFFFFFFFF by the packer): with
        // the leader's term below 0xFFFFFFFF, ring32 == term <=> term(i) == term. Two groups'
        // rings share one 128-B line, so a lane's pair of gathers costs one line, not two.
        fb = (aux == 0) | (aux >= 0xFFFFFFFFull) | (cin > last) || (last - cin > a.R);
        if (!fb && q > cin && q <= last) {
            const uint32_t lterm = static_cast<const uint32_t *>(a.ring)[g * a.R + (q & (uint64_t)(a.R - 1))];
            chg = lterm == (uint32_t)aux;
        }
    } else {
        // aux = the leader's term; the ring holds term(i) for i in (last - R, last]
        fb = (aux == 0) | (cin > last) || (last - cin > a.R);
        if (!fb && q > cin && q <= last) {
            const uint64_t lterm = static_cast<const uint64_t *>(a.ring)[g * a.R + (q & (uint64_t)(a.R - 1))];
            chg = lterm == aux;
        }
    }
    cout = chg ? q : cin;
}

// 1: the tile bodies issue every row load before the first compare (tile_blocks); 0 is the
// A/B baseline of profiles/r01i/kexp10_sched_barrier_ab.log
#ifndef HQ_TILE_SCHED_BARRIER
#define HQ_TILE_SCHED_BARRIER 1
#endif

// One 128-group tile starting at group `wbase` (a multiple of HQ_TILE_GROUPS), decided by one
// wave (`lane` = this lane). Row position 2i holds group i of the tile and position 2i + 1 group
// i + 64, so lane i's 16-byte load of a row brings groups i and i + 64. LEAD = 1: rows start at
// slot 1 (row s - 1 holds slot s) and m[0] = last_index (the leader's own match, raft.go:918,
// 1031). INPLACE: committed' is stored into the tile's committed row (a device-resident table).
// 8-byte store; WT: write-through (sc1, agent scope), so that a wave whose stores have drained
// (s_waitcnt vmcnt(0)) has made them visible with no release fence (the engine's per-step
// completion, hq_engine.hip; cdna_hip_programming.md Guideline 16 R1)
template <bool WT>
__device__ __forceinline__ void st8(uint64_t *p, uint64_t v) {
    if constexpr (WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

// SOFF: the full-tile path addresses every row and output as a uniform (SGPR) base plus this
// lane's 32-bit byte offset (global_load saddr + voffset), so no 64-bit per-lane address lives in
// VGPRs across the caller's loop (the persistent engine, hq_engine.hip: its step loop otherwise
// kept `match + 16 * lane` as a u64 pair and spilled it)
template <class T>
__device__ __forceinline__ T *byte_off(T *p, uint32_t off) {
    return reinterpret_cast<T *>(reinterpret_cast<
        typename std::conditional<std::is_const<T>::value, const char, char>::type *>(p) + off);
}

template <int N, int FORM, bool PERN, int LEAD, bool INPLACE, bool WT = false, bool SOFF = false>
__device__ __forceinline__ void commit_tile(const CommitK &a, uint64_t wbase, uint64_t lane) {
    constexpr uint64_t T = HQ_TILE_GROUPS, H = T / 2;
    constexpr int NR = N - LEAD;   // match rows in the tile
    const uint64_t *t = a.match + (wbase / T) * a.stride + lane * 2;
    const uint64_t ga = wbase + lane, gb = ga + H;
    bool ca = false, cb = false, fa = false, fb = false;
    if (wbase + T <= a.G) {
        // row r of the tile at lane's 16 bytes
        const uint64_t *tb = a.match + (wbase / T) * a.stride;   // uniform
        const uint32_t lo = (uint32_t)lane * 16u;
        auto row = [&](int r) -> const uint64_t * {
            if constexpr (SOFF) return byte_off(tb + r * T, lo);
            return t + r * T;
        };
        uint64_t m0[N], m1[N];
#pragma unroll
        for (int s = LEAD; s < N; ++s) {
            const u64x2 v = ld_stream2(row(s - LEAD));
            m0[s] = v.x;
            m1[s] = v.y;
        }
        const u64x2 ci = ld_stream2(row(NR)), la = ld_stream2(row(NR + 1));
        if constexpr (LEAD) {
            m0[0] = la.x;
            m1[0] = la.y;
        }
        u64x2 ax;
        if constexpr (FORM == HQ_FORM_TERM_MASK) {
            const uint32_t *mp =
                SOFF ? byte_off(reinterpret_cast<const uint32_t *>(tb + (NR + 2) * T), lo / 4)
                     : reinterpret_cast<const uint32_t *>(
                           reinterpret_cast<const uint16_t *>(t - lane * 2 + (NR + 2) * T) + lane * 2);
            const uint32_t mm = __builtin_nontemporal_load(mp);
            ax = (u64x2){mm & 0xFFFFu, mm >> 16};
        } else {
            ax = ld_stream2(row(NR + 2));
        }
#if HQ_TILE_SCHED_BARRIER
        // every row load of the tile is issued before the first compare: otherwise the
        // scheduler starts the network after two rows and issues the rows past the 4-KiB
        // immediate-offset range behind an s_waitcnt, one memory latency later (n <= 5: the
        // wider bodies would spill inside the 64-VGPR fused kernel)
        if constexpr (N <= 5) __builtin_amdgcn_sched_barrier(0);
#endif
        const int na = PERN ? (int)a.nv[ga] : N, nb = PERN ? (int)a.nv[gb] : N;
        uint64_t coa, cob;
#ifdef HQ_TILE_COPY   // tuning floor: the same loads and stores, no decision (wrong results)
        coa = ci.x ^ la.x ^ ax.x;
        cob = ci.y ^ la.y ^ ax.y;
#pragma unroll
        for (int s = LEAD; s < N; ++s) {
            coa ^= m0[s];
            cob ^= m1[s];
        }
        ca = coa & 1;
        cb = cob & 1;
        (void)na;
        (void)nb;
#else
        decide<N, FORM, PERN>(a, ga, m0, na, ci.x, la.x, ax.x, coa, ca, fa);
        decide<N, FORM, PERN>(a, gb, m1, nb, ci.y, la.y, ax.y, cob, cb, fb);
#endif
        if constexpr (INPLACE) {
            // the lane's 16 bytes of the committed row it has just read (groups ga, gb)
            uint64_t *cr = const_cast<uint64_t *>(row(NR));
            if constexpr (WT) {
                st8<true>(cr, coa);
                st8<true>(cr + 1, cob);
            } else {
                st_stream2(cr, (u64x2){coa, cob});
            }
        } else if constexpr (SOFF) {
            uint64_t *cb0 = a.cout + wbase;   // uniform
            st8<WT>(byte_off(cb0, lo / 2), coa);
            st8<WT>(byte_off(cb0 + H, lo / 2), cob);
        } else {
            st8<WT>(a.cout + ga, coa);
            st8<WT>(a.cout + gb, cob);
        }
    } else {   // the batch's last, partial tile: group by group
        auto single = [&](int j, bool &c, bool &f) {
            const uint64_t g = ga + H * j;
            uint64_t m[N];
            const uint64_t last = t[(NR + 1) * T + j];
#pragma unroll
            for (int s = LEAD; s < N; ++s) m[s] = t[(s - LEAD) * T + j];
            if constexpr (LEAD) m[0] = last;
            const uint64_t ax =
                FORM == HQ_FORM_TERM_MASK
                    ? (uint64_t)reinterpret_cast<const uint16_t *>(t - lane * 2 + (NR + 2) * T)[lane * 2 + j]
                    : t[(NR + 2) * T + j];
            uint64_t co;
            decide<N, FORM, PERN>(a, g, m, PERN ? (int)a.nv[g] : N, t[NR * T + j], last, ax,
                                  co, c, f);
            if constexpr (INPLACE) st8<WT>(const_cast<uint64_t *>(t) + NR * T + j, co);
            else st8<WT>(a.cout + g, co);
        };
        if (ga < a.G) single(0, ca, fa);
        if (gb < a.G) single(1, cb, fb);
    }
    const uint64_t ba = __ballot(ca), bb = __ballot(cb);
    const uint64_t xa = __ballot(fa), xb = __ballot(fb);
    const uint64_t w = (wbase >> 6) + lane;
    if (lane < 2 && w < ((a.G + 63) >> 6)) {
        if (a.changed) st8<WT>(a.changed + w, lane ? bb : ba);
        if (a.fallback) st8<WT>(a.fallback + w, lane ? xb : xa);
    }
}

}  // namespace
