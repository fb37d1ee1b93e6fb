// hq_table.hip — the device-resident progress table in the headline layout.
//
// The table IS the commit kernel's input: HQ_LAYOUT_TILES_LEADER tiles (128 groups per tile; rows
// match slot 1 .. n-1, committed, lastIndex, then term_start (u64) or the u16 term mask; row
// position 2i holds group i of the tile and 2i + 1 group i + 64), decided in place by
// hq_commit_dev with HQ_LAYOUT_TILES_LEADER | HQ_LAYOUT_IN_PLACE. The kernels here apply a step's
// deltas to it:
//   hq_table_ingest_match_dev / _lag_dev   remote.tryUpdate per accepted ReplicateResp
//                                          (remote.go:123-133, raft.go:1671-1700): match only rises
//   hq_table_append_dev / _append_count_dev appendEntries (raft.go:911-922): lastIndex, the term
//                                          bits of the new entries (the leader's own match is
//                                          lastIndex by construction of the layout, raft.go:918)
//   hq_table_committed_dev                 the committed row back in group order (readback)
//
// Every update is a max (match, lastIndex) or a sum (appended counts) per key, so the batch can
// be applied in any order. Default: one 64-bit atomic per record. HQ_INGEST_GROUPED (the
// records of one key adjacent in the batch, as a step worker emits them node by node): a wave
// reduces each run of equal keys with a segmented scan over shuffles and the run's last lane
// applies it with a plain read-modify-write; only the runs that touch the wave's first or last
// lane (they may continue in the neighbouring wave) use an atomic.
#include "hq_internal.h"

namespace {

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

constexpr int kTBlock = 256;
constexpr uint64_t kT = HQ_TILE_GROUPS;

unsigned tgrid(uint64_t lanes) {
    uint64_t b = (lanes + kTBlock - 1) / kTBlock;
    if (b < 1) b = 1;
    if (b > 256 * 64) b = 256 * 64;   // grid-stride beyond 64 workgroups per CU
    return (unsigned)b;
}

// The table of one launch: rows of 128 u64 per tile, tw words per tile.
struct TableK {
    uint64_t *tiles;
    uint64_t G, tw;
    uint32_t nr;     // match rows = n_max - 1 (slots 1 .. n_max - 1)
    uint32_t R;      // ring_len of the term mask
    uint32_t mask;   // 1: term-mask form (u16 row), 0: term-start form (u64 row, untouched)
    uint32_t flags;
};

// word offset of group g inside its tile's rows
__device__ __forceinline__ uint64_t tpos(uint64_t g) {
    const uint64_t i = g & (kT - 1);
    return 2 * (i & 63) + (i >> 6);
}
__device__ __forceinline__ uint64_t *trow(const TableK &t, uint64_t g, uint32_t row) {
    return t.tiles + (g / kT) * t.tw + (uint64_t)row * kT + tpos(g);
}
__device__ __forceinline__ uint16_t *tmask(const TableK &t, uint64_t g) {
    return reinterpret_cast<uint16_t *>(t.tiles + (g / kT) * t.tw + (uint64_t)(t.nr + 2) * kT) +
           tpos(g);
}

__device__ __forceinline__ void count_skip(uint64_t *n_skipped, bool skip) {
    const uint64_t m = __ballot(skip);
    if (n_skipped && m && (threadIdx.x & 63) == (uint32_t)(__ffsll((long long)m) - 1))
        atomicAdd(reinterpret_cast<unsigned long long *>(n_skipped),
                  (unsigned long long)__popcll(m));
}

// Inclusive segmented scan over the wave: v = op(v of every earlier lane with the same key),
// valid because equal keys are adjacent (HQ_INGEST_GROUPED): if lane - off has this key, so has
// every lane in between.
template <bool SUM>
__device__ __forceinline__ uint64_t seg_scan(uint64_t key, uint64_t v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint64_t ko = __shfl_up(key, off);
        const uint64_t vo = __shfl_up(v, off);
        if (lane >= off && ko == key) v = SUM ? v + vo : (vo > v ? vo : v);
    }
    return v;
}

// The lane that applies its key's run (the run's last lane) and whether the run may continue in
// a neighbouring wave (then an atomic applies it).
struct RunTail {
    bool tail, edge;
};
__device__ __forceinline__ RunTail run_tail(uint64_t key) {
    const int lane = threadIdx.x & 63;
    const uint64_t next = __shfl_down(key, 1);
    RunTail r;
    r.tail = lane == 63 || next != key;
    r.edge = key == __shfl(key, 0) || key == __shfl(key, 63);
    return r;
}

// the term-mask bits of the entries (prev, prev + n] (appendEntries at the leader's term)
__device__ __forceinline__ uint32_t append_bits(uint64_t prev, uint64_t n, uint32_t R) {
    if (n >= R) return R >= 32 ? 0xFFFFFFFFu : ((1u << R) - 1u);
    uint32_t bits = 0;
    for (uint64_t k = 1; k <= n; ++k) bits |= 1u << ((prev + k) & (R - 1));
    return bits;
}

// OR the u16 mask bits of group g: plain (the lane owns the u16) or atomic on the 32-bit word
// that holds it (positions 2i, 2i + 1 share a word)
__device__ __forceinline__ void or_mask(const TableK &t, uint64_t g, uint32_t bits, bool atomic) {
    uint16_t *m = tmask(t, g);
    if (atomic) {
        const uint64_t p = tpos(g);
        atomicOr(reinterpret_cast<unsigned int *>(m - (p & 1)), (bits & 0xFFFFu) << (16 * (p & 1)));
    } else {
        *m = (uint16_t)(*m | bits);
    }
}

// Records per lane of the ingest kernels: a wave takes V consecutive chunks of 64 records per
// iteration (lane l holds record l of each chunk) and issues every chunk's loads before the
// first dependent step, so a wave keeps V record loads and then V table loads in flight instead
// of one (the grouped ingest is a chain of dependent steps: record load -> scan -> table load
// -> store; with one record per lane its memory latency, not bandwidth, set the rate).
#ifndef HQ_INGEST_V
#define HQ_INGEST_V 4
#endif
constexpr int kIV = HQ_INGEST_V;

// One launch applies match raises: key = group << 8 | slot (match form) or group << 4 | slot
// (lag form), value = the acknowledged index. LAG: 8-byte records, index = lastIndex - lag.
// MODE: kAtomic (any batch), kGrouped (HQ_INGEST_GROUPED), kUnique (HQ_INGEST_UNIQUE: every key
// at most once, so each record is a plain read-modify-write of its own word)
enum IngestMode { kAtomic = 0, kGrouped = 1, kUnique = 2 };
template <int MODE, bool LAG>
__global__ __launch_bounds__(kTBlock) void k_table_ingest(const uint64_t *u, uint64_t count,
                                                          TableK t, uint64_t *n_skipped) {
    constexpr bool GROUPED = MODE == kGrouped;
    const uint64_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (kTBlock / 64) + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (kTBlock / 64);
    constexpr int SH = LAG ? 4 : 8;   // slot bits of the key
    for (uint64_t base = wave * 64 * kIV; base < count; base += nwaves * 64 * kIV) {
        uint64_t key[kIV], v[kIV], lag[kIV];
        bool in[kIV], ok[kIV];
#pragma unroll
        for (int c = 0; c < kIV; ++c) {
            const uint64_t i = base + 64 * c + lane;
            in[c] = i < count;
            key[c] = ~0ull;
            v[c] = lag[c] = 0;
            if (in[c]) {
                if constexpr (LAG) {
                    const uint64_t x = __builtin_nontemporal_load(u + i);
                    key[c] = x >> 28;   // group << 4 | slot
                    lag[c] = x & 0x0FFFFFFFull;
                } else {
                    const u64x2 x = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(u) + i);
                    key[c] = x.x;
                    v[c] = x.y;
                }
            }
        }
        bool skip[kIV];
#pragma unroll
        for (int c = 0; c < kIV; ++c) {
            const uint64_t g = key[c] >> SH, s = key[c] & ((1u << SH) - 1);
            // slot 0 is the leader: its match is lastIndex, no ReplicateResp comes from self
            ok[c] = in[c] && g < t.G && s >= 1 && s <= t.nr;
            skip[c] = in[c] && !ok[c];
        }
        if constexpr (LAG) {
            uint64_t last[kIV];
#pragma unroll
            for (int c = 0; c < kIV; ++c) last[c] = ok[c] ? *trow(t, key[c] >> 4, t.nr + 1) : 0;
#pragma unroll
            for (int c = 0; c < kIV; ++c) {
                // an ack above lastIndex is skipped; its value 0 leaves the run's max alone
                const bool above = ok[c] && lag[c] > last[c];
                v[c] = ok[c] && !above ? last[c] - lag[c] : 0;
                skip[c] |= above;
            }
        }
        if constexpr (GROUPED) {
            bool tail[kIV], edge[kIV];
            uint64_t *p[kIV], old[kIV];
#pragma unroll
            for (int c = 0; c < kIV; ++c) {
                v[c] = seg_scan<false>(key[c], v[c]);
                const RunTail r = run_tail(key[c]);
                tail[c] = ok[c] && r.tail;
                edge[c] = r.edge;
            }
#pragma unroll
            for (int c = 0; c < kIV; ++c) {
                p[c] = trow(t, key[c] >> SH, (uint32_t)(key[c] & ((1u << SH) - 1)) - 1);
#ifdef HQ_INGEST_NOLOAD      // timing probe (tools/lib_ingnoload): no table loads, wrong output
                old[c] = 0;
#else
                old[c] = tail[c] && !edge[c] ? *p[c] : 0;
#endif
            }
#pragma unroll
            for (int c = 0; c < kIV; ++c) {
                if (!tail[c]) continue;
#ifdef HQ_INGEST_NOSTORE     // timing probe (tools/lib_ingnostore): no table stores, wrong output
                if (v[c] == 0x5A5A5A5A5A5A5A5Aull) *p[c] = old[c];   // (keeps the loads live)
#else
                if (edge[c]) atomicMax(reinterpret_cast<unsigned long long *>(p[c]),
                                       (unsigned long long)v[c]);
                else if (v[c] > old[c]) *p[c] = v[c];
#endif
            }
        } else if constexpr (MODE == kUnique) {
            uint64_t *p[kIV], old[kIV];
#pragma unroll
            for (int c = 0; c < kIV; ++c) {        // every table load first, then the stores
                p[c] = trow(t, key[c] >> SH, (uint32_t)(key[c] & ((1u << SH) - 1)) - 1);
                old[c] = ok[c] && !skip[c] ? *p[c] : ~0ull;
            }
#pragma unroll
            for (int c = 0; c < kIV; ++c)
                if (ok[c] && !skip[c] && v[c] > old[c]) *p[c] = v[c];
        } else {
#pragma unroll
            for (int c = 0; c < kIV; ++c)
                if (ok[c] && !skip[c])
                    atomicMax(reinterpret_cast<unsigned long long *>(
                                  trow(t, key[c] >> SH, (uint32_t)(key[c] & ((1u << SH) - 1)) - 1)),
                              (unsigned long long)v[c]);
        }
#pragma unroll
        for (int c = 0; c < kIV; ++c) count_skip(n_skipped, skip[c]);
    }
}

// ---------------------------------------------------------------- binned ingest ---------------
// Records in any order, many per table slot (HQ_INGEST_BINNED, chosen by default for dense
// batches): a random 8-byte read-modify-write or 64-bit atomic per record moves whole lines at
// the memory side's random-access rate (one atomic per record: 10 % of HBM peak). Two streaming
// passes instead, no global atomics:
//   k_bin    each workgroup takes a chunk of kBinChunk records, counts them per bucket (a bucket =
//            2^tpb_shift consecutive tiles) in LDS, and writes the chunk back bucket by bucket as
//            8-byte entries (bucket-local key << 48 | index or lag), with each bucket's offset and
//            count in the chunk (meta[chunk][bucket]);
//   k_apply  one workgroup per bucket loads the bucket's match rows (and, for lags, its
//            lastIndex row) into LDS, applies every chunk's entries of the bucket with LDS 64-bit
//            max, and writes the rows back: every table line is read and written once per launch.
// The max commutes, so the result equals the sequential application in any order. Indexes of 2^48
// or more (never a real log index) do not fit an entry: k_bin applies those few with a global
// atomic, which k_apply's later read of the row sees (kernel boundary).
constexpr int kBinThreads = 1024;                                 // k_apply's workgroup
constexpr int kBinT = 1024;                                       // k_bin's workgroup
// records per thread and chunk (HQ_BIN_PER 16, chunks of 16 Ki with whole-wave segments in
// k_apply, HQ_APPLY_SEG 64: k_bin then holds 16 records' keys, values, buckets and ranks and
// spills 103 VGPRs — not measured)
#ifndef HQ_BIN_PER
#define HQ_BIN_PER 8
#endif
constexpr int kBinPer = HQ_BIN_PER;
constexpr uint64_t kBinChunk = (uint64_t)kBinT * kBinPer;         // 8192 records per chunk
constexpr uint32_t kBinMaxBuckets = 8192;                         // k_bin: 64 KB + 8 B per bucket

// HQ_BIN_PROF (tools/binprof.hip only): per-workgroup phase timestamps (wall_clock64) of the
// binned kernels' first loop iteration
#ifdef HQ_BIN_PROF
__device__ unsigned long long g_bin_prof[2][8192][8];
#define BIN_T(K, P) \
    if (threadIdx.x == 0 && blockIdx.x < 8192) g_bin_prof[K][blockIdx.x][P] = wall_clock64()
#else
#define BIN_T(K, P)
#endif

struct BinK {
    uint64_t *ent;       // [chunk][kBinChunk] entries, bucket order inside a chunk
    uint32_t *meta;      // [chunk][B]: offset | count << 16 of the bucket in the chunk
    uint64_t ntiles;
    uint32_t B;          // buckets
    uint32_t tpb_shift;  // tiles per bucket = 1 << tpb_shift
    uint32_t rows;       // LDS rows per tile in k_apply: the match rows (+ lastIndex for lags)
    uint32_t nchunks;    // chunks of this launch
};

// A workgroup barrier for LDS only: this wave's LDS operations done, then s_barrier.
// __syncthreads' release fence also waits for every outstanding global load and store of the
// wave (one vmcnt on gfx9), which would turn a prefetch issued before the barrier into a stall.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// exclusive scan of n (<= 8192) u32 counts in LDS into out (may not alias), block-wide; returns
// the total to every thread. Every thread must call it.
template <int T>
__device__ uint32_t block_scan(const uint32_t *in, uint32_t *out, uint32_t n, uint32_t *wtot) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint32_t per = (n + T - 1) / T, b0 = tid * per, b1 = min(b0 + per, n);
    uint32_t s = 0;
    for (uint32_t b = b0; b < b1; ++b) s += in[b];
    uint32_t x = s;                              // inclusive scan over the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        x += lane >= (uint32_t)d ? y : 0u;
    }
    if (lane == 63) wtot[wv] = x;
    lds_barrier();
    uint32_t wbase = 0, total = 0;
    for (uint32_t w = 0; w < T / 64; ++w) {
        const uint32_t v = wtot[w];
        wbase += w < wv ? v : 0u;
        total += v;
    }
    uint32_t run = wbase + x - s;
    for (uint32_t b = b0; b < b1; ++b) {
        out[b] = run;
        run += in[b];
    }
    lds_barrier();                             // wtot may be reused after the call
    return total;
}

// a chunk's records into registers: every load issued at once, unconditionally (a load inside
// `if (i < count)` is compiled as a branch that waits for it, one memory latency per record);
// positions past the end load the last record (the decode masks them)
template <bool LAG>
__device__ __forceinline__ void bin_load(const uint64_t *u, uint64_t count, uint64_t base,
                                         uint64_t (&key)[kBinPer], uint64_t (&v)[kBinPer]) {
#pragma unroll
    for (int r = 0; r < kBinPer; ++r) {
        const uint64_t i = base + (uint64_t)r * kBinT + threadIdx.x;
        const uint64_t ic = i < count ? i : count - 1;
        if constexpr (LAG) {
            const uint64_t x = __builtin_nontemporal_load(u + ic);
            key[r] = x >> 28;                          // group << 4 | slot
            v[r] = x & 0x0FFFFFFFull;                  // lag
        } else {
            const u64x2 x = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(u) + ic);
            key[r] = x.x;
            v[r] = x.y;                                // index
        }
    }
}

// One chunk k of k_bin: count its records per bucket, scan, write its meta row, scatter the
// entries into LDS bucket by bucket and write them out (key / v: its records, loaded earlier;
// then the records at `next`, unless ~0, are loaded into them)
template <bool LAG>
__device__ __forceinline__ void bin_chunk(uint64_t k, uint64_t count, const TableK &t,
                                          const BinK &bk, uint64_t *n_skipped, uint64_t *lds,
                                          uint64_t (&key)[kBinPer], uint64_t (&v)[kBinPer],
                                          uint64_t next, const uint64_t *u) {
    uint64_t *stage = lds;                                           // kBinChunk entries
    uint32_t *hist = reinterpret_cast<uint32_t *>(lds + kBinChunk);  // [B]
    uint32_t *hoff = hist + bk.B;                                    // [B]
    uint32_t *wtot = hoff + bk.B;                                    // [16]
    const uint32_t tid = threadIdx.x;
    constexpr int SH = LAG ? 4 : 8;
    const uint64_t base = k * kBinChunk;
    uint32_t bb[kBinPer], rk[kBinPer];
    for (uint32_t b = tid; b < bk.B; b += kBinT) hist[b] = 0;
    lds_barrier();
#pragma unroll
    for (int r = 0; r < kBinPer; ++r) {
        const bool in = base + (uint64_t)r * kBinT + tid < count;
        const uint64_t g = key[r] >> SH, s = key[r] & ((1u << SH) - 1);
        const bool ok = in && g < t.G && s >= 1 && s <= t.nr;
        count_skip(n_skipped, in && !ok);
        bb[r] = 0xFFFFFFFFu;
        rk[r] = 0;
        if (!ok) continue;
        if (!LAG && (v[r] >> 48)) {                    // no room in an entry: applied now
            atomicMax(reinterpret_cast<unsigned long long *>(trow(t, g, (uint32_t)s - 1)),
                      (unsigned long long)v[r]);
            continue;
        }
        const uint32_t b = (uint32_t)((g >> 7) >> bk.tpb_shift);
        const uint64_t lg = g - ((uint64_t)b << (7 + bk.tpb_shift));
        v[r] |= (lg << 3 | (s - 1)) << 48;             // the entry
        bb[r] = b;
        rk[r] = atomicAdd(&hist[b], 1u);               // LDS
    }
    lds_barrier();
    if (k == blockIdx.x) BIN_T(0, 1);
    const uint32_t total = block_scan<kBinT>(hist, hoff, bk.B, wtot);
    for (uint32_t b = tid; b < bk.B; b += kBinT)
        bk.meta[k * bk.B + b] = hoff[b] | hist[b] << 16;
#pragma unroll
    for (int r = 0; r < kBinPer; ++r)
        if (bb[r] != 0xFFFFFFFFu) stage[hoff[bb[r]] + rk[r]] = v[r];
    if (next != ~0ull) bin_load<LAG>(u, count, next, key, v);   // in flight from here on
    lds_barrier();
    if (k == blockIdx.x) BIN_T(0, 2);
    uint64_t *dst = bk.ent + base;
    for (uint32_t j = 2 * tid; j < total; j += 2 * kBinT) {
        if (j + 1 < total) {
            u64x2 x;
            x.x = stage[j];
            x.y = stage[j + 1];
            *reinterpret_cast<u64x2 *>(dst + j) = x;
        } else {
            dst[j] = stage[j];
        }
    }
    lds_barrier();                                     // stage and hist are reused next chunk
    if (k == blockIdx.x) BIN_T(0, 3);
}

// Persistent over the chunks (k = blockIdx.x, + gridDim.x, ...): the next chunk's records are
// loaded (into the registers this chunk's entries no longer need) before this chunk is written
template <bool LAG>
__global__ __launch_bounds__(kBinT) void k_bin(const uint64_t *u, uint64_t count, TableK t,
                                               BinK bk, uint64_t *n_skipped) {
    extern __shared__ uint64_t lds[];
    uint64_t key[kBinPer], v[kBinPer];
    BIN_T(0, 0);
    uint64_t k = blockIdx.x;
    if (k < bk.nchunks) bin_load<LAG>(u, count, k * kBinChunk, key, v);
    for (; k < bk.nchunks; k += gridDim.x)
        bin_chunk<LAG>(k, count, t, bk, n_skipped, lds, key, v,
                       k + gridDim.x < bk.nchunks ? (k + gridDim.x) * kBinChunk : ~0ull, u);
    BIN_T(0, 7);
}

// A/B builds (tools/): HQ_BIN_AB 1 = k_apply with plain LDS stores instead of the LDS max,
// 2 = without the entry gather, 3 = the rows' read and write alone; HQ_BIN_TPB_SHIFT = the
// largest region (2^shift tiles) tried
#ifndef HQ_BIN_AB
#define HQ_BIN_AB 0
#endif
#ifndef HQ_BIN_TPB_SHIFT
#define HQ_BIN_TPB_SHIFT 6
#endif
// one entry applied to the bucket's rows in LDS (64-bit LDS max); returns true for an ack above
// lastIndex (lags), which is skipped
template <bool LAG>
__device__ __forceinline__ bool bin_apply(const TableK &t, uint32_t R, uint64_t *rows, uint64_t e) {
    if (e == ~0ull) return false;
    const uint32_t lk = (uint32_t)(e >> 48);
    uint64_t v = e & 0xFFFFFFFFFFFFull;
    const uint32_t gl = lk >> 3, s1 = lk & 7, tl = gl >> 7;
    const uint32_t pos = (uint32_t)tpos(gl & 127);
    if constexpr (LAG) {
        const uint64_t last = rows[(tl * R + t.nr) * kT + pos];
        if (v > last) return true;
        v = last - v;
    }
#if HQ_BIN_AB == 1
    rows[(tl * R + s1) * kT + pos] = v;
#else
    atomicMax(reinterpret_cast<unsigned long long *>(rows + (tl * R + s1) * kT + pos),
              (unsigned long long)v);
#endif
    return false;
}

#ifndef HQ_APPLY_SEG
#define HQ_APPLY_SEG 32
#endif
constexpr int kApplyEnt = 6;                              // entries per thread and round
constexpr uint32_t kApplyLds = 128 * 1024;                // a bucket's rows in k_apply's LDS
constexpr int kApplyRows = (int)(kApplyLds / 16 / kBinThreads);  // row pairs per thread (8)
// T threads per k_apply workgroup: a bucket's rows take up to kApplyRows * 16 * T bytes of LDS
// (T = 1024: 128 KB, one workgroup per CU; T = 512: 64 KB, two per CU, so that one's latency
// phases can overlap the other's streaming)
template <int T>
constexpr uint32_t apply_lds() { return (uint32_t)kApplyRows * 16 * T; }

// the rows of bucket b (tile-major; row r < nr = match slot r + 1, row nr = lastIndex for lags)
// into registers, every load at once
template <int T>
__device__ __forceinline__ void apply_load_rows(const TableK &t, const BinK &bk, uint32_t b,
                                                u64x2 (&rv)[kApplyRows]) {
    const uint64_t tile0 = (uint64_t)b << bk.tpb_shift;
    const uint32_t nt = (uint32_t)min((uint64_t)1 << bk.tpb_shift, bk.ntiles - tile0);
    const uint32_t R = bk.rows, pairs = nt * R * 64;
#pragma unroll
    for (int k = 0; k < kApplyRows; ++k) {   // unconditional loads (see bin_load), clamped
        uint32_t w = threadIdx.x + (uint32_t)k * T;
        w = w < pairs ? w : pairs - 1;
        const uint32_t tl = w / (R * 64), r = (w / 64) % R, x = 2 * (w % 64);
        const uint32_t src = r < t.nr ? r : t.nr + 1;
        rv[k] = *reinterpret_cast<const u64x2 *>(t.tiles + (tile0 + tl) * t.tw +
                                                 (uint64_t)src * kT + x);
    }
}

// Persistent over the buckets, XCD-aware: workgroup i runs on XCD i % 8 and takes the buckets
// x * per + j, x * per + j + W, ... (x = i % 8, j = i / 8, W workgroups per XCD), so that the W
// workgroups of an XCD work on consecutive buckets at any time (the lines two neighbouring
// buckets share — an entry segment that straddles them, a meta row — are served by that XCD's L2
// once); the next bucket's rows are loaded while this one's entries are applied and its rows
// written back
template <bool LAG, int T = kBinThreads>
__global__ __launch_bounds__(T) void k_apply(TableK t, BinK bk, uint64_t *n_skipped) {
    extern __shared__ uint64_t lds[];
    uint64_t *rows = lds;                                                    // [nt][R][128]
    const uint32_t tid = threadIdx.x, R = bk.rows;
    uint32_t *M = reinterpret_cast<uint32_t *>(lds + ((size_t)R << (7 + bk.tpb_shift)));
    constexpr int NE = LAG ? 4 : kApplyEnt;    // (the lag form's extra row reads take registers)
    const uint32_t per = (bk.B + 7) / 8, x = blockIdx.x % 8, W = gridDim.x / 8;
    uint32_t j = blockIdx.x / 8;
    u64x2 rv[kApplyRows];
    BIN_T(1, 0);
    if (j < per && x * per + j < bk.B) apply_load_rows<T>(t, bk, x * per + j, rv);
    for (; j < per && x * per + j < bk.B; j += W) {
        const uint32_t b = x * per + j;
        const uint64_t tile0 = (uint64_t)b << bk.tpb_shift;
        const uint32_t nt = (uint32_t)min((uint64_t)1 << bk.tpb_shift, bk.ntiles - tile0);
        const uint32_t pairs = nt * R * 64;
        // every chunk's (offset, count) of this bucket into LDS: one load round for all of them
        for (uint32_t c = tid; c < bk.nchunks; c += T)
            M[c] = HQ_BIN_AB >= 2 ? 0u : bk.meta[(uint64_t)c * bk.B + b];
#pragma unroll
        for (int k = 0; k < kApplyRows; ++k) {
            const uint32_t w = tid + (uint32_t)k * T;
            if (w < pairs) {
                const uint32_t tl = w / (R * 64), r = (w / 64) % R, xx = 2 * (w % 64);
                rows[(tl * R + r) * kT + xx] = rv[k].x;
                rows[(tl * R + r) * kT + xx + 1] = rv[k].y;
            }
        }
        __syncthreads();                               // (waits for the meta loads too)
        if (j == blockIdx.x / 8) BIN_T(1, 1);
        // the entries: each half-wave takes one chunk's segment of the bucket at a time (lane l
        // its l-th entry; a segment averages kBinChunk / B entries), NE chunks per round with
        // every entry load issued before the first LDS max; segments longer than 32 entries
        // finish in a loop of their own
        // (HQ_APPLY_SEG = 64: a whole wave per segment, for chunks of 16 Ki records)
        constexpr uint32_t kSeg = HQ_APPLY_SEG;
        const uint32_t wv = tid >> 6, h = kSeg == 32 ? (tid >> 5) & 1 : 0, l = tid & (kSeg - 1);
        constexpr uint32_t kHalves = (64 / kSeg) * T / 64;   // segments in flight
        for (uint32_t c0 = 0; c0 < bk.nchunks; c0 += kHalves * NE) {
            uint32_t m[NE];
            uint64_t ent[NE];
#pragma unroll
            for (int u = 0; u < NE; ++u) {           // unconditional loads (see bin_load)
                const uint32_t c = c0 + (uint32_t)u * kHalves + (64 / kSeg) * wv + h;
                const uint32_t cc = c < bk.nchunks ? c : 0;
                m[u] = c < bk.nchunks ? M[c] : 0u;
                ent[u] = __builtin_nontemporal_load(bk.ent + (uint64_t)cc * kBinChunk +
                                                    (m[u] & 0xFFFFu) + l);
            }
            bool skip[NE];
#pragma unroll
            for (int u = 0; u < NE; ++u)
                skip[u] = bin_apply<LAG>(t, R, rows, l < (m[u] >> 16) ? ent[u] : ~0ull);
            if constexpr (LAG) {
#pragma unroll
                for (int u = 0; u < NE; ++u) count_skip(n_skipped, skip[u]);
            }
#pragma unroll
            for (int u = 0; u < NE; ++u) {           // the rare segments beyond 32 entries
                const uint32_t c = c0 + (uint32_t)u * kHalves + (64 / kSeg) * wv + h;
                for (uint32_t k = l + kSeg; k < (m[u] >> 16); k += kSeg) {
                    const bool sk = bin_apply<LAG>(
                        t, R, rows, bk.ent[(uint64_t)c * kBinChunk + (m[u] & 0xFFFFu) + k]);
                    if (LAG && sk && n_skipped)
                        atomicAdd(reinterpret_cast<unsigned long long *>(n_skipped), 1ull);
                }
            }
        }
        // the next bucket's rows, in flight while these are written back (issued after this
        // bucket's entry loads: the in-order load counter would make those wait for them)
        if (j + W < per && b + W < bk.B) apply_load_rows<T>(t, bk, b + W, rv);
        lds_barrier();
        if (j == blockIdx.x / 8) BIN_T(1, 2);
        // the match rows back
        const uint32_t mpairs = nt * t.nr * 64;
        for (uint32_t w = tid; w < mpairs; w += T) {
            const uint32_t tl = w / (t.nr * 64), r = (w / 64) % t.nr, xx = 2 * (w % 64);
            u64x2 v;
            v.x = rows[(tl * R + r) * kT + xx];
            v.y = rows[(tl * R + r) * kT + xx + 1];
            *reinterpret_cast<u64x2 *>(t.tiles + (tile0 + tl) * t.tw + (uint64_t)r * kT + xx) = v;
        }
        lds_barrier();                                 // the rows' LDS is reused next bucket
        if (j == blockIdx.x / 8) BIN_T(1, 3);
    }
    BIN_T(1, 7);
}

// one group's append of its run: lastIndex raised to new_last (16-byte form) or advanced by n
// (count form); the term-mask bits of the new entries set
template <bool COUNT>
__device__ __forceinline__ void apply_append(const TableK &t, uint64_t g, uint64_t v, bool atomic) {
    uint64_t *lp = trow(t, g, t.nr + 1);
    uint64_t prev, n;
    if (COUNT) {
        prev = atomic ? (uint64_t)atomicAdd(reinterpret_cast<unsigned long long *>(lp),
                                            (unsigned long long)v)
                      : *lp;
        if (!atomic) *lp = prev + v;
        n = v;
    } else {
        prev = atomic ? (uint64_t)atomicMax(reinterpret_cast<unsigned long long *>(lp),
                                            (unsigned long long)v)
                      : *lp;
        if (v <= prev) return;   // a stale append leaves the group unchanged
        if (!atomic) *lp = v;
        n = v - prev;
    }
    if (t.mask) or_mask(t, g, append_bits(prev, n, t.R), atomic);
}

// COUNT = 0: hq_append_update (group, new_last); 1: 8-byte group << 32 | n. Like the ingest, a
// wave takes kIV chunks of 64 records and issues every record load before the first dependent
// step (records read over PCIe from pinned host memory by the zero-copy pipeline would otherwise
// cost one round trip per record and lane).
template <bool COUNT, int MODE>
__global__ __launch_bounds__(kTBlock) void k_table_append(const uint64_t *u, uint64_t count,
                                                          TableK t, uint64_t *n_skipped) {
    constexpr bool GROUPED = MODE == kGrouped;
    const uint64_t lane = threadIdx.x & 63;
    const uint64_t wave = (uint64_t)blockIdx.x * (kTBlock / 64) + (threadIdx.x >> 6);
    const uint64_t nwaves = (uint64_t)gridDim.x * (kTBlock / 64);
    for (uint64_t base = wave * 64 * kIV; base < count; base += nwaves * 64 * kIV) {
        uint64_t key[kIV], v[kIV];
        bool in[kIV], ok[kIV];
#pragma unroll
        for (int c = 0; c < kIV; ++c) {
            const uint64_t i = base + 64 * c + lane;
            in[c] = i < count;
            key[c] = ~0ull;
            v[c] = 0;
            ok[c] = false;
            if (in[c]) {
                if (COUNT) {
                    const uint64_t x = __builtin_nontemporal_load(u + i);
                    key[c] = x >> 32;
                    v[c] = x & 0xFFFFFFFFull;
                    ok[c] = key[c] < t.G && v[c] != 0;
                } else {
                    const u64x2 x = __builtin_nontemporal_load(reinterpret_cast<const u64x2 *>(u + 2 * i));
                    key[c] = x.x;
                    v[c] = x.y;
                    ok[c] = key[c] < t.G;
                }
            }
        }
#pragma unroll
        for (int c = 0; c < kIV; ++c) {
            if constexpr (GROUPED) {
                // a skipped record keeps its key but adds nothing (0 is the sum's and max's
                // identity); a run crossing a chunk edge is applied atomically like one crossing
                // a wave edge
                const bool keyok = key[c] < t.G;
                const uint64_t x = seg_scan<COUNT>(key[c], ok[c] ? v[c] : 0);
                const RunTail r = run_tail(key[c]);
                if (keyok && r.tail && x) apply_append<COUNT>(t, key[c], x, r.edge);
            } else {
                if (ok[c]) apply_append<COUNT>(t, key[c], v[c], MODE == kAtomic);   // unique: plain
            }
            count_skip(n_skipped, in[c] && !ok[c]);
        }
    }
}

// the committed row of every tile back in group order: lane i of a wave reads the 16 bytes of
// groups i and i + 64 and writes them to their two column positions
__global__ __launch_bounds__(kTBlock) void k_table_committed(TableK t, uint64_t *out) {
    const uint64_t ntiles = (t.G + kT - 1) / kT;
    const uint64_t lane = threadIdx.x & 63;
    const uint64_t nw = (uint64_t)gridDim.x * (kTBlock / 64);
    for (uint64_t tile = (uint64_t)blockIdx.x * (kTBlock / 64) + (threadIdx.x >> 6); tile < ntiles;
         tile += nw) {
        const u64x2 v = __builtin_nontemporal_load(
            reinterpret_cast<const u64x2 *>(t.tiles + tile * t.tw + (uint64_t)t.nr * kT + 2 * lane));
        const uint64_t ga = tile * kT + lane, gb = ga + 64;
        if (ga < t.G) out[ga] = v.x;
        if (gb < t.G) out[gb] = v.y;
    }
}

int table_k(hq_ctx *ctx, const char *what, uint64_t *tiles, uint64_t G, uint32_t n_max,
            uint32_t form, uint32_t ring_len, uint32_t flags, TableK &t) {
    if (!tiles || !hq::aligned16(tiles))
        return hq::fail(ctx, HQ_E_INVAL, std::string(what) + ": tiles NULL or not 16-byte aligned");
    if (n_max < 1 || n_max > HQ_MAX_VOTERS)
        return hq::fail(ctx, HQ_E_INVAL, std::string(what) + ": n_max must be 1..8");
    if (form != HQ_FORM_TERM_START && form != HQ_FORM_TERM_MASK)
        return hq::fail(ctx, HQ_E_INVAL, std::string(what) + ": the table holds the term-start or "
                                                              "term-mask form");
    if (form == HQ_FORM_TERM_MASK &&
        (ring_len < 1 || ring_len > 16 || (ring_len & (ring_len - 1))))
        return hq::fail(ctx, HQ_E_INVAL, std::string(what) + ": ring_len must be a power of two <= 16");
    if (flags & ~(HQ_INGEST_GROUPED | HQ_INGEST_UNIQUE | HQ_INGEST_ATOMIC | HQ_INGEST_BINNED))
        return hq::fail(ctx, HQ_E_INVAL, std::string(what) + ": unknown flags");
    t.tiles = tiles;
    t.G = G;
    t.tw = hq_commit_tile_words_for(n_max, form, HQ_LAYOUT_TILES_LEADER);
    t.nr = n_max - 1;
    t.R = ring_len ? ring_len : 16;
    t.mask = form == HQ_FORM_TERM_MASK;
    t.flags = flags;
    return HQ_OK;
}

// The binned ingest's geometry for this batch, or false when the table is too large for it
// (more buckets than k_bin's LDS counts hold).
bool bin_plan(const hq_ctx *ctx, const TableK &t, uint64_t count, bool lag, BinK &bk,
              size_t &lds_bin, size_t &lds_apply, size_t &ws) {
    bk.ntiles = (t.G + kT - 1) / kT;
    bk.rows = t.nr + (lag ? 1u : 0u);
    const uint64_t chunks = (count + kBinChunk - 1) / kBinChunk;
    bk.nchunks = (uint32_t)std::min<uint64_t>(chunks, ctx->bin_launch_chunks);
    // k_apply's LDS: the bucket's rows, then a meta word per chunk
    const size_t meta_lds = 4 * (size_t)bk.nchunks;
    uint32_t sh = std::min<uint32_t>(HQ_BIN_TPB_SHIFT, ctx->bin_tpb_shift);   // <= 64 tiles
                                                       // (16-bit entry keys)
    const size_t cap = ctx->bin_apply_threads == 512 ? apply_lds<512>() : apply_lds<kBinThreads>();
    const size_t per_cu = ctx->bin_apply_threads == 512 ? 80 * 1024 : 160 * 1024;
    auto fits = [&](uint32_t sh) {
        const size_t rows = (size_t)bk.rows << (10 + sh);
        return rows <= cap && rows + meta_lds <= per_cu;
    };
    while (sh > 0 && !fits(sh)) --sh;
    if (!fits(sh)) return false;
    bk.tpb_shift = sh;
    const uint64_t B = (bk.ntiles + (1ull << sh) - 1) >> sh;
    if (B > kBinMaxBuckets || B == 0) return false;
    bk.B = (uint32_t)B;
    lds_bin = kBinChunk * 8 + 8 * (size_t)bk.B + 64;
    lds_apply = ((size_t)bk.rows << (10 + sh)) + meta_lds;
    // + 64 entries of padding: k_apply's unconditional loads read up to 31 entries past the last
    // chunk's last segment, which must stay inside the allocation
    ws = (size_t)bk.nchunks * kBinChunk * 8 + (size_t)bk.nchunks * bk.B * 4 + 64 * 8;
    return true;
}

// dense batches (>= 1 record per 8 table slots, >= 64 Ki records) in any order go binned
bool bin_default(const TableK &t, uint64_t count) {
    return count >= (1u << 16) && count * 8 >= t.G * t.nr;
}

template <bool LAG>
int ingest_binned(hq_ctx *ctx, const char *what, const uint64_t *u, uint64_t count, TableK &t,
                  BinK bk, size_t lds_bin, size_t lds_apply, size_t ws, uint64_t *n_skipped) {
    if (ctx->bin_ws_bytes < ws) {
        int rc = hq::check_hip(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
        if (rc) return rc;
        if (ctx->bin_ws) (void)hipFree(ctx->bin_ws);
        ctx->bin_ws = nullptr;
        ctx->bin_ws_bytes = 0;
        rc = hq::check_hip(ctx, hipMalloc(&ctx->bin_ws, ws), "hipMalloc(binned ingest)");
        if (rc) return rc;
        ctx->bin_ws_bytes = ws;
    }
    bk.ent = static_cast<uint64_t *>(ctx->bin_ws);
    bk.meta = reinterpret_cast<uint32_t *>(bk.ent + (size_t)bk.nchunks * kBinChunk);
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&k_bin<LAG>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bin);
    const bool half = ctx->bin_apply_threads == 512;
    (void)hipFuncSetAttribute(half ? reinterpret_cast<const void *>(&k_apply<LAG, 512>)
                                   : reinterpret_cast<const void *>(&k_apply<LAG>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_apply);
    const uint64_t per = (uint64_t)bk.nchunks * kBinChunk;   // records per launch pair
    for (uint64_t r0 = 0; r0 < count; r0 += per) {
        const uint64_t n = std::min(per, count - r0);
        BinK b = bk;
        b.nchunks = (uint32_t)((n + kBinChunk - 1) / kBinChunk);
        hipLaunchKernelGGL(k_bin<LAG>, dim3(std::min<uint32_t>(b.nchunks, ctx->bin_grid)),
                           dim3(kBinT), lds_bin, ctx->stream, u + r0 * (LAG ? 1 : 2), n, t,
                           b, n_skipped);
        int rc = hq::post_launch(ctx, what);
        if (!rc) rc = hq::pre_launch(ctx);
        if (rc) return rc;
        const dim3 ag(8 * std::min<uint32_t>((b.B + 7) / 8, ctx->bin_grid / 8));
        if (half)
            hipLaunchKernelGGL((k_apply<LAG, 512>), ag, dim3(512), lds_apply, ctx->stream, t, b,
                               n_skipped);
        else
            hipLaunchKernelGGL(k_apply<LAG>, ag, dim3(kBinThreads), lds_apply, ctx->stream, t, b,
                               n_skipped);
        rc = hq::post_launch(ctx, what);
        if (rc) return rc;
        if (r0 + per < count && (rc = hq::pre_launch(ctx))) return rc;
    }
    return HQ_OK;
}

// the ingest launch of any flags: binned (forced, or by default for a dense batch that is not
// grouped), else the per-record kernel
template <bool LAG>
int table_ingest(hq_ctx *ctx, const char *what, const uint64_t *u, uint64_t count, TableK &t,
                 uint32_t flags, uint64_t *n_skipped) {
    if ((flags & HQ_INGEST_ATOMIC) && (flags & (HQ_INGEST_BINNED | HQ_INGEST_GROUPED |
                                                HQ_INGEST_UNIQUE)))
        return hq::fail(ctx, HQ_E_INVAL, std::string(what) + ": HQ_INGEST_ATOMIC excludes the "
                                                              "other modes");
    if ((flags & HQ_INGEST_BINNED) && (flags & HQ_INGEST_GROUPED))
        return hq::fail(ctx, HQ_E_INVAL, std::string(what) + ": HQ_INGEST_BINNED excludes "
                                                              "HQ_INGEST_GROUPED");
    int rc = hq::pre_launch(ctx);
    if (rc) return rc;
    const bool want_bin = (flags & HQ_INGEST_BINNED) ||
                          (!(flags & (HQ_INGEST_ATOMIC | HQ_INGEST_GROUPED)) && bin_default(t, count));
    if (want_bin) {
        BinK bk{};
        size_t l1 = 0, l2 = 0, ws = 0;
        if (bin_plan(ctx, t, count, LAG, bk, l1, l2, ws))
            return ingest_binned<LAG>(ctx, what, u, count, t, bk, l1, l2, ws, n_skipped);
        if (flags & HQ_INGEST_BINNED)
            return hq::fail(ctx, HQ_E_INVAL, std::string(what) + ": table too large for "
                                                                  "HQ_INGEST_BINNED");
    }
    const dim3 grid(tgrid((count + kIV - 1) / kIV)), blk(kTBlock);
    if (flags & HQ_INGEST_UNIQUE)
        hipLaunchKernelGGL((k_table_ingest<kUnique, LAG>), grid, blk, 0, ctx->stream, u, count, t,
                           n_skipped);
    else if (flags & HQ_INGEST_GROUPED)
        hipLaunchKernelGGL((k_table_ingest<kGrouped, LAG>), grid, blk, 0, ctx->stream, u, count, t,
                           n_skipped);
    else
        hipLaunchKernelGGL((k_table_ingest<kAtomic, LAG>), grid, blk, 0, ctx->stream, u, count, t,
                           n_skipped);
    return hq::post_launch(ctx, "k_table_ingest");
}

}  // namespace

extern "C" {

int hq_table_ingest_match_dev(hq_ctx *ctx, const hq_match_update *updates, uint64_t count,
                              uint64_t *tiles, uint64_t G, uint32_t n_max, uint32_t form,
                              uint32_t flags, uint64_t *n_skipped) {
    if (!ctx) return HQ_E_INVAL;
    if (count == 0) return HQ_OK;
    TableK t;
    int rc = table_k(ctx, "hq_table_ingest_match_dev", tiles, G, n_max, form, 16, flags, t);
    if (rc) return rc;
    if (!updates || !hq::aligned16(updates))
        return hq::fail(ctx, HQ_E_INVAL, "hq_table_ingest_match_dev: updates NULL or misaligned");
    return table_ingest<false>(ctx, "hq_table_ingest_match_dev",
                               reinterpret_cast<const uint64_t *>(updates), count, t, flags,
                               n_skipped);
}

int hq_table_ingest_lag_dev(hq_ctx *ctx, const uint64_t *updates, uint64_t count,
                            uint64_t *tiles, uint64_t G, uint32_t n_max, uint32_t form,
                            uint32_t flags, uint64_t *n_skipped) {
    if (!ctx) return HQ_E_INVAL;
    if (count == 0) return HQ_OK;
    TableK t;
    int rc = table_k(ctx, "hq_table_ingest_lag_dev", tiles, G, n_max, form, 16, flags, t);
    if (rc) return rc;
    if (!updates) return hq::fail(ctx, HQ_E_INVAL, "hq_table_ingest_lag_dev: updates NULL");
    return table_ingest<true>(ctx, "hq_table_ingest_lag_dev", updates, count, t, flags, n_skipped);
}

static int table_append(hq_ctx *ctx, const char *what, const uint64_t *updates, uint64_t count,
                        bool counts, uint64_t *tiles, uint64_t G, uint32_t n_max, uint32_t form,
                        uint32_t ring_len, uint32_t flags, uint64_t *n_skipped) {
    if (!ctx) return HQ_E_INVAL;
    if (count == 0) return HQ_OK;
    TableK t;
    int rc = table_k(ctx, what, tiles, G, n_max, form, ring_len, flags, t);
    if (rc) return rc;
    if (flags & HQ_INGEST_BINNED)
        return hq::fail(ctx, HQ_E_INVAL, std::string(what) + ": HQ_INGEST_BINNED is for the ingests");
    if (!updates || (!counts && !hq::aligned16(updates)))
        return hq::fail(ctx, HQ_E_INVAL, std::string(what) + ": updates NULL or misaligned");
    if ((rc = hq::pre_launch(ctx))) return rc;
    const int mode = (flags & HQ_INGEST_UNIQUE) ? kUnique : (flags & HQ_INGEST_GROUPED) ? kGrouped
                                                                                         : kAtomic;
    const dim3 grid(tgrid((count + kIV - 1) / kIV)), blk(kTBlock);
#define HQ_APPEND(C, M) \
    hipLaunchKernelGGL((k_table_append<C, M>), grid, blk, 0, ctx->stream, updates, count, t, n_skipped)
    if (counts) {
        if (mode == kUnique) HQ_APPEND(true, kUnique);
        else if (mode == kGrouped) HQ_APPEND(true, kGrouped);
        else HQ_APPEND(true, kAtomic);
    } else {
        if (mode == kUnique) HQ_APPEND(false, kUnique);
        else if (mode == kGrouped) HQ_APPEND(false, kGrouped);
        else HQ_APPEND(false, kAtomic);
    }
#undef HQ_APPEND
    return hq::post_launch(ctx, "k_table_append");
}

int hq_table_append_dev(hq_ctx *ctx, const hq_append_update *updates, uint64_t count,
                        uint64_t *tiles, uint64_t G, uint32_t n_max, uint32_t form,
                        uint32_t ring_len, uint32_t flags, uint64_t *n_skipped) {
    return table_append(ctx, "hq_table_append_dev", reinterpret_cast<const uint64_t *>(updates),
                        count, false, tiles, G, n_max, form, ring_len, flags, n_skipped);
}

int hq_table_append_count_dev(hq_ctx *ctx, const uint64_t *updates, uint64_t count,
                              uint64_t *tiles, uint64_t G, uint32_t n_max, uint32_t form,
                              uint32_t ring_len, uint32_t flags, uint64_t *n_skipped) {
    return table_append(ctx, "hq_table_append_count_dev", updates, count, true, tiles, G, n_max,
                        form, ring_len, flags, n_skipped);
}

int hq_table_committed_dev(hq_ctx *ctx, const uint64_t *tiles, uint64_t G, uint32_t n_max,
                           uint32_t form, uint64_t *committed) {
    if (!ctx) return HQ_E_INVAL;
    if (G == 0) return HQ_OK;
    TableK t;
    int rc = table_k(ctx, "hq_table_committed_dev", const_cast<uint64_t *>(tiles), G, n_max, form,
                     16, 0, t);
    if (rc) return rc;
    if (!committed) return hq::fail(ctx, HQ_E_INVAL, "hq_table_committed_dev: committed NULL");
    if ((rc = hq::pre_launch(ctx))) return rc;
    const uint64_t ntiles = (G + kT - 1) / kT;
    hipLaunchKernelGGL(k_table_committed, dim3(tgrid(ntiles * 64)), dim3(kTBlock), 0, ctx->stream,
                       t, committed);
    return hq::post_launch(ctx, "k_table_committed");
}

}  // extern "C"
