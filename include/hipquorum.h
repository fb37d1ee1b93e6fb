/*
 * hipquorum.h — C-ABI of libhipquorum.so, the MI355X (gfx950) batched quorum engine for
 * dragonboat's multi-group Raft leader path.
 *
 * One call evaluates one quorum predicate for G independent Raft groups laid out as
 * structure-of-arrays in HBM. The entry points replace these reference interfaces
 * (paths relative to the dragonboat v3.3 tree):
 *
 *   hq_commit*        raft.tryCommit + sortMatchValues      internal/raft/raft.go:861-909
 *                     entryLog.tryCommit / term / commitTo  internal/raft/logentry.go:143-160,323-332,378-393
 *                     quorum / numVotingMembers             internal/raft/raft.go:368-378
 *   hq_readindex*     readIndex.confirm (quorum test)       internal/raft/readindex.go:77-116 (:84)
 *                     handleReadIndexLeaderConfirmation     internal/raft/raft.go:1740-1760
 *   hq_vote*          handleVoteResp / handleCandidateRequestVoteResp
 *                                                           internal/raft/raft.go:1062-1080,1968-1985
 *   hq_check_quorum*  leaderHasQuorum                       internal/raft/raft.go:380-390
 *   hq_readindex_multi*  readIndex.confirm prefix release   internal/raft/readindex.go:77-116
 *   hq_table_*        remote.tryUpdate, appendEntries       internal/raft/remote.go:123-133
 *                     (a device-resident progress table)    internal/raft/raft.go:911-922
 *   hq_worker_*       execEngine.processSteps ->            internal/execengine.go:923-1000
 *                     node.handleEvents -> raft.Handle      internal/node.go:1113-1157
 *   hq_events_*       the step worker's compact event stream (no reference counterpart)
 *   hq_wire_*         Transport.handleRequest,              internal/transport/transport.go:289-300
 *                     HandleMessageBatch, MessageBatch      nodehost.go:2021-2061, raftpb/raft.proto:154-203
 *
 * The reference has no plugin/FFI for this path (the quorum code lives in unexported methods of
 * the unexported raft struct, raft.go:198). The cgo binding a maintainer adds under
 * internal/hipquorum is shown in INTEGRATION.md; it follows the gorocksdb cgo conventions
 * (internal/logdb/kv/rocksdb/gorocksdb/db.go:3-9, errptr pattern db.go:241-253).
 *
 * Conventions
 *   - Every function returns an int status: HQ_OK (0) or a negative HQ_E_* code. The message of
 *     the last failure on a context is returned by hq_last_error(). Nothing aborts across the ABI.
 *   - A context owns one HIP stream on one GPU. A context is not thread-safe; use one per step
 *     worker (execengine.go:675-690). Different contexts may be used concurrently.
 *   - *_dev functions take DEVICE pointers (from hq_malloc_dev) and are asynchronous on the
 *     context's stream; call hq_sync() before reading results on the host.
 *     The functions without _dev take HOST pointers (pinned memory from hq_alloc_pinned is
 *     fastest), stage through the context's device workspace and return when results are on the
 *     host.
 *   - Bitmaps are arrays of uint64_t words, little-endian bit order: group g is bit (g % 64) of
 *     word g / 64. Bits of groups >= G in the last word are written as 0.
 *   - All arithmetic is unsigned 64-bit integer; results are bit-exact with the reference.
 */
#ifndef HIPQUORUM_H
#define HIPQUORUM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HQ_ABI_VERSION 21

/* status codes */
#define HQ_OK          0
#define HQ_E_INVAL    -1   /* bad argument (null pointer, bad size, misaligned, bad form) */
#define HQ_E_DEVICE   -2   /* HIP runtime error (launch failure, no device) */
#define HQ_E_NOMEM    -3   /* allocation failed */
#define HQ_E_STATE    -4   /* operation not valid in the context's current state */

/* maximum packed voting slots per group in the bitmap kernels (u8 bitmaps) and commit kernels */
#define HQ_MAX_VOTERS 8

/* commit term-check forms (see hq_commit_args) */
#define HQ_FORM_TERM_START 0  /* term(q)==term  <=>  term_start <= q <= last_index */
#define HQ_FORM_TERM_RING  1  /* term(q) gathered from a per-group ring of the last R terms */
#define HQ_FORM_TERM_MASK  2  /* term(q)==term read from a per-group bitmask over the last R */
#define HQ_FORM_TERM_RING32 3 /* the ring gather from a u32 ring (terms saturated at 2^32-1) */

/* commit input layouts (hq_commit_args.layout) */
#define HQ_LAYOUT_COLUMNS 0   /* one array per field (structure of arrays) */
#define HQ_LAYOUT_TILES   1   /* the same arrays cut into tiles of HQ_TILE_GROUPS groups */
#define HQ_LAYOUT_TILES_LEADER 2  /* tiles without the leader's match row (slot 0 = last_index) */
#define HQ_TILE_GROUPS  128   /* groups per tile: one wave64, two groups per lane */
/* flag OR-ed into HQ_LAYOUT_TILES_LEADER: the tiles are a device-resident progress table decided
 * in place — committed' is written into each tile's committed_in row (committed_out unused, may be
 * NULL; the tiles must be writable). Term-start and term-mask forms, hq_commit_dev only. */
#define HQ_LAYOUT_IN_PLACE 0x100u

/* vote outcomes, numerically equal to the reference State enum (internal/raft/raft.go:62-71) */
#define HQ_OUTCOME_FOLLOWER  0u   /* rejections reached quorum: becomeFollower (raft.go:1981-1984) */
#define HQ_OUTCOME_CANDIDATE 1u   /* undecided: stays candidate */
#define HQ_OUTCOME_LEADER    2u   /* grants reached quorum: becomeLeader (raft.go:1977-1980) */

typedef struct hq_ctx hq_ctx;

/* ---------------------------------------------------------------- context / memory ---------- */

/* Version of the ABI this library implements (HQ_ABI_VERSION). */
int hq_abi_version(void);
/* Number of visible GPUs. */
int hq_device_count(int *out);
/* PCI bus id ("dddd:bb:dd.f", NUL-terminated, len >= 13) of visible GPU `device`: lets a host
 * that opens one context per GPU (partition.go:38 sharding) show which physical
 * devices did the work. */
int hq_device_pci_bus_id(int device, char *out, int len);
/* What a pointer is to the GPU: HQ_PTR_PINNED_HOST (hq_alloc_pinned / hipHostMalloc memory, which
 * kernels may read and write over PCIe), HQ_PTR_DEVICE, or HQ_PTR_UNREGISTERED (pageable host
 * memory, NULL or unknown: a kernel touching it faults). Lets a zero-copy caller refuse ordinary
 * host arrays with an error instead of a GPU memory fault. */
#define HQ_PTR_UNREGISTERED 0
#define HQ_PTR_PINNED_HOST 1
#define HQ_PTR_DEVICE 2
int hq_pointer_kind(const void *p, int *kind);
/* Open a context (one HIP stream) on GPU `device`. flags: reserved, pass 0. */
int hq_open(int device, uint32_t flags, hq_ctx **out);
/* Destroy a context; waits for its stream. NULL is a no-op. */
void hq_close(hq_ctx *ctx);
/* Message of the last failure on ctx (never NULL; "" if none). ctx may be NULL for hq_open
 * failures: then the thread's last open error is returned. */
const char *hq_last_error(const hq_ctx *ctx);
/* Wait for all work queued on the context's stream. */
int hq_sync(hq_ctx *ctx);

/* Order ctx's stream after everything enqueued on other's stream so far (an event recorded on
 * other's stream, waited on by ctx's; no host synchronisation). Both contexts must be on one
 * device. Lets a step worker pipeline its steps over two contexts: step i+1's host-to-device
 * copies overlap step i's kernels and readback, its kernels still run after step i's. */
int hq_wait_for(hq_ctx *ctx, hq_ctx *other);

int hq_malloc_dev(hq_ctx *ctx, size_t bytes, void **out);
int hq_free_dev(hq_ctx *ctx, void *p);
int hq_alloc_pinned(hq_ctx *ctx, size_t bytes, void **out);
int hq_free_pinned(hq_ctx *ctx, void *p);
/* Asynchronous copies / fill on the context's stream. kind: 0 = H2D, 1 = D2H, 2 = D2D. */
int hq_memcpy_async(hq_ctx *ctx, void *dst, const void *src, size_t bytes, int kind);
int hq_memset_async(hq_ctx *ctx, void *dst, int value, size_t bytes);

/* Kernel timing: hq_timing_enable(ctx, 1) records a HIP event on the context's stream and opens
 * a timed region; every kernel launched in it is counted; hq_timing_enable(ctx, 0) (or
 * hq_timing_read) records the closing event. hq_timing_read() waits for it and returns the GPU
 * time of all closed regions (ms) and their launch count since the last reset, so
 * total_ms / launches is the mean launch-to-launch kernel time on the stream (back-to-back
 * kernels: kernel duration + the dependent-launch boundary). No per-launch events are recorded:
 * on gfx950 they add several microseconds to a ~10 us kernel. */
int hq_timing_enable(hq_ctx *ctx, int enable);
/* Open a timed region behind the next `launches` kernel launches on the context's stream: the
 * begin event is recorded right after the launches-th one (in stream order it fires when that
 * kernel ends), so a region over back-to-back launches enqueued in one go starts with the next
 * kernel already queued and measures no host launch latency. 0 = hq_timing_enable(ctx, 1). */
int hq_timing_begin_after(hq_ctx *ctx, uint64_t launches);
int hq_timing_read(hq_ctx *ctx, double *total_ms, uint64_t *launches);
int hq_timing_reset(hq_ctx *ctx);

/* ---------------------------------------------------------------- commit ------------------- */

/*
 * Batched leader commit decision, one Raft group per index g in [0, G).
 *
 * For each group (raft.go:888-909 + logentry.go:378-393):
 *   n  = n_voting ? n_voting[g] : n_max          voting members = remotes + witnesses
 *                                                (self included, observers never packed)
 *   q  = the (n/2+1)-th largest of match[0..n-1][g]     == matched[n - quorum] after sorting
 *   lt = term(q)                                    (0 outside [first-1, last], logentry.go:144)
 *   if q > committed_in[g] && lt == term[g]:  committed_out[g] = q, changed bit = 1
 *   else                                       committed_out[g] = committed_in[g], changed = 0
 *
 * term(q) == term is evaluated in one of two exact forms:
 *   HQ_FORM_TERM_START  term_start[g] = index of the leader's first entry of its current term (the
 *       no-op appended by becomeLeader, raft.go:987). Because entries carry the leader's term
 *       (raft.go:913-916) and log terms never decrease (entryutils.go:44-47):
 *       term(q) == term  <=>  term_start[g] <= q <= last_index[g].  `term`/`ring` unused.
 *   HQ_FORM_TERM_RING   ring[g * ring_len + (i % ring_len)] = term(i) for i in
 *       (last_index - ring_len, last_index]. The gather happens only when q > committed; it is
 *       exact when last_index[g] - committed_in[g] <= ring_len.
 *   HQ_FORM_TERM_MASK   bit (i % ring_len) of term_mask[g] = (term(i) == the leader's term) for
 *       i in (last_index - ring_len, last_index]; ring_len <= 16. The same per-index equality the
 *       ring gather tests, without the term values (no monotonicity assumption); exact when
 *       last_index[g] - committed_in[g] <= ring_len. `term`/`ring`/`term_start` unused.
 *   HQ_FORM_TERM_RING32 the ring form over ring32[g * ring_len + (i % ring_len)] =
 *       min(term(i), 0xFFFFFFFF) (hq_pack_ring32). For a leader's term below 0xFFFFFFFF the u32
 *       equality is the u64 one; a 64-B ring (R = 16) lets two groups share each gathered 128-B
 *       line. Groups whose term is >= 0xFFFFFFFF go to the fallback path.
 *
 * Groups that violate the contract are NOT decided: committed_out = committed_in, changed = 0 and
 * the fallback bit is set so the caller runs the CPU path (raft.go:888) for them:
 *   n == 0 or n > n_max;  RING form: term == 0, committed > last_index, or
 *   last_index - committed > ring_len;  RING32 form: as RING, and term >= 0xFFFFFFFF;  MASK form: committed > last_index or
 *   last_index - committed > ring_len.
 *
 * Layout HQ_LAYOUT_COLUMNS: match is slot-major, match[s * match_stride + g]; match_stride >= G.
 * committed_out may alias committed_in. changed / fallback may be NULL.
 *
 * Layout HQ_LAYOUT_TILES: the per-group input columns of 128 consecutive groups are stored as
 * one contiguous tile, so a wave reads its groups as ONE stream instead of n + 3 column streams
 * (6 % less time for the same bytes at 1 M groups x 3 voters, tools/kexp5.hip, git history). `match` points
 * to tile 0 (16-byte aligned); tile t = match + t * hq_commit_tile_words(n_max, form) holds
 * groups [128 t, 128 t + 128), each row 128 entries of one field, position 2i holding group
 * 128 t + i and position 2i + 1 group 128 t + 64 + i (lane i of a wave reads both with one
 * 16-byte load; its two ballots are then the tile's two bitmap words):
 *   rows 0 .. n_max-1   match of slot s (u64)
 *   row  n_max          committed_in (u64)
 *   row  n_max+1        last_index (u64)
 *   row  n_max+2        term_start (HQ_FORM_TERM_START) or the leader's term (RING, RING32),
 *                       u64; or the u16 term_mask (HQ_FORM_TERM_MASK, 256 bytes)
 * The last tile is padded to 128 groups (padding is never read into a decision).
 * match_stride, committed_in, last_index, term_start, term and term_mask are unused;
 * committed_out, n_voting, ring / ring32, changed and fallback stay separate arrays as above.
 *
 * Layout HQ_LAYOUT_TILES_LEADER: the tiles above without row 0. Slot 0 is the leader, and a
 * leader's own match is its lastIndex at every step (reset() sets it, raft.go:1031, and
 * appendEntries raises it with every append, raft.go:918), so the kernel takes slot 0's match
 * from the last_index row: rows 0 .. n_max-2 hold match slots 1 .. n_max-1, then committed_in,
 * last_index and the term row. 8 bytes less per group (48 instead of 56 at 3 voters), same
 * decision bit for bit whenever match[0] == last_index (hq_tile_commit_as_host checks it).
 */
typedef struct hq_commit_args {
    uint64_t G;               /* groups in this call */
    uint32_t n_max;           /* packed slots per group, 1..HQ_MAX_VOTERS */
    uint32_t form;            /* HQ_FORM_TERM_START or HQ_FORM_TERM_RING */
    uint32_t ring_len;        /* R for HQ_FORM_TERM_RING: power of two, 1..1024 */
    uint32_t layout;          /* HQ_LAYOUT_COLUMNS (0), HQ_LAYOUT_TILES or _TILES_LEADER */
    uint64_t match_stride;    /* elements between slot rows of match, >= G */
    const uint64_t *match;    /* [n_max][match_stride] */
    const uint8_t *n_voting;  /* [G] voting members per group, or NULL: all groups have n_max */
    const uint64_t *committed_in;   /* [G] */
    uint64_t *committed_out;        /* [G] (may alias committed_in) */
    const uint64_t *last_index;     /* [G] */
    const uint64_t *term_start;     /* [G] HQ_FORM_TERM_START */
    const uint64_t *term;           /* [G] HQ_FORM_TERM_RING: the leader's current term */
    const uint64_t *ring;           /* [G][ring_len] HQ_FORM_TERM_RING */
    uint64_t *changed;              /* [ceil(G/64)] or NULL */
    uint64_t *fallback;             /* [ceil(G/64)] or NULL */
    const uint16_t *term_mask;      /* [G] HQ_FORM_TERM_MASK */
    const uint32_t *ring32;         /* [G][ring_len] HQ_FORM_TERM_RING32 */
} hq_commit_args;

int hq_commit_dev(hq_ctx *ctx, const hq_commit_args *args);
int hq_commit(hq_ctx *ctx, const hq_commit_args *args);

/* u64 words of one HQ_LAYOUT_TILES tile of hq_commit_args with n_max slots and term form `form`:
 * (n_max + 3) rows of 128 u64, or (n_max + 2) rows + the 256-byte term_mask row. */
static inline uint64_t hq_commit_tile_words(uint32_t n_max, uint32_t form) {
    return form == HQ_FORM_TERM_MASK ? (uint64_t)(n_max + 2) * HQ_TILE_GROUPS + 32
                                     : (uint64_t)(n_max + 3) * HQ_TILE_GROUPS;
}
/* words of one tile in `layout` (HQ_LAYOUT_TILES or HQ_LAYOUT_TILES_LEADER) */
static inline uint64_t hq_commit_tile_words_for(uint32_t n_max, uint32_t form, uint32_t layout) {
    return hq_commit_tile_words((layout & 0xFFu) == HQ_LAYOUT_TILES_LEADER ? n_max - 1 : n_max,
                                form);
}
static inline uint64_t hq_commit_tiles(uint64_t G) {
    return (G + HQ_TILE_GROUPS - 1) / HQ_TILE_GROUPS;
}
/* Cut the input columns of a HQ_LAYOUT_COLUMNS batch (`columns`: match, committed_in,
 * last_index and the form's term_start / term / term_mask) into HQ_LAYOUT_TILES tiles at
 * `tiles` (hq_commit_tiles(G) * hq_commit_tile_words(n_max, form) u64, padding zeroed).
 * _dev: device pointers, async on the context's stream; _host: host pointers (a step worker
 * packing its staging buffer), no context needed. */
int hq_tile_commit_dev(hq_ctx *ctx, const hq_commit_args *columns, uint64_t *tiles);
int hq_tile_commit_host(const hq_commit_args *columns, uint64_t *tiles);
/* The same into `layout` = HQ_LAYOUT_TILES or HQ_LAYOUT_TILES_LEADER (tiles of
 * hq_commit_tile_words_for(n_max, form, layout) words; the leader layout drops match slot 0,
 * and the host packer returns HQ_E_INVAL if a group with n >= 1 has match[0] != last_index; the
 * device packer does not check it: it is meant for generated inputs whose slot 0 is lastIndex by
 * construction, and a real table must be cut by the host packer or kept in the leader layout
 * from the start, hq_table_* below). */
int hq_tile_commit_as_dev(hq_ctx *ctx, const hq_commit_args *columns, uint64_t *tiles,
                          uint32_t layout);
int hq_tile_commit_as_host(const hq_commit_args *columns, uint64_t *tiles, uint32_t layout);
/* `count` independent batches back to back on the context's stream (e.g. a step worker's
 * per-voter-count buckets of one step, or successive steps). Stops at the first invalid batch. */
int hq_commit_many_dev(hq_ctx *ctx, const hq_commit_args *args, uint32_t count);
/* The same `count` batches decided by ONE kernel launch when they can share it (2..32 batches,
 * uniform n (n_voting NULL), one form, 16-byte aligned columns, G > 0, not in place): a step
 * worker's voter-count buckets (groups bucketed by n for coalesced SoA, execengine.go:923
 * caller), or the independent batches that several step workers (or steps) have ready at once.
 * Batch i owns its own workgroups; results are identical to hq_commit_many_dev, which is what
 * runs when the batches cannot share a launch. */
int hq_commit_fused_dev(hq_ctx *ctx, const hq_commit_args *args, uint32_t count);

/* ---------------------------------------------------------------- persistent commit engine -- */
/*
 * A resident commit engine: ONE kernel launch decides a stream of posted commit batches
 * (hq_commit_dev's decision, bit for bit), so successive steps pay no dependent-launch boundary
 * and no grid fill / drain (≈ 2 us of a 1M-group launch). Step workers post the
 * batch of each step (raft.tryCommit over their leader groups, raft.go:888-909, logentry.go:378-393)
 * the way execEngine wakes its step workers (workReady.clusterReady -> stepWorkerMain,
 * execengine.go:115-123, 860-882): a 64-byte descriptor into a pinned ring, read by the resident
 * kernel. Wave w of the engine's grid decides tiles w, w + W, ... of every batch in post order,
 * so a device-resident table posted step after step (HQ_LAYOUT_IN_PLACE) is decided in order per
 * group with no grid-wide barrier between steps.
 *
 * Served: uniform n (n_voting NULL), HQ_FORM_TERM_START or HQ_FORM_TERM_MASK, layout
 * HQ_LAYOUT_TILES, HQ_LAYOUT_TILES_LEADER or HQ_LAYOUT_TILES_LEADER | HQ_LAYOUT_IN_PLACE, device
 * pointers. Every posted batch must have the engine's n_max, form, layout (and ring_len for the
 * mask form); its tiles and outputs must stay allocated until the step is complete.
 *
 * The engine has its own HIP stream and holds every CU of the GPU while it is resident (kernels
 * on other streams wait for it): hq_engine_drain() ends the resident launch, the next post
 * starts it again. A resident launch also ends by itself after idle_us without a post (1 ms by
 * default; every spin is bounded); steps posted meanwhile are run by a relaunch from
 * hq_engine_wait(). Engines of several processes on one GPU: give each max_workgroups = the
 * full grid / the processes, so that every grid is resident at once (a grid partly resident
 * beside another waits for its missing workgroups until one of them exits idle).
 */
#define HQ_ENGINE_SIGNAL 1u   /* per-step completion: hq_engine_wait(seq) returns as soon as step
                                 seq is done (else wait = drain: the steps complete as a whole) */
typedef struct hq_engine hq_engine;
typedef struct hq_engine_config {
    uint32_t n_max;          /* voting slots of every posted batch, 1..HQ_MAX_VOTERS */
    uint32_t form;           /* HQ_FORM_TERM_START or HQ_FORM_TERM_MASK */
    uint32_t layout;         /* HQ_LAYOUT_TILES, _TILES_LEADER or _TILES_LEADER | HQ_LAYOUT_IN_PLACE */
    uint32_t ring_len;       /* mask form: R (power of two <= 16); unused for term-start */
    uint32_t depth;          /* posted steps in flight: power of two 2..64 (0 = 64) */
    uint32_t flags;          /* HQ_ENGINE_SIGNAL */
    uint32_t idle_us;        /* polling time without a post before the resident launch ends (0 = 1000) */
    uint32_t max_workgroups; /* cap on the resident grid (0 = every CU at full occupancy) */
} hq_engine_config;
typedef struct hq_engine_stats {
    uint64_t posted;         /* steps posted (STOP steps of drains included) */
    uint64_t completed;      /* every step below this sequence number is known complete */
    uint64_t relaunches;     /* launches started by a wait because the grid had gone idle */
    uint32_t grid, block;    /* resident geometry */
    uint32_t depth, running;
} hq_engine_stats;
int hq_engine_open(hq_ctx *ctx, const hq_engine_config *cfg, hq_engine **out);
/* Post `count` batches as the next steps; *first_seq (may be NULL) = the sequence number of the
 * first. Blocks only when `depth` steps are in flight. Thread-safe (several step workers may
 * share one engine per GPU). */
int hq_engine_post(hq_engine *eng, const hq_commit_args *args, uint32_t count, uint64_t *first_seq);
/* Return when step `seq` is complete: its outputs are in device memory, visible to the host and
 * to every stream. */
int hq_engine_wait(hq_engine *eng, uint64_t seq);
/* Complete every posted step and end the resident launch (the CUs are free afterwards). */
int hq_engine_drain(hq_engine *eng);
/* A bounded run: post `count` batches, then drain. With no grid resident the launch's arguments
 * carry the steps and the STOP together (up to 32), so the grid ends as soon as the last step is
 * decided — a post followed by a drain launches on the post and the STOP reaches the running grid
 * through the ring (~20 us of relay and polling per launch, tools/engine_overhead.py). */
int hq_engine_run(hq_engine *eng, const hq_commit_args *args, uint32_t count, uint64_t *first_seq);
/* GPU time of the finished resident launches (HIP events around each), since the last reset. */
int hq_engine_timing(hq_engine *eng, uint64_t *launches, double *total_ms, int reset);
/* The device clock (s_memrealtime, 100 MHz) when step seq completed (HQ_ENGINE_SIGNAL). */
int hq_engine_done_clock(hq_engine *eng, uint64_t seq, uint64_t *ticks);
int hq_engine_info(hq_engine *eng, hq_engine_stats *out);
/* Diagnostic: the engine's state as the device holds it (readable while the grid runs): out[0]
 * posted (host ring), [1] relayed, [2] the relayed count the workgroups poll, [3] the exit
 * epoch, [4] launches, [5] grid, [6] completed, [7] running, then every workgroup's cursor (the
 * next step it takes at a launch), then the arrival counters ([depth][8] per shard, then [depth]
 * top). n_words >= 8 + grid + 9 * depth. */
int hq_engine_dump(hq_engine *eng, uint64_t *out, uint32_t n_words);
const char *hq_engine_last_error(const hq_engine *eng);
/* Drain and destroy. NULL is a no-op. */
void hq_engine_close(hq_engine *eng);

/* ---------------------------------------------------------------- commit over lags --------- */
/*
 * The same decision over a compact layout: every index is stored as its distance below the
 * group's lastIndex, as int32 ("lag"). The decision depends only on the order of the match
 * values, committed, term_start and lastIndex, and that order is kept by the lags:
 *   lag[s][g] = clamp(last_index - match_s)      (negative when match > last_index)
 *   cin_lag[g] = clamp(last_index - committed)
 *   ts_lag[g]  = clamp(last_index - term_start)  (HQ_FORM_TERM_START)
 *   lag_mask[g] bit k = (term(last_index - k) == the leader's term), k < ring_len
 *                                                 (HQ_FORM_TERM_MASK; the mask indexed by lag)
 * with clamp() saturating to [INT32_MIN, INT32_MAX]. Then (raft.go:888-909, logentry.go:378-393)
 *   d  = the (n/2+1)-th SMALLEST lag                   (= lastIndex - the quorum-th largest match)
 *   commit iff d < cin_lag && d >= 0 && (d <= ts_lag | bit d of lag_mask)
 *   cout_lag[g] = commit ? d : cin_lag[g];     committed' = lastIndex - cout_lag (hq_unpack_lags)
 * Saturation never changes a decision: a clamped lag is only ever compared against an unclamped
 * cin_lag. Fallback (not decided, as in hq_commit_dev): n == 0 or n > n_max; TERM_START:
 * cin_lag == INT32_MAX or INT32_MIN (committed not representable); TERM_MASK: cin_lag < 0 or
 * cin_lag > ring_len (the mask form's contract). A decided group's cout_lag is exact.
 * Bytes per group: 4n + 12 (term-start; 24 B at n = 3 against 56 B for hq_commit_dev) or
 * 4n + 10 (mask). Packed from the u64 columns by hq_pack_lags (host) or generated on the device.
 *
 * flags & HQ_LAG_LEADER_IMPLICIT: the lag rows start at slot 1 (row s - 1 = slot s) and slot 0's
 * lag is 0 — slot 0 is the leader, whose own match is its lastIndex at every step (reset,
 * raft.go:1031; appendEntries, raft.go:918). 4 bytes less per group (20 B at n = 3).
 */
#define HQ_LAG_LEADER_IMPLICIT 1u
typedef struct hq_commit_lag_args {
    uint64_t G;
    uint32_t n_max;           /* 1..HQ_MAX_VOTERS */
    uint32_t form;            /* HQ_FORM_TERM_START or HQ_FORM_TERM_MASK */
    uint32_t ring_len;        /* TERM_MASK: power of two <= 16 */
    uint32_t flags;           /* 0 or HQ_LAG_LEADER_IMPLICIT */
    uint64_t lag_stride;      /* elements between slot rows of lag, >= G */
    const int32_t *lag;       /* [n_max][lag_stride] */
    const uint8_t *n_voting;  /* [G] or NULL (all groups have n_max) */
    const int32_t *cin_lag;   /* [G] */
    int32_t *cout_lag;        /* [G] (may alias cin_lag) */
    const int32_t *ts_lag;    /* [G] TERM_START */
    const uint16_t *lag_mask; /* [G] TERM_MASK */
    uint64_t *changed;        /* [ceil(G/64)] or NULL */
    uint64_t *fallback;       /* [ceil(G/64)] or NULL */
} hq_commit_lag_args;

int hq_commit_lag_dev(hq_ctx *ctx, const hq_commit_lag_args *args);
/* hq_commit_fused_dev for the lag layout: 2..8 uniform-n batches of one form, aligned columns,
 * in one launch; otherwise one launch per batch, same results. */
int hq_commit_lag_fused_dev(hq_ctx *ctx, const hq_commit_lag_args *args, uint32_t count);

/* Host packer: the lag columns of *out (lag rows at out->lag_stride, cin_lag and ts_lag or
 * lag_mask per out->form) from u64 columns laid out as in hq_commit_args (match rows at
 * match_stride; term_start for TERM_START; term_mask (bit i % ring_len) for TERM_MASK).
 * Slots >= n_max of the lag rows are not written. With out->flags = HQ_LAG_LEADER_IMPLICIT slot 0
 * is not written (row s - 1 = slot s) and a group with n >= 1 (out->n_voting, if given) whose
 * match[0] != last_index is refused (HQ_E_INVAL). */
int hq_pack_lags(uint64_t G, uint32_t n_max, const uint64_t *match, uint64_t match_stride,
                 const uint64_t *committed, const uint64_t *last_index,
                 const uint64_t *term_start, const uint16_t *term_mask,
                 const hq_commit_lag_args *out);
/* committed[g] = last_index[g] - cout_lag[g] (the host's commitTo, logentry.go:323-332) for
 * every group whose fallback bit is clear (fallback may be NULL); fallback groups keep their
 * committed value for the CPU path. */
int hq_unpack_lags(uint64_t G, const uint64_t *last_index, const int32_t *cout_lag,
                   const uint64_t *fallback, uint64_t *committed);

/* ---------------------------------------------------------------- ReadIndex / vote ----------- */

/*
 * ReadIndex heartbeat-ack quorum, one pending ctx per group (readindex.go:77-116):
 *   confirmed bit = popcount(ack[g] & mask(n)) + 1 >= n/2 + 1     (the +1 is the leader, :84)
 * ack[g] bit s = voting slot s acknowledged the pending SystemCtx (distinct `from`); bits >= n are
 * ignored. n = n_voting ? n_voting[g] : n_uniform, valid 1..8; groups with an invalid n get
 * confirmed = 0 and, if `fallback` is non-NULL, a fallback bit.
 */
int hq_readindex_dev(hq_ctx *ctx, uint64_t G, const uint8_t *ack, const uint8_t *n_voting,
                     uint32_t n_uniform, uint64_t *confirmed, uint64_t *fallback);
int hq_readindex(hq_ctx *ctx, uint64_t G, const uint8_t *ack, const uint8_t *n_voting,
                 uint32_t n_uniform, uint64_t *confirmed, uint64_t *fallback);

/*
 * Vote tally (raft.go:1062-1080, 1968-1985). granted[g] bit s = slot s granted (the candidate's
 * own vote, campaign raft.go:1093, is a granted bit); rejected[g] bit s = slot s rejected.
 * First response wins (raft.go:1071-1073): a slot present in both is counted as granted.
 *   outcome = popcount(granted) >= q ? LEADER : popcount(rejected & ~granted) >= q ? FOLLOWER
 *                                                                            : CANDIDATE
 * Outcomes are 2-bit codes packed 32 per uint64_t word: group g at bits 2*(g%32) of word g/32.
 * Invalid n gives CANDIDATE (+ fallback bit).
 */
int hq_vote_dev(hq_ctx *ctx, uint64_t G, const uint8_t *granted, const uint8_t *rejected,
                const uint8_t *n_voting, uint32_t n_uniform, uint64_t *outcome,
                uint64_t *fallback);
int hq_vote(hq_ctx *ctx, uint64_t G, const uint8_t *granted, const uint8_t *rejected,
            const uint8_t *n_voting, uint32_t n_uniform, uint64_t *outcome, uint64_t *fallback);

/*
 * General ReadIndex with several pending ctxs per group (readindex.go:43-116).
 * Per group g: K = n_pending ? n_pending[g] : K_max ctxs in queue order (oldest first) with
 * indexes ctx_index[k * G + g] (non-decreasing, addRequest readindex.go:50-59); and
 * ack_ordinal[(k * n_max + s) * G + g] = the arrival ordinal (message sequence number within the
 * batch, 0 for acks carried over from earlier steps) of voting slot s's first HeartbeatResp for
 * ctx k, 0xFFFF = none. Replaying the messages in ordinal order through confirm() releases queue
 * prefixes; equivalently ctx k reaches quorum at t_k = the max(q-1, 1)-th smallest of its
 * ordinals and entry i is released at min_{k >= i} t_k with the index of the (first) ctx
 * attaining it (the rewrite of readindex.go:97-105).
 * Out: released_index[k * G + g] = rewritten index of entry k, or UINT64_MAX if not released;
 * released_count[g] = released prefix length; batch_end[g] (may be NULL) bit k = entry k is the
 * ctx whose confirm() released its batch — every released entry i belongs to the batch closed by
 * the first k >= i with bit k set, and the ReadIndexResp messages of that batch carry ctx k as
 * their hint (handleReadIndexLeaderConfirmation, raft.go:1740-1760). released_index may be NULL
 * when batch_end is not: it is then not written (32 of a K = 4 group's 34 output bytes), and the
 * caller, which holds ctx_index, derives it with hq_ri_released_host. n outside [1, n_max],
 * K > K_max or a decreasing ctx_index give fallback (nothing released). K_max <= 8, n_max <= 8;
 * ordinals distinct per group except 0 (ties at equal ordinals resolve in queue order).
 */
int hq_readindex_multi_dev(hq_ctx *ctx, uint64_t G, uint32_t K_max, uint32_t n_max,
                           const uint16_t *ack_ordinal, const uint64_t *ctx_index,
                           const uint8_t *n_pending, const uint8_t *n_voting, uint32_t n_uniform,
                           uint64_t *released_index, uint8_t *released_count,
                           uint8_t *batch_end, uint64_t *fallback);

/*
 * The same release over 128-group tiles: tile t starts at tiles + t * hq_ri_tile_bytes(K_max,
 * n_max, flags) and holds the rows ack_ordinal[k][s] (k < K_max, s < n_max; 128 u16 each, k-major),
 * ctx_index[k] (k < K_max; 128 u64 each), then with HQ_RI_TILE_PER_K n_pending (128 u8) and with
 * HQ_RI_TILE_PER_N n_voting (128 u8); group 128 t + j at entry j of every row (padding: ordinal
 * 0xFFFF, index 0, counts 0). One contiguous block per wave instead of K_max * (n_max + 1) column
 * streams. Outputs (columns) and semantics as hq_readindex_multi_dev; G even, released_index
 * 16-byte and released_count / batch_end 2-byte aligned.
 */
#define HQ_RI_TILE_GROUPS 128
#define HQ_RI_TILE_PER_K 1u
#define HQ_RI_TILE_PER_N 2u
static inline uint64_t hq_ri_tile_bytes(uint32_t K_max, uint32_t n_max, uint32_t flags) {
    return (uint64_t)K_max * n_max * 256 + (uint64_t)K_max * 1024 +
           ((flags & HQ_RI_TILE_PER_K) ? 128 : 0) + ((flags & HQ_RI_TILE_PER_N) ? 128 : 0);
}
int hq_readindex_multi_tiles_dev(hq_ctx *ctx, uint64_t G, uint32_t K_max, uint32_t n_max,
                                 const uint8_t *tiles, uint32_t flags, uint32_t n_uniform,
                                 uint64_t *released_index, uint8_t *released_count,
                                 uint8_t *batch_end, uint64_t *fallback);
/* Columns (as hq_readindex_multi_dev; n_pending / n_voting may be NULL, setting the flags) ->
 * tiles (ceil(G / 128) * hq_ri_tile_bytes(...) bytes, 16-byte aligned). _host: host pointers. */
int hq_tile_ri_multi_dev(hq_ctx *ctx, uint64_t G, uint32_t K_max, uint32_t n_max,
                         const uint16_t *ack_ordinal, const uint64_t *ctx_index,
                         const uint8_t *n_pending, const uint8_t *n_voting, uint8_t *tiles);
int hq_tile_ri_multi_host(uint64_t G, uint32_t K_max, uint32_t n_max,
                          const uint16_t *ack_ordinal, const uint64_t *ctx_index,
                          const uint8_t *n_pending, const uint8_t *n_voting, uint8_t *tiles);
/* released_index [K_max][G] from the compact outputs (released_count, batch_end) and the
 * caller's ctx_index [K_max][G]: entry k < released_count[g] gets ctx_index[k'][g] of the first
 * k' >= k with batch_end bit k' set (the index confirm() rewrote it to, readindex.go:96-104), the
 * other entries ~0 — the released_index the kernels write. Host pointers; HQ_E_INVAL when a
 * released entry has no closing ctx (batch_end not from the same call). */
int hq_ri_released_host(uint64_t G, uint32_t K_max, const uint64_t *ctx_index,
                        const uint8_t *released_count, const uint8_t *batch_end,
                        uint64_t *released_index);

/* ReadIndex confirmation and vote tally of the same groups in one pass over the shared n. */
int hq_readindex_vote_dev(hq_ctx *ctx, uint64_t G, const uint8_t *ack, const uint8_t *granted,
                          const uint8_t *rejected, const uint8_t *n_voting, uint32_t n_uniform,
                          uint64_t *confirmed, uint64_t *outcome, uint64_t *fallback);

/*
 * The same fused pass over a tiled bitmap layout: the bitmaps of 1024 consecutive groups (one
 * wave, 16 groups per lane) stored as one contiguous block of 1024-byte rows
 *   [n_voting (per_group_n only)] [ack] [granted] [rejected]
 * so a wave reads ONE stream instead of 3-4 columns (tools/kexp8.hip, git history: 14.5 vs 15.5 us per
 * 16M x 7 launch, 11.1 vs 11.9 us with uniform n). Tile t starts at tiles + t * rows * 1024,
 * byte (g & 1023) of each row is group g; the last tile is padded to 1024 groups (padding is
 * never decided). Outputs are the columns of hq_readindex_vote_dev. Same decisions as
 * readIndex.confirm's quorum test (readindex.go:84) and handleVoteResp / the candidate's tally
 * (raft.go:1062-1080, 1968-1985).
 */
#define HQ_BITS_TILE_GROUPS 1024
static inline uint64_t hq_bits_tiles(uint64_t G) {
    return (G + HQ_BITS_TILE_GROUPS - 1) / HQ_BITS_TILE_GROUPS;
}
int hq_readindex_vote_tiles_dev(hq_ctx *ctx, uint64_t G, const uint8_t *tiles,
                                uint32_t per_group_n, uint32_t n_uniform, uint64_t *confirmed,
                                uint64_t *outcome, uint64_t *fallback);
/* Columns -> bitmap tiles (hq_bits_tiles(G) * (n_voting ? 4 : 3) * 1024 bytes, padding zeroed).
 * _dev: device pointers, 16-byte aligned, async on the context's stream; _host: host pointers
 * (a step worker packing its staging buffer). */
int hq_tile_bits_dev(hq_ctx *ctx, uint64_t G, const uint8_t *ack, const uint8_t *granted,
                     const uint8_t *rejected, const uint8_t *n_voting, uint8_t *tiles);
int hq_tile_bits_host(uint64_t G, const uint8_t *ack, const uint8_t *granted,
                      const uint8_t *rejected, const uint8_t *n_voting, uint8_t *tiles);

/*
 * The same fused pass over 3-byte tiles: the leader's / candidate's own slot 0 carries no
 * information (it never acks its own ctx — readindex.go:84 counts it as the +1 — always grants
 * its own vote, campaign raft.go:1093, and never rejects it), so each group is 3 bytes instead
 * of 4: 1024-group tiles of rows [ack] [granted] [rejected], byte bits 0..6 = slots 1..7 and
 * bit 7 = one bit of n - 1 (ack row: bit 0, granted row: bit 1, rejected row: bit 2), n in
 * [1, 8]. Tile t starts at tiles + t * 3072. Same decisions as hq_readindex_vote_dev on groups
 * whose slot 0 is not acked, granted and not rejected; the packers give every other group (and
 * n outside [1, 8]) a fallback bit and zero bytes, and its decision must be ignored.
 */
int hq_readindex_vote_tiles3_dev(hq_ctx *ctx, uint64_t G, const uint8_t *tiles,
                                 uint64_t *confirmed, uint64_t *outcome);
/* Columns (n_voting, or n_uniform when NULL) -> 3-byte tiles (hq_bits_tiles(G) * 3072 bytes,
 * padding zeroed); fallback (may be NULL) receives the contract violations. */
int hq_tile_bits3_dev(hq_ctx *ctx, uint64_t G, const uint8_t *ack, const uint8_t *granted,
                      const uint8_t *rejected, const uint8_t *n_voting, uint32_t n_uniform,
                      uint8_t *tiles, uint64_t *fallback);
int hq_tile_bits3_host(uint64_t G, const uint8_t *ack, const uint8_t *granted,
                       const uint8_t *rejected, const uint8_t *n_voting, uint32_t n_uniform,
                       uint8_t *tiles, uint64_t *fallback);

/*
 * The same pass over bit-plane tiles: the 3-byte tiles' bits transposed so that the kernel
 * decides 32 groups per lane with bitwise adders (bit-sliced). A tile holds
 * HQ_PLANE_TILE_GROUPS groups as 24 planes of HQ_PLANE_TILE_GROUPS / 8 bytes: plane 8 r + b =
 * bit b of row r's byte of the 3-byte layout (r = 0 ack, 1 granted, 2 rejected), bit j of byte k
 * of a plane = the tile's group 8 k + j. Tile t starts at planes + t * 3 * HQ_PLANE_TILE_GROUPS.
 * Same decisions and contract as hq_readindex_vote_tiles3_dev.
 */
#define HQ_PLANE_TILE_GROUPS 2048
static inline uint64_t hq_plane_tiles(uint64_t G) {
    return (G + HQ_PLANE_TILE_GROUPS - 1) / HQ_PLANE_TILE_GROUPS;
}
int hq_readindex_vote_planes_dev(hq_ctx *ctx, uint64_t G, const uint8_t *planes,
                                 uint64_t *confirmed, uint64_t *outcome);
/* Columns -> bit-plane tiles (hq_plane_tiles(G) * 3 * HQ_PLANE_TILE_GROUPS bytes, padding
 * zeroed, 8-byte aligned); fallback (may be NULL) receives the contract violations. */
int hq_tile_planes_dev(hq_ctx *ctx, uint64_t G, const uint8_t *ack, const uint8_t *granted,
                       const uint8_t *rejected, const uint8_t *n_voting, uint32_t n_uniform,
                       uint8_t *planes, uint64_t *fallback);
int hq_tile_planes_host(uint64_t G, const uint8_t *ack, const uint8_t *granted,
                        const uint8_t *rejected, const uint8_t *n_voting, uint32_t n_uniform,
                        uint8_t *planes, uint64_t *fallback);

/*
 * CheckQuorum (raft.go:380-390): has_quorum bit = popcount(active[g] | 1 << self_slot) >= q,
 * then every active flag is reset (remote.go:196-198): active[g] is written back as 0.
 * self_slot is the leader's slot (the packer puts the leader in slot 0).
 */
int hq_check_quorum_dev(hq_ctx *ctx, uint64_t G, uint8_t *active, const uint8_t *n_voting,
                        uint32_t n_uniform, uint32_t self_slot, uint64_t *has_quorum,
                        uint64_t *fallback);

/*
 * The same decision over active-flag planes (raft.go:380-390; the leader's own slot always
 * counts, raft.go:384, so it is not stored). A tile holds HQ_PLANE_TILE_GROUPS groups as planes of
 * HQ_PLANE_TILE_GROUPS / 8 bytes, bit j of byte k of a plane = the tile's group 8 k + j:
 *   per-group n (n_uniform = 0): 10 planes — plane k < 7 = the active flag of the group's
 *     (k + 1)-th voting slot other than the leader's (slot order), planes 7..9 = bits 0..2 of n - 1;
 *   uniform n (n_uniform in 1..8): the n - 1 active planes only (none for n = 1).
 * has_quorum bit = 1 + (active other voting slots) >= n/2 + 1; every active plane of the batch is
 * then zeroed in place (setNotActive, remote.go:196-198). Planes 16-byte aligned, the tile size is
 * hq_cq_plane_bytes(G, n_uniform) / hq_plane_tiles(G). Nothing falls back: the packers flag the
 * groups whose columns break the contract (n outside 1..8, self_slot >= n), pack them as n = 1,
 * and the caller decides those on the CPU from its columns.
 */
static inline uint64_t hq_cq_plane_bytes(uint64_t G, uint32_t n_uniform) {
    return hq_plane_tiles(G) * (n_uniform ? n_uniform - 1 : 10) * (HQ_PLANE_TILE_GROUPS / 8);
}
int hq_check_quorum_planes_dev(hq_ctx *ctx, uint64_t G, uint8_t *planes, uint32_t n_uniform,
                               uint64_t *has_quorum);
/*
 * ReadIndex + vote + CheckQuorum in one pass (ABI 13): planes as hq_readindex_vote_planes_dev
 * (the groups' n from its n bits), active_planes = the CheckQuorum planes built with
 * n_uniform 8 and self_slot 0 (7 planes of HQ_PLANE_TILE_GROUPS / 8 bytes per tile, plane k = the
 * active flag of voting slot k + 1; hq_cq_plane_bytes(G, 8) bytes). Writes the confirmed and
 * outcome words of hq_readindex_vote_planes_dev and the has_quorum words of
 * hq_check_quorum_planes_dev, then zeroes the active planes (remote.go:196-198). Both plane
 * buffers 16-byte aligned. The ack / vote / active flags of slots >= n are ignored.
 */
int hq_readindex_vote_cq_planes_dev(hq_ctx *ctx, uint64_t G, const uint8_t *planes,
                                    uint8_t *active_planes, uint64_t *confirmed,
                                    uint64_t *outcome, uint64_t *has_quorum);
/* Columns (active u8 bitmap per group, bit s = voting slot s; n_voting, or n_uniform when NULL;
 * self_slot = the leader's slot) -> CheckQuorum planes (padding zeroed, 8-byte aligned);
 * fallback (may be NULL) receives the contract violations. */
int hq_tile_cq_planes_dev(hq_ctx *ctx, uint64_t G, const uint8_t *active, const uint8_t *n_voting,
                          uint32_t n_uniform, uint32_t self_slot, uint8_t *planes,
                          uint64_t *fallback);
int hq_tile_cq_planes_host(uint64_t G, const uint8_t *active, const uint8_t *n_voting,
                           uint32_t n_uniform, uint32_t self_slot, uint8_t *planes,
                           uint64_t *fallback);

/* ---------------------------------------------------------------- device-resident state ----- */
/*
 * Delta ingest into a device-resident progress table: the host ships only what
 * changed since the last step instead of re-packing whole batches over PCIe.
 *
 * hq_ingest_match_dev: for each update u, match[slot * match_stride + group] =
 *   max(match[...], u.index) — remote.tryUpdate (remote.go:123-133) raises match only, so any
 *   order of the batch (and duplicates) gives the sequential result. 64-bit atomic max.
 * hq_ingest_ack_dev: ack[group] |= 1 << slot — the confirmed-set insert of readIndex.confirm
 *   (readindex.go:83); idempotent, so duplicate acks never double count. ack must be 4-byte
 *   aligned (32-bit atomic OR on the containing word).
 * hq_append_dev: the leader appended entries at its current term up to new_last
 *   (appendEntries, raft.go:911-922): last_index = new_last, the leader's own match (slot 0) =
 *   new_last (raft.go:918), and the term-mask bits of (old_last, new_last] are set (ring_len <= 16).
 *   new_last <= last_index leaves the group unchanged. term_mask may be NULL.
 *
 * Updates whose group >= G or slot >= n_max are skipped and counted into *n_skipped (a device
 * uint64_t, may be NULL; accumulated, not reset).
 *
 * Padding: the ack and term_mask updates are 32-bit atomic ORs on the word that holds the target
 * byte / u16, so the ack array must be allocated to a multiple of 4 bytes and term_mask to an
 * even number of entries (hq_malloc_dev's rounding does it; a caller sub-allocating these arrays
 * must pad them itself). The bytes beyond G in that last word are never changed (OR with 0).
 */
typedef struct hq_match_update {
    uint64_t group_slot;   /* group << 8 | slot */
    uint64_t index;        /* ReplicateResp LogIndex accepted by the leader */
} hq_match_update;

typedef struct hq_append_update {
    uint64_t group;
    uint64_t new_last;
} hq_append_update;

int hq_ingest_match_dev(hq_ctx *ctx, const hq_match_update *updates, uint64_t count,
                        uint64_t *match, uint64_t match_stride, uint64_t G, uint32_t n_max,
                        uint64_t *n_skipped);
int hq_ingest_ack_dev(hq_ctx *ctx, const uint64_t *group_slot, uint64_t count, uint8_t *ack,
                      uint64_t G, uint32_t n_max, uint64_t *n_skipped);
int hq_append_dev(hq_ctx *ctx, const hq_append_update *updates, uint64_t count,
                  uint64_t *last_index, uint64_t *match_slot0, uint16_t *term_mask,
                  uint32_t ring_len, uint64_t G, uint64_t *n_skipped);

/*
 * The same two updates in 8 bytes each, for host-fed steps (PCIe is the bound there):
 * hq_ingest_lag_dev: update = group << 32 | slot << 28 | lag (28 bits): the follower in `slot`
 *   acknowledged index last_index[group] - lag, last_index as it stands when the kernel runs (after
 *   the step's appends); match = max(match, that index) as in hq_ingest_match_dev. A lag above
 *   last_index, group >= G or slot >= n_max is skipped and counted. Acks 2^28 or more below
 *   lastIndex need the 16-byte form.
 * hq_append_count_dev: update = group << 32 | n (n >= 1 entries appended at the leader's term):
 *   last_index += n (64-bit atomic add, so several appends of a group in one batch commute),
 *   the leader's match = the new last, term-mask bits of the n new indexes set. n == 0 or
 *   group >= G is skipped and counted.
 */
int hq_ingest_lag_dev(hq_ctx *ctx, const uint64_t *updates, uint64_t count, uint64_t *match,
                      uint64_t match_stride, const uint64_t *last_index, uint64_t G,
                      uint32_t n_max, uint64_t *n_skipped);
int hq_append_count_dev(hq_ctx *ctx, const uint64_t *updates, uint64_t count,
                        uint64_t *last_index, uint64_t *match_slot0, uint16_t *term_mask,
                        uint32_t ring_len, uint64_t G, uint64_t *n_skipped);

/* ---------------------------------------------------------------- progress table (tiles) ---- */
/*
 * The device-resident progress table in the headline layout: the commit kernel's own
 * HQ_LAYOUT_TILES_LEADER tiles of (n_max, form) — form HQ_FORM_TERM_START or HQ_FORM_TERM_MASK —
 * kept on the GPU across steps and decided in place (hq_commit_dev with layout
 * HQ_LAYOUT_TILES_LEADER | HQ_LAYOUT_IN_PLACE), so a step ships only its deltas and the decision
 * streams the same 8(n-1) + 26 or 8(n-1) + 32 bytes per group as the headline kernel. Build it
 * from columns with hq_tile_commit_as_host / _dev (HQ_LAYOUT_TILES_LEADER).
 *   hq_table_ingest_match_dev  remote.tryUpdate per ReplicateResp (remote.go:123-133):
 *                              match[slot] = max(match[slot], index); records as hq_match_update
 *                              (16-byte aligned); slot 0 (the leader, whose match is lastIndex)
 *                              and slot >= n_max are skipped and counted
 *   hq_table_ingest_lag_dev    the same from 8-byte records group << 32 | slot << 28 | lag
 *                              (index = lastIndex - lag as the table holds it when the kernel runs)
 *   hq_table_append_dev        appendEntries (raft.go:911-922): lastIndex = max(lastIndex,
 *                              new_last) and the term-mask bits of the new entries; records as
 *                              hq_append_update (16-byte aligned)
 *   hq_table_append_count_dev  the same from 8-byte records group << 32 | n: lastIndex += n
 *   hq_table_committed_dev     the committed row of every tile into committed[G], group order
 * flags: 0 = any batch (one 64-bit atomic per record, or binned: below); HQ_INGEST_GROUPED = the
 * caller guarantees
 * that the records of one key — (group, slot) for the ingests, group for the appends — are
 * adjacent in the batch (a step worker emitting node by node; a batch with unique keys is
 * grouped). Each wave then reduces its runs of equal keys with a segmented scan and applies a
 * run with one plain read-modify-write; runs that reach the wave's first or last lane (they may
 * continue in the next wave) use one atomic. Results equal the sequential application in any
 * order; a batch that is not grouped must not carry the flag. HQ_INGEST_UNIQUE = the caller
 * guarantees every key at most once in the batch (a step's final ack per (group, slot); one
 * append per group): each record is one plain read-modify-write of its own table word, no scan
 * and no atomic, in any order.
 * Ingests only (hq_table_ingest_match_dev / _lag_dev): HQ_INGEST_BINNED = records in any order
 * applied in two streaming passes without global atomics: the records are binned by table region
 * (2^k consecutive tiles) in LDS and written back bucket by bucket, then one workgroup per region
 * loads its match rows into LDS, applies every record of the region with LDS max and writes the
 * rows back (each table line read and written once). Chosen by default (flags 0 or
 * HQ_INGEST_UNIQUE) for a dense batch — at least 64 Ki records and one per 8 table slots — when
 * the table has at most 8192 regions (64 tiles each at n_max 3: 67 M groups); HQ_INGEST_BINNED
 * forces it (HQ_E_INVAL if the table is too large), HQ_INGEST_ATOMIC forces the per-record path.
 * Uses a device workspace of the context (8 bytes per record of a launch pair).
 */
#define HQ_INGEST_GROUPED 1u
#define HQ_INGEST_UNIQUE 2u
#define HQ_INGEST_ATOMIC 4u
#define HQ_INGEST_BINNED 8u
int hq_table_ingest_match_dev(hq_ctx *ctx, const hq_match_update *updates, uint64_t count,
                              uint64_t *tiles, uint64_t G, uint32_t n_max, uint32_t form,
                              uint32_t flags, uint64_t *n_skipped);
int hq_table_ingest_lag_dev(hq_ctx *ctx, const uint64_t *updates, uint64_t count,
                            uint64_t *tiles, uint64_t G, uint32_t n_max, uint32_t form,
                            uint32_t flags, uint64_t *n_skipped);
int hq_table_append_dev(hq_ctx *ctx, const hq_append_update *updates, uint64_t count,
                        uint64_t *tiles, uint64_t G, uint32_t n_max, uint32_t form,
                        uint32_t ring_len, uint32_t flags, uint64_t *n_skipped);
int hq_table_append_count_dev(hq_ctx *ctx, const uint64_t *updates, uint64_t count,
                              uint64_t *tiles, uint64_t G, uint32_t n_max, uint32_t form,
                              uint32_t ring_len, uint32_t flags, uint64_t *n_skipped);
int hq_table_committed_dev(hq_ctx *ctx, const uint64_t *tiles, uint64_t G, uint32_t n_max,
                           uint32_t form, uint64_t *committed);

/* ---------------------------------------------------------------- host-side packers --------- */
/*
 * The packers turn a step worker's per-group view — the membership maps r.remotes / r.observers
 * / r.witnesses (raft.go:206-208) and the response messages of the step — into the kernels' SoA
 * inputs, applying the reference's role rules. Host functions (no GPU); the caller owns every
 * array. Slot 0 is always the group's own node (the leader / candidate); then the other remotes,
 * then the witnesses, in member order; observers never get a slot (numVotingMembers,
 * raft.go:368-370; tryCommit raft.go:894-901). A group with more than n_max voting members, or
 * whose own node is not among its remotes, gets n_voting = 0 and a fallback bit, so the kernel
 * leaves it to the CPU path.
 */
#define HQ_ROLE_REMOTE   0u   /* full member (r.remotes) */
#define HQ_ROLE_OBSERVER 1u   /* non-voting member (r.observers) */
#define HQ_ROLE_WITNESS  2u   /* witness (r.witnesses): votes and counts, holds no data */

typedef struct hq_member {
    uint64_t node_id;
    uint64_t match;           /* remote.match (remote.go:62-69) */
    uint32_t role;            /* HQ_ROLE_* */
    uint32_t active;          /* remote.active (CheckQuorum) */
} hq_member;

typedef struct hq_group_view {
    uint64_t node_id;         /* this node: the leader (commit, ReadIndex) or candidate (vote) */
    uint64_t committed;       /* log.committed */
    uint64_t last_index;      /* log.lastIndex() */
    uint64_t term_start;      /* first index of the leader's term (term-start form) */
    uint64_t term;            /* r.term (ring form) */
    uint64_t ctx_low;         /* the pending ReadIndex SystemCtx (single-ctx form) */
    uint64_t ctx_high;
    uint16_t term_mask;       /* term-mask form */
    uint16_t reserved0;
    uint32_t reserved1;
    uint32_t first_member;    /* this group's members: members[first_member .. +n_members) */
    uint32_t n_members;
    uint32_t first_msg;       /* this group's step messages: msgs[first_msg .. +n_msgs) */
    uint32_t n_msgs;
} hq_group_view;

/* A response received in this step, in arrival order. RequestVoteResp: reject = m.Reject.
 * HeartbeatResp: hint_low / hint_high = m.Hint / m.HintHigh (the echoed SystemCtx). */
typedef struct hq_msg {
    uint64_t from;
    uint64_t hint_low;
    uint64_t hint_high;
    uint32_t reject;
    uint32_t reserved;
} hq_msg;

/* Commit inputs: match rows (n_max rows at args->match_stride), n_voting, committed_in,
 * last_index and, when non-NULL, term_start / term / term_mask of *args (host arrays).
 * args->G must equal G; args->fallback (may be NULL) receives the packing fallbacks. */
int hq_pack_commit(const hq_group_view *groups, uint64_t G, const hq_member *members,
                   hq_commit_args *args);

/* The u32 ring of HQ_FORM_TERM_RING32 from the u64 term ring (logentry.go:143-160 values):
 * ring32[i] = min(ring[i], 0xFFFFFFFF). `count` = G * ring_len entries. */
int hq_pack_ring32(const uint64_t *ring, uint64_t count, uint32_t *ring32);

/* Vote bitmaps: slot 0 granted (campaign's self vote, raft.go:1093); then every message from a
 * voting member sets its slot's granted or rejected bit if neither is set yet (first response
 * wins, raft.go:1071-1073); responses from observers (raft.go:1969-1972) and non-members
 * (Peer.Handle, peer.go:191-197) are dropped. */
int hq_pack_votes(const hq_group_view *groups, uint64_t G, const hq_member *members,
                  const hq_msg *msgs, uint8_t *granted, uint8_t *rejected, uint8_t *n_voting,
                  uint64_t *fallback);

/* ReadIndex ack bitmaps for the group's pending ctx: a HeartbeatResp from a voting member whose
 * hint equals (ctx_low, ctx_high) sets that member's slot (readindex.go:83; heartbeats carrying
 * a ctx go to voting members only, raft.go:836-848). Other hints, non-members and observers are
 * ignored. Also fills `active` from the members' active flags when non-NULL. */
int hq_pack_acks(const hq_group_view *groups, uint64_t G, const hq_member *members,
                 const hq_msg *msgs, uint8_t *ack, uint8_t *active, uint8_t *n_voting,
                 uint32_t n_max, uint64_t *fallback);

/* ---------------------------------------------------------------- step worker -------------- */
/*
 * The step worker is the caller side of the kernels: execEngine.processSteps (execengine.go:
 * 923-1000) for the quorum part of many Raft groups at once. It holds each group's quorum state
 * (raft.remotes / witnesses / observers, raft.go:206-208; entryLog committed / lastIndex and the
 * first index of the leader's term; readIndex, readindex.go:31-34; votes, raft.go:210) and takes
 * one step's events per group, in node.handleEvents order (node.go:1113-1157):
 *   1. the local ReadIndex           node.handleReadIndex -> Peer.ReadIndex (peer.go:297-303)
 *   2. received messages             handleReceivedMessages -> Peer.Handle (peer.go:186-198)
 *   3. tick messages                 CheckQuorum (raft.go:1582) / Election (raft.go:1485)
 *   4. proposals                     handleProposals -> handleLeaderPropose (raft.go:1590)
 * The input is laid out the way a step worker holds it: the groups that have events, each with
 * its event list (a node's message queue, node.mq), i.e. compressed rows over one event array.
 *
 * Membership filtering (Peer.Handle), the term check (onMessageTermNotMatched, raft.go:1416),
 * remote.tryUpdate, the confirmed-set inserts and first-response-wins votes are applied on the
 * host as the events are read; every quorum decision — tryCommit, the ReadIndex release with its
 * index rewrite, the vote outcome, leaderHasQuorum — is taken by the kernels above at the end of
 * a run of events. A run ends early only where a later event reads a decision (a ReadIndex
 * needs the committed index; a state change needs the vote / CheckQuorum outcome; a higher-term
 * message ends the group's leadership), so one step usually costs one GPU pass. Results equal
 * the reference processing the events one by one (tests/test_gpu_worker.py against
 * oracle/qref_step.c).
 *
 * Events the reference hands to code outside the quorum path without touching quorum state —
 * a follower or candidate forwarding or dropping a ReadIndex or a proposal — are returned as
 * `deferred`. Events the worker cannot take exactly suspend the group (`fallback`): an observer
 * acknowledging a pending ReadIndex ctx, a ReplicateResp above the leader's lastIndex, more
 * than 8 pending ReadIndex ctxs, an unknown message type or event kind. The group's events from
 * that one on are returned as deferred, its state is as of the event before, and it stays
 * suspended (its events deferred) until the caller re-syncs it with hq_worker_set_group.
 *
 * One worker per step worker goroutine; not thread-safe.
 */
#define HQ_STATE_FOLLOWER  0u
#define HQ_STATE_CANDIDATE 1u
#define HQ_STATE_LEADER    2u

/* raftpb.MessageType values (raftpb/raft.proto:26-52) the worker consumes */
#define HQ_MSG_REPLICATE_RESP    13u
#define HQ_MSG_REQUEST_VOTE_RESP 15u
#define HQ_MSG_HEARTBEAT_RESP    18u
#define HQ_MSG_READ_INDEX        19u

/* hq_event.kind */
#define HQ_EV_READ         1u  /* local ReadIndex: Peer.ReadIndex(ctx), From = NoNode; ctx in hint */
#define HQ_EV_MESSAGE      2u  /* a received pb.Message */
#define HQ_EV_CHECK_QUORUM 3u  /* the leader tick's CheckQuorum message (raft.go:1582-1588) */
#define HQ_EV_ELECTION     4u  /* the election tick's Election message (raft.go:1485-1515);
                                  issue it only when hasConfigChangeToApply() is false */
#define HQ_EV_PROPOSE      5u  /* a proposal of log_index entries (handleLeaderPropose) */

/* hq_state_change.reason */
#define HQ_REASON_VOTE         1u  /* vote outcome: became leader or follower */
#define HQ_REASON_CHECK_QUORUM 2u  /* leader lost quorum */
#define HQ_REASON_HIGHER_TERM  3u  /* a message with a higher term */
#define HQ_REASON_CAMPAIGN     4u  /* became candidate */
/* hq_dropped_read.reason (reportDroppedReadIndex) */
#define HQ_DROP_WITNESS   1u      /* ReadIndex from a witness (raft.go:1642-1643) */
#define HQ_DROP_NOT_READY 2u      /* no committed entry at the current term yet (:1645-1651) */

typedef struct hq_event {        /* one event of a group's step; messages carry the pb.Message
                                    fields the path reads (raft.proto:154-168) */
    uint32_t kind;               /* HQ_EV_* */
    uint32_t type;               /* HQ_EV_MESSAGE: HQ_MSG_* */
    uint64_t from;
    uint64_t term;
    uint64_t log_index;          /* HQ_EV_PROPOSE: number of entries */
    uint64_t hint;               /* HeartbeatResp / ReadIndex / HQ_EV_READ: SystemCtx.Low */
    uint64_t hint_high;          /* SystemCtx.High */
    uint32_t reject;
    uint32_t reserved;
} hq_event;

typedef struct hq_worker_group { /* a group's quorum state (add / set / get) */
    uint64_t cluster_id;
    uint64_t node_id;            /* this node; must be one of the group's remotes */
    uint64_t term;
    uint64_t committed;
    uint64_t last_index;
    uint64_t term_start;         /* leader: index of its first entry at `term` (its no-op) */
    uint32_t state;              /* HQ_STATE_* */
    uint32_t n_members;          /* remotes + witnesses + observers; at most 8 voting */
    uint32_t n_pending_reads;    /* get only */
    uint32_t suspended;          /* get only: 1 while the group is in fallback */
} hq_worker_group;

typedef struct hq_read_status {  /* readStatus (readindex.go:21-26), get only */
    uint64_t index;
    uint64_t from;
    uint64_t ctx_low;
    uint64_t ctx_high;
    uint32_t n_confirmed;
    uint32_t reserved;
} hq_read_status;

/* One step: group i of the list (a handle from hq_worker_add_group; each at most once) has the
 * events events[offsets[i] .. offsets[i + 1]) in the order above. */
typedef struct hq_step_input {
    uint64_t n_groups;
    const uint32_t *groups;
    const uint64_t *offsets;     /* [n_groups + 1], non-decreasing */
    const hq_event *events;
} hq_step_input;

typedef struct hq_commit_event { uint64_t cluster_id, committed; } hq_commit_event;
typedef struct hq_ready_to_read {   /* pb.ReadyToRead (raftpb/raft.go:54-57) */
    uint64_t cluster_id, index, ctx_low, ctx_high;
} hq_ready_to_read;
/* HQ_WORKER_READY_COMPACT: a ReadyToRead in 24 bytes. The host holds the rest: the group is the
 * pos-th of the step's list (its cluster id is the worker's), and the index is the group's
 * committed index before the step plus delta (a ReadIndex records the committed index when it
 * is received, raft.go:1636-1669; the host holds that committed index to apply entries) */
typedef struct hq_ready_compact {
    uint64_t ctx_low, ctx_high;
    uint32_t pos;
    int32_t delta;
} hq_ready_compact;
typedef struct hq_read_index_resp { /* ReadIndexResp to a remote requester (raft.go:1751-1757) */
    uint64_t cluster_id, to, log_index, hint, hint_high;
} hq_read_index_resp;
typedef struct hq_state_change {
    uint64_t cluster_id, term;
    uint32_t state, reason;
} hq_state_change;
typedef struct hq_dropped_read {
    uint64_t cluster_id, ctx_low, ctx_high, from;
    uint32_t reason, reserved;
} hq_dropped_read;

/* Results of one step; the arrays are owned by the worker and valid until its next call. Per
 * group, every list is in the order the reference produces it. `deferred` holds indexes into
 * the input's events array. */
typedef struct hq_step_output {
    const hq_commit_event *commits;        uint64_t n_commits;      /* committed index advanced */
    const hq_ready_to_read *ready;         uint64_t n_ready;
    const hq_read_index_resp *read_resps;  uint64_t n_read_resps;
    const hq_state_change *state_changes;  uint64_t n_state_changes;
    const hq_dropped_read *dropped_reads;  uint64_t n_dropped_reads;
    const uint64_t *deferred;              uint64_t n_deferred;
    const uint64_t *fallback_groups;       uint64_t n_fallback_groups;   /* cluster ids */
    uint64_t gpu_passes;        /* GPU passes (kernel batches + one sync each) of this step */
    uint64_t decisions;         /* group decisions taken on the GPU in this step */
    uint64_t handle_ns;         /* wall time: the host bookkeeping of the events */
    uint64_t pass_ns;           /* wall time: GPU passes (pack, copies, kernels, sync, apply) */
    uint64_t pack_ns;           /*   of which packing the kernels' SoA inputs */
    uint64_t device_ns;         /*   of which H2D + kernels + D2H + sync */
    uint64_t apply_ns;          /*   of which applying the decisions */
    /* (HQ_WORKER_ON_DEVICE workers: pack_ns = the host's time to queue the step's copies and
     * launches, device_ns = the thread's wait for the device after that (as for host workers:
     * the device's share of the pass, seen from the host), apply_ns = mapping the outputs after
     * the wait; gpu_ns below is the GPU's own time, so pass_ns - pack_ns - gpu_ns - apply_ns is
     * the wait the GPU's time does not explain: the waiting thread's wake-up and any queueing
     * ahead of the step) */
    /* HQ_WORKER_COMMIT_COLUMN workers only, else NULL: the step's commits as one word per
     * listed group (input order), its new committed index or 0 (no commit: a commit never sets
     * 0); `commits` is then NULL and n_commits counts the nonzero words */
    const uint64_t *committed_column;
    /* HQ_WORKER_COMMIT_ADVANCE workers only, else NULL: the step's commits as one 4-byte word per
     * listed group (input order), how far its committed index advanced (new - previous; 0: no
     * commit) — the host adds it to the committed index it already holds (entries (prev, prev +
     * advance] are committed); `commits` and `committed_column` are then NULL and n_commits
     * counts the nonzero words */
    const uint32_t *committed_advance;
    /* HQ_WORKER_READY_COMPACT workers only, else NULL: the step's ReadyToReads as 24-byte
     * records (hq_ready_compact, in the order of `ready`); `ready` is then NULL and n_ready
     * counts them. A step in which some record's delta does not fit 32 bits keeps `ready` */
    const hq_ready_compact *ready_compact;
    /* ABI 21. Device workers (0 otherwise): the step's clocks. device_ns above is the thread's
     * wait for the device (the time from the last queued operation to the wait's return);
     * gpu_ns the GPU's time between the step's timing events — with hq_worker_step_jobs the
     * shared launches' time, the same in each of the gpu_jobs workers' outputs (count it once).
     * The wait polled for wait_poll_ns, then slept wait_sleep_ns (wait_sleeps times: a blocking
     * wait is one); wait_end_ns is the host's steady clock at its return and, with HQ_WAIT_CLOCK,
     * device_end_ticks the device's 100-MHz constant clock after the step's last kernel (the
     * difference between the two over steps is the wake-up's lateness, hq_worker_set_wait). */
    uint64_t gpu_ns;
    uint32_t gpu_jobs;
    uint32_t wait_sleeps;
    uint64_t wait_poll_ns, wait_sleep_ns, wait_end_ns, device_end_ticks;
    /* HQ_WORKER_READY_SLOTS workers, a step that wrote slots (else NULL / 0): the single ReadyToRead
     * of every listed group whose only other record is its commit, as hq_ready_compact records in
     * per-tile slots — tile t (listed groups 256 t .. 256 t + 255) holds ready_slot_counts[t]
     * records at ready_slots[256 t ..], in group order; n_ready_slotted in all. They are not in
     * `ready` / `ready_compact` (n_ready counts the list only). A group's records are all in one
     * of the two; the step's ReadyToReads in the reference's order (group order) are the two merged
     * by the record's group position (`pos`; a 32-byte list record's group is its cluster id). */
    const hq_ready_compact *ready_slots;
    const uint32_t *ready_slot_counts;
    uint64_t n_ready_tiles, n_ready_slotted;
    /* HQ_WAIT_CLOCK, the jobs path: the device's 100-MHz clock before the step's first kernel (a
     * one-thread kernel ahead of it): (device_end_ticks - device_start_ticks) x 10 ns against
     * gpu_ns tells a step that waited in the device's queue from one whose kernels ran late */
    uint64_t device_start_ticks;
} hq_step_output;

typedef struct hq_worker hq_worker;

/* n_max: voting slots per group (1..8). */
int hq_worker_open(int device, uint32_t n_max, hq_worker **out);
/* flags: 0 (= hq_worker_open) or HQ_WORKER_ON_DEVICE — the groups' quorum state stays on the GPU
 * and hq_worker_step takes every event there: one thread per group handles its events one at a
 * time as the reference does (membership filter, term check, tryUpdate + tryCommit, the
 * confirmed-set insert + readIndex.confirm, handleLeaderReadIndex, the vote tally, CheckQuorum,
 * campaign, appendEntries, the state transitions), each decision at the event that triggers
 * it; the host ships the step's event rows and reads the result lists back (one launch pair,
 * two synchronisations). Same results as the host worker; groups of at most 16 members.
 * add/set/get_group work on a host mirror refreshed from the device when needed. */
#define HQ_WORKER_ON_DEVICE 1u
/* with HQ_WORKER_ON_DEVICE: a step in which more than half of the listed groups commit returns
 * its commits as hq_step_output.committed_column (8 bytes per listed group across PCIe instead
 * of a 16-byte record per commit); other steps keep the list */
#define HQ_WORKER_COMMIT_COLUMN 2u
/* with HQ_WORKER_ON_DEVICE: a step in which more than a quarter of the listed groups commit
 * returns its commits as hq_step_output.committed_advance (4 bytes per listed group); other steps,
 * and a step in which some group's committed index advances by 2^32 or more, keep the list */
#define HQ_WORKER_COMMIT_ADVANCE 4u
/* with HQ_WORKER_ON_DEVICE: the ReadyToReads as hq_step_output.ready_compact (24 bytes each
 * across PCIe instead of 32: the cluster id and the index are the host's already) */
#define HQ_WORKER_READY_COMPACT 8u
/* with HQ_WORKER_ON_DEVICE and HQ_WORKER_COMMIT_ADVANCE: the single ReadyToReads in per-tile slots
 * (hq_step_output.ready_slots): the engine's first pass writes them while it still reads the
 * step's stream (the host link's other direction) instead of a pass after it. Taken by sized
 * stream steps (hq_worker_step_stream / _step_jobs with sizes or sizes16; other inputs keep the
 * list); a record whose index - the group's committed index before the step does not fit 32
 * bits stays in the list */
#define HQ_WORKER_READY_SLOTS 16u
int hq_worker_open_ex(int device, uint32_t n_max, uint32_t flags, hq_worker **out);
void hq_worker_close(hq_worker *w);
const char *hq_worker_last_error(const hq_worker *w);
/* Add a group; members[0 .. g->n_members); *handle (may be NULL) receives its handle, the
 * group's index in the order of addition. Fails if the cluster exists, the node is not one of
 * its remotes or it has more than n_max voting members. */
int hq_worker_add_group(hq_worker *w, const hq_worker_group *g, const hq_member *members,
                        uint32_t *handle);
/* Add `count` groups (handles continue in order); group i's members follow group i-1's in
 * `members`. Stops at the first group that fails (the groups before it stay added). */
int hq_worker_add_groups(hq_worker *w, const hq_worker_group *groups, uint64_t count,
                         const hq_member *members);
/* The handle of a cluster. */
int hq_worker_find(hq_worker *w, uint64_t cluster_id, uint32_t *handle);
/* The worker's groups (handles 0 .. *n - 1; ABI 21). */
int hq_worker_group_count(hq_worker *w, uint64_t *n);
/* Overwrite a group's state (re-sync after fallback); clears its read queue and votes and
 * resumes it. */
int hq_worker_set_group(hq_worker *w, const hq_worker_group *g, const hq_member *members);
/* Read a group's state: members (up to cap) in the order given at add/set, and its pending
 * ReadIndex queue (up to reads_cap) in queue order. Either array may be NULL. */
int hq_worker_get_group(hq_worker *w, uint64_t cluster_id, hq_worker_group *g,
                        hq_member *members, uint32_t cap, hq_read_status *reads,
                        uint32_t reads_cap);
int hq_worker_step(hq_worker *w, const hq_step_input *in, hq_step_output *out);
/* How a device worker's thread waits for its step (ABI 21):
 *   HQ_WAIT_BLOCK  poll for poll_us, then sleep on a blocking-sync HIP event (the runtime's
 *                  interrupt wait) — the default, poll_us 50
 *   HQ_WAIT_SLEEP  poll for poll_us, then check every sleep_us microseconds, asleep in between
 *                  (a timer wake-up)
 *   HQ_WAIT_SPIN   poll (yielding) until the step is done: one host core per waiting worker
 *   HQ_WAIT_ADAPT  sleep once until poll_us (at least 100) before the end the previous step's wait
 *                  predicts, then poll (yielding); a step running past twice the prediction
 *                  sleeps on the blocking-sync event (the first step waits as HQ_WAIT_BLOCK)
 * | HQ_WAIT_CLOCK: a one-thread kernel behind each step stamps the device's constant clock
 *   (hq_step_output.device_end_ticks). The jobs path (hq_worker_step_jobs) waits with the first
 *   job's worker's policy. HQ_E_INVAL for a host worker or an unknown mode. */
#define HQ_WAIT_BLOCK 0u
#define HQ_WAIT_SLEEP 1u
#define HQ_WAIT_SPIN  2u
#define HQ_WAIT_ADAPT 3u
#define HQ_WAIT_CLOCK 0x100u
int hq_worker_set_wait(hq_worker *w, uint32_t mode, uint32_t poll_us, uint32_t sleep_us);

/* ---------------------------------------------------------------- event streams ------------- */
/*
 * The same step as a compact byte stream: group i's events are bytes[boffsets[i] ..
 * boffsets[i + 1]), one after another, each a header byte and LEB128 varints of exactly the
 * fields its handler reads. A steady-state leader step (ReplicateResp / HeartbeatResp /
 * proposals at the group's term) takes 3-7 bytes per event instead of the 56-byte row, so a
 * device worker's step crosses PCIe ~10x faster; the producer (a transport decoder, the caller's
 * own event queue, hq_wire_step_stream) writes it directly, or hq_events_encode turns rows into it.
 *
 *   header  bits 0-2  kind (HQ_EV_*; 0, 6, 7: not a valid kind -> the group falls back)
 *           bits 3-5  HQ_EV_MESSAGE: type code 0 ReplicateResp, 1 RequestVoteResp,
 *                     2 HeartbeatResp, 3 ReadIndex, 4 ReplicateResp whose log_index repeats
 *                     the group's previous ReplicateResp in the stream (its varint left out:
 *                     the followers of a steady leader ack the same index), 5 HeartbeatResp
 *                     whose hint / hint_high repeat the group's previous HeartbeatResp in the
 *                     stream (0 / 0 before the first: ctx-less acks and every follower's ack of
 *                     the same ctx), 7 another type (its varint follows). "Previous" counts
 *                     only events written with codes 0 / 4 (ReplicateResp) and 2 / 5
 *                     (HeartbeatResp): a ReplicateResp or HeartbeatResp written with code 7 does
 *                     not set the index / ctx that a later code 4 / 5 repeats (the encoder never
 *                     writes those two types with code 7); 6 a run (ABI 17): the next m events
 *                     repeat the group's previous message — a ReplicateResp or HeartbeatResp
 *                     written with codes 0 / 4 / 2 / 5 or in a run: its type, term, reject and
 *                     log_index / ctx — with other senders; a varint m >= 1, then m sender
 *                     varints (bit 6 of a run's header is 0; bit 7 0). Bit 7 set (ABI 21): the
 *                     consecutive form, senders s0, s0 + 1, .., s0 + m - 1 — a varint m, then s0
 *                     alone (s0 + m < 2^32). The acks of a steady leader's followers come as
 *                     runs: 2 + m bytes for m one-byte senders instead of 2 m, 3 bytes when the
 *                     followers' node ids are consecutive.
 *                     The encoders write a run for 3 to 6 such events (6: a run with 10-byte
 *                     senders still fits HQ_EVENT_STREAM_MAX)
 *           bit 6     reject
 *           bit 7     term repeats the group's previous message term in the stream (0 before
 *                     its first message): the term varint is left out
 *   READ: hint, hint_high      PROPOSE: log_index      CHECK_QUORUM, ELECTION: nothing
 *   MESSAGE: [type], from, [term], then ReplicateResp: log_index; RequestVoteResp: nothing;
 *            HeartbeatResp, ReadIndex: hint, hint_high; another type: log_index, hint, hint_high;
 *            codes 4 and 5: nothing more
 * Fields a handler does not read are not carried (hq_events_decode returns them as 0). Event
 * indexes (offsets, deferred) count events as in hq_step_input.
 */
#define HQ_EVENT_STREAM_MAX 64u   /* bytes one event (or one run) takes at most */

typedef struct hq_step_stream {
    uint64_t n_groups;
    const uint32_t *groups;
    const uint64_t *offsets;     /* [n_groups + 1] event index prefix, as hq_step_input */
    const uint64_t *boffsets;    /* [n_groups + 1] byte prefix into bytes, non-decreasing */
    const uint8_t *bytes;
    /* Sized form (sizes != NULL; offsets / boffsets are then not read): per group one word,
     * events | bytes << 16 (each < 2^16), and the totals over the step — 4 bytes per group
     * cross PCIe instead of the 16 of the two prefix arrays, and the device engine scans them.
     * Event indexes (deferred) count from 0 in group order as with offsets[0] = 0. In this form
     * `groups` may be NULL: the step lists the handles 0 .. n_groups - 1 in order (a worker
     * that steps all its groups every time; a group without events has size 0). */
    const uint32_t *sizes;
    uint64_t n_events, n_bytes;
    /* ABI 21, the sized form with 2-byte words (sizes NULL): per group its byte count (< 2^16)
     * only — 2 bytes per group cross the link instead of 4. The events are the group's bytes
     * decoded to their end, counted by the engine (n_events must still be their total); a
     * group's bytes that do not decode make the step HQ_E_INVAL (as a host worker's decoder
     * does), not a fallback of the group. */
    const uint16_t *sizes16;
} hq_step_stream;

/* Encode rows (offsets as in hq_step_input) into out[0 .. cap) and boffsets[0 .. n_groups];
 * HQ_E_STATE when fewer than HQ_EVENT_STREAM_MAX bytes are left before an event (size out for
 * HQ_EVENT_STREAM_MAX per event to never hit it). */
int hq_events_encode(uint64_t n_groups, const uint64_t *offsets, const hq_event *events,
                     uint8_t *out, uint64_t cap, uint64_t *boffsets);
/* The same with per-group size words (sizes[i] = events | bytes << 16, the hq_step_stream sized
 * form) and the byte total instead of boffsets; HQ_E_INVAL when a group has 2^16 or more events
 * or bytes (use boffsets for such a step). */
int hq_events_encode_sized(uint64_t n_groups, const uint64_t *offsets, const hq_event *events,
                           uint8_t *out, uint64_t cap, uint32_t *sizes, uint64_t *n_bytes);
/* Compact messages. A producer that keeps a step's messages as 16-byte records instead of the
 * 56-byte rows (what it must hold of a received pb.Message, raft.proto:154-168, for this path)
 * hands them to hq_events16_encode_sized, which writes the same stream bytes as encoding the
 * equivalent rows. A record is one event, or the escape HQ_EV16_FULL followed by the event as an
 * hq_event row in the next 4 records (64 bytes; the last 8 unused) when a field does not fit. */
typedef struct hq_event16 {
    uint8_t kind;       /* bits 0-2 HQ_EV_*, bit 3 reject, HQ_EV16_READ_CTX, HQ_EV16_FULL */
    uint8_t type;       /* HQ_EV_MESSAGE: HQ_MSG_* (< 256) */
    uint16_t from;      /* sender node id (< 2^16) */
    uint32_t term;      /* message term (< 2^32); HQ_EV_READ: SystemCtx.High (< 2^32) */
    uint64_t value;     /* ReplicateResp, other types, HQ_EV_PROPOSE: log_index; HQ_EV_READ:
                           SystemCtx.Low; HeartbeatResp / ReadIndex: SystemCtx.Low with High 0 */
} hq_event16;
/* a HeartbeatResp / ReadIndex whose ctx is that of the group's latest HQ_EV_READ record before it
 * in the call (0 / 0 if none): the acks of the heartbeat a ReadIndex broadcast (raft.go:836-848);
 * `value` is then not read */
#define HQ_EV16_READ_CTX 0x10u
#define HQ_EV16_FULL     0x80u   /* escape: the next 4 records hold the event as an hq_event */
/* Encode compact records: group i's records are recs[offsets16[i] .. offsets16[i + 1]) (an
 * escape and its 4 records are one event). Writes the sized form as hq_events_encode_sized does
 * for the equivalent rows (the same bytes and size words) and the event and byte totals.
 * threads > 1: that many native threads (a persistent pool shared by concurrent calls; a caller
 * runs only its own call's ranges), each encoding a range of groups into its own scratch before
 * the ranges are copied into place (0 or 1: the calling thread only). HQ_E_INVAL on a malformed
 * escape or a group of 2^16 events or bytes; HQ_E_STATE when fewer than HQ_EVENT_STREAM_MAX bytes
 * of out (cap bytes) are left before an event — the same rule at every thread count, as
 * hq_events_encode_sized (size out for HQ_EVENT_STREAM_MAX per event to never hit it). */
int hq_events16_encode_sized(uint64_t n_groups, const uint64_t *offsets16, const hq_event16 *recs,
                             uint8_t *out, uint64_t cap, uint32_t *sizes, uint64_t *n_events,
                             uint64_t *n_bytes, uint32_t threads);
/* Several streams at once — the steps of a GPU's step workers (execengine.go:675-690), one
 * stream each: hq_events16_encode_sized for every job, the groups of all jobs split into
 * `threads` ranges of about equal records (a range may cross from one job into the next), so
 * that the threads stay evenly loaded whatever the number of jobs (one call per job on a shared
 * pool queues the jobs past the threads' count: 16 workers on 14 threads took two rounds).
 * Every job's bytes, sizes and totals equal its own hq_events16_encode_sized call's; each job's
 * rc is its own (HQ_E_INVAL / HQ_E_STATE as there), the call returns the first job's failure. */
typedef struct hq_encode16_job {
    uint64_t n_groups;
    const uint64_t *offsets16;
    const hq_event16 *recs;
    uint8_t *out;
    uint64_t cap;
    uint32_t *sizes;
    uint64_t n_events, n_bytes;  /* out */
    int rc;                      /* out */
    int reserved;
    uint16_t *sizes16;           /* ABI 21: when not NULL, the 2-byte words (hq_step_stream.sizes16)
                                    are written here instead (sizes may then be NULL) */
} hq_encode16_job;
int hq_events16_encode_sized_multi(hq_encode16_job *jobs, uint32_t count, uint32_t threads);
/* Phase clocks of the threaded hq_events16_encode_sized calls (diagnostic; process-wide sums
 * since the last reset): wall = encode + copy phase per call; a range ("task") queued for the
 * pool waits `lag` from the call's queueing until a pool thread starts it (`helped` such starts;
 * the others ran on the caller); `run` = the tasks' own time. */
typedef struct hq_encode_stats {
    uint64_t calls, tasks, helped;
    uint64_t wall_ns, encode_ns, copy_ns;
    uint64_t lag_ns, max_lag_ns, run_ns;
} hq_encode_stats;
int hq_encode_stats_read(hq_encode_stats *out, int reset);
/* Rows to compact records: group i's events (offsets as in hq_step_input) become records
 * out[offsets16[i] .. offsets16[i + 1]) (an event that does not fit takes an escape: 5 records).
 * HQ_E_STATE when cap records cannot hold them (5 per event always can). */
int hq_events_to16(uint64_t n_groups, const uint64_t *offsets, const hq_event *events,
                   hq_event16 *out, uint64_t cap, uint64_t *offsets16);
/* Count each group's events in a stream (group i's bytes: bytes[boffsets[i] .. boffsets[i + 1])):
 * offsets[0] = 0, offsets[i + 1] = offsets[i] + its events — the event prefix of a stream given
 * with 2-byte size words. HQ_E_INVAL when a group's bytes do not decode to whole events. */
int hq_events_count(uint64_t n_groups, const uint64_t *boffsets, const uint8_t *bytes,
                    uint64_t *offsets);
/* Decode a stream back into rows events[offsets[0] .. offsets[n_groups]); HQ_E_INVAL when a
 * group's bytes do not hold exactly its events. */
int hq_events_decode(uint64_t n_groups, const uint64_t *offsets, const uint64_t *boffsets,
                     const uint8_t *bytes, hq_event *events);
/* hq_worker_step over a stream. An HQ_WORKER_ON_DEVICE worker ships the bytes and its device
 * engine decodes them (a group whose bytes are malformed falls back at the event that fails to
 * decode); a host worker decodes them into rows first (HQ_E_INVAL on malformed bytes). Inputs in
 * pinned memory (hq_alloc_pinned) copy fastest. */
int hq_worker_step_stream(hq_worker *w, const hq_step_stream *in, hq_step_output *out);

/* Several workers stepped at once, one native thread each (job 0 on the calling thread, the rest
 * on a process-wide pool): what a host's step-worker goroutines do when each calls its own
 * worker (execengine.go:923-1000). Each job names one of rows / stream. Every job's rc is set;
 * returns the first failing rc (HQ_E_INVAL, nothing run, if a worker appears twice). */
typedef struct hq_step_job {
    hq_worker *worker;
    const hq_step_input *rows;
    const hq_step_stream *stream;
    hq_step_output *out;
    int rc;
    int reserved;
} hq_step_job;
int hq_worker_step_jobs(hq_step_job *jobs, uint32_t count);

/* ---------------------------------------------------------------- wire decode --------------- */
/*
 * The step worker's input from the wire. A host receives raftpb.MessageBatch bytes (the protobuf
 * encoding of raftpb/raft.proto:154-168 Message and :191-196 MessageBatch, marshalled by
 * raft.pb.go Message.MarshalTo :2232 / MessageBatch.MarshalTo :2417) over the reference's TCP
 * transport; these functions turn them into hq_step_input rows the way the reference turns them
 * into Peer.Handle calls:
 *   Transport.handleRequest (internal/transport/transport.go:289-300): a batch whose
 *     deployment_id is not this host's or whose bin_ver is not HQ_RPC_BIN_VERSION is dropped;
 *   messageHandler.HandleMessageBatch (nodehost.go:2021-2061): SnapshotReceived messages are
 *     handled aside (not queued), messages of clusters this worker does not run are dropped,
 *     the rest are queued per cluster in arrival order;
 *   node.handleEvents (node.go:1113-1157) / handleReceivedMessages (:1257-1287): per cluster, the
 *     local ReadIndex first, then the received messages in arrival order, then the ticks
 *     (CheckQuorum / Election), then the proposals.
 * Any valid proto2 encoding is accepted (fields in any order, unknown fields skipped, entries and
 * snapshots counted but not decoded — the quorum path reads Type, From, Term, LogIndex, Reject,
 * Hint, HintHigh). A malformed batch (truncated, bad varint, wrong wire type of a known field)
 * is rejected whole with HQ_E_INVAL.
 */
#define HQ_RPC_BIN_VERSION 210u   /* raftio.RPCBinVersion (raftio/binversion.go:30) */

typedef struct hq_wire_message {  /* one decoded pb.Message */
    hq_event ev;                  /* kind HQ_EV_MESSAGE; type, from, term, log_index, hint,
                                     hint_high, reject */
    uint64_t cluster_id;
    uint64_t to;
    uint64_t log_term;
    uint64_t commit;
    uint32_t n_entries;           /* entries carried (field 11), not decoded */
    uint32_t has_snapshot;        /* field 12 present */
} hq_wire_message;

typedef struct hq_wire_batch_info {
    uint64_t n_messages;
    uint64_t deployment_id;
    uint64_t source_address_len;
    uint32_t bin_ver;
    uint32_t reserved;
} hq_wire_batch_info;

typedef struct hq_wire_stats {    /* counters since the last hq_wire_reset */
    uint64_t batches, bytes, messages, entries;
    uint64_t snapshot_received;   /* SnapshotReceived messages (handled aside by the host) */
    uint64_t dropped_batches;     /* foreign deployment id / binary version */
    uint64_t dropped_messages;    /* the messages of those batches */
    uint64_t dropped_no_cluster;  /* events of clusters the worker does not run */
} hq_wire_stats;

/* Stateless: decode one MessageBatch into out[0 .. min(count, cap)) (out may be NULL to count).
 * *count = messages in the batch; HQ_E_STATE if they do not fit cap. */
int hq_wire_decode_batch(const uint8_t *bytes, size_t len, hq_wire_message *out, uint64_t cap,
                         uint64_t *count, hq_wire_batch_info *info);

/* The sending side (ABI 21; benchmarks and tests): msgs[0 .. n) marshalled as one MessageBatch
 * exactly as MessageBatch.MarshalTo / Message.MarshalTo write it (raft.pb.go:2417-2445,
 * :2232-2296: every nullable=false field in field order, the empty Snapshot), then deployment_id,
 * source_address and HQ_RPC_BIN_VERSION. Messages with entries are HQ_E_INVAL (not marshalled);
 * HQ_E_STATE when cap is short (160 bytes per message and source_len + 24 always suffice). */
int hq_wire_encode_batch(const hq_wire_message *msgs, uint64_t n, uint64_t deployment_id,
                         const uint8_t *source, size_t source_len, uint8_t *out, uint64_t cap,
                         uint64_t *len);

typedef struct hq_wire hq_wire;
int hq_wire_open(uint64_t deployment_id, hq_wire **out);
void hq_wire_close(hq_wire *w);
const char *hq_wire_last_error(const hq_wire *w);
/* Start a step: forget every queued event. */
int hq_wire_reset(hq_wire *w);
/* Local events of a cluster for this step (HQ_EV_READ, HQ_EV_CHECK_QUORUM, HQ_EV_ELECTION,
 * HQ_EV_PROPOSE), in their order within each kind. */
int hq_wire_add_local(hq_wire *w, uint64_t cluster_id, const hq_event *events, uint64_t count);
/* Decode one received MessageBatch and queue its messages. */
int hq_wire_add_batch(hq_wire *w, const uint8_t *bytes, size_t len);
/* The step's hq_step_input for `worker`: clusters in order of first appearance, each with its
 * events in node.handleEvents order. Arrays owned by w until its next reset / step_input. */
int hq_wire_step_input(hq_wire *w, hq_worker *worker, hq_step_input *out, hq_wire_stats *stats);
/* The same step as an event stream (see "event streams" above); arrays owned by w likewise. */
int hq_wire_step_stream(hq_wire *w, hq_worker *worker, hq_step_stream *out, hq_wire_stats *stats);
/* Local events of many clusters at once: cluster c's are events[offsets[c] .. offsets[c + 1]). */
int hq_wire_add_locals(hq_wire *w, uint64_t n, const uint64_t *cluster_ids, const uint64_t *offsets,
                       const hq_event *events);
/* ABI 21, the step worker's production feed: the step in the worker's handle order, straight into
 * a sized stream. hq_wire_attach binds a worker (before events are queued): from then on every
 * message's cluster is resolved to the worker's handle as its batch is decoded (through a table
 * the wire keeps across steps — handles never change), messages of clusters the worker does not
 * run are dropped at once, and hq_wire_step_input / _step_stream are HQ_E_STATE. Each step:
 * hq_wire_reset, hq_wire_add_batch / hq_wire_add_locals, then hq_wire_step_sized writes every
 * handle h in 0 .. n - 1 (n = hq_worker_group_count) — its events in node.handleEvents order as
 * stream bytes into bytes[0 .. cap) and their byte count into sizes16[h] (0: no event) — and fills
 * *out as hq_step_stream's sized form with 2-byte words and groups = NULL, ready for
 * hq_worker_step_stream / hq_worker_step_jobs (bytes and sizes16 in pinned memory are read by
 * the device in place). HQ_E_STATE when cap runs short (HQ_EVENT_STREAM_MAX bytes per event
 * always suffice), HQ_E_INVAL when sizes16 has fewer than n words (n_cap) or a group reaches 2^16
 * events or bytes. The batch acceptance and per-cluster order are hq_wire_step_input's. */
int hq_wire_attach(hq_wire *w, hq_worker *worker);
int hq_wire_step_sized(hq_wire *w, uint8_t *bytes, uint64_t cap, uint16_t *sizes16, uint64_t n_cap,
                       hq_step_stream *out, hq_wire_stats *stats);

/* ---------------------------------------------------------------- synthetic inputs ---------- */

/*
 * Deterministic synthetic inputs generated on the device (benchmarks and parity tests; inputs
 * never cross PCIe). Group j of the call has clusterID cid = cid_base + j * cid_stride and draws
 * from splitmix64 seeded with (seed ^ cid). The byte-identical CPU generator is oracle/qgen.c;
 * the recipe is DESIGN.md "Synthetic inputs".
 */
typedef struct hq_synth_spec {
    uint64_t seed;
    uint64_t G;
    uint64_t cid_base;        /* clusterID of group 0 (>= 1; 0 is NoNode, raft.go:48) */
    uint64_t cid_stride;      /* clusterID step between consecutive groups (>= 1) */
    uint32_t n_max;           /* slots per group */
    uint32_t mixed_n;         /* 0: every group has n_max voters; 1: n = {3,5,7}[cid % 3] */
    uint32_t ring_len;        /* R: spread of committed/term_start below last, ring length */
    uint32_t parity_extras;   /* 1: add the rare edge cases (q > last, committed == last) */
} hq_synth_spec;

/* Fills match (n_max rows at args->match_stride), n_voting (if non-NULL), committed_in,
 * last_index, term_start, term, ring and term_mask (each if non-NULL) of *args; args->form is
 * ignored. term_mask needs spec->ring_len <= 16. */
int hq_synth_commit_dev(hq_ctx *ctx, const hq_synth_spec *spec, const hq_commit_args *args);
/* Fills the ack / granted / rejected bitmaps and n_voting (each if non-NULL). */
/* The same generated batch in the lag layout (hq_commit_lag_args; lag rows, cin_lag, ts_lag and
 * lag_mask, each if non-NULL); last_index (if non-NULL) receives the groups' lastIndex. */
int hq_synth_commit_lag_dev(hq_ctx *ctx, const hq_synth_spec *spec,
                            const hq_commit_lag_args *args, uint64_t *last_index);
int hq_synth_bitmaps_dev(hq_ctx *ctx, const hq_synth_spec *spec, uint8_t *ack, uint8_t *granted,
                         uint8_t *rejected, uint8_t *n_voting);

#ifdef __cplusplus
}
#endif
#endif /* HIPQUORUM_H */
