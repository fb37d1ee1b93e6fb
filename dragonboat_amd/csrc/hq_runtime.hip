// hq_runtime.hip — contexts, memory, timing and the host-pointer entry points of
// libhipquorum.so. Kernels and their _dev launchers live in hq_kernels.hip.
#include <cstdlib>
#include <cstring>
#include <new>

#include "hq_internal.h"

namespace {
thread_local std::string g_open_error;  // hq_open failures (no context yet)
}

namespace hq {

int fail(hq_ctx *ctx, int code, const std::string &msg) {
    if (ctx) ctx->err = msg;
    else g_open_error = msg;
    return code;
}

int check_hip(hq_ctx *ctx, hipError_t e, const char *what) {
    if (e == hipSuccess) return HQ_OK;
    return fail(ctx, e == hipErrorOutOfMemory ? HQ_E_NOMEM : HQ_E_DEVICE,
                std::string(what) + ": " + hipGetErrorString(e));
}

int pre_launch(hq_ctx *ctx) {
    int rc = check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (!rc && ctx->timing) ctx->region_launches++;
    return rc;
}

int post_launch(hq_ctx *ctx, const char *what) {
    int rc = check_hip(ctx, hipGetLastError(), what);
    // hq_timing_begin_after: the region opens behind the n-th launch, in stream order, so the
    // begin event fires when that launch ends and the next one is already queued
    if (!rc && ctx->begin_after && --ctx->begin_after == 0) {
        rc = check_hip(ctx, hipEventRecord(ctx->ev_begin, ctx->stream), "hipEventRecord");
        if (!rc) {
            ctx->timing = true;
            ctx->region_launches = 0;
        }
    }
    return rc;
}

int ensure_workspace(hq_ctx *ctx, size_t bytes) {
    if (ctx->ws_bytes >= bytes) return HQ_OK;
    if (ctx->ws) {
        int rc = check_hip(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
        if (rc) return rc;
        (void)hipFree(ctx->ws);
        ctx->ws = nullptr;
        ctx->ws_bytes = 0;
    }
    int rc = check_hip(ctx, hipMalloc(&ctx->ws, bytes), "hipMalloc(workspace)");
    if (rc) return rc;
    ctx->ws_bytes = bytes;
    return HQ_OK;
}

}  // namespace hq

extern "C" {

int hq_abi_version(void) { return HQ_ABI_VERSION; }

int hq_device_count(int *out) {
    if (!out) return HQ_E_INVAL;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *out = n;
    return HQ_OK;
}

int hq_device_pci_bus_id(int device, char *out, int len) {
    if (!out || len < 13) return HQ_E_INVAL;   // "dddd:bb:dd.f" + NUL
    out[0] = '\0';
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return HQ_E_DEVICE;
    if (device < 0 || device >= n) return HQ_E_INVAL;
    return hipDeviceGetPCIBusId(out, len, device) == hipSuccess ? HQ_OK : HQ_E_DEVICE;
}

int hq_pointer_kind(const void *p, int *kind) {
    if (!kind) return HQ_E_INVAL;
    *kind = HQ_PTR_UNREGISTERED;
    if (!p) return HQ_OK;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();   // pageable host memory reports an error: clear it
        return HQ_OK;
    }
    if (at.type == hipMemoryTypeDevice || at.type == hipMemoryTypeManaged)
        *kind = HQ_PTR_DEVICE;
    else if (at.type == hipMemoryTypeHost)
        *kind = HQ_PTR_PINNED_HOST;
    return HQ_OK;
}

int hq_open(int device, uint32_t flags, hq_ctx **out) {
    (void)flags;
    if (!out) return hq::fail(nullptr, HQ_E_INVAL, "hq_open: out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return hq::fail(nullptr, HQ_E_DEVICE, "hq_open: no HIP device visible");
    if (device < 0 || device >= n)
        return hq::fail(nullptr, HQ_E_INVAL, "hq_open: device index out of range");
    hq_ctx *ctx = new (std::nothrow) hq_ctx();
    if (!ctx) return hq::fail(nullptr, HQ_E_NOMEM, "hq_open: out of host memory");
    ctx->device = device;
    if (const char *b = std::getenv("HQ_BITS_BLOCK")) {
        const int v = std::atoi(b);
        if (v == 256 || v == 512 || v == 1024) ctx->bits_block = v;
    }
    if (const char *r = std::getenv("HQ_RI_PAIRS")) ctx->ri_pairs = std::atoi(r) != 0;
    if (const char *r = std::getenv("HQ_RI_UNIFORM")) ctx->ri_uniform = std::atoi(r) != 0;
    if (const char *gd = std::getenv("HQ_BIN_GRID")) {
        const int v = std::atoi(gd);
        if (v >= 8 && v <= 4096) ctx->bin_grid = (uint32_t)(v & ~7);
    }
    if (const char *tp = std::getenv("HQ_BIN_TPB")) {
        const int v = std::atoi(tp);
        if (v >= 0 && v <= 6) ctx->bin_tpb_shift = (uint32_t)v;
    }
    if (const char *at = std::getenv("HQ_BIN_APPLY_T")) {
        const int v = std::atoi(at);
        if (v == 512 || v == 1024) ctx->bin_apply_threads = (uint32_t)v;
    }
    if (const char *c = std::getenv("HQ_BIN_LAUNCH_CHUNKS")) {
        const int v = std::atoi(c);
        if (v >= 1 && v <= 4096) ctx->bin_launch_chunks = (uint32_t)v;
    }
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        std::string msg = std::string("hq_open: ") + hipGetErrorString(e);
        delete ctx;
        return hq::fail(nullptr, HQ_E_DEVICE, msg);
    }
    *out = ctx;
    return HQ_OK;
}

void hq_close(hq_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    if (ctx->ev_begin) (void)hipEventDestroy(ctx->ev_begin);
    if (ctx->ev_end) (void)hipEventDestroy(ctx->ev_end);
    if (ctx->ev_order) (void)hipEventDestroy(ctx->ev_order);
    if (ctx->ws) (void)hipFree(ctx->ws);
    if (ctx->bin_ws) (void)hipFree(ctx->bin_ws);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char *hq_last_error(const hq_ctx *ctx) {
    return ctx ? ctx->err.c_str() : g_open_error.c_str();
}

int hq_sync(hq_ctx *ctx) {
    if (!ctx) return HQ_E_INVAL;
    int rc = hq::check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (rc) return rc;
    return hq::check_hip(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
}

int hq_wait_for(hq_ctx *ctx, hq_ctx *other) {
    if (!ctx || !other) return HQ_E_INVAL;
    if (other == ctx) return HQ_OK;  // a stream is already ordered after itself
    if (other->device != ctx->device)
        return hq::fail(ctx, HQ_E_INVAL, "hq_wait_for: contexts on different devices");
    int rc = hq::check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (!rc && !other->ev_order)
        rc = hq::check_hip(ctx, hipEventCreateWithFlags(&other->ev_order, hipEventDisableTiming),
                           "hipEventCreateWithFlags");
    // the wait captures the event as just recorded, so re-recording it later is safe
    if (!rc) rc = hq::check_hip(ctx, hipEventRecord(other->ev_order, other->stream), "hipEventRecord");
    if (!rc)
        rc = hq::check_hip(ctx, hipStreamWaitEvent(ctx->stream, other->ev_order, 0),
                           "hipStreamWaitEvent");
    return rc;
}

int hq_malloc_dev(hq_ctx *ctx, size_t bytes, void **out) {
    if (!ctx || !out) return HQ_E_INVAL;
    *out = nullptr;
    int rc = hq::check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (rc) return rc;
    return hq::check_hip(ctx, hipMalloc(out, bytes ? bytes : 1), "hipMalloc");
}

int hq_free_dev(hq_ctx *ctx, void *p) {
    if (!ctx) return HQ_E_INVAL;
    if (!p) return HQ_OK;
    int rc = hq::check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (rc) return rc;
    return hq::check_hip(ctx, hipFree(p), "hipFree");
}

int hq_alloc_pinned(hq_ctx *ctx, size_t bytes, void **out) {
    if (!ctx || !out) return HQ_E_INVAL;
    *out = nullptr;
    return hq::check_hip(ctx, hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault),
                         "hipHostMalloc");
}

int hq_free_pinned(hq_ctx *ctx, void *p) {
    if (!ctx) return HQ_E_INVAL;
    if (!p) return HQ_OK;
    return hq::check_hip(ctx, hipHostFree(p), "hipHostFree");
}

int hq_memcpy_async(hq_ctx *ctx, void *dst, const void *src, size_t bytes, int kind) {
    if (!ctx) return HQ_E_INVAL;
    if (bytes == 0) return HQ_OK;
    if (!dst || !src) return hq::fail(ctx, HQ_E_INVAL, "hq_memcpy_async: NULL pointer");
    hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice
                    : kind == 1 ? hipMemcpyDeviceToHost
                    : kind == 2 ? hipMemcpyDeviceToDevice
                                : hipMemcpyDefault;
    if (kind < 0 || kind > 2) return hq::fail(ctx, HQ_E_INVAL, "hq_memcpy_async: bad kind");
    int rc = hq::check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (rc) return rc;
    return hq::check_hip(ctx, hipMemcpyAsync(dst, src, bytes, k, ctx->stream), "hipMemcpyAsync");
}

int hq_memset_async(hq_ctx *ctx, void *dst, int value, size_t bytes) {
    if (!ctx) return HQ_E_INVAL;
    if (bytes == 0) return HQ_OK;
    if (!dst) return hq::fail(ctx, HQ_E_INVAL, "hq_memset_async: NULL pointer");
    int rc = hq::check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (rc) return rc;
    return hq::check_hip(ctx, hipMemsetAsync(dst, value, bytes, ctx->stream), "hipMemsetAsync");
}

static int timing_close(hq_ctx *ctx) {
    ctx->begin_after = 0;   // a region that never opened records nothing
    if (!ctx->timing) return HQ_OK;
    int rc = hq::check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (!rc) rc = hq::check_hip(ctx, hipEventRecord(ctx->ev_end, ctx->stream), "hipEventRecord");
    if (rc) return rc;
    ctx->timing = false;
    ctx->region_done = true;
    return HQ_OK;
}

static int timing_fold(hq_ctx *ctx) {
    if (!ctx->region_done) return HQ_OK;
    int rc = hq::check_hip(ctx, hipEventSynchronize(ctx->ev_end), "hipEventSynchronize");
    if (rc) return rc;
    float ms = 0.f;
    rc = hq::check_hip(ctx, hipEventElapsedTime(&ms, ctx->ev_begin, ctx->ev_end),
                       "hipEventElapsedTime");
    if (rc) return rc;
    ctx->timed_ms += ms;
    ctx->timed_launches += ctx->region_launches;
    ctx->region_launches = 0;
    ctx->region_done = false;
    return HQ_OK;
}

int hq_timing_enable(hq_ctx *ctx, int enable) {
    if (!ctx) return HQ_E_INVAL;
    if (!enable) return timing_close(ctx);
    if (ctx->timing) return HQ_OK;
    int rc = timing_fold(ctx);  // a previous region is accumulated before its events are reused
    if (rc) return rc;
    rc = hq::check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (!rc && !ctx->ev_begin) rc = hq::check_hip(ctx, hipEventCreate(&ctx->ev_begin), "hipEventCreate");
    if (!rc && !ctx->ev_end) rc = hq::check_hip(ctx, hipEventCreate(&ctx->ev_end), "hipEventCreate");
    if (!rc) rc = hq::check_hip(ctx, hipEventRecord(ctx->ev_begin, ctx->stream), "hipEventRecord");
    if (rc) return rc;
    ctx->timing = true;
    ctx->region_launches = 0;
    return HQ_OK;
}

int hq_timing_begin_after(hq_ctx *ctx, uint64_t launches) {
    if (!ctx) return HQ_E_INVAL;
    if (launches == 0) return hq_timing_enable(ctx, 1);
    if (ctx->timing || ctx->begin_after)
        return hq::fail(ctx, HQ_E_STATE, "hq_timing_begin_after: a timed region is already open");
    int rc = timing_fold(ctx);
    if (rc) return rc;
    rc = hq::check_hip(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    if (!rc && !ctx->ev_begin) rc = hq::check_hip(ctx, hipEventCreate(&ctx->ev_begin), "hipEventCreate");
    if (!rc && !ctx->ev_end) rc = hq::check_hip(ctx, hipEventCreate(&ctx->ev_end), "hipEventCreate");
    if (rc) return rc;
    ctx->begin_after = launches;
    return HQ_OK;
}

int hq_timing_read(hq_ctx *ctx, double *total_ms, uint64_t *launches) {
    if (!ctx) return HQ_E_INVAL;
    int rc = timing_close(ctx);
    if (!rc) rc = timing_fold(ctx);
    if (rc) return rc;
    if (total_ms) *total_ms = ctx->timed_ms;
    if (launches) *launches = ctx->timed_launches;
    return HQ_OK;
}

int hq_timing_reset(hq_ctx *ctx) {
    if (!ctx) return HQ_E_INVAL;
    int rc = timing_close(ctx);
    if (!rc) rc = timing_fold(ctx);
    if (rc) return rc;
    ctx->timed_ms = 0.0;
    ctx->timed_launches = 0;
    return HQ_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- host-pointer entry points --
// Stage host arrays through the context's device workspace: H2D, kernel, D2H, synchronise.

namespace {

struct Stage {
    hq_ctx *ctx;
    char *base;
    size_t off = 0;
    explicit Stage(hq_ctx *c) : ctx(c), base(static_cast<char *>(c->ws)) {}
    static size_t pad(size_t b) { return (b + 255) & ~size_t(255); }
    template <class T>
    T *take(size_t bytes) {
        T *p = reinterpret_cast<T *>(base + off);
        off += pad(bytes);
        return p;
    }
};

int h2d(hq_ctx *ctx, void *d, const void *h, size_t b) { return hq_memcpy_async(ctx, d, h, b, 0); }
int d2h(hq_ctx *ctx, void *h, const void *d, size_t b) { return hq_memcpy_async(ctx, h, d, b, 1); }

// HQ_LAYOUT_TILES(_LEADER) from host memory: the tiles are one block, so the whole input is one
// H2D copy
int commit_tiles_host(hq_ctx *ctx, const hq_commit_args *a) {
    if (!a->match || !a->committed_out || a->n_max < 1 || a->n_max > HQ_MAX_VOTERS ||
        a->form > HQ_FORM_TERM_RING32)
        return hq_commit_dev(ctx, a);  // same validation and message
    const bool ring = a->form == HQ_FORM_TERM_RING, ring32 = a->form == HQ_FORM_TERM_RING32;
    if ((ring && !a->ring) || (ring32 && !a->ring32)) return hq_commit_dev(ctx, a);
    if ((ring || ring32) && (a->ring_len < 1 || a->ring_len > 1024)) return hq_commit_dev(ctx, a);
    const uint64_t G = a->G, nw = hq::words64(G);
    const size_t tiles =
        hq_commit_tiles(G) * hq_commit_tile_words_for(a->n_max, a->form, a->layout) * 8;
    const size_t ring_bytes = ring ? G * 8 * a->ring_len : ring32 ? G * 4 * a->ring_len : 0;
    const size_t need = Stage::pad(tiles) + Stage::pad(G * 8) + 2 * Stage::pad(nw * 8) +
                        Stage::pad(G) + Stage::pad(ring_bytes);
    int rc = hq::ensure_workspace(ctx, need);
    if (rc) return rc;
    Stage s(ctx);
    hq_commit_args d = *a;
    uint64_t *dt = s.take<uint64_t>(tiles), *dco = s.take<uint64_t>(G * 8);
    d.match = dt;
    d.committed_out = dco;
    rc = h2d(ctx, dt, a->match, tiles);
    if (ring || ring32) {
        void *dr = s.take<char>(ring_bytes);
        if (ring) d.ring = static_cast<const uint64_t *>(dr);
        else d.ring32 = static_cast<const uint32_t *>(dr);
        if (!rc) rc = h2d(ctx, dr, ring ? (const void *)a->ring : (const void *)a->ring32,
                          ring_bytes);
    }
    uint8_t *dnv = s.take<uint8_t>(G);
    if (a->n_voting) {
        d.n_voting = dnv;
        if (!rc) rc = h2d(ctx, dnv, a->n_voting, G);
    }
    uint64_t *dchg = s.take<uint64_t>(nw * 8), *dfb = s.take<uint64_t>(nw * 8);
    d.changed = a->changed ? dchg : nullptr;
    d.fallback = a->fallback ? dfb : nullptr;
    if (!rc) rc = hq_commit_dev(ctx, &d);
    if (!rc) rc = d2h(ctx, a->committed_out, dco, G * 8);
    if (!rc && a->changed) rc = d2h(ctx, a->changed, dchg, nw * 8);
    if (!rc && a->fallback) rc = d2h(ctx, a->fallback, dfb, nw * 8);
    if (!rc) rc = hq_sync(ctx);
    return rc;
}

}  // namespace

extern "C" {

int hq_commit(hq_ctx *ctx, const hq_commit_args *a) {
    if (!ctx) return HQ_E_INVAL;
    if (!a) return hq::fail(ctx, HQ_E_INVAL, "hq_commit: args is NULL");
    if (a->G == 0) return HQ_OK;
    if (a->layout & HQ_LAYOUT_IN_PLACE)
        return hq::fail(ctx, HQ_E_INVAL,
                        "hq_commit: HQ_LAYOUT_IN_PLACE is a device-resident table (hq_commit_dev)");
    if (a->layout == HQ_LAYOUT_TILES || a->layout == HQ_LAYOUT_TILES_LEADER)
        return commit_tiles_host(ctx, a);
    if (!a->match || !a->committed_in || !a->committed_out || !a->last_index ||
        a->n_max < 1 || a->n_max > HQ_MAX_VOTERS || a->match_stride < a->G)
        return hq_commit_dev(ctx, a);  // same validation and message
    const uint64_t G = a->G, nw = hq::words64(G);
    const bool ring = a->form == HQ_FORM_TERM_RING;
    const bool ring32 = a->form == HQ_FORM_TERM_RING32;
    const bool mask = a->form == HQ_FORM_TERM_MASK;
    if (a->form > HQ_FORM_TERM_RING32) return hq_commit_dev(ctx, a);
    if (ring && (!a->ring || !a->term)) return hq_commit_dev(ctx, a);
    if (ring32 && (!a->ring32 || !a->term)) return hq_commit_dev(ctx, a);
    if (mask && !a->term_mask) return hq_commit_dev(ctx, a);
    if (!ring && !ring32 && !mask && !a->term_start) return hq_commit_dev(ctx, a);
    if ((ring || ring32) && (a->ring_len < 1 || a->ring_len > 1024)) return hq_commit_dev(ctx, a);
    const size_t col = G * 8;
    const size_t ring_bytes = ring ? col * a->ring_len : ring32 ? G * 4 * a->ring_len : 0;
    size_t need = Stage::pad(col * a->n_max) + 4 * Stage::pad(col) + 2 * Stage::pad(nw * 8) +
                  Stage::pad(G) + Stage::pad(ring_bytes);
    int rc = hq::ensure_workspace(ctx, need);
    if (rc) return rc;
    Stage s(ctx);
    hq_commit_args d = *a;
    uint64_t *dm = s.take<uint64_t>(col * a->n_max);
    d.match = dm;
    d.match_stride = G;
    for (uint32_t k = 0; k < a->n_max && !rc; ++k)
        rc = h2d(ctx, dm + (size_t)k * G, a->match + (size_t)k * a->match_stride, col);
    uint64_t *dci = s.take<uint64_t>(col), *dco = s.take<uint64_t>(col);
    uint64_t *dlast = s.take<uint64_t>(col), *daux = s.take<uint64_t>(col);
    d.committed_in = dci;
    d.committed_out = dco;
    d.last_index = dlast;
    if (!rc) rc = h2d(ctx, dci, a->committed_in, col);
    if (!rc) rc = h2d(ctx, dlast, a->last_index, col);
    if (ring) {
        d.term = daux;
        uint64_t *dring = s.take<uint64_t>(col * a->ring_len);
        d.ring = dring;
        if (!rc) rc = h2d(ctx, daux, a->term, col);
        if (!rc) rc = h2d(ctx, dring, a->ring, col * a->ring_len);
    } else if (ring32) {
        d.term = daux;
        uint32_t *dring = s.take<uint32_t>(ring_bytes);
        d.ring32 = dring;
        if (!rc) rc = h2d(ctx, daux, a->term, col);
        if (!rc) rc = h2d(ctx, dring, a->ring32, ring_bytes);
    } else if (mask) {
        d.term_mask = reinterpret_cast<uint16_t *>(daux);
        if (!rc) rc = h2d(ctx, daux, a->term_mask, G * 2);
    } else {
        d.term_start = daux;
        if (!rc) rc = h2d(ctx, daux, a->term_start, col);
    }
    uint8_t *dnv = s.take<uint8_t>(G);
    if (a->n_voting) {
        d.n_voting = dnv;
        if (!rc) rc = h2d(ctx, dnv, a->n_voting, G);
    }
    uint64_t *dchg = s.take<uint64_t>(nw * 8), *dfb = s.take<uint64_t>(nw * 8);
    d.changed = a->changed ? dchg : nullptr;
    d.fallback = a->fallback ? dfb : nullptr;
    if (!rc) rc = hq_commit_dev(ctx, &d);
    if (!rc) rc = d2h(ctx, a->committed_out, dco, col);
    if (!rc && a->changed) rc = d2h(ctx, a->changed, dchg, nw * 8);
    if (!rc && a->fallback) rc = d2h(ctx, a->fallback, dfb, nw * 8);
    if (!rc) rc = hq_sync(ctx);
    return rc;
}

static int bits_host(hq_ctx *ctx, uint64_t G, const uint8_t *const *ins, int nin,
                     const uint8_t *nv, uint8_t **dins, uint8_t **dnv, uint64_t **dout,
                     int nout, const size_t *out_bytes) {
    size_t need = Stage::pad(G) * (nin + 1);
    for (int i = 0; i < nout; ++i) need += Stage::pad(out_bytes[i]);
    int rc = hq::ensure_workspace(ctx, need);
    if (rc) return rc;
    Stage s(ctx);
    for (int i = 0; i < nin && !rc; ++i) {
        dins[i] = s.take<uint8_t>(G);
        rc = h2d(ctx, dins[i], ins[i], G);
    }
    *dnv = s.take<uint8_t>(G);
    if (nv && !rc) rc = h2d(ctx, *dnv, nv, G);
    if (!nv) *dnv = nullptr;
    for (int i = 0; i < nout; ++i) dout[i] = s.take<uint64_t>(out_bytes[i]);
    return rc;
}

int hq_readindex(hq_ctx *ctx, uint64_t G, const uint8_t *ack, const uint8_t *n_voting,
                 uint32_t n_uniform, uint64_t *confirmed, uint64_t *fallback) {
    if (!ctx) return HQ_E_INVAL;
    if (G == 0) return HQ_OK;
    if (!ack || !confirmed) return hq::fail(ctx, HQ_E_INVAL, "hq_readindex: NULL ack/confirmed");
    const size_t wb = hq::words64(G) * 8;
    const uint8_t *ins[1] = {ack};
    uint8_t *dins[1], *dnv;
    uint64_t *dout[2];
    size_t ob[2] = {wb, wb};
    int rc = bits_host(ctx, G, ins, 1, n_voting, dins, &dnv, dout, 2, ob);
    if (!rc) rc = hq_readindex_dev(ctx, G, dins[0], dnv, n_uniform, dout[0],
                                   fallback ? dout[1] : nullptr);
    if (!rc) rc = d2h(ctx, confirmed, dout[0], wb);
    if (!rc && fallback) rc = d2h(ctx, fallback, dout[1], wb);
    if (!rc) rc = hq_sync(ctx);
    return rc;
}

int hq_vote(hq_ctx *ctx, uint64_t G, const uint8_t *granted, const uint8_t *rejected,
            const uint8_t *n_voting, uint32_t n_uniform, uint64_t *outcome, uint64_t *fallback) {
    if (!ctx) return HQ_E_INVAL;
    if (G == 0) return HQ_OK;
    if (!granted || !rejected || !outcome)
        return hq::fail(ctx, HQ_E_INVAL, "hq_vote: NULL granted/rejected/outcome");
    const size_t wb = hq::words64(G) * 8, ob2 = hq::words32(G) * 8;
    const uint8_t *ins[2] = {granted, rejected};
    uint8_t *dins[2], *dnv;
    uint64_t *dout[2];
    size_t ob[2] = {ob2, wb};
    int rc = bits_host(ctx, G, ins, 2, n_voting, dins, &dnv, dout, 2, ob);
    if (!rc) rc = hq_vote_dev(ctx, G, dins[0], dins[1], dnv, n_uniform, dout[0],
                              fallback ? dout[1] : nullptr);
    if (!rc) rc = d2h(ctx, outcome, dout[0], ob2);
    if (!rc && fallback) rc = d2h(ctx, fallback, dout[1], wb);
    if (!rc) rc = hq_sync(ctx);
    return rc;
}

}  // extern "C"
