/*
 * qgen.c — CPU twin of the device synthetic-input generator (hq_synth_*_dev). TEST
 * INFRASTRUCTURE ONLY. The recipe (DESIGN.md "Synthetic inputs") is restated
 * here independently of the HIP code; the GPU parity tests compare both generators' outputs
 * byte for byte before comparing decisions.
 */
#include "qref.h"

uint64_t qgen_splitmix64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int group_n(const qgen_spec *s, uint64_t cid) {
    static const int mixed[3] = {3, 5, 7};
    return s->mixed_n ? mixed[cid % 3] : (int)s->n_max;
}

int qgen_commit(const qgen_spec *s, const qref_commit_args *o) {
    const uint64_t R = s->ring_len;
    if (R < 1 || (R & (R - 1)) || s->n_max < 1 || s->n_max > 8 || s->cid_stride < 1) return -1;
    if (s->mixed_n && s->n_max < 7) return -1;
    for (uint64_t j = 0; j < s->G; j++) {
        const uint64_t cid = s->cid_base + j * s->cid_stride;
        uint64_t st = s->seed ^ cid;
        const int n = group_n(s, cid);
        const uint64_t term = 2 + qgen_splitmix64(&st) % ((1ull << 20) - 2);
        const uint64_t last = (1ull << 20) + qgen_splitmix64(&st) % (1ull << 40);
        uint64_t committed = last - qgen_splitmix64(&st) % R;
        const uint64_t term_start = last - qgen_splitmix64(&st) % R + 1;
        if (s->parity_extras) {
            uint64_t x = qgen_splitmix64(&st);
            if (x % 100 == 0) committed = last;
        }
        for (int k = 0; k < (int)s->n_max; k++) {
            uint64_t m;
            if (k >= n) {
                m = 0;
            } else if (k == 0) {
                m = last;                       /* leader's own remote: lastIndex (raft.go:918) */
            } else {
                uint64_t a = qgen_splitmix64(&st);
                uint64_t b = qgen_splitmix64(&st);
                m = committed - a % 4 + b % (last - committed + 4);
                if (m > last) m = last;
                if (s->parity_extras) {
                    uint64_t c = qgen_splitmix64(&st);
                    if (c % 100 == 0) m = last + 1 + (c / 100) % 3;
                }
            }
            if (o->match) ((uint64_t *)o->match)[(uint64_t)k * o->match_stride + j] = m;
        }
        if (o->n_voting) ((uint8_t *)o->n_voting)[j] = (uint8_t)n;
        if (o->committed_in) ((uint64_t *)o->committed_in)[j] = committed;
        if (o->last_index) ((uint64_t *)o->last_index)[j] = last;
        if (o->term_start) ((uint64_t *)o->term_start)[j] = term_start;
        if (o->term) ((uint64_t *)o->term)[j] = term;
        if (o->ring || o->term_mask) {
            uint64_t cur = term;
            uint32_t mask = 0;
            for (uint64_t k = 0; k < R; k++) {
                const uint64_t i = last - k;
                uint64_t t;
                if (i >= term_start) {
                    t = term;
                } else {
                    uint64_t x = qgen_splitmix64(&st);
                    uint64_t dec = (i + 1 == term_start) ? 1 + (x & 1) : (x & 1);
                    cur = cur > dec ? cur - dec : 1;
                    t = cur;
                }
                if (o->ring) ((uint64_t *)o->ring)[j * R + (i & (R - 1))] = t;
                mask |= (uint32_t)(t == term) << (i & (R - 1));
            }
            if (o->term_mask) ((uint16_t *)o->term_mask)[j] = (uint16_t)mask;
        }
    }
    return 0;
}

int qgen_c1_stream(uint64_t seed, uint64_t T, uint64_t committed0, uint64_t last0,
                   uint64_t *match, uint64_t *last) {
    uint64_t st = seed ^ 1;   /* clusterID 1 */
    uint64_t m[3] = {last0, committed0, committed0};
    uint64_t l = last0;
    for (uint64_t t = 0; t < T; t++) {
        uint64_t x = qgen_splitmix64(&st);
        if (t % 8 == 7) {                          /* leader appends 1..4 entries */
            l += 1 + (x >> 8) % 4;
            m[0] = l;
        }
        int slot = 1 + (int)(x & 1);               /* one follower's ReplicateResp */
        uint64_t nm = m[slot] + (x >> 1) % 4;
        m[slot] = nm > l ? l : nm;
        for (int s = 0; s < 3; s++) match[(uint64_t)s * T + t] = m[s];
        last[t] = l;
    }
    return 0;
}

/* 16-bit Bernoulli draws carved from successive splitmix64 outputs */
typedef struct { uint64_t st, buf; int avail; } bern_t;
static int bern(bern_t *b, uint32_t thr16) {
    if (b->avail == 0) { b->buf = qgen_splitmix64(&b->st); b->avail = 4; }
    uint32_t v = (uint32_t)(b->buf & 0xFFFF);
    b->buf >>= 16;
    b->avail--;
    return v < thr16;
}

#define P60 39322u   /* 0.6 * 65536 */
#define P30 19661u   /* 0.3 * 65536 */

int qgen_bitmaps(const qgen_spec *s, uint8_t *ack, uint8_t *granted, uint8_t *rejected,
                 uint8_t *n_voting) {
    if (s->n_max < 1 || s->n_max > 8 || s->cid_stride < 1) return -1;
    if (s->mixed_n && s->n_max < 7) return -1;
    for (uint64_t j = 0; j < s->G; j++) {
        const uint64_t cid = s->cid_base + j * s->cid_stride;
        bern_t b = {s->seed ^ cid, 0, 0};
        const int n = group_n(s, cid);
        uint32_t a = 0, g = 1, r = 0;     /* self (slot 0) votes for itself, never acks */
        for (int k = 1; k < n; k++) if (bern(&b, P60)) a |= 1u << k;
        for (int k = 1; k < n; k++) if (bern(&b, P60)) g |= 1u << k;
        for (int k = 1; k < n; k++) if (!((g >> k) & 1) && bern(&b, P30)) r |= 1u << k;
        if (s->parity_extras) {
            uint64_t x = qgen_splitmix64(&b.st);
            if (x % 50 == 0) r |= g & ~1u;          /* overlapping grant+reject: first wins */
            if (x % 50 == 1) a |= 1u;               /* self bit in ack: counted literally */
            if (x % 50 == 2) a |= 0xFFu & ~((1u << n) - 1);   /* bits beyond n: ignored */
        }
        if (ack) ack[j] = (uint8_t)a;
        if (granted) granted[j] = (uint8_t)g;
        if (rejected) rejected[j] = (uint8_t)r;
        if (n_voting) n_voting[j] = (uint8_t)n;
    }
    return 0;
}
