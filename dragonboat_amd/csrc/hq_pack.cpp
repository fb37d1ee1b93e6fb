// hq_pack.cpp — host-side packers of libhipquorum.so: a step worker's per-group membership and
// step messages -> the kernels' structure-of-arrays inputs, with the reference's role rules
// (include/hipquorum.h "host-side packers"). Plain C++ on the host; no GPU calls.
#include <cstdint>
#include <cstring>

#include "../../include/hipquorum.h"

namespace {

// Voting slots of one group: slot 0 = the group's own node (must be a remote), then the other
// remotes, then the witnesses, in member order. Observers get no slot (raft.go:368-370).
struct Slots {
    int n = 0;
    int member[HQ_MAX_VOTERS];
    bool ok = false;
};

Slots voting_slots(const hq_group_view &v, const hq_member *m, uint32_t n_max) {
    Slots s;
    const hq_member *mm = m + v.first_member;
    int self = -1, count = 0;
    for (uint32_t i = 0; i < v.n_members; ++i) {
        if (mm[i].role == HQ_ROLE_OBSERVER) continue;
        if (mm[i].role != HQ_ROLE_REMOTE && mm[i].role != HQ_ROLE_WITNESS) return s;  // unknown role
        ++count;
        if (mm[i].role == HQ_ROLE_REMOTE && mm[i].node_id == v.node_id) self = (int)i;
    }
    if (self < 0 || count > (int)n_max || count > HQ_MAX_VOTERS) return s;
    s.member[s.n++] = self;
    for (uint32_t pass = 0; pass < 2; ++pass) {
        const uint32_t role = pass == 0 ? HQ_ROLE_REMOTE : HQ_ROLE_WITNESS;
        for (uint32_t i = 0; i < v.n_members; ++i)
            if (mm[i].role == role && (int)i != self) s.member[s.n++] = (int)i;
    }
    s.ok = true;
    return s;
}

// slot of `from` among the voting members, -1 for observers and non-members
int slot_of(const Slots &s, const hq_group_view &v, const hq_member *m, uint64_t from) {
    for (int k = 0; k < s.n; ++k)
        if (m[v.first_member + s.member[k]].node_id == from) return k;
    return -1;
}

inline void set_bit(uint64_t *bm, uint64_t g) {
    if (bm) bm[g >> 6] |= 1ull << (g & 63);
}

}  // namespace

extern "C" int hq_pack_commit(const hq_group_view *groups, uint64_t G, const hq_member *members,
                              hq_commit_args *a) {
    if (G == 0) return HQ_OK;
    if (!groups || !members || !a || !a->match || !a->committed_in || !a->last_index ||
        !a->n_voting || a->G != G || a->match_stride < G || a->n_max < 1 ||
        a->n_max > HQ_MAX_VOTERS)
        return HQ_E_INVAL;
    uint64_t *match = const_cast<uint64_t *>(a->match);
    uint8_t *nv = const_cast<uint8_t *>(a->n_voting);
    if (a->fallback) std::memset(a->fallback, 0, ((G + 63) / 64) * 8);
    for (uint64_t g = 0; g < G; ++g) {
        const hq_group_view &v = groups[g];
        const Slots s = voting_slots(v, members, a->n_max);
        for (uint32_t k = 0; k < a->n_max; ++k)
            match[k * a->match_stride + g] =
                (s.ok && (int)k < s.n) ? members[v.first_member + s.member[k]].match : 0;
        nv[g] = s.ok ? (uint8_t)s.n : 0;
        if (!s.ok) set_bit(a->fallback, g);
        const_cast<uint64_t *>(a->committed_in)[g] = v.committed;
        const_cast<uint64_t *>(a->last_index)[g] = v.last_index;
        if (a->term_start) const_cast<uint64_t *>(a->term_start)[g] = v.term_start;
        if (a->term) const_cast<uint64_t *>(a->term)[g] = v.term;
        if (a->term_mask) const_cast<uint16_t *>(a->term_mask)[g] = v.term_mask;
    }
    return HQ_OK;
}

extern "C" int hq_pack_votes(const hq_group_view *groups, uint64_t G, const hq_member *members,
                             const hq_msg *msgs, uint8_t *granted, uint8_t *rejected,
                             uint8_t *n_voting, uint64_t *fallback) {
    if (G == 0) return HQ_OK;
    if (!groups || !members || !granted || !rejected || !n_voting) return HQ_E_INVAL;
    if (fallback) std::memset(fallback, 0, ((G + 63) / 64) * 8);
    for (uint64_t g = 0; g < G; ++g) {
        const hq_group_view &v = groups[g];
        const Slots s = voting_slots(v, members, HQ_MAX_VOTERS);
        uint32_t gr = 0, rj = 0;
        if (s.ok) {
            gr = 1;  // campaign: the candidate votes for itself (raft.go:1093)
            for (uint32_t i = 0; i < v.n_msgs; ++i) {
                if (!msgs) return HQ_E_INVAL;
                const hq_msg &mm = msgs[v.first_msg + i];
                const int k = slot_of(s, v, members, mm.from);  // observers / non-members dropped
                if (k < 0 || ((gr | rj) >> k) & 1) continue;    // first response wins
                if (mm.reject) rj |= 1u << k;
                else gr |= 1u << k;
            }
        } else {
            set_bit(fallback, g);
        }
        granted[g] = (uint8_t)gr;
        rejected[g] = (uint8_t)rj;
        n_voting[g] = s.ok ? (uint8_t)s.n : 0;
    }
    return HQ_OK;
}

extern "C" int hq_pack_acks(const hq_group_view *groups, uint64_t G, const hq_member *members,
                            const hq_msg *msgs, uint8_t *ack, uint8_t *active, uint8_t *n_voting,
                            uint32_t n_max, uint64_t *fallback) {
    if (G == 0) return HQ_OK;
    if (!groups || !members || !ack || !n_voting || n_max < 1 || n_max > HQ_MAX_VOTERS)
        return HQ_E_INVAL;
    if (fallback) std::memset(fallback, 0, ((G + 63) / 64) * 8);
    for (uint64_t g = 0; g < G; ++g) {
        const hq_group_view &v = groups[g];
        const Slots s = voting_slots(v, members, n_max);
        uint32_t a = 0, act = 0;
        if (s.ok) {
            for (uint32_t i = 0; i < v.n_msgs; ++i) {
                if (!msgs) return HQ_E_INVAL;
                const hq_msg &mm = msgs[v.first_msg + i];
                if (mm.hint_low != v.ctx_low || mm.hint_high != v.ctx_high) continue;
                const int k = slot_of(s, v, members, mm.from);
                if (k >= 0) a |= 1u << k;   // the confirmed set (readindex.go:83)
            }
            for (int k = 0; k < s.n; ++k)
                act |= (uint32_t)(members[v.first_member + s.member[k]].active != 0) << k;
        } else {
            set_bit(fallback, g);
        }
        ack[g] = (uint8_t)a;
        if (active) active[g] = (uint8_t)act;
        n_voting[g] = s.ok ? (uint8_t)s.n : 0;
    }
    return HQ_OK;
}

extern "C" int hq_pack_ring32(const uint64_t *ring, uint64_t count, uint32_t *ring32) {
    if (count == 0) return HQ_OK;
    if (!ring || !ring32) return HQ_E_INVAL;
    // terms at or above 0xFFFFFFFF saturate: never equal to a term the kernel decides for
    for (uint64_t i = 0; i < count; ++i)
        ring32[i] = ring[i] < 0xFFFFFFFFull ? (uint32_t)ring[i] : 0xFFFFFFFFu;
    return HQ_OK;
}

namespace {

int32_t lag_of(uint64_t last, uint64_t x) {  // clamp(last - x) to int32
    if (x <= last) {
        const uint64_t d = last - x;
        return d >= (uint64_t)INT32_MAX ? INT32_MAX : (int32_t)d;
    }
    const uint64_t d = x - last;
    return d >= (uint64_t)INT32_MAX + 1 ? INT32_MIN : -(int32_t)d;
}

}  // namespace

extern "C" int hq_pack_lags(uint64_t G, uint32_t n_max, const uint64_t *match,
                            uint64_t match_stride, const uint64_t *committed,
                            const uint64_t *last_index, const uint64_t *term_start,
                            const uint16_t *term_mask, const hq_commit_lag_args *out) {
    if (G == 0) return HQ_OK;
    if (!match || !committed || !last_index || !out || !out->lag || !out->cin_lag ||
        match_stride < G || out->lag_stride < G || n_max < 1 || n_max > out->n_max)
        return HQ_E_INVAL;
    const bool ts = out->form == HQ_FORM_TERM_START;
    if (ts ? (!term_start || !out->ts_lag) : (!term_mask || !out->lag_mask)) return HQ_E_INVAL;
    const uint32_t R = out->ring_len;
    if (!ts && (R < 1 || R > 16 || (R & (R - 1)))) return HQ_E_INVAL;
    int32_t *lag = const_cast<int32_t *>(out->lag);
    if (out->flags & ~HQ_LAG_LEADER_IMPLICIT) return HQ_E_INVAL;
    // HQ_LAG_LEADER_IMPLICIT: slot 0 is not stored; it must be the leader's lastIndex
    // (raft.go:918, 1031) for every group that has a slot 0
    const uint32_t lead = (out->flags & HQ_LAG_LEADER_IMPLICIT) ? 1 : 0;
    if (lead)
        for (uint64_t g = 0; g < G; ++g)
            if ((!out->n_voting || out->n_voting[g] >= 1) && match[g] != last_index[g])
                return HQ_E_INVAL;
    for (uint32_t s = lead; s < n_max; ++s)
        for (uint64_t g = 0; g < G; ++g)
            lag[(s - lead) * out->lag_stride + g] =
                lag_of(last_index[g], match[s * match_stride + g]);
    for (uint64_t g = 0; g < G; ++g) {
        const uint64_t last = last_index[g];
        const_cast<int32_t *>(out->cin_lag)[g] = lag_of(last, committed[g]);
        if (ts) {
            const_cast<int32_t *>(out->ts_lag)[g] = lag_of(last, term_start[g]);
        } else {
            // bit (i % R) of the u64-layout mask -> bit k = last - i of the lag-indexed mask
            uint32_t m = 0;
            for (uint32_t k = 0; k < R; ++k) m |= ((term_mask[g] >> ((last - k) & (R - 1))) & 1u) << k;
            const_cast<uint16_t *>(out->lag_mask)[g] = (uint16_t)m;
        }
    }
    return HQ_OK;
}

extern "C" int hq_unpack_lags(uint64_t G, const uint64_t *last_index, const int32_t *cout_lag,
                              const uint64_t *fallback, uint64_t *committed) {
    if (G == 0) return HQ_OK;
    if (!last_index || !cout_lag || !committed) return HQ_E_INVAL;
    // a decided group's cout_lag is d (>= 0) or its own unclamped cin_lag: last - lag is exact
    for (uint64_t g = 0; g < G; ++g)
        if (!fallback || !((fallback[g >> 6] >> (g & 63)) & 1))
            committed[g] = last_index[g] - (uint64_t)(int64_t)cout_lag[g];
    return HQ_OK;
}

// Columns -> HQ_LAYOUT_TILES tiles on the host (the twin of k_tile_commit): a step worker that
// packs columns can hand the kernel one contiguous staging block per 128 groups instead.
extern "C" int hq_tile_commit_host(const hq_commit_args *a, uint64_t *tiles) {
    return hq_tile_commit_as_host(a, tiles, HQ_LAYOUT_TILES);
}

// HQ_LAYOUT_TILES_LEADER drops slot 0's row, which the layout defines as last_index (the
// leader's own match, raft.go:918 appendEntries / :1031 reset). A group with n >= 1 whose
// slot 0 differs is refused (HQ_E_INVAL): the layout cannot carry it.
extern "C" int hq_tile_commit_as_host(const hq_commit_args *a, uint64_t *tiles, uint32_t layout) {
    if (!a || !tiles || a->layout != HQ_LAYOUT_COLUMNS || a->n_max < 1 ||
        a->n_max > HQ_MAX_VOTERS || a->form > HQ_FORM_TERM_RING32 ||
        (layout != HQ_LAYOUT_TILES && layout != HQ_LAYOUT_TILES_LEADER))
        return HQ_E_INVAL;
    if (a->G == 0) return HQ_OK;
    const bool mask = a->form == HQ_FORM_TERM_MASK;
    const uint64_t *aux = a->form == HQ_FORM_TERM_START ? a->term_start : a->term;
    if (!a->match || !a->committed_in || !a->last_index || a->match_stride < a->G ||
        (mask ? !a->term_mask : !aux))
        return HQ_E_INVAL;
    const uint32_t lead = layout == HQ_LAYOUT_TILES_LEADER ? 1 : 0;
    if (lead)
        for (uint64_t g = 0; g < a->G; ++g)
            if ((!a->n_voting || a->n_voting[g] >= 1) && a->match[g] != a->last_index[g])
                return HQ_E_INVAL;
    const uint32_t n = a->n_max - lead;   // match rows per tile
    const uint64_t tw = hq_commit_tile_words_for(a->n_max, a->form, layout), T = HQ_TILE_GROUPS;
    for (uint64_t t = 0; t < hq_commit_tiles(a->G); ++t) {
        uint64_t *tile = tiles + t * tw;
        std::memset(tile, 0, tw * 8);
        uint16_t *mrow = reinterpret_cast<uint16_t *>(tile + (n + 2) * T);
        // row position p holds group (p >> 1) + 64 * (p & 1) of the tile
        for (uint64_t p = 0; p < T; ++p) {
            const uint64_t g = t * T + (p >> 1) + (T / 2) * (p & 1);
            if (g >= a->G) continue;
            for (uint32_t s = 0; s < n; ++s)
                tile[s * T + p] = a->match[(s + lead) * a->match_stride + g];
            tile[n * T + p] = a->committed_in[g];
            tile[(n + 1) * T + p] = a->last_index[g];
            if (mask) mrow[p] = a->term_mask[g];
            else tile[(n + 2) * T + p] = aux[g];
        }
    }
    return HQ_OK;
}

// Bitmap columns -> 1024-group tiles on the host (the twin of k_tile_bits).
extern "C" int hq_tile_bits_host(uint64_t G, const uint8_t *ack, const uint8_t *granted,
                                 const uint8_t *rejected, const uint8_t *n_voting,
                                 uint8_t *tiles) {
    if (G == 0) return HQ_OK;
    if (!ack || !granted || !rejected || !tiles) return HQ_E_INVAL;
    const uint8_t *cols[4] = {n_voting, ack, granted, rejected};
    const uint32_t rows = n_voting ? 4 : 3;
    const uint64_t T = HQ_BITS_TILE_GROUPS;
    for (uint64_t t = 0; t < hq_bits_tiles(G); ++t) {
        const uint64_t g0 = t * T, cnt = G - g0 < T ? G - g0 : T;
        uint8_t *tile = tiles + t * rows * T;
        for (uint32_t r = 0; r < rows; ++r) {
            std::memcpy(tile + r * T, cols[r + 4 - rows] + g0, cnt);
            std::memset(tile + r * T + cnt, 0, T - cnt);
        }
    }
    return HQ_OK;
}

// Bitmap columns -> 3-byte tiles on the host (the twin of k_tile_bits3): rows ack, granted,
// rejected of 1024 groups, bits of slots 1..7 in bits 0..6 and one bit of n - 1 in bit 7
// (include/hipquorum.h hq_readindex_vote_tiles3_dev). Groups outside the contract get a fallback
// bit and zero bytes.
extern "C" int hq_tile_bits3_host(uint64_t G, const uint8_t *ack, const uint8_t *granted,
                                  const uint8_t *rejected, const uint8_t *n_voting,
                                  uint32_t n_uniform, uint8_t *tiles, uint64_t *fallback) {
    if (G && (!ack || !granted || !rejected || !tiles)) return HQ_E_INVAL;
    const uint64_t total = (G + 1023) / 1024 * 1024;
    if (fallback) std::memset(fallback, 0, ((G + 63) / 64) * 8);
    for (uint64_t g = 0; g < total; ++g) {
        uint32_t A = 0, Gr = 0, Rj = 0;
        if (g < G) {
            const uint32_t n = n_voting ? n_voting[g] : n_uniform;
            const uint32_t a = ack[g], x = granted[g], r = rejected[g];
            if (n < 1 || n > 8 || (a & 1) || !(x & 1) || (r & 1)) {
                if (fallback) set_bit(fallback, g);
            } else {
                const uint32_t keep = (1u << n) - 2u, m = n - 1;
                A = ((a & keep) >> 1) | ((m & 1) << 7);
                Gr = ((x & keep) >> 1) | (((m >> 1) & 1) << 7);
                Rj = ((r & keep) >> 1) | (((m >> 2) & 1) << 7);
            }
        }
        uint8_t *row = tiles + (g >> 10) * 3072 + (g & 1023);
        row[0] = (uint8_t)A;
        row[1024] = (uint8_t)Gr;
        row[2048] = (uint8_t)Rj;
    }
    return HQ_OK;
}

// Bitmap columns -> bit-plane tiles on the host (the twin of k_tile_planes): each group's three
// bytes as in hq_tile_bits3_host, bit b of row r set in plane 8 r + b.
extern "C" int hq_tile_planes_host(uint64_t G, const uint8_t *ack, const uint8_t *granted,
                                   const uint8_t *rejected, const uint8_t *n_voting,
                                   uint32_t n_uniform, uint8_t *planes, uint64_t *fallback) {
    if (G && (!ack || !granted || !rejected || !planes)) return HQ_E_INVAL;
    constexpr uint64_t T = HQ_PLANE_TILE_GROUPS;
    const uint64_t total = (G + T - 1) / T * T;
    std::memset(planes, 0, total * 3);
    if (fallback) std::memset(fallback, 0, ((G + 63) / 64) * 8);
    for (uint64_t g = 0; g < G; ++g) {
        const uint32_t n = n_voting ? n_voting[g] : n_uniform;
        const uint32_t a = ack[g], x = granted[g], r = rejected[g];
        if (n < 1 || n > 8 || (a & 1) || !(x & 1) || (r & 1)) {
            if (fallback) set_bit(fallback, g);
            continue;
        }
        const uint32_t keep = (1u << n) - 2u, m = n - 1;
        const uint32_t bytes = (((a & keep) >> 1) | ((m & 1) << 7)) |
                               ((((x & keep) >> 1) | (((m >> 1) & 1) << 7)) << 8) |
                               ((((r & keep) >> 1) | (((m >> 2) & 1) << 7)) << 16);
        uint8_t *tile = planes + (g / T) * (3 * T);
        const uint64_t j = g % T;
        for (uint32_t q = 0; q < 24; ++q)
            if ((bytes >> q) & 1) tile[q * (T / 8) + j / 8] |= (uint8_t)(1u << (j % 8));
    }
    return HQ_OK;
}

// Active flags -> CheckQuorum planes on the host (the twin of k_tile_cq_planes;
// include/hipquorum.h hq_check_quorum_planes_dev).
extern "C" int hq_tile_cq_planes_host(uint64_t G, const uint8_t *active, const uint8_t *n_voting,
                                      uint32_t n_uniform, uint32_t self_slot, uint8_t *planes,
                                      uint64_t *fallback) {
    if (n_voting ? n_uniform != 0 : (n_uniform < 1 || n_uniform > HQ_MAX_VOTERS)) return HQ_E_INVAL;
    if (!n_voting && self_slot >= n_uniform) return HQ_E_INVAL;
    const uint64_t NP = n_voting ? 10 : n_uniform - 1;
    if (G && (!active || (NP && !planes))) return HQ_E_INVAL;
    constexpr uint64_t T = HQ_PLANE_TILE_GROUPS;
    const uint64_t total = (G + T - 1) / T * T;
    if (NP) std::memset(planes, 0, total / 8 * NP);
    if (fallback) std::memset(fallback, 0, ((G + 63) / 64) * 8);
    for (uint64_t g = 0; g < G; ++g) {
        const uint32_t n = n_voting ? n_voting[g] : n_uniform;
        if (n < 1 || n > 8 || self_slot >= n) {
            if (fallback) set_bit(fallback, g);
            continue;
        }
        const uint32_t a = active[g] & ((1u << n) - 1u);
        uint32_t bits = (a & ((1u << self_slot) - 1u)) | ((a >> (self_slot + 1)) << self_slot);
        if (n_voting) bits |= (n - 1) << 7;
        uint8_t *tile = planes + (g / T) * (NP * T / 8);
        const uint64_t j = g % T;
        for (uint64_t q = 0; q < NP; ++q)
            if ((bits >> q) & 1) tile[q * (T / 8) + j / 8] |= (uint8_t)(1u << (j % 8));
    }
    return HQ_OK;
}

// Multi-ctx ReadIndex columns -> 128-group tiles on the host (the twin of k_tile_ri_multi;
// include/hipquorum.h hq_readindex_multi_tiles_dev).
extern "C" int hq_tile_ri_multi_host(uint64_t G, uint32_t K_max, uint32_t n_max,
                                     const uint16_t *ord, const uint64_t *idx, const uint8_t *np,
                                     const uint8_t *nv, uint8_t *tiles) {
    if (G && (!ord || !idx || !tiles)) return HQ_E_INVAL;
    if (K_max < 1 || K_max > 8 || n_max < 1 || n_max > 8) return HQ_E_INVAL;
    constexpr uint64_t T = HQ_RI_TILE_GROUPS;
    const uint32_t flags = (np ? HQ_RI_TILE_PER_K : 0) | (nv ? HQ_RI_TILE_PER_N : 0);
    const uint64_t tb = hq_ri_tile_bytes(K_max, n_max, flags);
    const uint64_t ntiles = (G + T - 1) / T, rows = (uint64_t)K_max * n_max;
    for (uint64_t t = 0; t < ntiles; ++t) {
        uint8_t *b = tiles + t * tb;
        for (uint64_t j = 0; j < T; ++j) {
            const uint64_t g = t * T + j;
            const bool in = g < G;
            // voter-major: voter s's block of K_max * 256 bytes, the pair j / 2's K_max dwords,
            // ctx k's dword holding groups 2 (j / 2) and 2 (j / 2) + 1
            for (uint64_t k = 0; k < K_max; ++k)
                for (uint64_t s = 0; s < n_max; ++s) {
                    const uint16_t x = in ? ord[(k * n_max + s) * G + g] : 0xFFFFu;
                    std::memcpy(b + s * K_max * 256 + (j / 2) * 4 * K_max + 4 * k + 2 * (j % 2),
                                &x, 2);
                }
            for (uint64_t k = 0; k < K_max; ++k) {
                const uint64_t x = in ? idx[k * G + g] : 0;
                std::memcpy(b + rows * 256 + k * 1024 + 8 * j, &x, 8);
            }
            uint8_t *u = b + rows * 256 + K_max * 1024ull;   // the u8 rows
            if (np) {
                u[j] = in ? np[g] : 0;
                u += T;
            }
            if (nv) u[j] = in ? nv[g] : 0;
        }
    }
    return HQ_OK;
}

// released_index from the compact ReadIndex outputs (include/hipquorum.h hq_ri_released_host): a
// downward scan per group carries the index of the nearest closing ctx at or above entry k.
extern "C" int hq_ri_released_host(uint64_t G, uint32_t K_max, const uint64_t *ctx_index,
                                   const uint8_t *released_count, const uint8_t *batch_end,
                                   uint64_t *released_index) {
    if (G && (!ctx_index || !released_count || !batch_end || !released_index)) return HQ_E_INVAL;
    if (K_max < 1 || K_max > 8) return HQ_E_INVAL;
    for (uint64_t g = 0; g < G; ++g) {
        const uint32_t cnt = released_count[g], be = batch_end[g];
        if (cnt > K_max) return HQ_E_INVAL;
        uint64_t cur = ~0ull;
        bool closed = false;
        for (int k = (int)K_max - 1; k >= 0; --k) {
            if ((be >> k) & 1) {
                cur = ctx_index[(uint64_t)k * G + g];
                closed = true;
            }
            const bool rel = (uint32_t)k < cnt;
            if (rel && !closed) return HQ_E_INVAL;
            released_index[(uint64_t)k * G + g] = rel ? cur : ~0ull;
        }
    }
    return HQ_OK;
}
