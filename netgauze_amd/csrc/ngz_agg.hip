// Flow aggregation on the device: the collector's windowed FlowAggregator
// (crates/collector/src/flow/aggregation/aggregator.rs) over the columns the
// decode path leaves in HBM.  C ABI: include/ngz/flow_aggregate.h.
//
// Pipeline of one ngz_agg_push (one stream; the push is all-or-nothing):
//   k_agg_dgram   datagrams that carry >= 1 data record (aggregator.rs:308
//                 yields one item per record)
//   hipcub max-scan over export times -> k_agg_late: lateness per datagram
//                 (aggregation.rs:139-141: ts < current_time - lateness, with
//                 current_time the running max of the earlier non-late items)
//                 and its observation-domain dictionary entry (new domains are
//                 listed for the host, which assigns them: k_agg_domfix)
//   hipcub sum-scan over set record counts -> k_agg_recinfo: every set's first row, times,
//                 plan and datagram info (16 bytes), and the set holding every 256th record;
//                 a record kernel finds its record's set from those (ctx_of), cached loads only
//   k_agg_claim   one lane per record: its group's slot in the HBM table
//                 (open addressing; a new group's first record claims a slot
//                 with a CAS on the 64-bit tag and writes the exact key).  Keys
//                 that fit 63 bits are their own tag.  Other keys are hashed:
//                 k_agg_check compares every record's key with its slot's key,
//                 and records of a key whose hash collided re-probe comparing
//                 keys (k_agg_claim in exact mode) until every record sits in
//                 its own key's slot -- groups are exact, collisions only cost
//                 probes.
//   validation    table full / too many groups / dictionaries full: the slots
//                 claimed by this push are released and the dictionaries put
//                 back, so a failed push leaves the aggregator as it was
//   k_agg_apply   FlowCacheRecord::reduce (aggregator.rs:159-198) of every
//                 record into its group: wave and workgroup pre-aggregation,
//                 then atomics on the group row (integer Add wraps like
//                 release-mode `+=`; Min / Max / BoolMapOr)
//   k_agg_ordered reductions whose result depends on record order (float Add,
//                 float Min / Max ties, IPv6 Min / Max): records sorted by group
//                 (stable radix sort), one sequential fold per group in record
//                 order, starting from the group's value -- the reference's
//                 order exactly
// Windows close as the event time advances (aggregation.rs:154-160): their
// groups are handed out by ngz_agg_emit and their slots freed (tombstones;
// the table is rebuilt when they pile up).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "ngz/flow_aggregate.h"
#include "ngz/flow_decode.h"
#include "ngz_host.h"

namespace {

constexpr uint32_t ROW_HDR = 88;  // sizeof(ngz_agg_row)
constexpr uint32_t OWN_OFF = 88;  // device bookkeeping after the header: the record owning the row in this push
constexpr uint32_t KEY0 = 96;     // first key byte
static_assert(sizeof(ngz_agg_row) == ROW_HDR, "ngz_agg_row layout");
constexpr uint32_t DOM_SLOTS = 128;
constexpr uint32_t SET_BITS = 64;
constexpr uint32_t NEWDOM_SLOTS = 256;  // distinct new observation domains one push may bring
constexpr uint64_t TAG_EMPTY = 0, TAG_TOMB = 1;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t OWN_BIT = 0x80000000u;  // rec_g: the record is its group's owner (slots < 2^31)

// dginfo bits (per datagram)
constexpr uint16_t DG_USE = 1, DG_LATE = 2, DG_MISSING = 0x200;  // domain index in bits 2..8

// value classes: how a column value becomes the accumulator operand
enum : uint8_t {
    VC_UINT = 0,   // unsigned integer / ipv4 / boolean / dateTimeSeconds (min/max/add/or in u64)
    VC_SINT = 1,   // signed integer, dateTimeMilliseconds (sign-extended; min/max with the sign bit flipped)
    VC_DTFRAC = 2, // dateTime micro/nanoseconds: (secs << 32 | nanos), ordered like DateTime
    VC_BYTES = 3,  // byte-wise OR (octetArray, macAddress, ipv6Address, unsigned256)
    VC_RANK = 4,   // sub-registry enum / TCPHeaderFlags Min-Max: the value's rank in the Rust Ord
    VC_F32 = 5,    // OrderedFloat<f32> (ordered path)
    VC_F64 = 6,    // OrderedFloat<f64> (ordered path)
    VC_IPV6 = 7,   // Ipv6Addr Min / Max (16 bytes, big-endian order; ordered path)
    VC_VBYTES = 8, // octetArray BoolMapOr, any length: the group keeps its first value's length and ORs
                   // the others into it, zipped (`lhs.iter_mut().zip(rhs)`, generator.rs:1051-1059);
                   // BVAL row form (below); ordered path
    VC_VLIST = 9,  // basicList / subTemplateList / subTemplateMultiList Min / Max: Box<[u8]>'s
                   // lexicographic Ord; BVAL row form; ordered path
};
__host__ __device__ inline bool vc_ordered(uint8_t vc) {
    return vc == VC_F32 || vc == VC_F64 || vc == VC_IPV6 || vc == VC_VBYTES || vc == VC_VLIST;
}

// key kinds: canonical key bytes in the row
enum : uint8_t {
    KK_FIXED = 0,  // the column cell, zero padded
    KK_BYTES = 3,  // a byte value of any length (string / octetArray / list / unknown IEs): BVAL row form.
                   // A string is its text: a fixed-length cell up to its first NUL (Field::String,
                   // generator.rs:1654-1669), a variable-length one as sent; octets / lists / unknown
                   // IEs their bytes (Box<[u8]> compares the length too)
};

// BVAL row form of a byte value: u32 length n, u32 arena offset of bytes 32.. (when n > 32), the
// first 32 bytes zero padded.  Values longer than 32 bytes keep their tail in the aggregator's
// byte arena (bump-allocated per group, compacted when the table is rebuilt, emptied by flush).
constexpr uint32_t BVAL_BYTES = 40, BVAL_INLINE = 32;
// Arena bytes a BVAL value of n > 32 bytes takes: its tail, rounded to 8 bytes.  Row offsets are
// in 8-byte units (a u32 addresses 32 GiB of arena; a push that would pass it fails, NGZ_E_LIMIT)
constexpr uint64_t ARENA_MAX = 1ull << 35;
__host__ __device__ __forceinline__ uint64_t tail_span(uint32_t n) {
    return n > BVAL_INLINE ? ((uint64_t)(n - BVAL_INLINE) + 7) & ~7ull : 0;
}

struct AggSlotPlan {            // per batch slot, built on the host every push
    const uint8_t *key_col[NGZ_AGG_MAX_KEYS];   // null: the record has no such field (None)
    const uint8_t *val_col[NGZ_AGG_MAX_VALUES];
    uint32_t key_w[NGZ_AGG_MAX_KEYS];           // 32-bit: a kernel reading the plan with scalar loads
    uint32_t val_w[NGZ_AGG_MAX_VALUES];         // gets them without a vector load (SMEM is dword-wide)
    uint64_t tpl_bit;
    uint32_t proto;
    uint32_t usable;                            // 0: slot not aggregated (no records / not device-decoded)
    const uint8_t *bytes;                       // the batch bytes (variable-length cells point into them)
    uint32_t key_vlen, val_vlen;                // bit k / v: a variable-length column ({u64 offset, u32 length})
};

struct AggParams {
    uint32_t n_keys, n_vals;
    uint32_t key_off[NGZ_AGG_MAX_KEYS];
    uint32_t key_slot[NGZ_AGG_MAX_KEYS];   // row bytes of the key (multiple of 4)
    uint8_t key_kind[NGZ_AGG_MAX_KEYS];
    uint32_t key_pw[NGZ_AGG_MAX_KEYS];     // packed mode: the IE's fixed column width
    uint32_t val_off[NGZ_AGG_MAX_VALUES];
    uint8_t val_op[NGZ_AGG_MAX_VALUES];
    uint8_t val_vc[NGZ_AGG_MAX_VALUES];
    uint8_t val_tcp[NGZ_AGG_MAX_VALUES];   // VC_RANK of TCPHeaderFlags (else a sub-registry)
    const uint32_t *rank_known[NGZ_AGG_MAX_VALUES];  // VC_RANK sub-registry: bitmap of registered values
    uint32_t row_bytes;
    uint64_t mask;              // table slots - 1
    uint32_t push_id;
    uint32_t port_bit;
    uint32_t peer;              // the push's peer IP (entry of the aggregator's peer dictionary)
    uint32_t peer_bits;         // packed tags: bits of the peer entry (log2 of max_peers)
    uint64_t coll_flip;         // collection time ms, sign bit flipped (unsigned order == signed order)
    uint32_t lds_ok;            // 1: no byte-wise OR values (wave results may be combined in LDS)
    uint32_t packed;            // 1: the whole group key packs into 63 bits (exact tag)
    uint64_t hash_mask;         // hashed keys: bits of the hash kept (NGZ_AGG_OPT_HASH_BITS: tests force collisions)
    uint32_t own;               // 1: one record per group and push (its owner) reduces with plain stores
    uint32_t kw_n;              // hashed keys of at most 8 words: their count (key words held in registers), else 0
    uint8_t kw_key[8], kw_idx[8];  // key word j: its key field and its word within the field
    uint64_t unit_op[2];        // owner path: 4-bit op of each 8-byte unit of the row (units 0-15, 16-31)
    uint64_t unit_src[2];       // ... and its operand (U_SRC_*)
    uint32_t key_str;           // bit k: key k is a string (KK_BYTES text: fixed cells NUL-truncated)
    uint32_t has_bytes;         // some key / value is in the BVAL form
    uint8_t *arena;             // byte arena: tails of BVAL values longer than 32 bytes
    uint64_t arena_cap;
    unsigned long long *arena_used;  // device bump counter (bytes)
    const unsigned long long *rank_nested[NGZ_AGG_MAX_VALUES];  // VC_RANK of a nested sub-registry: rank of
                                                                 // values 0..255, [256]: outer Unassigned
    uint8_t op_off[8], op_w[8];  // partitioned path: operand v's byte offset and width in a payload (0: none)
};

__device__ __forceinline__ uint64_t mix64(uint64_t h, uint64_t v) {
    h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h *= 0xBF58476D1CE4E5B9ull;
    return h ^ (h >> 31);
}

__host__ __device__ __forceinline__ uint64_t slot_of(uint64_t h) {  // table position of a tag
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    return h ^ (h >> 33);
}

__device__ __forceinline__ bool tag_live(uint64_t t) { return t > TAG_TOMB; }

// word j (4 bytes, little-endian, zero padded past w) of a w-byte cell; str: NUL truncated
__device__ __forceinline__ uint32_t cell_word(const uint8_t *p, uint32_t w, uint32_t j, bool str, bool &nul) {
    if ((w & 3) == 0 && !str && 4 * j < w) return *(const uint32_t *)(p + 4 * j);
    uint32_t r = 0;
#pragma unroll
    for (uint32_t b = 0; b < 4; ++b) {
        const uint32_t i = 4 * j + b;
        uint32_t c = i < w ? p[i] : 0u;
        if (str) {
            if (nul) c = 0;
            else if (c == 0) nul = true;
        }
        r |= c << (8 * b);
    }
    return r;
}

// canonical key word j of a fixed key cell
struct KeyWords {
    const uint8_t *p;
    uint32_t w;
    bool nul = false;
    __device__ uint32_t operator()(uint32_t j) { return cell_word(p, w, j, false, nul); }
};

// A byte value of a record: where its bytes are and how many (BVAL keys and values)
struct Span {
    const uint8_t *p;
    uint32_t n;
};

__device__ __forceinline__ Span cell_span(const uint8_t *col, uint32_t w, bool vlen, bool str, const uint8_t *bytes,
                                          uint64_t row) {
    if (vlen) {  // {u64 offset into the batch bytes, u32 length, u32 0} (NGZ_K_VLEN)
        const uint8_t *c = col + row * 16;
        return Span{bytes + *(const uint64_t *)c, *(const uint32_t *)(c + 8)};
    }
    const uint8_t *q = col + row * w;
    uint32_t n = w;
    if (str) {  // a fixed-length string is its text up to the first NUL
        n = 0;
        while (n < w && q[n]) ++n;
    }
    return Span{q, n};
}

__device__ __forceinline__ Span key_span(const AggSlotPlan &sp, const AggParams &P, uint32_t k, uint64_t row) {
    return cell_span(sp.key_col[k], sp.key_w[k], (sp.key_vlen >> k) & 1, (P.key_str >> k) & 1, sp.bytes, row);
}

__device__ __forceinline__ Span val_span(const AggSlotPlan &sp, uint32_t v, uint64_t row) {
    return cell_span(sp.val_col[v], sp.val_w[v], (sp.val_vlen >> v) & 1, false, sp.bytes, row);
}

// word j (little-endian) of bytes [0, n) of p, zero past n
__device__ __forceinline__ uint32_t span_word(const uint8_t *p, uint32_t n, uint32_t j) {
    uint32_t r = 0;
#pragma unroll
    for (uint32_t b = 0; b < 4; ++b) {
        const uint32_t i = 4 * j + b;
        if (i < n) r |= (uint32_t)p[i] << (8 * b);
    }
    return r;
}

// A BVAL value in a row: byte i is inline (i < 32) or in the arena
struct BRef {
    const uint8_t *a, *b;  // bytes [0, split) at a, [split, n) at b - split
    uint32_t split, n;
    __device__ __forceinline__ uint8_t at(uint32_t i) const { return i < split ? a[i] : b[i - split]; }
};

__device__ __forceinline__ BRef bval_ref(const uint8_t *slot, const AggParams &P) {
    const uint32_t n = *(const uint32_t *)slot, off = *(const uint32_t *)(slot + 4);
    return BRef{slot + 8, P.arena + ((uint64_t)off << 3), BVAL_INLINE, n};
}

// Box<[u8]> / [u8] Ord: lexicographic, then by length
__device__ __forceinline__ int bytes_cmp(const BRef &x, const BRef &y) {
    const uint32_t m = min(x.n, y.n);
    for (uint32_t i = 0; i < m; ++i) {
        const uint8_t a = x.at(i), b = y.at(i);
        if (a != b) return a < b ? -1 : 1;
    }
    return x.n < y.n ? -1 : (x.n > y.n ? 1 : 0);
}

// Writes a record's byte value in the BVAL form at slot (tail bytes into the arena).  The
// push sized the arena for every tail it can write (k_agg_tail_need); err bit 64 if not.
__device__ __forceinline__ void bval_write(uint8_t *slot, const Span s, const AggParams &P,
                                           unsigned int *__restrict__ err) {
    uint32_t *d = (uint32_t *)slot;
    d[0] = s.n;
    d[1] = 0;
#pragma unroll
    for (uint32_t j = 0; j < BVAL_INLINE / 4; ++j) d[2 + j] = span_word(s.p, min(s.n, BVAL_INLINE), j);
    if (s.n > BVAL_INLINE) {
        const uint64_t need = tail_span(s.n);
        const uint64_t off = atomicAdd(P.arena_used, (unsigned long long)need);
        if (off + need > P.arena_cap) {
            atomicOr(err, 64u);
            return;
        }
        for (uint32_t i = 0; i < s.n - BVAL_INLINE; ++i) P.arena[off + i] = s.p[BVAL_INLINE + i];
        d[1] = (uint32_t)(off >> 3);
    }
}

// Canonical key words of a record held in registers (hashed keys of at most 8 words): the
// record's columns are read once, and the slot's key is compared with a few wide loads
struct KeyVal {
    uint32_t w[8];
};

__device__ __forceinline__ void key_words(const AggSlotPlan &sp, const AggParams &P, uint64_t row, KeyVal &kv) {
    bool nul = false;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
        kv.w[j] = 0;
        if (j >= P.kw_n) continue;
        const uint32_t k = P.kw_key[j], i = P.kw_idx[j];
        const uint8_t *c = sp.key_col[k];
        if (!c) continue;
        const uint32_t w = sp.key_w[k];
        if (i == 0) nul = false;
        kv.w[j] = cell_word(c + row * w, w, i, false, nul);  // KeyVal keys are fixed cells
    }
}

// row header word 1 (ngz_agg_row bytes 4-7): flow type, reserved byte, peer entry
__device__ __forceinline__ uint32_t hdr_word(const AggSlotPlan &sp, const AggParams &P) {
    return sp.proto | (P.peer << 16);
}

__device__ __forceinline__ uint64_t key_tag(const AggSlotPlan &sp, const AggParams &P, uint64_t row, uint32_t win,
                                            uint32_t &present, KeyVal &kv) {
    present = 0;
    if (P.packed) {  // exact tag: bit 63 | window/60 | flow type | peer | per key: presence bit + value bits
        uint64_t x = ((((uint64_t)(win / 60) << 1) | (sp.proto == 9)) << P.peer_bits) | P.peer;
        for (uint32_t k = 0; k < P.n_keys; ++k) {
            const uint8_t *c = sp.key_col[k];
            const uint32_t w = sp.key_w[k];
            uint64_t v = 0;
            if (c) {
                present |= 1u << k;
                const uint8_t *q = c + row * w;
                v = w == 4 ? *(const uint32_t *)q : w == 2 ? *(const uint16_t *)q : w == 8 ? *(const uint64_t *)q : *q;
            }
            x = (((x << 1) | (c != nullptr)) << (8 * P.key_pw[k])) | v;
        }
        return x | (1ull << 63);
    }
    uint64_t h = mix64(0x4E475A41474731ull, ((uint64_t)win << 32) | hdr_word(sp, P));
    if (P.kw_n) {
        key_words(sp, P, row, kv);
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j) {
            if (j >= P.kw_n) continue;
            const uint32_t k = P.kw_key[j];
            const bool has = sp.key_col[k] != nullptr;
            if (P.kw_idx[j] == 0) {
                h = mix64(h, has ? 0x100u : 0u);
                if (has) present |= 1u << k;
            }
            if (has) h = mix64(h, kv.w[j]);
        }
    } else {
        for (uint32_t k = 0; k < P.n_keys; ++k) {
            const uint8_t *c = sp.key_col[k];
            h = mix64(h, c ? 0x100u : 0u);
            if (!c) continue;
            present |= 1u << k;
            if (P.key_kind[k] == KK_BYTES) {  // its length and every byte
                const Span s = key_span(sp, P, k, row);
                h = mix64(h, s.n);
                for (uint32_t j = 0; j < (s.n + 3) / 4; ++j) h = mix64(h, span_word(s.p, s.n, j));
                continue;
            }
            KeyWords kw{c + row * sp.key_w[k], sp.key_w[k]};
            for (uint32_t j = 0; j < P.key_slot[k] / 4; ++j) h = mix64(h, kw(j));
        }
    }
    h &= P.hash_mask;
    return h < 2 ? h + 2 : h;  // 0 / 1 are the empty and tombstone tags
}

// A slot's header and first 8 key words (KeyVal keys), loaded with three 16-byte loads
struct KeyRow {
    uint4 h0, k0, k1;
};

__device__ __forceinline__ KeyRow key_row_load(const uint8_t *R, const AggParams &P) {
    KeyRow kr;
    kr.h0 = *(const uint4 *)R;
    kr.k0 = *(const uint4 *)(R + KEY0);
    kr.k1 = make_uint4(0, 0, 0, 0);
    if (P.kw_n > 4) kr.k1 = *(const uint4 *)(R + KEY0 + 16);
    return kr;
}

__device__ __forceinline__ bool key_row_equal(const KeyRow &kr, const AggSlotPlan &sp, const AggParams &P,
                                              uint32_t win, uint32_t kp, const KeyVal &kv) {
    // an absent key's words are zero in the row and in kv
    const uint32_t rw[8] = {kr.k0.x, kr.k0.y, kr.k0.z, kr.k0.w, kr.k1.x, kr.k1.y, kr.k1.z, kr.k1.w};
    bool same = kr.h0.x == win && kr.h0.y == hdr_word(sp, P) && kr.h0.z == kp;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j)
        if (j < P.kw_n) same = same && rw[j] == kv.w[j];
    return same;
}

__device__ __forceinline__ bool key_equal(const uint8_t *R, const AggSlotPlan &sp, const AggParams &P, uint64_t row,
                                          uint32_t win, uint32_t kp, const KeyVal &kv) {
    if (P.kw_n) return key_row_equal(key_row_load(R, P), sp, P, win, kp, kv);
    bool same = *(const uint32_t *)(R + 0) == win && *(const uint32_t *)(R + 4) == hdr_word(sp, P) &&
                *(const uint32_t *)(R + 8) == kp;
    for (uint32_t k = 0; k < P.n_keys && same; ++k) {
        const uint8_t *c = sp.key_col[k];
        if (!c) continue;
        const uint32_t *rk = (const uint32_t *)(R + P.key_off[k]);
        if (P.key_kind[k] == KK_BYTES) {
            const Span s = key_span(sp, P, k, row);
            same = rk[0] == s.n;
            for (uint32_t j = 0; j < BVAL_INLINE / 4 && same; ++j)
                same = rk[2 + j] == span_word(s.p, min(s.n, BVAL_INLINE), j);
            if (same && s.n > BVAL_INLINE) {
                const uint8_t *t = P.arena + ((uint64_t)rk[1] << 3);
                for (uint32_t i = BVAL_INLINE; i < s.n && same; ++i) same = t[i - BVAL_INLINE] == s.p[i];
            }
            continue;
        }
        KeyWords kw{c + row * sp.key_w[k], sp.key_w[k]};
        for (uint32_t j = 0; j < P.key_slot[k] / 4 && same; ++j) same = rk[j] == kw(j);
    }
    return same;
}

__device__ __forceinline__ void key_write(uint8_t *R, const AggSlotPlan &sp, const AggParams &P, uint64_t row,
                                          uint32_t win, uint32_t kp, const KeyVal &kv, unsigned int *__restrict__ err) {
    *(uint32_t *)(R + 0) = win;
    *(uint32_t *)(R + 4) = hdr_word(sp, P);
    *(uint32_t *)(R + 8) = kp;
    if (P.kw_n) {
#pragma unroll
        for (uint32_t j = 0; j < 8; ++j)
            if (j < P.kw_n) ((uint32_t *)(R + KEY0))[j] = kv.w[j];
        return;
    }
    for (uint32_t k = 0; k < P.n_keys; ++k) {
        uint32_t *dst = (uint32_t *)(R + P.key_off[k]);
        const uint8_t *c = sp.key_col[k];
        if (!c) {
            for (uint32_t j = 0; j < P.key_slot[k] / 4; ++j) dst[j] = 0;
            continue;
        }
        if (P.key_kind[k] == KK_BYTES) {
            bval_write((uint8_t *)dst, key_span(sp, P, k, row), P, err);
            continue;
        }
        KeyWords kw{c + row * sp.key_w[k], sp.key_w[k]};
        for (uint32_t j = 0; j < P.key_slot[k] / 4; ++j) dst[j] = kw(j);
    }
}

__device__ __forceinline__ uint64_t load_value(const uint8_t *p, uint32_t w, uint8_t vc) {
    if (vc == VC_DTFRAC) {  // {u32 secs, u32 nanos} -> ordered (secs, nanos)
        const uint32_t s = *(const uint32_t *)p, ns = *(const uint32_t *)(p + 4);
        return ((uint64_t)s << 32) | ns;
    }
    uint64_t v = 0;
    if (w == 8) v = *(const uint64_t *)p;
    else if (w == 4) v = *(const uint32_t *)p;
    else if (w == 2) v = *(const uint16_t *)p;
    else v = *p;
    if (vc == VC_SINT && w < 8) {  // sign-extend to 64 bits
        const uint32_t sh = 64 - 8 * w;
        v = (uint64_t)(((int64_t)(v << sh)) >> sh);
    }
    return v;
}

__host__ __device__ __forceinline__ uint32_t bitrev8(uint32_t x) {
    x = ((x & 0xF0u) >> 4) | ((x & 0x0Fu) << 4);
    x = ((x & 0xCCu) >> 2) | ((x & 0x33u) << 2);
    return ((x & 0xAAu) >> 1) | ((x & 0x55u) << 1);
}

// Operand of value v for the atomic path.  Signed min/max: sign bit flipped so unsigned order
// holds.  Ranks: TCPHeaderFlags derives Ord over (FIN, SYN, ..., CWR) in declaration order, so
// FIN is the most significant (iana/src/tcp.rs:41-70); a sub-registry enum orders by its
// discriminant: a registered value is its own discriminant, Unassigned(x) comes after every
// registered variant (generator_sub_registries.rs: `Unassigned(ty)` declared last).  A nested
// sub-registry (forwardingStatus) orders by its outer variant (one per 64-value group, then
// Unassigned), then by the reason enum's discriminant, then by the value: a host-built table
// (rank_nested, the value in the low 32 bits).
// value_operand from a cell's bytes already loaded (raw: the w-byte cell, little-endian, zero-extended)
__device__ __forceinline__ uint64_t operand_of_raw(const AggSlotPlan &sp, const AggParams &P, uint32_t v, uint64_t raw) {
    const uint8_t vc = P.val_vc[v];
    const uint32_t w = sp.val_w[v];
    uint64_t x = raw;
    if (vc == VC_DTFRAC) x = (raw << 32) | (raw >> 32);  // {u32 secs, u32 nanos} -> (secs, nanos), as load_value
    else if (vc == VC_SINT && w < 8) {
        const uint32_t sh = 64 - 8 * w;
        x = (uint64_t)(((int64_t)(x << sh)) >> sh);
    }
    if (vc == VC_SINT && (P.val_op[v] == NGZ_AGG_MIN || P.val_op[v] == NGZ_AGG_MAX)) x ^= 1ull << 63;
    if (vc == VC_RANK) {
        if (P.val_tcp[v]) x = bitrev8((uint32_t)x & 0xFF);
        else if (const unsigned long long *nr = P.rank_nested[v]) x = x < 256 ? nr[x] : nr[256] | x;
        else {
            const uint32_t *known = P.rank_known[v];
            const bool reg = x < 65536 && known && ((known[x >> 5] >> (x & 31)) & 1);
            if (!reg) x |= 1ull << 32;
        }
    }
    return x;
}

__device__ __forceinline__ uint64_t value_operand(const AggSlotPlan &sp, const AggParams &P, uint32_t v, uint64_t row) {
    const uint8_t vc = P.val_vc[v];
    uint64_t x = load_value(sp.val_col[v] + row * sp.val_w[v], sp.val_w[v], vc == VC_RANK ? VC_UINT : vc);
    if (vc == VC_SINT && (P.val_op[v] == NGZ_AGG_MIN || P.val_op[v] == NGZ_AGG_MAX)) x ^= 1ull << 63;
    if (vc == VC_RANK) {
        if (P.val_tcp[v]) x = bitrev8((uint32_t)x & 0xFF);
        else if (const unsigned long long *nr = P.rank_nested[v]) x = x < 256 ? nr[x] : nr[256] | x;
        else {
            const uint32_t *known = P.rank_known[v];
            const bool reg = x < 65536 && known && ((known[x >> 5] >> (x & 31)) & 1);
            if (!reg) x |= 1ull << 32;
        }
    }
    return x;
}

__global__ void k_agg_dgram(const ngz_set_info *__restrict__ sets, uint32_t n_sets, uint32_t n_dgrams,
                            uint32_t *__restrict__ has_rec) {
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < n_sets; s += gridDim.x * blockDim.x)
        if (sets[s].n && sets[s].dgram < n_dgrams) has_rec[sets[s].dgram] = 1;
}

__global__ void k_agg_ts(const ngz_dgram_hdr *__restrict__ hdr, const uint32_t *__restrict__ has_rec, uint32_t n,
                         uint32_t *__restrict__ ts) {
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < n; d += gridDim.x * blockDim.x)
        ts[d] = (hdr[d].status == NGZ_DG_OK && has_rec[d]) ? hdr[d].time : 0u;
}

__device__ __forceinline__ int dom_find(const unsigned long long *dict, uint32_t id) {
    const unsigned long long key = (1ull << 32) | id;
    for (int i = 0; i < (int)DOM_SLOTS; ++i)
        if (dict[i] == key) return i;
    return -1;
}

__global__ void k_agg_late(const ngz_dgram_hdr *__restrict__ hdr, const uint32_t *__restrict__ has_rec,
                           const uint32_t *__restrict__ pmax, uint32_t n, uint32_t state_ct, uint64_t lateness_ms,
                           const unsigned long long *__restrict__ dom_dict, uint16_t *__restrict__ dginfo,
                           unsigned long long *__restrict__ newdom, unsigned int *__restrict__ err) {
    __shared__ unsigned long long dict[DOM_SLOTS];
    for (uint32_t i = threadIdx.x; i < DOM_SLOTS; i += blockDim.x) dict[i] = dom_dict[i];
    __syncthreads();
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
        const uint32_t d = base + threadIdx.x;
        if (d >= n) continue;
        uint16_t info = 0;
        if (hdr[d].status == NGZ_DG_OK && has_rec[d]) {
            uint32_t ct = state_ct;
            if (d > 0 && pmax[d - 1] > ct) ct = pmax[d - 1];
            const bool late = ct != 0 && (int64_t)hdr[d].time * 1000 < (int64_t)ct * 1000 - (int64_t)lateness_ms;
            if (late) {
                info = DG_LATE;
            } else {
                const uint32_t id = hdr[d].domain;
                const int i = dom_find(dict, id);
                if (i >= 0) {
                    info = (uint16_t)(DG_USE | (i << 2));
                } else {
                    // not in the dictionary yet: list it for the host (set of distinct ids)
                    info = DG_USE | DG_MISSING;
                    const unsigned long long key = (1ull << 32) | id;
                    uint32_t j = (id * 2654435761u) % NEWDOM_SLOTS, probes = 0;
                    for (;;) {
                        unsigned long long cur = newdom[j];
                        if (cur == 0) {
                            cur = atomicCAS(&newdom[j], 0ull, key);
                            if (cur == 0) break;
                        }
                        if (cur == key) break;
                        j = (j + 1) % NEWDOM_SLOTS;
                        if (++probes == NEWDOM_SLOTS) { atomicOr(err, 1u); break; }
                    }
                }
            }
        }
        dginfo[d] = info;
    }
}

__global__ void k_agg_domfix(const ngz_dgram_hdr *__restrict__ hdr, const unsigned long long *__restrict__ dom_dict,
                             uint16_t *__restrict__ dginfo, uint32_t n, unsigned int *__restrict__ err) {
    __shared__ unsigned long long dict[DOM_SLOTS];
    for (uint32_t i = threadIdx.x; i < DOM_SLOTS; i += blockDim.x) dict[i] = dom_dict[i];
    __syncthreads();
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
        const uint32_t d = base + threadIdx.x;
        if (d >= n || !(dginfo[d] & DG_MISSING)) continue;
        const int i = dom_find(dict, hdr[d].domain);
        if (i < 0) { atomicOr(err, 16u); continue; }
        dginfo[d] = (uint16_t)(DG_USE | (i << 2));
    }
}

// Per-record context, 16 bytes, written once per push so the record kernels reach a record's
// row, times, plan and datagram info with one coalesced load instead of a chain of lookups
// (set index -> set -> datagram header / info -> plan):
//   x: row in the slot's columns   y: export time   z: sys-up time (NetFlow v9, else 0)
//   w: slot (bits 0-15) | datagram info (bits 16-31, DG_VALID: aggregated)
constexpr uint16_t DG_VALID = 0x8000;
// The context of each set (one thread per set): {first row, export time, sys-up time (NetFlow v9),
// slot | datagram info << 16}; and bset[b]: the set holding record 256 b (the last set starting at
// or before it: empty sets share their successor's start)
__global__ void k_agg_recinfo(const ngz_set_info *__restrict__ sets, uint32_t n_sets, const ngz_dgram_hdr *__restrict__ hdr,
                              const uint16_t *__restrict__ dginfo, const AggSlotPlan *__restrict__ plans,
                              uint32_t n_dgrams, uint32_t n_slots, uint4 *__restrict__ sctx, unsigned int *__restrict__ err) {
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < n_sets; s += gridDim.x * blockDim.x) {
        const ngz_set_info si = sets[s];
        uint32_t ts = 0, sysup = 0, w = 0;
        if (si.n && (si.dgram >= n_dgrams || si.slot >= n_slots)) {
            atomicOr(err, 16u);
        } else if (si.n) {
            const ngz_dgram_hdr &h = hdr[si.dgram];
            ts = h.time;
            sysup = h.version == 9 ? h.sys_up_time : 0u;
            uint16_t info = dginfo[si.dgram];
            if ((info & DG_USE) && plans[si.slot].usable) info |= DG_VALID;
            w = si.slot | ((uint32_t)info << 16);
        }
        sctx[s] = make_uint4(si.rec0, ts, sysup, w);
    }
}

// last s in [lo, hi] with rstart[s] <= t
__device__ __forceinline__ uint32_t set_search(const uint32_t *__restrict__ rstart, uint32_t lo, uint32_t hi, uint64_t t) {
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (rstart[mid] <= t) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__global__ void k_agg_bset(const uint32_t *__restrict__ rstart, uint32_t n_sets, uint64_t n_blocks,
                           uint32_t *__restrict__ bset) {
    for (uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; b < n_blocks; b += (uint64_t)gridDim.x * blockDim.x)
        bset[b] = set_search(rstart, 0, n_sets - 1, b << 8);
}

// Everything the record kernels share
struct RecCtx {
    const uint4 *sctx;       // per set: {first row, export time, sys-up time, slot | info << 16}
    const uint32_t *rstart;  // per set: its first record (exclusive scan of the set sizes)
    const uint32_t *bset;    // per 256 records: the set holding the first
    uint32_t n_sets;
    uint64_t n_rec;
    const AggSlotPlan *plans;
};

// Record t's context {row, export time, sys-up time, slot | info << 16}: its set is between the
// sets of records 256 floor(t / 256) and 256 (floor(t / 256) + 1), so a wave of consecutive records
// reads the same few cached entries (a per-record table was 16 bytes of HBM per record and pass)
__device__ __forceinline__ uint4 ctx_of(const RecCtx &C, uint64_t t) {
    if (t >= C.n_rec) return make_uint4(0, 0, 0, 0);
    const uint64_t b = t >> 8;
    const uint32_t lo = C.bset[b], hi = ((b + 1) << 8) < C.n_rec ? C.bset[b + 1] : C.n_sets - 1;
    const uint32_t s = set_search(C.rstart, lo, hi, t);
    const uint4 c = C.sctx[s];
    return make_uint4(c.x + (uint32_t)(t - C.rstart[s]), c.y, c.z, c.w);
}

// The slot every active lane of the wave holds (as a wave-uniform value the compiler keeps in an
// SGPR), or NONE when they differ
__device__ __forceinline__ uint32_t wave_uniform_slot(uint32_t slot, bool active) {
    const uint64_t m = __ballot(active);
    if (!m) return NONE;
    const int l0 = __ffsll((unsigned long long)m) - 1;
    const uint32_t s0 = (uint32_t)__shfl((int)slot, l0);
    if (!__all(!active || slot == s0)) return NONE;
    return __builtin_amdgcn_readfirstlane(s0);
}

// ctx_of for a caller whose lanes' records all lie in one 256-record block (t >> 8 equal across
// the wave): the block's set bounds come through scalar loads
__device__ __forceinline__ uint4 ctx_of_block(const RecCtx &C, uint64_t t) {
    if (t >= C.n_rec) return make_uint4(0, 0, 0, 0);
    const uint64_t b = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(t >> 40)) << 32) |
                       __builtin_amdgcn_readfirstlane((uint32_t)(t >> 8));
    const uint32_t lo = C.bset[b], hi = ((b + 1) << 8) < C.n_rec ? C.bset[b + 1] : C.n_sets - 1;
    const uint32_t s = set_search(C.rstart, lo, hi, t);
    const uint4 c = C.sctx[s];
    return make_uint4(c.x + (uint32_t)(t - C.rstart[s]), c.y, c.z, c.w);
}

struct Rec {
    bool valid = false, late = false;
    uint32_t slot = 0, ts = 0, sysup = 0;
    uint16_t info = 0;
    uint64_t row = 0;
};

__device__ __forceinline__ Rec rec_from(const uint4 p) {
    Rec r;
    r.row = p.x;
    r.ts = p.y;
    r.sysup = p.z;
    r.slot = p.w & 0xFFFF;
    r.info = (uint16_t)(p.w >> 16);
    r.late = (r.info & DG_LATE) != 0;
    r.valid = (r.info & DG_VALID) != 0;
    return r;
}

__device__ __forceinline__ Rec rec_of(const RecCtx &C, uint64_t t, unsigned int *) {
    Rec r;
    if (t >= C.n_rec) return r;
    const uint4 p = ctx_of(C, t);
    r.row = p.x;
    r.ts = p.y;
    r.sysup = p.z;
    r.slot = p.w & 0xFFFF;
    r.info = (uint16_t)(p.w >> 16);
    r.late = (r.info & DG_LATE) != 0;
    r.valid = (r.info & DG_VALID) != 0;
    return r;
}

// Appends v to list for every lane that wants to, with one counter atomic per wave (the
// counters are single words: one atomic per record would serialise on them)
template <class CT>
__device__ __forceinline__ void wave_append(uint32_t *__restrict__ list, CT *__restrict__ counter, bool want,
                                            uint32_t v) {
    const uint64_t m = __ballot(want);
    if (!m) return;
    const int lane = (int)__lane_id(), l0 = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if (lane == l0) base = (uint32_t)atomicAdd(counter, (CT)__popcll(m));
    base = (uint32_t)__shfl((int)base, l0);
    if (want) list[base + __popcll(m & ((1ull << lane) - 1))] = v;
}

// Open-addressing probe for one record's group.  Claiming a free slot: CAS on the tag, then
// the key bytes.  At a slot whose tag equals the record's, hashed keys are compared when the
// slot's key is known to be written: its group was reduced by an earlier push (the row's
// per-push marker is set), or exact = true (records whose hash collided, re-probed after the
// pass that wrote every key).  A slot claimed by another record of this same pass is taken
// tentatively (*tentative): k_agg_check compares the keys once the pass is over.
template <bool EXACT>
__device__ __forceinline__ uint32_t probe(const AggSlotPlan &sp, const AggParams &P, uint64_t row, uint32_t win,
                                          uint32_t kp, const KeyVal &kv, uint64_t h,
                                          unsigned long long *__restrict__ tags, uint8_t *__restrict__ rows,
                                          unsigned int *__restrict__ err, bool *tentative, bool *claimed) {
    uint64_t g = slot_of(h) & P.mask;
    *tentative = *claimed = false;
    for (uint64_t probes = 0; probes <= P.mask; ++probes, g = (g + 1) & P.mask) {
        unsigned long long cur = tags[g];
        if (cur == TAG_EMPTY) {
            cur = atomicCAS(&tags[g], TAG_EMPTY, (unsigned long long)h);
            if (cur == TAG_EMPTY) {
                key_write(rows + g * P.row_bytes, sp, P, row, win, kp, kv, err);
                *claimed = true;
                return (uint32_t)g;
            }
        }
        if (cur != h) continue;
        if (P.packed) return (uint32_t)g;
        const uint8_t *R = rows + g * P.row_bytes;
        // the marker is written by k_agg_apply* only: stable during this pass (loaded with the key)
        const uint32_t mark = EXACT ? 1u : *(const uint32_t *)(R + 36);
        const bool eq = key_equal(R, sp, P, row, win, kp, kv);
        if (mark != 0) {
            if (eq) return (uint32_t)g;
            continue;
        }
        *tentative = true;
        return (uint32_t)g;
    }
    atomicOr(err, 2u);  // table full
    return NONE;
}

// First pass: every record of the push
__global__ __launch_bounds__(256) void k_agg_claim(const RecCtx C, const AggParams P,
                                                   unsigned long long *__restrict__ tags, uint8_t *__restrict__ rows,
                                                   uint32_t *__restrict__ rec_g, uint32_t *__restrict__ claims,
                                                   unsigned long long *__restrict__ n_claims,
                                                   unsigned long long *__restrict__ late_count,
                                                   uint32_t *__restrict__ tent, unsigned int *__restrict__ n_tent,
                                                   unsigned int *__restrict__ err) {
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < C.n_rec; base += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t t = base + threadIdx.x;
        const Rec r = rec_from(ctx_of_block(C, t));  // base: a multiple of 256
        const uint64_t late_mask = __ballot(r.late);
        if ((threadIdx.x & 63) == 0 && late_mask) atomicAdd(late_count, (unsigned long long)__popcll(late_mask));
        const uint32_t su = wave_uniform_slot(r.slot, r.valid);  // the wave's template, in an SGPR
        if (t >= C.n_rec) continue;
        uint32_t g = NONE;
        bool tentative = false, claimed = false;
        if (r.valid) {
            auto go = [&](const AggSlotPlan &sp) {
                const uint32_t ts = r.ts, win = ts - ts % 60;  // get_window_start
                uint32_t kp;
                KeyVal kv;
                const uint64_t h = key_tag(sp, P, r.row, win, kp, kv);
                g = probe<false>(sp, P, r.row, win, kp, kv, h, tags, rows, err, &tentative, &claimed);
            };
            if (su != NONE) go(C.plans[su]);
            else go(C.plans[r.slot]);
            // every record of the group writes itself as the owner; the last store wins
            if (P.own && g != NONE) *(uint32_t *)(rows + (uint64_t)g * P.row_bytes + OWN_OFF) = (uint32_t)t;
        }
        wave_append(tent, n_tent, tentative, (uint32_t)t);
        wave_append(claims, n_claims, claimed, g);
        rec_g[t] = g;
    }
}

// Hashed keys: compare each record's key with its slot's (all slots' keys are written by now);
// a record on another key's slot (64-bit tag collision) is listed for the exact re-probe.
// list == null: every record; else the records listed.
__global__ __launch_bounds__(256) void k_agg_check(const RecCtx C, const AggParams P, const uint8_t *__restrict__ rows,
                                                   uint32_t *__restrict__ rec_g, const uint32_t *__restrict__ list,
                                                   uint32_t n_list, uint32_t *__restrict__ collided,
                                                   unsigned int *__restrict__ n_collided,
                                                   unsigned int *__restrict__ err) {
    const uint64_t n = list ? n_list : C.n_rec;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t t = list ? list[i] : i;
        const uint32_t g = rec_g[t];
        if (g == NONE) continue;
        const Rec r = rec_of(C, t, err);
        if (!r.valid) continue;
        const AggSlotPlan &sp = C.plans[r.slot];
        const uint32_t ts = r.ts, win = ts - ts % 60;
        uint32_t kp;
        KeyVal kv;
        (void)key_tag(sp, P, r.row, win, kp, kv);
        if (!key_equal(rows + (uint64_t)g * P.row_bytes, sp, P, r.row, win, kp, kv)) {
            rec_g[t] = NONE;
            collided[atomicAdd(n_collided, 1u)] = (uint32_t)t;  // rare (64-bit tag collisions)
        }
    }
}

// Exact re-probe of the listed records
__global__ __launch_bounds__(256) void k_agg_reprobe(const RecCtx C, const AggParams P,
                                                     unsigned long long *__restrict__ tags, uint8_t *__restrict__ rows,
                                                     uint32_t *__restrict__ rec_g, const uint32_t *__restrict__ list,
                                                     uint32_t n_list, uint32_t *__restrict__ claims,
                                                     unsigned long long *__restrict__ n_claims,
                                                     unsigned int *__restrict__ err) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n_list; i += gridDim.x * blockDim.x) {
        const uint64_t t = list[i];
        const Rec r = rec_of(C, t, err);
        bool tentative = false, claimed = false;
        uint32_t g = NONE;
        if (r.valid) {
            const AggSlotPlan &sp = C.plans[r.slot];
            const uint32_t ts = r.ts, win = ts - ts % 60;
            uint32_t kp;
            KeyVal kv;
            const uint64_t h = key_tag(sp, P, r.row, win, kp, kv);
            g = probe<true>(sp, P, r.row, win, kp, kv, h, tags, rows, err, &tentative, &claimed);
            rec_g[t] = g;
        }
        wave_append(claims, n_claims, claimed, g);
    }
}

// A failed push releases the slots it claimed (their rows still hold the identity values:
// a claim writes only the key)
__global__ void k_agg_unclaim(unsigned long long *__restrict__ tags, const uint32_t *__restrict__ claims, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        tags[claims[i]] = TAG_EMPTY;
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const int lo = __shfl_xor((int)(uint32_t)v, m), hi = __shfl_xor((int)(uint32_t)(v >> 32), m);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
    const int lo = __shfl((int)(uint32_t)v, lane), hi = __shfl((int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
enum { R_ADD, R_MIN, R_MAX, R_OR };
template <int OP>
__device__ __forceinline__ uint64_t wave_reduce(uint64_t v) {  // butterfly over the 64 lanes
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint64_t o = shfl_xor64(v, m);
        v = OP == R_ADD ? v + o : OP == R_MIN ? (o < v ? o : v) : OP == R_MAX ? (o > v ? o : v) : (v | o);
    }
    return v;
}

// Conditional atomics: a plain load of the accumulator first.  Min / max / OR only ever
// move one way between table resets, so a stale value can only cause an unneeded atomic,
// never a skipped one; after a group's first few records most of them are skipped.
__device__ __forceinline__ uint32_t peek32(const uint8_t *p) { return *(const volatile uint32_t *)p; }
__device__ __forceinline__ uint64_t peek64(const uint8_t *p) { return *(const volatile uint64_t *)p; }
__device__ __forceinline__ void min32(uint8_t *p, uint32_t v) { if (v < peek32(p)) atomicMin((unsigned int *)p, v); }
__device__ __forceinline__ void max32(uint8_t *p, uint32_t v) { if (v > peek32(p)) atomicMax((unsigned int *)p, v); }
__device__ __forceinline__ void or32(uint8_t *p, uint32_t v) {
    if (v & ~peek32(p)) atomicOr((unsigned int *)p, v);
}
__device__ __forceinline__ void or64(uint8_t *p, uint64_t v) {
    if (v & ~peek64(p)) atomicOr((unsigned long long *)p, (unsigned long long)v);
}

__device__ __forceinline__ void apply_value(uint8_t *dst, uint8_t op, uint64_t x) {
    switch (op) {
    case NGZ_AGG_ADD: if (x) atomicAdd((unsigned long long *)dst, (unsigned long long)x); break;
    case NGZ_AGG_MIN: if (x < peek64(dst)) atomicMin((unsigned long long *)dst, (unsigned long long)x); break;
    case NGZ_AGG_MAX: if (x > peek64(dst)) atomicMax((unsigned long long *)dst, (unsigned long long)x); break;
    default: or64(dst, x); break;
    }
}

__device__ __forceinline__ void apply_value_hot(uint8_t *dst, uint8_t op, uint64_t x) {
    switch (op) {
    case NGZ_AGG_ADD: atomicAdd((unsigned long long *)dst, (unsigned long long)x); break;
    case NGZ_AGG_MIN: atomicMin((unsigned long long *)dst, (unsigned long long)x); break;
    case NGZ_AGG_MAX: atomicMax((unsigned long long *)dst, (unsigned long long)x); break;
    default: if (x) atomicOr((unsigned long long *)dst, (unsigned long long)x); break;
    }
}

__device__ __forceinline__ void apply_push_constants(uint8_t *R, const AggParams &P) {
    // per-push constants once per (group, push): collection time bounds, peer port
    if (peek32(R + 36) != P.push_id && atomicExch((unsigned int *)(R + 36), P.push_id) != P.push_id) {
        atomicMin((unsigned long long *)(R + 40), (unsigned long long)P.coll_flip);
        atomicMax((unsigned long long *)(R + 48), (unsigned long long)P.coll_flip);
        atomicOr((unsigned long long *)(R + 64), 1ull << P.port_bit);
    }
}

// One lane per record, its group's row known (k_agg_claim).  Lanes of a wave that share a
// group are first reduced across the wave and applied by one lane (wave pre-aggregation:
// low-cardinality keys would otherwise serialise on a few hot rows); once the largest
// remaining group of the wave has fewer than 4 records, every remaining lane applies its own
// record.  Wave results are combined further in a per-workgroup LDS table (CN entries) across
// all the tiles the workgroup walks, and applied to HBM once per workgroup.  Values of the
// ordered classes are left to k_agg_ordered.
constexpr int CN = 64;
constexpr int CN_PROBES = 8;  // a group's entry sits within this many slots of its home slot
template <int MAXV>  // aggregated fields held in registers (value loads issued together, before any atomic)
__global__ __launch_bounds__(256, 4) void k_agg_apply(const RecCtx C, const AggParams P,
                                                    uint32_t *__restrict__ rec_g, uint8_t *__restrict__ rows,
                                                    const uint32_t *__restrict__ list,
                                                    const unsigned int *__restrict__ n_list,
                                                    unsigned int *__restrict__ err) {
    __shared__ uint32_t c_g[CN];
    __shared__ unsigned long long c_cnt[CN], c_tpl[CN], c_d0[CN], c_d1[CN];
    __shared__ unsigned long long c_val[CN][NGZ_AGG_MAX_VALUES];
    __shared__ uint32_t c_tmin[CN], c_tmax[CN], c_smax[CN], c_vp[CN], c_wt[CN];
    for (int e = threadIdx.x; e < CN; e += blockDim.x) {
        c_g[e] = NONE;
        c_wt[e] = NONE;
        c_cnt[e] = c_tpl[e] = c_d0[e] = c_d1[e] = 0;
        c_tmin[e] = 0xFFFFFFFFu;
        c_tmax[e] = c_smax[e] = c_vp[e] = 0;
        for (uint32_t v = 0; v < P.n_vals; ++v) c_val[e][v] = P.val_op[v] == NGZ_AGG_MIN ? ~0ull : 0ull;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    // list: the records k_agg_own left (not their group's owner), else every record
    const uint64_t n = list ? *n_list : C.n_rec;
    // the next tile's record index, group and context are loaded while this tile is reduced
    // (one dependent round trip less per tile: the kernel is latency-bound)
    auto fetch = [&](uint64_t tile, uint64_t &t, uint32_t &g, uint4 &ctx) {
        const uint64_t i = tile * blockDim.x + threadIdx.x;
        t = i < n ? (list ? list[i] : i) : C.n_rec;
        g = t < C.n_rec ? rec_g[t] : NONE;
        ctx = ctx_of(C, t);
    };
    uint64_t t_next;
    uint32_t g_next;
    uint4 c_next;
    if ((uint64_t)blockIdx.x * blockDim.x < n) fetch(blockIdx.x, t_next, g_next, c_next);
    for (uint64_t tile = blockIdx.x; tile * blockDim.x < n; tile += gridDim.x) {
        const uint64_t t = t_next;
        uint32_t g = g_next;
        const uint4 ctx = c_next;
        if ((tile + gridDim.x) * blockDim.x < n) fetch(tile + gridDim.x, t_next, g_next, c_next);
        const uint32_t wave_tile = (uint32_t)(tile * (blockDim.x / 64) + threadIdx.x / 64);  // unique per block
        Rec r;
        if (g != NONE) {  // rec_of from the prefetched context
            r.row = ctx.x;
            r.ts = ctx.y;
            r.sysup = ctx.z;
            r.slot = ctx.w & 0xFFFF;
            r.info = (uint16_t)(ctx.w >> 16);
            r.late = (r.info & DG_LATE) != 0;
            r.valid = (r.info & DG_VALID) != 0;
        }
        if (!list && g != NONE && P.own && r.valid &&
            *(const uint32_t *)(rows + (uint64_t)g * P.row_bytes + OWN_OFF) == (uint32_t)t) {
            // the group's owner record is left to k_agg_apply_own, which runs after this kernel
            rec_g[t] = g | OWN_BIT;
            g = NONE;
        }
        const bool valid = g != NONE && r.valid;
        if (!valid) g = NONE;
        const AggSlotPlan &sp = C.plans[valid ? r.slot : 0];
        const uint64_t row = r.row;
        uint32_t ts = 0, sysup = 0;
        uint64_t tpl = 0, dom0 = 0, dom1 = 0;
        if (valid) {
            ts = r.ts;
            sysup = r.sysup;
            tpl = sp.tpl_bit;
            const uint32_t db = (r.info >> 2) & 0x7F;
            (db < 64 ? dom0 : dom1) = 1ull << (db & 63);
        }
        uint64_t xv[MAXV];
        uint32_t hv = 0, hb = 0;  // aggregated fields present: numeric (in xv) / byte-wise OR
#pragma unroll
        for (int v = 0; v < MAXV; ++v) {
            xv[v] = 0;
            if (valid && v < (int)P.n_vals && sp.val_col[v] && !vc_ordered(P.val_vc[v])) {
                if (P.val_vc[v] == VC_BYTES) hb |= 1u << v;
                else { xv[v] = value_operand(sp, P, v, row); hv |= 1u << v; }
            }
        }
        uint64_t todo = __ballot(valid);
        // records of one datagram share export time, sys-up time, template and domain: when the
        // whole wave does, the wave reductions of those are skipped
        bool hdr_uniform = false;
        if (todo) {
            const int l0 = __ffsll((unsigned long long)todo) - 1;
            const uint64_t u0 = readlane64(((uint64_t)ts << 32) | sysup, l0), u1 = readlane64(tpl, l0),
                           u2 = readlane64(dom0 | (dom1 ? (1ull << 63) | dom1 : 0ull), l0);
            const bool same = !valid || ((((uint64_t)ts << 32) | sysup) == u0 && tpl == u1 &&
                                         (dom0 | (dom1 ? (1ull << 63) | dom1 : 0ull)) == u2);
            hdr_uniform = __ballot(!same) == 0;
        }
        if (P.lds_ok && todo) {
            // lanes whose group already has an entry in the workgroup's table apply their own
            // record there, all lanes at once (one LDS atomic per field and lane; lanes of one
            // group collide on its entry, which the LDS serialises far faster than the leader
            // loop below walks the groups one by one); the loop is left with the other lanes
            int e = -1;
            if (valid) {
                int i = (int)(slot_of(g) & (CN - 1));
                for (int probes = 0; probes < CN_PROBES; ++probes, i = (i + 1) & (CN - 1)) {
                    const uint32_t cur = c_g[i];
                    if (cur == g) { e = i; break; }
                    if (cur == NONE) break;
                }
            }
            const uint64_t hits = __ballot(e >= 0);
            if (hits) {
                todo &= ~hits;
                if (e >= 0) {
                    atomicAdd(&c_cnt[e], 1ull);
                    // the header fields once per (entry, wave tile) when the wave shares them
                    const bool hdr = !hdr_uniform || atomicExch(&c_wt[e], wave_tile) != wave_tile;
                    if (hdr) {
                        atomicMin(&c_tmin[e], ts);
                        atomicMax(&c_tmax[e], ts);
                        if (sysup) atomicMax(&c_smax[e], sysup);
                        atomicOr(&c_tpl[e], (unsigned long long)tpl);
                        if (dom0) atomicOr(&c_d0[e], (unsigned long long)dom0);
                        if (dom1) atomicOr(&c_d1[e], (unsigned long long)dom1);
                    }
#pragma unroll
                    for (int v = 0; v < MAXV; ++v) {
                        if (v >= (int)P.n_vals) break;
                        if (!((hv >> v) & 1)) continue;
                        unsigned long long *c = &c_val[e][v];
                        switch (P.val_op[v]) {
                        case NGZ_AGG_ADD: if (xv[v]) atomicAdd(c, (unsigned long long)xv[v]); break;
                        case NGZ_AGG_MIN: atomicMin(c, (unsigned long long)xv[v]); break;
                        case NGZ_AGG_MAX: atomicMax(c, (unsigned long long)xv[v]); break;
                        default: atomicOr(c, (unsigned long long)xv[v]); break;
                        }
                    }
                    if (hv) atomicOr(&c_vp[e], hv);
                }
            }
        }
        while (todo) {
            const int leader = __ffsll((unsigned long long)todo) - 1;
            const uint32_t lg = (uint32_t)__shfl((int)g, leader);
            const bool mine = valid && ((todo >> lane) & 1) && g == lg;
            const uint64_t match = __ballot(mine);
            if (__popcll(match) < 4) break;
            todo &= ~match;
            const uint64_t cnt = __popcll(match);
            uint8_t *R = rows + (uint64_t)lg * P.row_bytes;
            if (P.lds_ok) {
                // combine-table path: the leader claims the group's LDS entry and every matching
                // lane applies its own record with LDS atomics (no cross-lane reductions)
                int e0 = -1;
                if (lane == leader) {
                    int i = (int)(slot_of(lg) & (CN - 1));
                    for (int probes = 0; probes < CN_PROBES; ++probes, i = (i + 1) & (CN - 1)) {
                        uint32_t cur = c_g[i];
                        if (cur == NONE) {
                            cur = atomicCAS(&c_g[i], NONE, lg);
                            if (cur == NONE) { e0 = i; break; }
                        }
                        if (cur == lg) { e0 = i; break; }
                    }
                }
                const int e = __shfl(e0, leader);
                if (e >= 0) {
                    if (lane == leader) atomicAdd(&c_cnt[e], (unsigned long long)cnt);
                    if (hdr_uniform ? lane == leader : mine) {
                        atomicMin(&c_tmin[e], ts);
                        atomicMax(&c_tmax[e], ts);
                        if (sysup) atomicMax(&c_smax[e], sysup);
                        atomicOr(&c_tpl[e], (unsigned long long)tpl);
                        if (dom0) atomicOr(&c_d0[e], (unsigned long long)dom0);
                        if (dom1) atomicOr(&c_d1[e], (unsigned long long)dom1);
                    }
                    uint32_t vp = 0;
#pragma unroll
                    for (int v = 0; v < MAXV; ++v) {
                        if (v >= (int)P.n_vals) break;
                        const bool hasn = mine && ((hv >> v) & 1);
                        if (__ballot(hasn)) vp |= 1u << v;
                        if (hasn) {
                            unsigned long long *c = &c_val[e][v];
                            switch (P.val_op[v]) {
                            case NGZ_AGG_ADD: atomicAdd(c, (unsigned long long)xv[v]); break;
                            case NGZ_AGG_MIN: atomicMin(c, (unsigned long long)xv[v]); break;
                            case NGZ_AGG_MAX: atomicMax(c, (unsigned long long)xv[v]); break;
                            default: atomicOr(c, (unsigned long long)xv[v]); break;
                            }
                        }
                    }
                    if (lane == leader && vp) atomicOr(&c_vp[e], vp);
                    continue;  // the wave's next group
                }
            }
            uint64_t tmin = ts, tmax = ts, smax = sysup, tpls = tpl, d0 = dom0, d1 = dom1;  // (leader's own)
            if (!hdr_uniform) {
                tmin = wave_reduce<R_MIN>(mine ? ts : 0xFFFFFFFFull);
                tmax = wave_reduce<R_MAX>(mine ? ts : 0ull);
                smax = wave_reduce<R_MAX>(mine ? sysup : 0ull);
                tpls = wave_reduce<R_OR>(mine ? tpl : 0ull);
                d0 = wave_reduce<R_OR>(mine ? dom0 : 0ull);
                d1 = wave_reduce<R_OR>(mine ? dom1 : 0ull);
            }
            if (lane == leader) {
                // hot rows: fire-and-forget atomics (a load of a contended line costs more)
                atomicAdd((unsigned long long *)(R + 16), (unsigned long long)cnt);
                atomicMin((unsigned int *)(R + 24), (uint32_t)tmin);
                atomicMax((unsigned int *)(R + 28), (uint32_t)tmax);
                if (smax) atomicMax((unsigned int *)(R + 32), (uint32_t)smax);
                atomicOr((unsigned long long *)(R + 56), (unsigned long long)tpls);
                if (d0) atomicOr((unsigned long long *)(R + 72), (unsigned long long)d0);
                if (d1) atomicOr((unsigned long long *)(R + 80), (unsigned long long)d1);
                apply_push_constants(R, P);
            }
            uint32_t vp = 0;
#pragma unroll
            for (int v = 0; v < MAXV; ++v) {
                if (v >= (int)P.n_vals) break;
                const bool hasn = mine && ((hv >> v) & 1), bytes = mine && ((hb >> v) & 1);
                const bool any_num = __ballot(hasn) != 0, any_bytes = __ballot(bytes) != 0;
                if (!any_num && !any_bytes) continue;
                vp |= 1u << v;
                const uint8_t op = P.val_op[v];
                const uint64_t x = hasn ? xv[v] : (op == NGZ_AGG_MIN ? ~0ull : 0ull);
                uint64_t rr = 0;
                if (any_num) switch (op) {
                case NGZ_AGG_ADD: rr = wave_reduce<R_ADD>(x); break;
                case NGZ_AGG_MIN: rr = wave_reduce<R_MIN>(x); break;
                case NGZ_AGG_MAX: rr = wave_reduce<R_MAX>(x); break;
                default: rr = wave_reduce<R_OR>(x); break;
                }
                if (lane == leader && any_num) apply_value_hot(R + P.val_off[v], op, rr);
                if (bytes) {  // byte ORs: each matching lane ORs its words into the row
                    const uint32_t w = sp.val_w[v];
                    bool nul = false;
                    for (uint32_t j = 0; j < (w + 3) / 4; ++j)
                        or32(R + P.val_off[v] + 4 * j, cell_word(sp.val_col[v] + row * w, w, j, false, nul));
                }
            }
            if (lane == leader && vp) atomicOr((unsigned int *)(R + 12), vp);
        }
        if (!(valid && ((todo >> lane) & 1))) continue;
        // per-record path
        uint8_t *R = rows + (uint64_t)g * P.row_bytes;
        atomicAdd((unsigned long long *)(R + 16), 1ull);
        min32(R + 24, ts);
        max32(R + 28, ts);
        max32(R + 32, sysup);
        or64(R + 56, tpl);
        or64(R + (dom0 ? 72 : 80), dom0 | dom1);
        apply_push_constants(R, P);
#pragma unroll
        for (int v = 0; v < MAXV; ++v) {
            if (v >= (int)P.n_vals) break;
            uint8_t *dst = R + P.val_off[v];
            if ((hv >> v) & 1) {
                apply_value(dst, P.val_op[v], xv[v]);
            } else if ((hb >> v) & 1) {  // BoolMapOr over bytes (mac, mpls label, octetArray, u256)
                const uint32_t w = sp.val_w[v];
                bool nul = false;
                for (uint32_t j = 0; j < (w + 3) / 4; ++j) or32(dst + 4 * j, cell_word(sp.val_col[v] + row * w, w, j, false, nul));
            }
        }
        or32(R + 12, hv | hb);
    }  // tiles
    __syncthreads();
    for (int e = threadIdx.x; e < CN; e += blockDim.x) {  // the workgroup's combined groups -> HBM
        const uint32_t gg = c_g[e];
        if (gg == NONE) continue;
        uint8_t *R = rows + (uint64_t)gg * P.row_bytes;
        atomicAdd((unsigned long long *)(R + 16), c_cnt[e]);
        min32(R + 24, c_tmin[e]);
        max32(R + 28, c_tmax[e]);
        max32(R + 32, c_smax[e]);
        or64(R + 56, c_tpl[e]);
        or64(R + 72, c_d0[e]);
        or64(R + 80, c_d1[e]);
        apply_push_constants(R, P);
        const uint32_t vp = c_vp[e];
        for (uint32_t v = 0; v < P.n_vals; ++v)
            if ((vp >> v) & 1) apply_value(R + P.val_off[v], P.val_op[v], c_val[e][v]);
        or32(R + 12, vp);
    }
}

// Owner path ops, one per 8-byte unit of the row (AggParams::unit_op / unit_src)
enum : uint8_t { U_KEEP = 0, U_ADD = 1, U_MIN = 2, U_MAX = 3, U_OR = 4, U_VP = 5, U_TS = 6, U_SYS = 7 };
constexpr int OWN_ROUNDS = 2;  // k_agg_apply_own: rounds of eight owners whose rows are in flight together
// k_agg_apply_own's LDS row per record: aggregated-field operands 0-7, then export | sys-up time,
// template bit, domain bits, present-value bits
enum : uint32_t { OP_TS = 8, OP_TPL = 9, OP_D0 = 10, OP_D1 = 11, OP_HV = 12, OPW = 13 };
enum : uint8_t { U_SRC_ONE = 8, U_SRC_COLL = 9, U_SRC_PORT = 10, U_SRC_TPL = 11, U_SRC_DOM0 = 12, U_SRC_DOM1 = 13 };

// The owner record of each group: its whole reduction with plain loads and stores, eight
// lanes per record, each lane one 16-byte piece of the row (two with rows over 128 bytes), so
// one wave instruction moves eight rows.  A row is touched by no other lane in this kernel.
//
// FUSED (default): runs first.  Every valid record is taken; the row's owner word, read with
// the row, decides; the records that are not their group's owner are listed in rest for
// k_agg_apply's atomics, which run after this kernel.  The owner test costs no read of its own
// (5-tuple: 3.3 ms of k_agg_apply per 10^8 records saved).  !FUSED (NGZ_AGG_OWN_SPLIT): runs
// after k_agg_apply, which tested every record's owner word and applied the others.
template <bool FUSED>
__global__ __launch_bounds__(256) void k_agg_apply_own(const RecCtx C, const AggParams P,
                                                       uint32_t *__restrict__ rec_g, uint8_t *__restrict__ rows,
                                                       uint32_t *__restrict__ rest, unsigned int *__restrict__ n_rest,
                                                       unsigned int *__restrict__ err) {
    const uint32_t lane = threadIdx.x & 63, piece = lane & 7, np = P.row_bytes / 16;
    const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t n_waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    // 64 records per wave step.  Every lane first loads its own record's operands (coalesced,
    // all in flight together) and puts them in the wave's LDS rows; the owners among them are
    // then taken eight at a time, one per lane octet, and each lane reads from LDS just the
    // operands of its own row piece's units (the op table is per lane), so each round waits on
    // its rows only.  (Handing all operands over by lane shuffles took ~25 bpermutes per round
    // and 16 more VGPRs.)
    __shared__ unsigned long long opnd[4][64][OPW];
    unsigned long long (*ops)[OPW] = opnd[(threadIdx.x >> 6) & 3];
    // the lane's four 8-byte units (2p, 2p+1 in the first line, 2p+16, 2p+17 in the second):
    // op, and the operand column of the LDS row (OPW: none)
    uint32_t uop[4], ucol[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t u = 2 * piece + (j & 1) + (j >= 2 ? 16 : 0);
        uop[j] = (uint32_t)(P.unit_op[u >> 4] >> (4 * (u & 15))) & 15;
        const uint32_t sv = (uint32_t)(P.unit_src[u >> 4] >> (4 * (u & 15))) & 15;
        ucol[j] = uop[j] == U_KEEP ? OPW : uop[j] == U_VP ? OP_HV : (uop[j] == U_TS || uop[j] == U_SYS) ? OP_TS
                : sv < 8 ? sv : sv == U_SRC_TPL ? OP_TPL : sv == U_SRC_DOM0 ? OP_D0 : sv == U_SRC_DOM1 ? OP_D1 : OPW;
    }
    for (uint64_t base = wave * 64; base < C.n_rec; base += n_waves * 64) {
        const uint32_t mine = base + lane < C.n_rec ? rec_g[base + lane] : NONE;
        Rec r;
        if (FUSED && mine != NONE) r = rec_from(ctx_of_block(C, base + lane));  // base: a multiple of 64
        const bool owner = FUSED ? mine != NONE && r.valid : mine != NONE && (mine & OWN_BIT);
        uint64_t m = __ballot(owner);
        if (!m) continue;
        if (!FUSED && owner) rec_g[base + lane] = mine & ~OWN_BIT;  // plain group index again (k_agg_ordered sorts on it)
        if (!FUSED && owner) r = rec_from(ctx_of_block(C, base + lane));
        const uint32_t su = wave_uniform_slot(r.slot, r.valid);
        {
            const AggSlotPlan &sp = su != NONE ? C.plans[su] : C.plans[r.slot];
            const uint32_t db = (r.info >> 2) & 0x7F;
            uint32_t hv = 0;
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                uint64_t x = 0;
                if (r.valid && v < (int)P.n_vals && sp.val_col[v] && !vc_ordered(P.val_vc[v])) {
                    x = value_operand(sp, P, v, r.row);
                    hv |= 1u << v;
                }
                ops[lane][v] = x;
            }
            ops[lane][OP_TS] = ((uint64_t)r.sysup << 32) | r.ts;
            ops[lane][OP_TPL] = r.valid ? sp.tpl_bit : 0ull;
            ops[lane][OP_D0] = db < 64 ? 1ull << db : 0ull;
            ops[lane][OP_D1] = db < 64 ? 0ull : 1ull << (db & 63);
            ops[lane][OP_HV] = hv;
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t vmask = r.valid ? 1u : 0u;
        while (m) {
            // up to OWN_ROUNDS rounds of eight owners: every round's rows are loaded before any
            // is reduced, so OWN_ROUNDS x 8 rows per wave are in flight
            int src[OWN_ROUNDS];
            bool one[OWN_ROUNDS], two[OWN_ROUNDS];
            uint4 *q[OWN_ROUNDS];
            uint4 w0[OWN_ROUNDS], w1[OWN_ROUNDS];
#pragma unroll
            for (int k = 0; k < OWN_ROUNDS; ++k) {
                // octet o takes the o-th lowest owner left in m
                uint64_t mm = m;
                for (uint32_t o = lane >> 3; o > 0 && mm; --o) mm &= mm - 1;
                const bool act = mm != 0;
                src[k] = act ? __ffsll((unsigned long long)mm) - 1 : 0;
                for (int j = 0; j < 8 && m; ++j) m &= m - 1;
                // every lane takes part in the shuffles (a lane left out by a short-circuit
                // would read 0 from an inactive source lane)
                const uint32_t g = (uint32_t)__shfl((int)mine, src[k]) & ~OWN_BIT;
                const uint32_t s_valid = (uint32_t)__shfl((int)vmask, src[k]);
                const bool ok = act && s_valid != 0;
                q[k] = (uint4 *)(rows + (uint64_t)g * P.row_bytes);
                one[k] = ok && piece < np;
                two[k] = ok && piece + 8 < np;
                w0[k] = w1[k] = make_uint4(0, 0, 0, 0);
                if (one[k]) w0[k] = q[k][piece];
                if (two[k]) w1[k] = q[k][piece + 8];
            }
            if (FUSED) {
#pragma unroll
                for (int k = 0; k < OWN_ROUNDS; ++k) {
                    // the owner word (byte OWN_OFF = 88: piece 5, third dword), from the octet's lane 5
                    const uint32_t ownw = (uint32_t)__shfl((int)w0[k].z, (int)((lane & ~7u) + OWN_OFF / 16));
                    const uint32_t t = (uint32_t)(base + src[k]);
                    // the octet holds a valid record (its lane 0 loaded piece 0)
                    const uint32_t cand = (uint32_t)__shfl((int)(one[k] ? 1 : 0), (int)(lane & ~7u));
                    const bool is_owner = cand && ownw == t;
                    wave_append(rest, n_rest, cand && !is_owner && piece == 0, t);
                    one[k] = one[k] && is_owner;
                    two[k] = two[k] && is_owner;
                }
            }
#pragma unroll
            for (int k = 0; k < OWN_ROUNDS; ++k) {
                const unsigned long long *o = ops[src[k]];
                const uint32_t s_hv = (uint32_t)o[OP_HV];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if (!(h ? two[k] : one[k])) continue;
                    uint4 &wv = h ? w1[k] : w0[k];
                    uint32_t *c = (uint32_t *)&wv;
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        const int j = 2 * h + e;
                        const uint32_t op = uop[j];
                        if (op == U_KEEP) continue;
                        uint32_t &lo = c[2 * e], &hi = c[2 * e + 1];
                        const uint32_t col = ucol[j];
                        const uint64_t x = col < OPW ? o[col] : 0ull;
                        if (op == U_VP) { hi |= s_hv; continue; }
                        if (op == U_TS) { lo = min(lo, (uint32_t)x); hi = max(hi, (uint32_t)x); continue; }
                        if (op == U_SYS) { lo = max(lo, (uint32_t)(x >> 32)); hi = P.push_id; continue; }
                        uint64_t y;
                        if (col < 8) {
                            if (!((s_hv >> col) & 1)) continue;  // the record lacks the field (None)
                            y = x;
                        } else if (col < OPW) {
                            y = x;
                        } else {  // per-push constants
                            const uint32_t u = 2 * piece + (j & 1) + (j >= 2 ? 16 : 0);
                            const uint32_t sv = (uint32_t)(P.unit_src[u >> 4] >> (4 * (u & 15))) & 15;
                            y = sv == U_SRC_ONE ? 1ull : sv == U_SRC_COLL ? P.coll_flip : 1ull << P.port_bit;
                        }
                        uint64_t cur = ((uint64_t)hi << 32) | lo;
                        cur = op == U_ADD ? cur + y : op == U_MIN ? (y < cur ? y : cur) : op == U_MAX ? (y > cur ? y : cur)
                                                                                                       : (cur | y);
                        lo = (uint32_t)cur;
                        hi = (uint32_t)(cur >> 32);
                    }
                    q[k][piece + 8 * h] = wv;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

__global__ void k_agg_iota(uint32_t *__restrict__ x, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        x[i] = (uint32_t)i;
}

// OrderedFloat's Ord (ordered_float: NaN equals NaN and is greater than every number; -0 == +0)
template <class F>
__device__ __forceinline__ int ofloat_cmp(F a, F b) {
    const bool na = a != a, nb = b != b;
    if (na || nb) return na == nb ? 0 : (na ? 1 : -1);
    return a < b ? -1 : (a > b ? 1 : 0);
}

// Ord::min / Ord::max (core::cmp::min_by / max_by): on equal, min keeps the first argument
// (the group's value) and max takes the second (the record's) -- `*v1 = (*v1).min(*v2)`
__device__ __forceinline__ bool take_new(uint8_t op, int cmp_cur_new) {
    return op == NGZ_AGG_MIN ? cmp_cur_new > 0 : cmp_cur_new <= 0;
}

// One thread per group present in the sorted record list: the ordered reductions folded in
// record order (the stable sort kept it within a group), from the group's value.
__global__ __launch_bounds__(256) void k_agg_ordered(const RecCtx C, const AggParams P,
                                                     const uint32_t *__restrict__ sg, const uint32_t *__restrict__ sr,
                                                     uint64_t n, uint8_t *__restrict__ rows,
                                                     unsigned int *__restrict__ err) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t g = sg[i];
        if (g == NONE || (i > 0 && sg[i - 1] == g)) continue;  // not the first record of its group
        uint8_t *R = rows + (uint64_t)g * P.row_bytes;
        uint32_t vp = *(const uint32_t *)(R + 12);
        for (uint32_t v = 0; v < P.n_vals; ++v) {
            const uint8_t vc = P.val_vc[v];
            if (!vc_ordered(vc)) continue;
            const uint8_t op = P.val_op[v];
            bool have = (vp >> v) & 1;
            uint8_t *dst = R + P.val_off[v];
            if (vc == VC_VBYTES) {
                // octetArray `|=`: the first value keeps its length, later ones OR in their zipped
                // prefix (generator.rs:1051-1059); the tail of a value longer than 32 bytes is ORed
                // in place in the arena
                uint32_t *d = (uint32_t *)dst;
                uint32_t n0 = have ? d[0] : 0u, inl[BVAL_INLINE / 4];
#pragma unroll
                for (uint32_t j = 0; j < BVAL_INLINE / 4; ++j) inl[j] = have ? d[2 + j] : 0u;
                for (uint64_t j = i; j < n && sg[j] == g; ++j) {
                    const Rec r = rec_of(C, sr[j], err);
                    if (!r.valid) continue;
                    const AggSlotPlan &sp = C.plans[r.slot];
                    if (!sp.val_col[v]) continue;
                    const Span s = val_span(sp, v, r.row);
                    if (!have) {
                        bval_write(dst, s, P, err);  // the group's first value, tail included
                        n0 = s.n;
#pragma unroll
                        for (uint32_t q = 0; q < BVAL_INLINE / 4; ++q) inl[q] = d[2 + q];
                        have = true;
                        continue;
                    }
                    const uint32_t m = min(n0, s.n);
#pragma unroll
                    for (uint32_t q = 0; q < BVAL_INLINE / 4; ++q) inl[q] |= span_word(s.p, min(m, BVAL_INLINE), q);
                    if (m > BVAL_INLINE) {
                        uint8_t *t = P.arena + ((uint64_t)d[1] << 3);
                        for (uint32_t b = BVAL_INLINE; b < m; ++b) t[b - BVAL_INLINE] |= s.p[b];
                    }
                }
                if (have) {
#pragma unroll
                    for (uint32_t q = 0; q < BVAL_INLINE / 4; ++q) d[2 + q] = inl[q];
                    vp |= 1u << v;
                }
                continue;
            }
            if (vc == VC_VLIST) {
                // Box<[u8]> Min / Max: the best value so far is the group's (in the row) or a record's
                // (in the batch); written once at the end
                BRef best = have ? bval_ref(dst, P) : BRef{nullptr, nullptr, 0, 0};
                bool from_rec = false;
                Span bs{nullptr, 0};
                for (uint64_t j = i; j < n && sg[j] == g; ++j) {
                    const Rec r = rec_of(C, sr[j], err);
                    if (!r.valid) continue;
                    const AggSlotPlan &sp = C.plans[r.slot];
                    if (!sp.val_col[v]) continue;
                    const Span s = val_span(sp, v, r.row);
                    const BRef x{s.p, nullptr, s.n, s.n};
                    if (!have || take_new(op, bytes_cmp(best, x))) {
                        best = x;
                        bs = s;
                        from_rec = true;
                    }
                    have = true;
                }
                if (from_rec) {
                    bval_write(dst, bs, P, err);
                    vp |= 1u << v;
                }
                continue;
            }
            double cd = 0;
            float cf = 0;
            uint8_t c6[16];
            if (have) {
                if (vc == VC_F64) memcpy(&cd, dst, 8);
                else if (vc == VC_F32) memcpy(&cf, dst, 4);
                else memcpy(c6, dst, 16);
            }
            for (uint64_t j = i; j < n && sg[j] == g; ++j) {
                const Rec r = rec_of(C, sr[j], err);
                if (!r.valid) continue;
                const AggSlotPlan &sp = C.plans[r.slot];
                if (!sp.val_col[v]) continue;
                const uint8_t *cell = sp.val_col[v] + r.row * sp.val_w[v];
                if (vc == VC_F64) {
                    double x;
                    memcpy(&x, cell, 8);
                    if (!have) cd = x;
                    else if (op == NGZ_AGG_ADD) cd = cd + x;
                    else if (take_new(op, ofloat_cmp(cd, x))) cd = x;
                } else if (vc == VC_F32) {
                    float x;
                    memcpy(&x, cell, 4);
                    if (!have) cf = x;
                    else if (op == NGZ_AGG_ADD) cf = cf + x;
                    else if (take_new(op, ofloat_cmp(cf, x))) cf = x;
                } else {  // Ipv6Addr: octets in order
                    int c = 0;
                    if (have)
                        for (int b = 0; b < 16 && c == 0; ++b) c = (int)c6[b] - (int)cell[b];
                    if (!have || take_new(op, c)) memcpy(c6, cell, 16);
                }
                have = true;
            }
            if (have) {
                if (vc == VC_F64) memcpy(dst, &cd, 8);
                else if (vc == VC_F32) { memcpy(dst, &cf, 4); memset(dst + 4, 0, 4); }
                else memcpy(dst, c6, 16);
                vp |= 1u << v;
            }
        }
        *(uint32_t *)(R + 12) = vp;
    }
}

// ---- Partitioned reduction: many groups, several records each per push ----
// Groups far beyond a workgroup's LDS table (protocol + port: 393 216 groups of ~250 records per
// push) leave k_agg_apply with ~3 device atomics per record, each a memory round trip.  Instead
// the records are partitioned by table slot range: partition p is slots [p, p + 1) * PART_SLOTS,
// so its groups fit one workgroup's LDS table indexed by slot.  A histogram pass (partition-major
// counts per tile of records), one scan and a scatter pass copy every record's operands into its
// partition's run; one workgroup per partition then reduces its run in LDS and updates its rows
// with plain loads and stores (no other workgroup touches them).  Per record: its operands read
// once, a payload written and read once, instead of ~3 atomics and ~8 row peeks.  The order of
// records within a run is not kept: only order-free reductions run here (ordered classes are
// k_agg_ordered's).
constexpr uint32_t PART_SLOTS = 512, PART_SHIFT = 9;
constexpr uint32_t PART_TILE = 65536;  // records per histogram / scatter workgroup (grid size; at most
                                       // 2048 workgroups)

// Workgroup w of the histogram and scatter passes takes rounds w, w + G, w + 2G, ... of PART_ROUND
// records (G workgroups): at any time the grid works on one contiguous stretch of records, so the
// operand columns are read as a few sequential streams (tiles of contiguous records per workgroup
// made ~10 000 concurrent column streams, and the operand loads ran at under 1 TB/s)
constexpr uint32_t PART_RPT = 4;                      // records per thread and round
#ifndef NGZ_SCATTER_ATTRIB
#define NGZ_SCATTER_ATTRIB 0  // timing-attribution variants of k_agg_part_scatter (experiment builds; wrong output)
#endif
constexpr uint32_t PART_ROUND = 256 * PART_RPT;

// counts[p * G + w]: workgroup w's records headed for partition p (a record has a group only if
// the claim found it valid)
__global__ __launch_bounds__(256) void k_agg_part_hist(const RecCtx C, const uint32_t *__restrict__ rec_g, uint32_t n_part,
                                                       uint32_t *__restrict__ counts) {
    extern __shared__ uint32_t h[];
    for (uint32_t i = threadIdx.x; i < n_part; i += blockDim.x) h[i] = 0;
    __syncthreads();
    for (uint64_t r0 = (uint64_t)blockIdx.x * PART_ROUND; r0 < C.n_rec; r0 += (uint64_t)gridDim.x * PART_ROUND)
        for (uint32_t k = 0; k < PART_RPT; ++k) {
            const uint64_t t = r0 + k * 256 + threadIdx.x;
            const uint32_t g = t < C.n_rec ? rec_g[t] : NONE;
            if (g != NONE) atomicAdd(&h[g >> PART_SHIFT], 1u);
        }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < n_part; i += blockDim.x) counts[(uint64_t)i * gridDim.x + blockIdx.x] = h[i];
}

// Payload of one record (pb = 16 NP bytes, a multiple of 32): {group, export time, sys-up time,
// slot | info << 16}, then the operands of the order-free aggregated fields at their own widths
// (P.op_off / op_w: 8-byte operands first, then 4, 2, 1; an unsigned field's operand is its column
// width, others 8 bytes), zero padded.  A payload fills whole 32-byte sectors, so one written in
// pieces needs no read-modify-write in DRAM (80-byte payloads of 7 u64 operands straddled sectors:
// 113 bytes of WRITE_SIZE per payload).  Each thread builds PART_RPT payloads a round, every load of
// the round issued before the first payload is assembled, and stores each as NP 16-byte pieces.
template <uint32_t NP>
__global__ __launch_bounds__(256) void k_agg_part_scatter(const RecCtx C, const AggParams P, const uint32_t *__restrict__ rec_g,
                                                          uint32_t n_part, const uint32_t *__restrict__ offs,
                                                          uint8_t *__restrict__ pay) {
    extern __shared__ uint32_t cur[];
    __shared__ uint4 stage[256 * NP];  // per wave: 64 payload rows (the store transpose)
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i = threadIdx.x; i < n_part; i += blockDim.x) cur[i] = offs[(uint64_t)i * gridDim.x + blockIdx.x];
    __syncthreads();
    // thread i of a round takes records r0 + 4i .. r0 + 4i + 3 (a wave: one aligned 256-record
    // block): its group ids come in one 16-byte load and, when the four are consecutive rows of one
    // template, each operand column in one load of 4 cells (4, 8, 16 or 2x16 bytes) -- a quarter of
    // the load instructions of a record per lane
    for (uint64_t r0 = (uint64_t)blockIdx.x * PART_ROUND; r0 < C.n_rec; r0 += (uint64_t)gridDim.x * PART_ROUND) {
        const uint64_t t0 = r0 + PART_RPT * threadIdx.x;
        uint32_t g[PART_RPT];
        uint4 c[PART_RPT];
        if (t0 + PART_RPT <= C.n_rec) {
            const uint4 gg = *(const uint4 *)(rec_g + t0);
            g[0] = gg.x;
            g[1] = gg.y;
            g[2] = gg.z;
            g[3] = gg.w;
        } else {
#pragma unroll
            for (uint32_t k = 0; k < PART_RPT; ++k) g[k] = t0 + k < C.n_rec ? rec_g[t0 + k] : NONE;
        }
#pragma unroll
        for (uint32_t k = 0; k < PART_RPT; ++k)
#if NGZ_SCATTER_ATTRIB & 1  // timing attribution (experiment variants only): no context chain
            c[k] = g[k] != NONE ? make_uint4((uint32_t)(t0 + k), 0, 0, C.sctx[0].w) : make_uint4(0, 0, 0, 0);
#else
            c[k] = g[k] != NONE ? ctx_of_block(C, t0 + k) : make_uint4(0, 0, 0, 0);
#endif
        uint64_t x[PART_RPT][8];
        const uint32_t slot0 = c[0].w & 0xFFFF;
        bool quad = true;
#pragma unroll
        for (uint32_t k = 0; k < PART_RPT; ++k)
            quad = quad && g[k] != NONE && (c[k].w & 0xFFFF) == slot0 && c[k].x == c[0].x + k;
        quad = quad && (c[0].x & 3) == 0;
        const uint32_t suq = wave_uniform_slot(slot0, quad);
        if (quad && suq != NONE) {
            const AggSlotPlan &sp = C.plans[suq];
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                uint64_t raw[PART_RPT] = {0, 0, 0, 0};
                const uint32_t wv = sp.val_w[v];
                if (P.op_w[v] && sp.val_col[v] && wv != 1 && wv != 2 && wv != 4 && wv != 8) {
                    // other widths (byte-wise OR of a 3..7-byte cell): cell by cell
#pragma unroll
                    for (uint32_t k = 0; k < PART_RPT; ++k) x[k][v] = value_operand(sp, P, v, c[k].x);
                    continue;
                }
                if (P.op_w[v] && sp.val_col[v] && !(NGZ_SCATTER_ATTRIB & 2)) {  // (2: no operand loads)
                    const uint32_t w = wv;
                    const uint8_t *b = sp.val_col[v] + (uint64_t)c[0].x * w;
                    if (w == 1) {
                        const uint32_t q = *(const uint32_t *)b;
                        raw[0] = q & 0xFF; raw[1] = (q >> 8) & 0xFF; raw[2] = (q >> 16) & 0xFF; raw[3] = q >> 24;
                    } else if (w == 2) {
                        const uint2 q = *(const uint2 *)b;
                        raw[0] = q.x & 0xFFFF; raw[1] = q.x >> 16; raw[2] = q.y & 0xFFFF; raw[3] = q.y >> 16;
                    } else if (w == 4) {
                        const uint4 q = *(const uint4 *)b;
                        raw[0] = q.x; raw[1] = q.y; raw[2] = q.z; raw[3] = q.w;
                    } else {
                        const uint4 q0 = *(const uint4 *)b, q1 = *(const uint4 *)(b + 16);
                        raw[0] = ((uint64_t)q0.y << 32) | q0.x; raw[1] = ((uint64_t)q0.w << 32) | q0.z;
                        raw[2] = ((uint64_t)q1.y << 32) | q1.x; raw[3] = ((uint64_t)q1.w << 32) | q1.z;
                    }
                }
#pragma unroll
                for (uint32_t k = 0; k < PART_RPT; ++k)
                    x[k][v] = P.op_w[v] && sp.val_col[v] ? operand_of_raw(sp, P, v, raw[k]) : 0ull;
            }
        } else {
#pragma unroll
            for (uint32_t k = 0; k < PART_RPT; ++k) {
                const uint32_t slot = c[k].w & 0xFFFF;
                const AggSlotPlan &sp = C.plans[slot];
#pragma unroll
                for (int v = 0; v < 8; ++v)
                    x[k][v] = g[k] != NONE && P.op_w[v] && sp.val_col[v] ? value_operand(sp, P, v, c[k].x) : 0ull;
            }
        }
#pragma unroll
        for (uint32_t k = 0; k < PART_RPT; ++k) {
            const bool has = g[k] != NONE;
            const uint32_t pos = has ? atomicAdd(&cur[g[k] >> PART_SHIFT], 1u) : 0u;
            uint32_t wd[NP * 4];
            wd[0] = g[k];
            wd[1] = c[k].y;
            wd[2] = c[k].z;
            wd[3] = c[k].w;
#pragma unroll
            for (uint32_t j = 4; j < NP * 4; ++j) wd[j] = 0;
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                const uint32_t ow = P.op_w[v];
                if (!ow) continue;
                const uint64_t xv = x[k][v];
                // the operand's dword: a wave-uniform index into the payload registers (one indexed
                // move each, not a compare and select per payload dword)
                const uint32_t o = P.op_off[v], j0 = __builtin_amdgcn_readfirstlane(o >> 2), sh = 8 * (o & 3);
                const uint32_t lo = ow >= 4 ? (uint32_t)xv : ow == 2 ? ((uint32_t)xv & 0xFFFFu) << sh : ((uint32_t)xv & 0xFFu) << sh;
                wd[j0] |= lo;
                if (ow == 8) wd[j0 + 1] = (uint32_t)(xv >> 32);
            }
            if (NGZ_SCATTER_ATTRIB & 4) continue;  // (4: no payload stores)
            // The payloads go out whole: lane l's row of the wave's LDS stage, then each store
            // instruction writes 64 / NP payloads with NP consecutive lanes per payload (piece
            // lane % NP of payload lane / NP).  A store of one piece per lane wrote 64 payloads, 64
            // scattered lines per instruction: the stores were 70 % of this kernel (5.4 -> 1.8 ms
            // without them, profiles/r5/agg_scatter_attrib)
            uint4 *row = &stage[(threadIdx.x & ~63u) * NP + lane * NP];
#pragma unroll
            for (uint32_t j = 0; j < NP; ++j) row[j] = make_uint4(wd[4 * j], wd[4 * j + 1], wd[4 * j + 2], wd[4 * j + 3]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint64_t hm = __builtin_amdgcn_ballot_w64(has);
            constexpr uint32_t R = 64 / NP;  // payloads per store instruction
#pragma unroll
            for (uint32_t s0 = 0; s0 < 64; s0 += R) {
                const uint32_t m = s0 + lane / NP, j = lane % NP;
                const uint32_t pm = (uint32_t)__shfl((int)pos, (int)(m & 63), 64);
                if (lane / NP < R && m < 64 && ((hm >> m) & 1))
                    ((uint4 *)(pay + (uint64_t)pm * (16 * NP)))[j] = stage[(threadIdx.x & ~63u) * NP + m * NP + j];
            }
            // the next record's rows overwrite the stage: every lane's reads of it are done
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
    }
}

// One workgroup per partition: its run reduced into an LDS table indexed by slot, then every
// touched row updated in place (the reductions of FlowCacheRecord::reduce, aggregator.rs:159-198)
template <uint32_t NP, uint32_t RPT>
__global__ __launch_bounds__(1024) void k_agg_part_reduce(const AggParams P, const AggSlotPlan *__restrict__ plans,
                                                         const uint32_t *__restrict__ offs, uint32_t n_tiles,
                                                         const uint8_t *__restrict__ pay, uint8_t *__restrict__ rows) {
    __shared__ uint32_t e_cnt[PART_SLOTS], e_tmin[PART_SLOTS], e_tmax[PART_SLOTS], e_smax[PART_SLOTS], e_vp[PART_SLOTS];
    __shared__ unsigned long long e_tpl[PART_SLOTS], e_d0[PART_SLOTS], e_d1[PART_SLOTS];
    __shared__ unsigned long long e_val[8][PART_SLOTS];
    for (uint32_t e = threadIdx.x; e < PART_SLOTS; e += blockDim.x) {
        e_cnt[e] = e_smax[e] = e_vp[e] = e_tmax[e] = 0;
        e_tmin[e] = 0xFFFFFFFFu;
        e_tpl[e] = e_d0[e] = e_d1[e] = 0;
#pragma unroll
        for (int v = 0; v < 8; ++v) e_val[v][e] = v < (int)P.n_vals && P.val_op[v] == NGZ_AGG_MIN ? ~0ull : 0ull;
    }
    __syncthreads();
    const uint32_t p = blockIdx.x;
    const uint64_t beg = offs[(uint64_t)p * n_tiles], end = offs[(uint64_t)(p + 1) * n_tiles];
    // RPT payloads per thread and round, all loaded before the first is reduced (one round
    // trip per round, not per record)
    for (uint64_t i0 = beg; i0 < end; i0 += (uint64_t)RPT * blockDim.x) {
        uint4 q[RPT][NP];
#pragma unroll
        for (uint32_t k = 0; k < RPT; ++k) {
            const uint64_t i = i0 + k * blockDim.x + threadIdx.x;
#pragma unroll
            for (uint32_t j = 0; j < NP; ++j) q[k][j] = i < end ? ((const uint4 *)(pay + i * 16 * NP))[j] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (uint32_t k = 0; k < RPT; ++k) {
        if (i0 + k * blockDim.x + threadIdx.x >= end) continue;
        uint32_t wd[NP * 4];
#pragma unroll
        for (uint32_t j = 0; j < NP; ++j) {
            wd[4 * j] = q[k][j].x;
            wd[4 * j + 1] = q[k][j].y;
            wd[4 * j + 2] = q[k][j].z;
            wd[4 * j + 3] = q[k][j].w;
        }
        const uint4 h = make_uint4(wd[0], wd[1], wd[2], wd[3]);
        uint64_t x[8];
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            // the operand's dwords by a wave-uniform index (k_agg_part_scatter's layout)
            const uint32_t ow = P.op_w[v], o = P.op_off[v], j0 = __builtin_amdgcn_readfirstlane(o >> 2), sh = 8 * (o & 3);
            const uint32_t lo = ow ? wd[j0] : 0u, hi = ow == 8 ? wd[j0 + 1] : 0u;
            x[v] = ow == 8 ? ((uint64_t)hi << 32) | lo : ow == 4 ? (uint64_t)lo : ow == 2 ? (uint64_t)((lo >> sh) & 0xFFFFu)
                 : ow == 1 ? (uint64_t)((lo >> sh) & 0xFFu) : 0ull;
        }
        const uint32_t e = h.x & (PART_SLOTS - 1), ts = h.y, sysup = h.z, slot = h.w & 0xFFFF, info = h.w >> 16;
        const uint32_t su = wave_uniform_slot(slot, true);
        const AggSlotPlan &sp = su != NONE ? plans[su] : plans[slot];
        const uint32_t db = (info >> 2) & 0x7F;
        // Min / Max / Or only move one way: an entry the record cannot change (read first) takes no
        // atomic.  After a group's first records that is most of them, and the LDS atomics (a dozen
        // per record, 64-bit ones at half rate) were what bounded this kernel
        atomicAdd(&e_cnt[e], 1u);
        if (ts < e_tmin[e]) atomicMin(&e_tmin[e], ts);
        if (ts > e_tmax[e]) atomicMax(&e_tmax[e], ts);
        if (sysup > e_smax[e]) atomicMax(&e_smax[e], sysup);
        const unsigned long long tb = sp.tpl_bit;
        if ((e_tpl[e] & tb) != tb) atomicOr(&e_tpl[e], tb);
        unsigned long long *dd = db < 64 ? &e_d0[e] : &e_d1[e];
        const unsigned long long dbit = 1ull << (db & 63);
        if (!(*dd & dbit)) atomicOr(dd, dbit);
        uint32_t hv = 0;
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            if (v >= (int)P.n_vals || !sp.val_col[v] || vc_ordered(P.val_vc[v])) continue;
            hv |= 1u << v;
            unsigned long long *c = &e_val[v][e];
            const unsigned long long xv = x[v];
            switch (P.val_op[v]) {
            case NGZ_AGG_ADD: if (xv) atomicAdd(c, xv); break;
            case NGZ_AGG_MIN: if (xv < *c) atomicMin(c, xv); break;
            case NGZ_AGG_MAX: if (xv > *c) atomicMax(c, xv); break;
            default: if ((*c | xv) != *c) atomicOr(c, xv); break;
            }
        }
        if ((e_vp[e] & hv) != hv) atomicOr(&e_vp[e], hv);
        }
    }
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < PART_SLOTS; e += blockDim.x) {
        const uint32_t cnt = e_cnt[e];
        if (!cnt) continue;
        uint8_t *R = rows + (uint64_t)(p * PART_SLOTS + e) * P.row_bytes;
        uint32_t *u = (uint32_t *)R;
        uint64_t *w = (uint64_t *)R;
        w[2] += cnt;                      // record_count (16)
        u[6] = min(u[6], e_tmin[e]);      // min / max export time (24, 28)
        u[7] = max(u[7], e_tmax[e]);
        u[8] = max(u[8], e_smax[e]);      // max sys-up time (32)
        u[9] = P.push_id;                 // per-push marker (36): the push constants are applied here
        w[5] = min(w[5], P.coll_flip);    // min / max collection time, flipped (40, 48)
        w[6] = max(w[6], P.coll_flip);
        w[7] |= e_tpl[e];                 // template, peer port, domain sets (56, 64, 72, 80)
        w[8] |= 1ull << P.port_bit;
        w[9] |= e_d0[e];
        w[10] |= e_d1[e];
        const uint32_t vp = e_vp[e];
        u[3] |= vp;                       // val_present (12)
        for (uint32_t v = 0; v < P.n_vals && v < 8; ++v) {
            if (!((vp >> v) & 1)) continue;
            uint64_t *dst = (uint64_t *)(R + P.val_off[v]);
            const uint64_t xv = e_val[v][e], c = *dst;
            switch (P.val_op[v]) {
            case NGZ_AGG_ADD: *dst = c + xv; break;
            case NGZ_AGG_MIN: *dst = xv < c ? xv : c; break;
            case NGZ_AGG_MAX: *dst = xv > c ? xv : c; break;
            default: *dst = c | xv; break;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Low-cardinality pushes (packed keys, few distinct key tuples): one pass over
// the key and value columns, no per-record context, slot claim or HBM atomic.
//
// k_agg_lc_part: one wave per workgroup walks its sets (XCD-aware), 256 records
// per pass (4 rows per lane, rows 64 apart: every column load of the wave is one
// contiguous run) with every key and value column of the pass loaded together
// and the next pass of the set prefetched.  The wave finds its key tuples as it
// goes (a wave-uniform list of at most LC_NK per window context) and reduces each
// record into lane-private LDS cells, cell (tuple, field, lane): one LDS atomic
// per record and aggregated field, no conflicts between lanes.  Per-set header
// fields (export time bounds, sys-up time, template and domain sets) are uniform
// per set and kept per tuple in lane `tuple`'s registers.  When its sets move to
// another window context, and at its end, the wave reduces its cells and
// appends one partial entry per tuple to a small list.
//
// k_agg_lc_merge (one workgroup): the partial entries, a few per wave, combined
// per exact tag in LDS; then each distinct tag finds or claims its group in the
// HBM table and is applied to the row.  A push that needs more than the
// capacity, or meets a full table, releases its claims and changes nothing.
//
// A wave that meets more than LC_NK key tuples in one window context (or an
// entry list that would overflow) raises the overflow flag: every wave stops,
// the merge does nothing, and the push takes the general path from the start.
// ---------------------------------------------------------------------------
constexpr uint32_t LC_SLOTS = 256;    // merge: open-addressing table of the push's distinct tags
constexpr uint32_t LC_MAX_TAGS = 64;  // more distinct tags in one push: the general path
constexpr int LC_NK = 8;              // key tuples a wave accumulates per window context (more: general path)
constexpr int LC_MAXV = 8;            // aggregated fields (more: the general path)
constexpr int LC_CELLS = 32;          // lane-private cells per (tuple, field): lanes l and l + 32 share
                                      // one (they reach the LDS in different cycles, no conflict)

struct LcEntry {  // one wave's partial group (128 B)
    unsigned long long tag;  // exact packed tag (window / 60, flow type, peer, keys)
    unsigned long long cnt;
    uint32_t tmin, tmax, smax, vp;
    unsigned long long tpl, d0, d1;
    unsigned long long acc[LC_MAXV];
    unsigned long long pad;
};
static_assert(sizeof(LcEntry) == 128, "LcEntry");

// The buffer resource of a column's rows from A to the set's end (rounded up to 16 rows:
// range checks are per dword, so the set's last rows are never in a partly covered dword;
// in bounds, capacities being whole 256-row windows).  Reads past it return 0, so lanes past
// the set's end need no clamp, and an absent field (col null) is a resource of 0 bytes.
// Every input provably wave-uniform: a resource the compiler takes for a divergent one gets
// a waterfall loop around each load.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t lc_rsrc(const uint8_t *col, uint32_t w, uint64_t A, uint64_t end) {
    const int bytes = __builtin_amdgcn_readfirstlane(
        col ? (int)min<uint64_t>((((end + 15) & ~15ull) - A) * w, 0x7FFFFFF0ull) : 0);
    const uint64_t base = (uint64_t)(col ? col + A * w : nullptr);
    const uint64_t ub = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(base >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)base);
    return __builtin_amdgcn_make_buffer_rsrc((void *)ub, (short)0, bytes, 0x00020000);
}

constexpr int LC_G = 4;  // groups of 4 consecutive rows per lane and block: 1024 rows per block

// The lane's rows of a W-byte column: group q holds rows A + 256 q + 4 lane + (0..3), 4W bytes
// (4W-aligned), one 4-, 8- or 16-byte load (two for W = 8) per group, all in flight together.
// Each width has its own instantiation, and the caller consumes the words inside it: loads
// whose results merged across a branch on the width made the compiler wait on each at once.
template <int W>
struct LcCol {
    static constexpr int NW = W;  // dwords per group
    uint32_t d[LC_G][NW];
    __device__ __forceinline__ void load(const __amdgpu_buffer_rsrc_t r, uint32_t lane) {
        typedef unsigned int v2u __attribute__((ext_vector_type(2)));
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int q = 0; q < LC_G; ++q) {
            const uint32_t o = (256u * q + 4u * lane) * W;
            if constexpr (W == 1) {
                d[q][0] = __builtin_amdgcn_raw_buffer_load_b32(r, o, 0, 0);
            } else if constexpr (W == 2) {
                const v2u t = __builtin_amdgcn_raw_buffer_load_b64(r, o, 0, 0);
                d[q][0] = t.x, d[q][1] = t.y;
            } else {
#pragma unroll
                for (int h = 0; h < W / 4; ++h) {
                    const v4u t = __builtin_amdgcn_raw_buffer_load_b128(r, o + 16 * h, 0, 0);
                    d[q][4 * h] = t.x, d[q][4 * h + 1] = t.y, d[q][4 * h + 2] = t.z, d[q][4 * h + 3] = t.w;
                }
            }
        }
    }
    // row i (0-3) of group q, little-endian
    __device__ __forceinline__ uint64_t cell(int q, int i) const {
        if constexpr (W == 8) return d[q][2 * i] | ((uint64_t)d[q][2 * i + 1] << 32);
        else if constexpr (W == 4) return d[q][i];
        else if constexpr (W == 2) return (d[q][i >> 1] >> (16 * (i & 1))) & 0xFFFFu;
        else return (d[q][0] >> (8 * i)) & 0xFFu;
    }
};

// value_operand of a cell already loaded (raw: the w column bytes, little-endian)
__device__ __forceinline__ uint64_t lc_operand(const AggParams &P, uint32_t v, uint64_t raw, uint32_t w) {
    const uint8_t vc = P.val_vc[v];
    uint64_t x = raw;
    if (vc == VC_DTFRAC) {
        x = (raw << 32) | (raw >> 32);  // {u32 secs, u32 nanos} -> (secs, nanos) ordered
    } else if (vc == VC_SINT && w < 8) {
        const uint32_t sh = 64 - 8 * w;
        x = (uint64_t)(((int64_t)(raw << sh)) >> sh);
    }
    if (vc == VC_SINT && (P.val_op[v] == NGZ_AGG_MIN || P.val_op[v] == NGZ_AGG_MAX)) x ^= 1ull << 63;
    if (vc == VC_RANK) {
        if (P.val_tcp[v]) x = bitrev8((uint32_t)x & 0xFF);
        else if (const unsigned long long *nr = P.rank_nested[v]) x = x < 256 ? nr[x] : nr[256] | x;
        else {
            const uint32_t *known = P.rank_known[v];
            const bool reg = x < 65536 && known && ((known[x >> 5] >> (x & 31)) & 1);
            if (!reg) x |= 1ull << 32;
        }
    }
    return x;
}

__device__ __forceinline__ uint64_t lc_identity(uint8_t op) { return op == NGZ_AGG_MIN ? ~0ull : 0ull; }

constexpr int LC_MAXK = 4;  // key fields (packed keys: at most 35 bits of them)

// One set as k_agg_lc_part needs it, resolved ahead (no dependent chain set -> datagram
// -> plan per set in the reduce loop): 32 B, one scalar load
struct LcSet {
    uint32_t rec0, n, ts, sysup;
    uint32_t slot;  // NONE: no records aggregated (empty, late, failed datagram, slot not aggregated)
    uint32_t info;  // bits 0-6: observation domain entry
    uint32_t pad[2];
};
static_assert(sizeof(LcSet) == 32, "LcSet");

// a descriptor through the constant address space (scalar loads; the set index is uniform)
__device__ __forceinline__ LcSet lc_desc(const LcSet *p) {
    typedef const __attribute__((address_space(4))) LcSet *cset;
    const cset q = (cset)p;
    LcSet d;
    d.rec0 = q->rec0;
    d.n = q->n;
    d.ts = q->ts;
    d.sysup = q->sysup;
    d.slot = q->slot;
    d.info = q->info;
    d.pad[0] = d.pad[1] = 0;
    return d;
}

__global__ __launch_bounds__(256) void k_agg_lc_sets(const ngz_set_info *__restrict__ sets, uint32_t n_sets,
                                                     const ngz_dgram_hdr *__restrict__ hdr,
                                                     const uint16_t *__restrict__ dginfo,
                                                     const AggSlotPlan *__restrict__ plans, uint32_t n_dgrams,
                                                     uint32_t n_slots, LcSet *__restrict__ out,
                                                     unsigned long long *__restrict__ late_count,
                                                     unsigned int *__restrict__ err) {
    for (uint32_t s0 = blockIdx.x * blockDim.x; s0 < n_sets; s0 += gridDim.x * blockDim.x) {
    const uint32_t s = s0 + threadIdx.x;
    uint64_t late_n = 0;
    if (s < n_sets) {
        const ngz_set_info si = sets[s];
        LcSet d{si.rec0, si.n, 0, 0, NONE, 0, {0, 0}};
        if (si.n) {
            if (si.dgram >= n_dgrams || si.slot >= n_slots) {
                atomicOr(err, 16u);
            } else {
                const uint16_t info = dginfo[si.dgram];
                if (info & DG_LATE) {
                    late_n = si.n;
                } else if ((info & DG_USE) && plans[si.slot].usable) {
                    const ngz_dgram_hdr &h = hdr[si.dgram];
                    d.ts = h.time;
                    d.sysup = h.version == 9 ? h.sys_up_time : 0u;
                    d.slot = si.slot;
                    d.info = (info >> 2) & 0x7F;
                }
            }
        }
        out[s] = d;
    }
    late_n = wave_reduce<R_ADD>(late_n);  // one counter atomic per wave
    if ((threadIdx.x & 63) == 0 && late_n) atomicAdd(late_count, (unsigned long long)late_n);
    }
}

// One aggregated field of a block, W-byte column: the block's loads, then one LDS atomic per
// row into the row's tuple cell (rows outside the set have the spare tuple LC_NK)
template <int W>
__device__ __forceinline__ void lc_reduce_field(const __amdgpu_buffer_rsrc_t r, const AggParams &P, uint32_t v,
                                                uint32_t lane, const uint32_t (&cell)[LC_G * 4],
                                                unsigned long long *__restrict__ cv) {
    LcCol<W> c;
    c.load(r, lane);
    const uint8_t op = P.val_op[v], vc = P.val_vc[v];
    const bool plain = vc == VC_UINT || (vc == VC_SINT && W == 8 && op != NGZ_AGG_MIN && op != NGZ_AGG_MAX);
    uint64_t x[LC_G * 4];
#pragma unroll
    for (int q = 0; q < LC_G; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) x[4 * q + i] = c.cell(q, i);
    if (!plain) {
#pragma unroll
        for (int j = 0; j < LC_G * 4; ++j) x[j] = lc_operand(P, v, x[j], W);
    }
    switch (op) {
    case NGZ_AGG_ADD:
#pragma unroll
        for (int j = 0; j < LC_G * 4; ++j) atomicAdd(cv + cell[j], (unsigned long long)x[j]);
        break;
    case NGZ_AGG_MIN:
#pragma unroll
        for (int j = 0; j < LC_G * 4; ++j) atomicMin(cv + cell[j], (unsigned long long)x[j]);
        break;
    case NGZ_AGG_MAX:
#pragma unroll
        for (int j = 0; j < LC_G * 4; ++j) atomicMax(cv + cell[j], (unsigned long long)x[j]);
        break;
    default:
#pragma unroll
        for (int j = 0; j < LC_G * 4; ++j) atomicOr(cv + cell[j], (unsigned long long)x[j]);
        break;
    }
}

// One key field of a block into the packed keys: key = ((key << 1) | present) << 8W | value
template <int W>
__device__ __forceinline__ void lc_key_field(const __amdgpu_buffer_rsrc_t r, uint32_t lane, uint64_t has,
                                             uint64_t (&key)[LC_G * 4]) {
    LcCol<W> c;
    c.load(r, lane);
#pragma unroll
    for (int q = 0; q < LC_G; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) key[4 * q + i] = (((key[4 * q + i] << 1) | has) << (8 * W)) | c.cell(q, i);
}

// LDS per wave: value cells [tuple 0..LC_NK][field][LC_CELLS] (u64; tuple LC_NK takes the
// rows outside the set and is never read), then counts [tuple][LC_CELLS] (u32)
__host__ __device__ constexpr size_t lc_lds_bytes(uint32_t nv) {
    return (size_t)(LC_NK + 1) * nv * LC_CELLS * 8 + (size_t)(LC_NK + 1) * LC_CELLS * 4;
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) void k_agg_lc_part(
    const LcSet *__restrict__ descs, uint32_t n_sets, const AggSlotPlan *__restrict__ plans, const AggParams P,
    uint32_t key_bits, LcEntry *__restrict__ out, unsigned int *__restrict__ n_out, uint32_t cap,
    unsigned int *__restrict__ flag) {
    extern __shared__ unsigned long long lc_cells[];
    const uint32_t nv = P.n_vals, lane = threadIdx.x, cl = lane & (LC_CELLS - 1);
    unsigned int *lc_cnt = (unsigned int *)(lc_cells + (size_t)(LC_NK + 1) * nv * LC_CELLS);
    uint64_t kl[LC_NK];  // the wave's key tuples of the current window context (wave-uniform)
    uint32_t nkw = 0;
    // lane k: header fields of tuple k
    uint32_t h_tmin = 0xFFFFFFFFu, h_tmax = 0, h_smax = 0, h_vp = 0;
    uint64_t h_tpl = 0, h_d0 = 0, h_d1 = 0;
#pragma unroll
    for (int k = 0; k < LC_NK; ++k) kl[k] = 0;
    auto reset = [&]() {
        for (uint32_t c = 0; c < (uint32_t)(LC_NK + 1) * nv; ++c)
            lc_cells[c * LC_CELLS + cl] = lc_identity(P.val_op[c % nv]);
        for (uint32_t k = 0; k <= (uint32_t)LC_NK; ++k) lc_cnt[k * LC_CELLS + cl] = 0;
        nkw = 0;
        h_tmin = 0xFFFFFFFFu;
        h_tmax = h_smax = h_vp = 0;
        h_tpl = h_d0 = h_d1 = 0;
    };
    // the cells of window context ctx -> one entry per key tuple; false: the list is full
    auto flush = [&](uint64_t ctx) -> bool {
        if (!nkw) return true;
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(n_out, nkw);
        base = (uint32_t)__shfl((int)base, 0);
        if (base + nkw > cap) {
            if (lane == 0) atomicOr(flag, 1u);
            return false;
        }
#pragma unroll
        for (int k = 0; k < LC_NK; ++k) {
            if (k >= (int)nkw) break;
            const uint64_t total = wave_reduce<R_ADD>(lane < LC_CELLS ? (uint64_t)lc_cnt[k * LC_CELLS + cl] : 0ull);
            LcEntry *e = out + base + k;
            if (lane == (uint32_t)k) {  // the tuple's header lives in lane k
                e->tag = (ctx << key_bits) | kl[k] | (1ull << 63);  // key_tag's exact tag
                e->cnt = total;
                e->tmin = h_tmin;
                e->tmax = h_tmax;
                e->smax = h_smax;
                e->vp = h_vp;
                e->tpl = h_tpl;
                e->d0 = h_d0;
                e->d1 = h_d1;
            }
            for (uint32_t v = 0; v < nv; ++v) {
                const uint8_t op = P.val_op[v];
                const uint64_t a = lane < LC_CELLS ? lc_cells[(k * nv + v) * LC_CELLS + cl] : lc_identity(op);
                uint64_t r;
                switch (op) {
                case NGZ_AGG_ADD: r = wave_reduce<R_ADD>(a); break;
                case NGZ_AGG_MIN: r = wave_reduce<R_MIN>(a); break;
                case NGZ_AGG_MAX: r = wave_reduce<R_MAX>(a); break;
                default: r = wave_reduce<R_OR>(a); break;
                }
                if (lane == 0) e->acc[v] = r;
            }
        }
        return true;
    };
    reset();
    uint64_t cur = ~0ull;  // current window context (window / 60, flow type, peer); none yet
    // one wave per workgroup: the set sequence, the set and its plan are wave-uniform (scalar
    // loads, no EXEC masking around them); XCD-aware: workgroup b walks the (b % 8)-th eighth
    const uint32_t G = gridDim.x, X = (G % 8 == 0 && G >= 8) ? 8u : 1u;
    const uint32_t per = (n_sets + X - 1) / X, s_end = min(n_sets, (blockIdx.x % X) * per + per);
    typedef const __attribute__((address_space(4))) AggSlotPlan *cplan;
    const uint32_t s0 = (blockIdx.x % X) * per + blockIdx.x / X, step = G / X;
    LcSet dn{};  // the next set's descriptor, loaded one set ahead
    if (s0 < s_end) dn = lc_desc(descs + s0);
    uint32_t it = 0;
    for (uint32_t s = s0; s < s_end; s += step, ++it) {
        // some wave overflowed: the general path takes the push (checked every 16 sets)
        if ((it & 15) == 15 && *(volatile unsigned int *)flag) return;
        const LcSet d = dn;
        if (s + step < s_end) dn = lc_desc(descs + s + step);
        if (d.slot == NONE) continue;
        // the plan through the constant address space: its fields are wave-uniform and read
        // with scalar loads, also at a runtime field index
        const auto &sp = ((cplan)plans)[d.slot];
        const uint32_t ts = d.ts, win = ts - ts % 60;
        const uint64_t ctx = ((((uint64_t)(win / 60) << 1) | (sp.proto == 9)) << P.peer_bits) | P.peer;
        if (ctx != cur) {
            if (cur != ~0ull && !flush(cur)) return;
            reset();
            cur = ctx;
        }
        uint32_t hv = 0;  // aggregated fields the set's template has (Some)
        for (uint32_t v = 0; v < nv; ++v)
            if (sp.val_col[v]) hv |= 1u << v;
        const uint64_t end = (uint64_t)d.rec0 + d.n;
        uint32_t pres = 0;  // key tuples this lane saw in the set
        // blocks of 1024 rows from the set's first row rounded down to 4: lane l takes rows
        // A + 256 q + 4 l + i, so every column load is 4W-aligned and one wave instruction
        // covers 256 W contiguous bytes
        for (uint64_t A = d.rec0 & ~3ull; A < end; A += 256 * LC_G) {
            const uint32_t lo = (uint32_t)(d.rec0 > A ? d.rec0 - A : 0), hi = (uint32_t)min<uint64_t>(end - A, 256 * LC_G);
            uint64_t key[LC_G * 4];
#pragma unroll
            for (int j = 0; j < LC_G * 4; ++j) key[j] = 0;
            for (uint32_t k = 0; k < P.n_keys; ++k) {  // key_tag's packing of the key fields
                const uint8_t *col = sp.key_col[k];
                const __amdgpu_buffer_rsrc_t r = lc_rsrc(col, P.key_pw[k], A, end);
                const uint64_t has = col != nullptr;
                switch (P.key_pw[k]) {
                case 1: lc_key_field<1>(r, lane, has, key); break;
                case 2: lc_key_field<2>(r, lane, has, key); break;
                default: lc_key_field<4>(r, lane, has, key); break;
                }
            }
            // each row's tuple in the wave's list, extended by any tuple it has not met yet;
            // rows outside the set: the spare tuple LC_NK
            uint32_t kid[LC_G * 4], vm = 0;
#pragma unroll
            for (int j = 0; j < LC_G * 4; ++j) {
                const uint32_t rel = 256u * (j >> 2) + 4u * lane + (j & 3);
                if (rel - lo < hi - lo) vm |= 1u << j;  // lo <= rel < hi
                kid[j] = LC_NK;
            }
            // the wave's tuples one at a time (a uniform exit after the last one met)
#pragma unroll
            for (int k = 0; k < LC_NK; ++k) {
                if (k >= (int)nkw) break;
#pragma unroll
                for (int j = 0; j < LC_G * 4; ++j) kid[j] = key[j] == kl[k] ? (uint32_t)k : kid[j];
            }
            uint32_t unmatched = 0;
#pragma unroll
            for (int j = 0; j < LC_G * 4; ++j) unmatched |= kid[j] == LC_NK ? 1u << j : 0u;
            // rows whose tuple the wave has not met yet (rare): one tuple at a time, taken from the
            // first such row of the first such lane, entered into the list, matched everywhere
            uint32_t um = unmatched & vm;
            while (__ballot(um != 0)) {
                const int l0 = __ffsll((unsigned long long)__ballot(um != 0)) - 1;
                const uint32_t j0 = (uint32_t)__shfl((int)(um ? __builtin_ctz(um) : 0), l0);
                uint64_t kj = 0;
#pragma unroll
                for (int j = 0; j < LC_G * 4; ++j) kj = (uint32_t)j == j0 ? key[j] : kj;
                const uint64_t t = readlane64(kj, l0);
                if (nkw == (uint32_t)LC_NK) {
                    if (lane == 0) atomicOr(flag, 1u);
                    return;
                }
#pragma unroll
                for (int k = 0; k < LC_NK; ++k)
                    if (k == (int)nkw) kl[k] = t;
#pragma unroll
                for (int i = 0; i < LC_G * 4; ++i)
                    if (((um >> i) & 1) && key[i] == t) {
                        kid[i] = nkw;
                        um &= ~(1u << i);
                    }
                ++nkw;
            }
            uint32_t cell[LC_G * 4];
#pragma unroll
            for (int j = 0; j < LC_G * 4; ++j) {
                if (!((vm >> j) & 1)) kid[j] = LC_NK;
                pres |= (1u << kid[j]);
                atomicAdd(&lc_cnt[kid[j] * LC_CELLS + cl], 1u);
                cell[j] = kid[j] * nv * LC_CELLS + cl;
            }
            // field by field: the field's loads for the block in flight together, then its
            // LDS updates (the width's own instantiation; a runtime loop over the fields)
            for (uint32_t v = 0; v < nv; ++v) {
                if (!((hv >> v) & 1)) continue;
                const uint32_t w = sp.val_w[v];
                const __amdgpu_buffer_rsrc_t r = lc_rsrc(sp.val_col[v], w, A, end);
                unsigned long long *cv = lc_cells + v * LC_CELLS;
                switch (w) {
                case 8: lc_reduce_field<8>(r, P, v, lane, cell, cv); break;
                case 4: lc_reduce_field<4>(r, P, v, lane, cell, cv); break;
                case 2: lc_reduce_field<2>(r, P, v, lane, cell, cv); break;
                default: lc_reduce_field<1>(r, P, v, lane, cell, cv); break;
                }
            }
        }
        // key tuples present in the set: OR over the wave; lane k updates tuple k's header
        uint32_t mset = pres & ((1u << LC_NK) - 1);
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) mset |= (uint32_t)__shfl_xor((int)mset, m);
        if (lane < nkw && ((mset >> lane) & 1)) {
            const uint32_t db = d.info;
            h_tmin = min(h_tmin, ts);
            h_tmax = max(h_tmax, ts);
            h_smax = max(h_smax, d.sysup);
            h_tpl |= sp.tpl_bit;
            if (db < 64) h_d0 |= 1ull << db;
            else h_d1 |= 1ull << (db & 63);
            h_vp |= hv;
        }
    }
    if (cur != ~0ull) flush(cur);
}

// The key bytes of a packed tag into a claimed row (key_write's layout for packed keys)
__device__ __forceinline__ void lc_key_write(uint8_t *R, const AggParams &P, uint64_t tag) {
    uint64_t x = tag & ~(1ull << 63);
    uint32_t kp = 0;
    for (int k = (int)P.n_keys - 1; k >= 0; --k) {
        const uint32_t bits = 8 * P.key_pw[k];
        const uint64_t v = bits >= 64 ? x : (x & ((1ull << bits) - 1));
        x = bits >= 64 ? 0 : x >> bits;
        const bool present = x & 1;
        x >>= 1;
        if (present) kp |= 1u << k;
        uint32_t *dst = (uint32_t *)(R + P.key_off[k]);
        for (uint32_t j = 0; j < P.key_slot[k] / 4; ++j) dst[j] = present && j < 2 ? (uint32_t)(v >> (32 * j)) : 0u;
    }
    const uint32_t peer = (uint32_t)(x & ((1ull << P.peer_bits) - 1));
    x >>= P.peer_bits;
    const uint32_t proto = (x & 1) ? 9u : 10u;
    *(uint32_t *)(R + 0) = (uint32_t)(x >> 1) * 60u;
    *(uint32_t *)(R + 4) = proto | (peer << 16);
    *(uint32_t *)(R + 8) = kp;
}

// The partial entries, a few per wave, combined per exact tag: LCM_BLOCKS workgroups each
// combine a slice in LDS and write one entry per tag they met; the workgroup that finishes last
// combines those, then each distinct tag finds or claims its group and is applied to the row.
// err bits: 2 table full, 32 capacity (both: nothing claimed, nothing applied)
constexpr int LCM_THREADS = 256;
constexpr int LCM_BLOCKS = 64;

struct LcMergeLds {
    unsigned long long t_tag[LC_SLOTS];
    uint32_t t_idx[LC_SLOTS];
    unsigned long long m_tag[LC_MAX_TAGS], m_cnt[LC_MAX_TAGS], m_tpl[LC_MAX_TAGS], m_d0[LC_MAX_TAGS],
        m_d1[LC_MAX_TAGS], m_acc[LC_MAX_TAGS][LC_MAXV];
    uint32_t m_tmin[LC_MAX_TAGS], m_tmax[LC_MAX_TAGS], m_smax[LC_MAX_TAGS], m_vp[LC_MAX_TAGS], m_g[LC_MAX_TAGS],
        m_claimed[LC_MAX_TAGS];
    uint32_t n_tags, s_full, s_new, s_last;
};

// entries i = first, first + stride, ... < n of `in` combined into L; false: more than
// LC_MAX_TAGS distinct tags
__device__ bool lc_combine(LcMergeLds &L, const LcEntry *__restrict__ in, uint32_t first, uint32_t stride, uint32_t n,
                           const AggParams &P) {
    const uint32_t tid = threadIdx.x, nv = P.n_vals;
    for (uint32_t i = tid; i < LC_SLOTS; i += blockDim.x) {
        L.t_tag[i] = 0;
        L.t_idx[i] = NONE;
    }
    if (tid == 0) L.n_tags = 0;
    __syncthreads();
    auto find = [&](uint64_t tag, bool insert) -> uint32_t {
        uint32_t i = (uint32_t)(slot_of(tag) & (LC_SLOTS - 1));
        for (uint32_t probes = 0; probes < LC_SLOTS; ++probes, i = (i + 1) & (LC_SLOTS - 1)) {
            unsigned long long c = L.t_tag[i];
            if (c == 0 && insert) c = atomicCAS(&L.t_tag[i], 0ull, (unsigned long long)tag);
            if (c == 0) return insert ? i : NONE;
            if (c == tag) return i;
        }
        return NONE;
    };
    for (uint32_t i = first + tid * stride; i < n; i += blockDim.x * stride)
        if (in[i].tag) find(in[i].tag, true);  // tag 0: an unused slice entry
    __syncthreads();
    for (uint32_t i = tid; i < LC_SLOTS; i += blockDim.x) {
        if (!L.t_tag[i]) continue;
        const uint32_t m = atomicAdd(&L.n_tags, 1u);
        if (m >= LC_MAX_TAGS) continue;
        L.t_idx[i] = m;
        L.m_tag[m] = L.t_tag[i];
        L.m_cnt[m] = L.m_tpl[m] = L.m_d0[m] = L.m_d1[m] = 0;
        L.m_tmin[m] = 0xFFFFFFFFu;
        L.m_tmax[m] = L.m_smax[m] = L.m_vp[m] = 0;
        for (uint32_t v = 0; v < nv; ++v) L.m_acc[m][v] = lc_identity(P.val_op[v]);
    }
    __syncthreads();
    if (L.n_tags > LC_MAX_TAGS) return false;
    for (uint32_t i = first + tid * stride; i < n; i += blockDim.x * stride) {
        const LcEntry &e = in[i];
        if (!e.tag) continue;
        const uint32_t m = L.t_idx[find(e.tag, false)];
        atomicAdd(&L.m_cnt[m], e.cnt);
        atomicMin(&L.m_tmin[m], e.tmin);
        atomicMax(&L.m_tmax[m], e.tmax);
        atomicMax(&L.m_smax[m], e.smax);
        atomicOr(&L.m_vp[m], e.vp);
        atomicOr(&L.m_tpl[m], e.tpl);
        atomicOr(&L.m_d0[m], e.d0);
        atomicOr(&L.m_d1[m], e.d1);
        for (uint32_t v = 0; v < nv; ++v) {
            switch (P.val_op[v]) {
            case NGZ_AGG_ADD: atomicAdd(&L.m_acc[m][v], e.acc[v]); break;
            case NGZ_AGG_MIN: atomicMin(&L.m_acc[m][v], e.acc[v]); break;
            case NGZ_AGG_MAX: atomicMax(&L.m_acc[m][v], e.acc[v]); break;
            default: atomicOr(&L.m_acc[m][v], e.acc[v]); break;
            }
        }
    }
    __syncthreads();
    return true;
}

// part: LCM_BLOCKS * LC_MAX_TAGS entries of scratch; cnt: [0] entries written by
// k_agg_lc_part, [1] overflow flag, [2] workgroups done (zeroed before the launch)
__global__ __launch_bounds__(LCM_THREADS) void k_agg_lc_merge(const LcEntry *__restrict__ in, uint32_t cap,
                                                              LcEntry *__restrict__ part,
                                                              unsigned int *__restrict__ cnt, const AggParams P,
                                                              unsigned long long *__restrict__ tags,
                                                              uint8_t *__restrict__ rows, uint64_t room,
                                                              uint32_t *__restrict__ claims,
                                                              unsigned long long *__restrict__ n_claims,
                                                              unsigned int *__restrict__ err) {
    __shared__ LcMergeLds L;
    unsigned int *flag = cnt + 1;
    if (*(volatile unsigned int *)flag) return;  // uniform per launch: every workgroup returns
    const uint32_t tid = threadIdx.x, nv = P.n_vals;
    const uint32_t n_in = min(*(volatile unsigned int *)cnt, cap);
    // 1. this workgroup's slice (entries b, b + LCM_BLOCKS, ...) -> one entry per tag
    const bool ok = lc_combine(L, in, blockIdx.x, gridDim.x, n_in, P);
    LcEntry *mine = part + (size_t)blockIdx.x * LC_MAX_TAGS;
    const uint32_t nt = ok ? L.n_tags : 0;
    if (!ok && tid == 0) atomicOr(flag, 1u);
    for (uint32_t m = tid; m < LC_MAX_TAGS; m += blockDim.x) {
        LcEntry &e = mine[m];
        e.tag = m < nt ? L.m_tag[m] : 0ull;  // tag 0: no entry
        if (m >= nt) continue;
        e.cnt = L.m_cnt[m];
        e.tmin = L.m_tmin[m];
        e.tmax = L.m_tmax[m];
        e.smax = L.m_smax[m];
        e.vp = L.m_vp[m];
        e.tpl = L.m_tpl[m];
        e.d0 = L.m_d0[m];
        e.d1 = L.m_d1[m];
        for (uint32_t v = 0; v < nv; ++v) e.acc[v] = L.m_acc[m][v];
    }
    // 2. the last workgroup to finish combines the slices.  Release: every thread fences its own
    // slice stores at agent scope before the barrier (whichever waves wrote slice entries), then
    // one thread arrives; acquire: the last workgroup's loads after every arrival
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    if (tid == 0)
        L.s_last = __hip_atomic_fetch_add(cnt + 2, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    __syncthreads();
    if (!L.s_last) return;
    __atomic_thread_fence(__ATOMIC_ACQUIRE);  // every thread of the last workgroup
    if (*(volatile unsigned int *)flag) return;
    // slices' tag-0 entries (none) fall in their own LDS slot and are skipped below
    if (!lc_combine(L, part, 0, 1, gridDim.x * LC_MAX_TAGS, P)) {
        if (tid == 0) atomicOr(flag, 1u);  // too many groups for this path: the general path
        return;
    }
    if (tid == 0) L.s_full = L.s_new = 0;
    __syncthreads();
    // 3. each tag's group: found, or claimed (this workgroup is the push's only claimer)
    const uint32_t n_tags = L.n_tags;
    for (uint32_t m = tid; m < n_tags; m += blockDim.x) {
        L.m_g[m] = NONE;
        L.m_claimed[m] = 0;
        const uint64_t h = L.m_tag[m];
        if (!h) continue;
        uint64_t g = slot_of(h) & P.mask;
        uint32_t found = NONE, claimed = 0;
        for (uint64_t probes = 0; probes <= P.mask; ++probes, g = (g + 1) & P.mask) {
            unsigned long long c = tags[g];
            if (c == TAG_EMPTY) {
                c = atomicCAS(&tags[g], TAG_EMPTY, (unsigned long long)h);
                if (c == TAG_EMPTY) {
                    lc_key_write(rows + g * P.row_bytes, P, h);
                    found = (uint32_t)g;
                    claimed = 1;
                    break;
                }
            }
            if (c == h) {
                found = (uint32_t)g;
                break;
            }
        }
        L.m_g[m] = found;
        L.m_claimed[m] = claimed;
        if (found == NONE) atomicOr(&L.s_full, 1u);
        if (claimed) atomicAdd(&L.s_new, 1u);
    }
    __syncthreads();
    if (L.s_full || L.s_new > room) {  // nothing changes: release this push's claims
        for (uint32_t m = tid; m < n_tags; m += blockDim.x)
            if (L.m_claimed[m]) tags[L.m_g[m]] = TAG_EMPTY;
        if (tid == 0) atomicOr(err, L.s_full ? 2u : 32u);
        return;
    }
    // 4. the rows
    for (uint32_t m = tid; m < n_tags; m += blockDim.x) {
        if (!L.m_tag[m]) continue;
        const uint32_t g = L.m_g[m];
        if (L.m_claimed[m]) claims[atomicAdd(n_claims, 1ull)] = g;
        uint8_t *R = rows + (uint64_t)g * P.row_bytes;
        atomicAdd((unsigned long long *)(R + 16), L.m_cnt[m]);
        atomicMin((unsigned int *)(R + 24), L.m_tmin[m]);
        atomicMax((unsigned int *)(R + 28), L.m_tmax[m]);
        if (L.m_smax[m]) atomicMax((unsigned int *)(R + 32), L.m_smax[m]);
        atomicOr((unsigned long long *)(R + 56), L.m_tpl[m]);
        if (L.m_d0[m]) atomicOr((unsigned long long *)(R + 72), L.m_d0[m]);
        if (L.m_d1[m]) atomicOr((unsigned long long *)(R + 80), L.m_d1[m]);
        apply_push_constants(R, P);
        const uint32_t vp = L.m_vp[m];
        if (vp) atomicOr((unsigned int *)(R + 12), vp);
        for (uint32_t v = 0; v < nv; ++v)
            if ((vp >> v) & 1) apply_value_hot(R + P.val_off[v], P.val_op[v], L.m_acc[m][v]);
    }
}

__global__ void k_agg_init(uint8_t *__restrict__ rows, uint64_t n_groups, uint32_t row_bytes,
                           const uint32_t *__restrict__ ident, uint32_t ident_words) {
    // every row <- the identity row (min fields at their maximum)
    const uint64_t n_words = n_groups * (row_bytes / 4);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_words;
         i += (uint64_t)gridDim.x * blockDim.x)
        ((uint32_t *)rows)[i] = ident[i % ident_words];
}

// groups selected for output: every live group (cut == nullptr) or the closed windows, each
// group against its own peer's cutoff (cut[peer], INT64_MIN: the peer closed nothing)
__device__ __forceinline__ bool selected(uint64_t tag, const uint8_t *R, const int64_t *__restrict__ cut) {
    if (!tag_live(tag)) return false;
    if (!cut) return true;
    const uint32_t peer = *(const uint16_t *)(R + 6);
    return (int64_t)*(const uint32_t *)R <= cut[peer];
}

__global__ void k_agg_count(const unsigned long long *__restrict__ tags, const uint8_t *__restrict__ rows,
                            uint64_t n_slots, uint32_t row_bytes, const int64_t *__restrict__ cut,
                            unsigned long long *__restrict__ cursor) {
    uint32_t c = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n_slots;
         g += (uint64_t)gridDim.x * blockDim.x)
        c += selected(tags[g], rows + g * row_bytes, cut);
    if (c) atomicAdd(cursor, (unsigned long long)c);
}

// copies the selected groups to out; tomb: their slots become tombstones (closed windows)
__global__ void k_agg_take(unsigned long long *__restrict__ tags, const uint8_t *__restrict__ rows, uint64_t n_slots,
                           uint32_t row_bytes, const int64_t *__restrict__ cut, int tomb, uint8_t *__restrict__ out,
                           unsigned long long *__restrict__ cursor) {
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n_slots;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t *R = rows + g * row_bytes;
        if (!selected(tags[g], R, cut)) continue;
        const uint64_t o = atomicAdd(cursor, 1ull);
        const uint32_t *src = (const uint32_t *)R;
        uint32_t *dst = (uint32_t *)(out + o * row_bytes);
        for (uint32_t i = 0; i < row_bytes / 4; ++i) dst[i] = src[i];
        if (tomb) tags[g] = TAG_TOMB;
    }
}

// OR of the set bitmaps of every live group (dictionary entries still in use)
__global__ void k_agg_bits(const unsigned long long *__restrict__ tags, const uint8_t *__restrict__ rows,
                           uint64_t n_slots, uint32_t row_bytes, unsigned long long *__restrict__ used) {
    unsigned long long tpl = 0, port = 0, d0 = 0, d1 = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n_slots;
         g += (uint64_t)gridDim.x * blockDim.x) {
        if (!tag_live(tags[g])) continue;
        const uint8_t *R = rows + g * row_bytes;
        tpl |= *(const uint64_t *)(R + 56);
        port |= *(const uint64_t *)(R + 64);
        d0 |= *(const uint64_t *)(R + 72);
        d1 |= *(const uint64_t *)(R + 80);
    }
    if (tpl) atomicOr(&used[0], tpl);
    if (port) atomicOr(&used[1], port);
    if (d0) atomicOr(&used[2], d0);
    if (d1) atomicOr(&used[3], d1);
}

// rehash the live groups into an empty table (drops the tombstones)
__global__ void k_agg_rehash(const unsigned long long *__restrict__ tags, const uint8_t *__restrict__ rows,
                             uint64_t n_slots, uint32_t row_bytes, unsigned long long *__restrict__ ntags,
                             uint8_t *__restrict__ nrows, unsigned int *__restrict__ err) {
    const uint64_t mask = n_slots - 1;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n_slots;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long h = tags[g];
        if (!tag_live(h)) continue;
        uint64_t s = slot_of(h) & mask, probes = 0;
        while (atomicCAS(&ntags[s], TAG_EMPTY, h) != TAG_EMPTY) {  // every live group is distinct
            s = (s + 1) & mask;
            if (++probes > mask) { atomicOr(err, 2u); break; }
        }
        const uint32_t *src = (const uint32_t *)(rows + g * row_bytes);
        uint32_t *dst = (uint32_t *)(nrows + s * row_bytes);
        for (uint32_t i = 0; i < row_bytes / 4; ++i) dst[i] = src[i];
    }
}

// ---- byte values (BVAL) longer than 32 bytes: their tails in the byte arena ----
// Tail bytes a push can write at most: need[0] the tails of every present BVAL key and value of
// every valid record, need[1] the longest one (a group's claim writes one tail per key field, its
// ordered fold at most one per value field, so a push writes at most slots x fields x longest)
__global__ void k_agg_tail_need(const RecCtx C, const AggParams P, unsigned long long *__restrict__ need) {
    uint64_t mine = 0, longest = 0;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < C.n_rec; t += (uint64_t)gridDim.x * blockDim.x) {
        const Rec r = rec_of(C, t, nullptr);
        if (!r.valid) continue;
        const AggSlotPlan &sp = C.plans[r.slot];
        for (uint32_t k = 0; k < P.n_keys; ++k)
            if (P.key_kind[k] == KK_BYTES && sp.key_col[k]) {
                const Span s = key_span(sp, P, k, r.row);
                mine += tail_span(s.n);
                longest = max(longest, tail_span(s.n));
            }
        for (uint32_t v = 0; v < P.n_vals; ++v)
            if ((P.val_vc[v] == VC_VBYTES || P.val_vc[v] == VC_VLIST) && sp.val_col[v]) {
                const Span s = val_span(sp, v, r.row);
                mine += tail_span(s.n);
                longest = max(longest, tail_span(s.n));
            }
    }
    for (int m = 32; m >= 1; m >>= 1) {
        mine += (uint64_t)__shfl_xor((long long)mine, m);
        longest = max(longest, (uint64_t)__shfl_xor((long long)longest, m));
    }
    if ((threadIdx.x & 63) == 0 && mine) {
        atomicAdd(need, (unsigned long long)mine);
        atomicMax(need + 1, (unsigned long long)longest);
    }
}

// Moves the tails of one row's BVAL keys / values from arena `from` to `to` (bump cursor),
// rewriting the row's offsets
__device__ __forceinline__ void move_tails(uint8_t *R, const AggParams &P, const uint8_t *__restrict__ from,
                                           uint8_t *__restrict__ to, unsigned long long *__restrict__ cursor) {
    const uint32_t kp = *(const uint32_t *)(R + 8), vp = *(const uint32_t *)(R + 12);
    auto one = [&](uint8_t *slot) {
        uint32_t *d = (uint32_t *)slot;
        if (d[0] <= BVAL_INLINE) return;
        const uint64_t n = d[0] - BVAL_INLINE, src = (uint64_t)d[1] << 3;
        const uint64_t off = atomicAdd(cursor, (unsigned long long)tail_span(d[0]));
        for (uint64_t i = 0; i < n; ++i) to[off + i] = from[src + i];
        d[1] = (uint32_t)(off >> 3);
    };
    for (uint32_t k = 0; k < P.n_keys; ++k)
        if (P.key_kind[k] == KK_BYTES && ((kp >> k) & 1)) one(R + P.key_off[k]);
    for (uint32_t v = 0; v < P.n_vals; ++v)
        if ((P.val_vc[v] == VC_VBYTES || P.val_vc[v] == VC_VLIST) && ((vp >> v) & 1)) one(R + P.val_off[v]);
}

// output rows (k_agg_take) -> their tails gathered into one buffer the host copies out
__global__ void k_agg_out_tails(uint8_t *__restrict__ out_rows, uint64_t n, const AggParams P,
                                uint8_t *__restrict__ tails, unsigned long long *__restrict__ cursor) {
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (uint64_t)gridDim.x * blockDim.x)
        move_tails(out_rows + g * P.row_bytes, P, P.arena, tails, cursor);
}

// arena compaction: the live rows' tails into a fresh arena (emitted groups' tails dropped)
__global__ void k_agg_compact(const unsigned long long *__restrict__ tags, uint8_t *__restrict__ rows, uint64_t n_slots,
                              const AggParams P, uint8_t *__restrict__ to, unsigned long long *__restrict__ cursor) {
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n_slots; g += (uint64_t)gridDim.x * blockDim.x)
        if (tag_live(tags[g])) move_tails(rows + g * P.row_bytes, P, P.arena, to, cursor);
}

}  // namespace

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
struct ngz_agg {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    std::string last_error;
    bool poisoned = false;
    std::vector<ngz_agg_field> keys, vals;
    uint64_t window_ms = 0, lateness_ms = 0;
    uint64_t slots = 0;      // table slots (power of two)
    uint64_t limit = 0;      // groups held at most (the capacity asked for)
    uint64_t live = 0, tombs = 0;
    AggParams P{};
    // fixed at first sight: column width and decoded kind of every key / value
    std::vector<int> val_w, key_w, key_kind_seen, val_kind_seen;
    // dictionaries: entry = value, -1 = free (bits of groups refer to entry positions)
    std::vector<int64_t> templates, ports, domains;
    // the dictionaries as of the last flush / emit (the rows it returned refer to them)
    std::vector<int64_t> out_templates, out_ports, out_domains;
    // exporter peers: the IP keys groups and windows (aggregator.rs:119-124, aggregation.rs:96-108);
    // entry i is the rows' peer field.  Each peer has its own event time (seconds, 0 = none yet)
    uint32_t max_peers = NGZ_AGG_MAX_PEERS;
    std::vector<ngz_peer> peers, out_peers;
    std::vector<uint32_t> peer_time;
    std::map<std::string, uint32_t> peer_index;
    uint32_t push_id = 0;
    float t_push = 0;
    // device
    unsigned long long *tags = nullptr;
    uint8_t *rows = nullptr;
    uint32_t *ident = nullptr;
    unsigned long long *dom_dict = nullptr;
    unsigned long long *newdom = nullptr;
    unsigned int *err = nullptr;
    unsigned long long *late = nullptr;
    unsigned long long *cursor = nullptr;
    unsigned long long *n_claims = nullptr;
    unsigned int *n_coll = nullptr;
    unsigned long long *used = nullptr;
    // byte arena of BVAL tails (values longer than 32 bytes): bump-allocated by the kernels
    // (arena_used[0]); arena_used[1] is the push's tail-byte bound (k_agg_tail_need).  arena_mark:
    // the bytes in use after the last push (a failed push puts the counter back to it)
    uint8_t *arena = nullptr;
    uint64_t arena_cap = 0, arena_mark = 0;
    unsigned long long *arena_used = nullptr;
    std::vector<uint8_t> out_tails;  // tails of the rows last returned by flush / emit
    uint32_t take_id = 0;            // flush / emit calls so far: the last one's rows carry it (ngz_agg_row.take_id)
    int64_t *cut = nullptr;         // per-peer window cutoffs of ngz_agg_closed / ngz_agg_emit
    uint32_t cut_cap = 0;
    uint32_t *rank_maps = nullptr;  // one 65536-bit map per VC_RANK sub-registry value
    AggSlotPlan *plans = nullptr;
    uint32_t plans_cap = 0;
    // scratch, grown on demand
    void *scratch = nullptr;
    size_t scratch_cap = 0;
    uint8_t *rec_buf = nullptr;  // record contexts, rec_g, claims, collided lists, sort buffers
    size_t rec_cap = 0;
    uint8_t *part_buf = nullptr;  // partitioned reduction: counts, offsets, scan scratch, payloads
    size_t part_cap = 0;
    LcEntry *lc = nullptr;        // low-cardinality path: the waves' partial groups
    uint32_t lc_cap = 0;          // ... entries allocated
    unsigned int *lc_cnt = nullptr;  // [0] entries written, [1] overflow flag, [2] merge workgroups done
    LcSet *lc_sets = nullptr;     // ... the push's set descriptors
    uint32_t lc_sets_cap = 0;
    const char *last_path = "";   // the reduction path of the last push ("lowcard" / "general")
    int opt_lowcard = -1;         // NGZ_AGG_OPT_LOWCARD: -1 by size, 0 never, 1 at any size
    int opt_partition = -1;       // NGZ_AGG_OPT_PARTITION: -1 by groups and records, 0 never, 1 always
    bool opt_owner = true;        // NGZ_AGG_OPT_OWNER
    uint32_t lc_skip = 0;         // pushes left before the low-cardinality scan is tried again
};

namespace {

int fail(ngz_agg *a, int rc, const std::string &msg) {
    if (a) a->last_error = msg;
    return rc;
}

#define AGG_HIP(a, x)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            (a)->poisoned = true;                                                         \
            return fail(a, NGZ_E_DEVICE, std::string(#x ": ") + hipGetErrorString(e_));   \
        }                                                                                 \
    } while (0)

uint32_t grid_for(uint64_t n, uint32_t block = 256, uint32_t max_blocks = 8192) {
    uint64_t g = (n + block - 1) / block;
    if (g == 0) g = 1;
    return (uint32_t)std::min<uint64_t>(g, max_blocks);
}

int reset_rows(ngz_agg *a, unsigned long long *tags, uint8_t *rows) {
    AGG_HIP(a, hipMemsetAsync(tags, 0, a->slots * 8, a->stream));
    hipLaunchKernelGGL(k_agg_init, dim3(8192), dim3(256), 0, a->stream, rows, a->slots, a->P.row_bytes, a->ident,
                       a->P.row_bytes / 4);
    AGG_HIP(a, hipGetLastError());
    return NGZ_OK;
}

// Value class of (IE, op), following IE::supports_{arithmetic,comparison,bitwise}_ops
// (generator.rs:1176-1272) for acceptance and the generated Field ops (generator.rs:580-629,
// 896-1080) for the arithmetic.  Returns the value class or -1 (rejected by the reference's
// validate_operation_compatibility, config.rs:212-250).
int value_class(const ngzh::IeRow *r, uint8_t op, std::string &why) {
    using namespace ngzh;
    const uint8_t dt = r ? r->dtype : DT_octetArray;  // IE::Unknown: octetArray
    const bool subreg = r && (r->flags & 4);
    const bool tcp = r && (r->flags & 2);
    const bool ident_or_flags = r && (r->flags & (8 | 16));
    const bool integer = dt == DT_unsigned8 || dt == DT_unsigned16 || dt == DT_unsigned32 || dt == DT_unsigned64 ||
                         dt == DT_signed8 || dt == DT_signed16 || dt == DT_signed32 || dt == DT_signed64;
    const bool sgn = dt == DT_signed8 || dt == DT_signed16 || dt == DT_signed32 || dt == DT_signed64;
    const bool flt = dt == DT_float32 || dt == DT_float64;
    switch (op) {
    case NGZ_AGG_ADD:
        if (ident_or_flags || subreg || !(integer || flt)) { why = "field does not support arithmetic operations"; return -1; }
        if (flt) return dt == DT_float32 ? VC_F32 : VC_F64;
        return sgn ? VC_SINT : VC_UINT;
    case NGZ_AGG_MIN:
    case NGZ_AGG_MAX:
        if (!(integer || flt || dt == DT_dateTimeSeconds || dt == DT_dateTimeMilliseconds ||
              dt == DT_dateTimeMicroseconds || dt == DT_dateTimeNanoseconds || dt == DT_ipv4Address ||
              dt == DT_ipv6Address || dt == DT_basicList || dt == DT_subTemplateList || dt == DT_subTemplateMultiList)) {
            why = "field does not support comparison operations";
            return -1;
        }
        if (dt == DT_basicList || dt == DT_subTemplateList || dt == DT_subTemplateMultiList) return VC_VLIST;
        if (flt) return dt == DT_float32 ? VC_F32 : VC_F64;
        if (dt == DT_ipv6Address) return VC_IPV6;
        if (tcp || subreg) return VC_RANK;  // nested sub-registries (forwardingStatus) get a rank table
        if (integer || dt == DT_ipv4Address || dt == DT_dateTimeSeconds) return sgn ? VC_SINT : VC_UINT;
        if (dt == DT_dateTimeMilliseconds) return VC_SINT;
        return VC_DTFRAC;
    case NGZ_AGG_OR:
        if (flt || dt == DT_string || dt == DT_basicList || dt == DT_subTemplateList || dt == DT_subTemplateMultiList ||
            dt == DT_dateTimeSeconds || dt == DT_dateTimeMilliseconds || dt == DT_dateTimeMicroseconds ||
            dt == DT_dateTimeNanoseconds) {
            why = "field does not support bitwise operations";
            return -1;
        }
        // sub-registry enums OR their raw values (generator_sub_registries.rs: BitOrAssign)
        if (integer || dt == DT_boolean || dt == DT_ipv4Address) return VC_UINT;
        // octetArray as Box<[u8]> (any length, IE::Unknown included); the MPLS label stacks are [u8; 3]
        if (dt == DT_octetArray && !(r && (r->flags & 1))) return VC_VBYTES;
        return VC_BYTES;  // macAddress, ipv6Address, unsigned256, MPLS label
    }
    why = "unknown op";
    return -1;
}

uint32_t value_slot_bytes(int vc) {
    return vc == VC_VBYTES || vc == VC_VLIST ? BVAL_BYTES : vc == VC_BYTES ? 32 : vc == VC_IPV6 ? 16 : 8;
}

// dictionary entry for value x (reusing a free position), or -1 when all SET_BITS / cap are used
int dict_put(std::vector<int64_t> &d, int64_t x, uint32_t cap) {
    for (size_t i = 0; i < d.size(); ++i)
        if (d[i] == x) return (int)i;
    for (size_t i = 0; i < d.size(); ++i)
        if (d[i] < 0) { d[i] = x; return (int)i; }
    if (d.size() >= cap) return -1;
    d.push_back(x);
    return (int)d.size() - 1;
}

// Frees the dictionary entries no live group refers to any more (set bits of the live rows).
int dict_gc(ngz_agg *a) {
    AGG_HIP(a, hipMemsetAsync(a->used, 0, 32, a->stream));
    hipLaunchKernelGGL(k_agg_bits, dim3(grid_for(a->slots, 256, 2048)), dim3(256), 0, a->stream, a->tags, a->rows,
                       a->slots, a->P.row_bytes, a->used);
    unsigned long long used[4];
    AGG_HIP(a, hipMemcpyAsync(used, a->used, 32, hipMemcpyDeviceToHost, a->stream));
    AGG_HIP(a, hipStreamSynchronize(a->stream));
    for (size_t i = 0; i < a->templates.size(); ++i)
        if (!(used[0] >> i & 1)) a->templates[i] = -1;
    for (size_t i = 0; i < a->ports.size(); ++i)
        if (!(used[1] >> i & 1)) a->ports[i] = -1;
    for (size_t i = 0; i < a->domains.size(); ++i)
        if (!((i < 64 ? used[2] >> i : used[3] >> (i - 64)) & 1)) a->domains[i] = -1;
    return NGZ_OK;
}

int upload_domains(ngz_agg *a) {
    unsigned long long tab[DOM_SLOTS] = {};
    for (size_t i = 0; i < a->domains.size() && i < DOM_SLOTS; ++i)
        if (a->domains[i] >= 0) tab[i] = (1ull << 32) | (uint64_t)a->domains[i];
    AGG_HIP(a, hipMemcpyAsync(a->dom_dict, tab, sizeof tab, hipMemcpyHostToDevice, a->stream));
    return NGZ_OK;
}

// rebuild the table without its tombstones (same size)
int rehash(ngz_agg *a) {
    unsigned long long *ntags = nullptr;
    uint8_t *nrows = nullptr;
    if (hipMalloc(&ntags, a->slots * 8) != hipSuccess || hipMalloc(&nrows, a->slots * a->P.row_bytes) != hipSuccess) {
        hipFree(ntags);
        hipFree(nrows);
        return NGZ_OK;  // keep the tombstones (correct, only slower probes); retried at the next emit
    }
    int rc = reset_rows(a, ntags, nrows);
    if (rc) { hipFree(ntags); hipFree(nrows); return rc; }
    AGG_HIP(a, hipMemsetAsync(a->err, 0, 4, a->stream));
    hipLaunchKernelGGL(k_agg_rehash, dim3(grid_for(a->slots)), dim3(256), 0, a->stream, a->tags, a->rows, a->slots,
                       a->P.row_bytes, ntags, nrows, a->err);
    unsigned int e = 0;
    AGG_HIP(a, hipMemcpyAsync(&e, a->err, 4, hipMemcpyDeviceToHost, a->stream));
    AGG_HIP(a, hipStreamSynchronize(a->stream));
    if (e) {
        hipFree(ntags);
        hipFree(nrows);
        a->poisoned = true;
        return fail(a, NGZ_E_DEVICE, "rehash lost groups");
    }
    hipFree(a->tags);
    hipFree(a->rows);
    a->tags = ntags;
    a->rows = nrows;
    a->tombs = 0;
    if (a->arena_mark) {
        // the emitted groups' tails are garbage: move the live ones into a fresh arena
        uint8_t *to = nullptr;
        if (hipMalloc(&to, a->arena_cap) != hipSuccess) return NGZ_OK;  // keep the garbage (retried next time)
        unsigned long long used = 0;
        AGG_HIP(a, hipMemsetAsync(a->arena_used + 1, 0, 8, a->stream));
        hipLaunchKernelGGL(k_agg_compact, dim3(grid_for(a->slots)), dim3(256), 0, a->stream, a->tags, a->rows, a->slots,
                           a->P, to, a->arena_used + 1);
        AGG_HIP(a, hipMemcpyAsync(&used, a->arena_used + 1, 8, hipMemcpyDeviceToHost, a->stream));
        AGG_HIP(a, hipMemcpyAsync(a->arena_used, a->arena_used + 1, 8, hipMemcpyDeviceToDevice, a->stream));
        AGG_HIP(a, hipStreamSynchronize(a->stream));
        hipFree(a->arena);
        a->arena = a->P.arena = to;
        a->arena_mark = used;
    }
    return NGZ_OK;
}

// Byte arena: room for `need` more bytes after the ones in use (grown to at least twice its size,
// the bytes in use moved over)
int arena_reserve(ngz_agg *a, uint64_t need) {
    // row offsets are u32 counts of 8-byte units (tail_span): the arena ends at 32 GiB
    if (a->arena_mark + need > ARENA_MAX)
        return fail(a, NGZ_E_LIMIT, "byte arena: the push could need more than 32 GiB of value tails");
    if (a->arena_mark + need <= a->arena_cap) return NGZ_OK;
    const uint64_t cap = std::min<uint64_t>(ARENA_MAX, std::max<uint64_t>({a->arena_mark + need, 2 * a->arena_cap, 1u << 20}));
    uint8_t *p = nullptr;
    if (hipMalloc(&p, cap) != hipSuccess) return fail(a, NGZ_E_NOMEM, "byte arena");
    if (a->arena_mark) AGG_HIP(a, hipMemcpyAsync(p, a->arena, a->arena_mark, hipMemcpyDeviceToDevice, a->stream));
    AGG_HIP(a, hipStreamSynchronize(a->stream));
    hipFree(a->arena);
    a->arena = p;
    a->arena_cap = cap;
    a->P.arena = p;
    a->P.arena_cap = cap;
    return NGZ_OK;
}

// every group gone (flush / reset): the arena starts over
int arena_clear(ngz_agg *a) {
    a->arena_mark = 0;
    AGG_HIP(a, hipMemsetAsync(a->arena_used, 0, 8, a->stream));
    return NGZ_OK;
}

// host finish of output rows: collection times back to signed, per-push marker cleared,
// values at the IE width, ranks back to values
void finish_rows(ngz_agg *a, uint8_t *dst, int64_t n) {
    const uint32_t RB = a->P.row_bytes;
    for (int64_t g = 0; g < n; ++g) {
        uint8_t *R = dst + (uint64_t)g * RB;
        uint64_t c;
        memcpy(&c, R + 40, 8); c ^= 1ull << 63; memcpy(R + 40, &c, 8);
        memcpy(&c, R + 48, 8); c ^= 1ull << 63; memcpy(R + 48, &c, 8);
        memcpy(R + 36, &a->take_id, 4);  // ngz_agg_row.take_id (the device's per-push marker there is done)
        uint32_t vp;
        memcpy(&vp, R + 12, 4);
        for (uint32_t v = 0; v < a->P.n_vals; ++v) {
            const int vc = a->P.val_vc[v];
            uint8_t *p = R + a->P.val_off[v];
            if (!(vp >> v & 1)) { memset(p, 0, value_slot_bytes(vc)); continue; }
            if (vc == VC_BYTES || vc == VC_IPV6 || vc == VC_F32 || vc == VC_F64 || vc == VC_VBYTES || vc == VC_VLIST)
                continue;
            uint64_t x;
            memcpy(&x, p, 8);
            const uint8_t op = a->P.val_op[v];
            if (vc == VC_SINT && (op == NGZ_AGG_MIN || op == NGZ_AGG_MAX)) x ^= 1ull << 63;
            if (vc == VC_RANK) x = a->P.val_tcp[v] ? bitrev8((uint32_t)x & 0xFF) : (x & 0xFFFFFFFFull);
            const int w = a->val_w[v];
            if (vc != VC_DTFRAC && w > 0 && w < 8) {  // wrap at the Rust width (release-mode +=), then extend
                const uint32_t sh = 64 - 8 * w;
                x = vc == VC_SINT ? (uint64_t)(((int64_t)(x << sh)) >> sh) : (x << sh) >> sh;
            }
            memcpy(p, &x, 8);
        }
    }
}

// groups selected by per-peer cutoffs (device array; nullptr: every group) -> dst (host);
// tomb: free their slots
int64_t take_rows(ngz_agg *a, void *dst, uint64_t cap, const int64_t *cut, bool tomb) {
    AGG_HIP(a, hipSetDevice(a->device));
    unsigned long long n = 0;
    AGG_HIP(a, hipMemsetAsync(a->cursor, 0, 8, a->stream));
    hipLaunchKernelGGL(k_agg_count, dim3(grid_for(a->slots)), dim3(256), 0, a->stream, a->tags, a->rows, a->slots,
                       a->P.row_bytes, cut, a->cursor);
    AGG_HIP(a, hipMemcpyAsync(&n, a->cursor, 8, hipMemcpyDeviceToHost, a->stream));
    AGG_HIP(a, hipStreamSynchronize(a->stream));
    const uint32_t RB = a->P.row_bytes;
    if ((uint64_t)n * RB > cap || (n && !dst)) return fail(a, NGZ_E_INVALID, "output buffer too small");
    if (++a->take_id == 0) a->take_id = 1;  // earlier rows' byte values are gone from here on
    a->out_tails.clear();
    if (n) {
        uint8_t *tmp = nullptr;
        if (hipMalloc(&tmp, (uint64_t)n * RB) != hipSuccess) return fail(a, NGZ_E_NOMEM, "output staging");
        AGG_HIP(a, hipMemsetAsync(a->cursor, 0, 8, a->stream));
        hipLaunchKernelGGL(k_agg_take, dim3(grid_for(a->slots)), dim3(256), 0, a->stream, a->tags, a->rows, a->slots, RB,
                           cut, tomb ? 1 : 0, tmp, a->cursor);
        // byte values longer than 32 bytes: their tails gathered for the host (ngz_agg_row_bytes),
        // the rows' offsets rewritten to point there
        uint8_t *tails = nullptr;
        unsigned long long nt = 0;
        hipError_t e = hipSuccess;
        a->out_tails.clear();
        if (a->arena_mark) {
            e = hipMalloc(&tails, a->arena_mark);
            if (e == hipSuccess) e = hipMemsetAsync(a->arena_used + 1, 0, 8, a->stream);
            if (e == hipSuccess) {
                hipLaunchKernelGGL(k_agg_out_tails, dim3(grid_for(n)), dim3(256), 0, a->stream, tmp, (uint64_t)n, a->P,
                                   tails, a->arena_used + 1);
                e = hipMemcpyAsync(&nt, a->arena_used + 1, 8, hipMemcpyDeviceToHost, a->stream);
            }
            if (e == hipSuccess) e = hipStreamSynchronize(a->stream);
            if (e == hipSuccess && nt) {
                a->out_tails.resize(nt);
                e = hipMemcpyAsync(a->out_tails.data(), tails, nt, hipMemcpyDeviceToHost, a->stream);
            }
        }
        if (e == hipSuccess) e = hipMemcpyAsync(dst, tmp, (uint64_t)n * RB, hipMemcpyDeviceToHost, a->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(a->stream);
        hipFree(tmp);
        hipFree(tails);
        if (e != hipSuccess) { a->poisoned = true; return fail(a, NGZ_E_DEVICE, hipGetErrorString(e)); }
        finish_rows(a, (uint8_t *)dst, (int64_t)n);
    }
    a->out_templates = a->templates;
    a->out_ports = a->ports;
    a->out_domains = a->domains;
    a->out_peers = a->peers;
    return (int64_t)n;
}

int64_t floordiv64(int64_t x, int64_t d) { return x / d - ((x % d != 0) && ((x < 0) != (d < 0))); }

// Windows a peer's event time has closed (aggregation.rs:154-160): starts <= cutoff =
// get_window_start(current_time - lateness) - window_duration, in seconds (floored).
int64_t cutoff_s(const ngz_agg *a, uint32_t peer) {
    const uint32_t ct = a->peer_time[peer];
    if (!ct) return INT64_MIN;
    const int64_t t = (int64_t)ct * 1000 - (int64_t)a->lateness_ms;
    const int64_t cut_ms = floordiv64(t, 60000) * 60000 - (int64_t)a->window_ms;
    return floordiv64(cut_ms, 1000);
}

// every peer's cutoff into the device array a->cut; false: no peer has an event time
int upload_cutoffs(ngz_agg *a, bool *any) {
    *any = false;
    const uint32_t n = (uint32_t)a->peers.size();
    std::vector<int64_t> c(std::max<uint32_t>(n, 1), INT64_MIN);
    for (uint32_t i = 0; i < n; ++i) {
        c[i] = cutoff_s(a, i);
        *any = *any || c[i] != INT64_MIN;
    }
    if (!*any) return NGZ_OK;
    if (n > a->cut_cap) {
        hipFree(a->cut);
        a->cut = nullptr;
        a->cut_cap = 0;
        const uint32_t want = std::max<uint32_t>(n, 64);
        if (hipMalloc(&a->cut, 8ull * want) != hipSuccess) return fail(a, NGZ_E_NOMEM, "cutoff table");
        a->cut_cap = want;
    }
    AGG_HIP(a, hipMemcpyAsync(a->cut, c.data(), 8ull * n, hipMemcpyHostToDevice, a->stream));
    return NGZ_OK;
}

void forget_peers(ngz_agg *a) {
    a->peers.clear();
    a->peer_time.clear();
    a->peer_index.clear();
}

std::string peer_key(const ngz_peer &p) {
    return std::string(1, (char)p.family) + std::string((const char *)p.addr, p.family == 4 ? 4 : 16);
}

}  // namespace

extern "C" {

int ngz_agg_abi_version(void) { return NGZ_AGG_ABI_VERSION; }

int ngz_agg_create(int device, const ngz_agg_field *fields, uint32_t n_fields, uint64_t window_ms,
                   uint64_t lateness_ms, uint64_t capacity, uint32_t max_peers, ngz_agg **out) {
    if (!out || (n_fields && !fields)) return NGZ_E_INVALID;
    *out = nullptr;
    if (window_ms == 0 || lateness_ms > window_ms) return NGZ_E_INVALID;  // AggregationConfig::validate
    if (max_peers > NGZ_AGG_MAX_PEERS) return NGZ_E_LIMIT;
    ngz_agg *a = new ngz_agg();
    a->device = device;
    a->max_peers = max_peers ? max_peers : NGZ_AGG_MAX_PEERS;
    a->window_ms = window_ms;
    a->lateness_ms = lateness_ms;
    std::vector<int> vcs;
    for (uint32_t i = 0; i < n_fields; ++i) {
        const ngz_agg_field &f = fields[i];
        if (f.op > NGZ_AGG_OR) { delete a; return NGZ_E_INVALID; }
        if (f.op == NGZ_AGG_KEY) { a->keys.push_back(f); continue; }
        std::string why;
        const int vc = value_class(ngzh::ie_find(f.pen, f.ie_id), f.op, why);
        if (vc == -1) { delete a; return NGZ_E_INVALID; }
        a->vals.push_back(f);
        vcs.push_back(vc);
    }
    if (a->keys.size() > NGZ_AGG_MAX_KEYS || a->vals.size() > NGZ_AGG_MAX_VALUES) { delete a; return NGZ_E_LIMIT; }
    a->key_w.assign(a->keys.size(), -1);
    a->key_kind_seen.assign(a->keys.size(), -1);
    a->val_w.assign(a->vals.size(), -1);
    a->val_kind_seen.assign(a->vals.size(), -1);
    // row layout: header, keys (canonical bytes, slot a multiple of 4), values (8 B; IPv6 16 B;
    // byte ORs up to 32 B)
    uint32_t off = KEY0;
    AggParams &P = a->P;
    P.n_keys = (uint32_t)a->keys.size();
    P.n_vals = (uint32_t)a->vals.size();
    for (uint32_t k = 0; k < P.n_keys; ++k) {
        const ngzh::IeRow *r = ngzh::ie_find(a->keys[k].pen, a->keys[k].ie_id);
        uint32_t slot = BVAL_BYTES;
        uint8_t kind = KK_BYTES;  // IE::Unknown / vendor Unknown: raw bytes
        int fw = 0;  // packed-key eligibility: IEs whose column width is fixed by the Rust type (1/2/4/8 bytes)
        if (r) {
            kind = KK_FIXED;
            switch (r->dtype) {
            case ngzh::DT_unsigned8: case ngzh::DT_signed8: case ngzh::DT_boolean: slot = 4; fw = 1; break;
            case ngzh::DT_unsigned16: slot = 4; fw = (r->flags & 2) ? 1 : 2; break;  // tcpControlBits column is u8
            case ngzh::DT_signed16: slot = 4; fw = 2; break;
            case ngzh::DT_unsigned32: case ngzh::DT_signed32: case ngzh::DT_float32: case ngzh::DT_ipv4Address:
            case ngzh::DT_dateTimeSeconds: slot = 4; fw = 4; break;
            case ngzh::DT_unsigned64: case ngzh::DT_signed64: case ngzh::DT_float64:
            case ngzh::DT_dateTimeMilliseconds: case ngzh::DT_dateTimeMicroseconds:
            case ngzh::DT_dateTimeNanoseconds: slot = 8; break;
            case ngzh::DT_macAddress: slot = 8; break;
            case ngzh::DT_ipv6Address: slot = 16; break;
            case ngzh::DT_unsigned256: slot = 32; break;
            case ngzh::DT_string: slot = BVAL_BYTES; kind = KK_BYTES; P.key_str |= 1u << k; break;
            default: slot = BVAL_BYTES; kind = KK_BYTES; break;  // octetArray, lists: Box<[u8]>
            }
            if ((r->flags & 1) && r->dtype == ngzh::DT_octetArray) { slot = 4; kind = KK_FIXED; }  // [u8; 3]
        }
        if (kind == KK_BYTES) P.has_bytes = 1;
        P.key_off[k] = off;
        P.key_slot[k] = slot;
        P.key_kind[k] = kind;
        P.key_pw[k] = (uint32_t)fw;
        off += slot;
    }
    if (off - KEY0 > NGZ_AGG_MAX_KEY_BYTES + 64) { delete a; return NGZ_E_LIMIT; }
    off = (off + 7) & ~7u;
    bool ranks = false;
    for (uint32_t v = 0; v < P.n_vals; ++v) {
        const ngzh::IeRow *r = ngzh::ie_find(a->vals[v].pen, a->vals[v].ie_id);
        P.val_off[v] = off;
        P.val_op[v] = a->vals[v].op;
        P.val_vc[v] = (uint8_t)vcs[v];
        P.val_tcp[v] = vcs[v] == VC_RANK && r && (r->flags & 2);
        ranks = ranks || (vcs[v] == VC_RANK && !P.val_tcp[v]);
        if (vcs[v] == VC_VBYTES || vcs[v] == VC_VLIST) P.has_bytes = 1;
        off += value_slot_bytes(vcs[v]);
    }
    // whole 128-byte lines: a row at a random slot then touches ceil(row/128) lines, not one
    // more when it straddles (176-byte rows at a 176-byte stride cover 2.4 lines on average);
    // NGZ_AGG_ROW_PACK keeps whole 16-byte pieces only (k_agg_apply_own's unit)
    P.row_bytes = ngz_knob("NGZ_AGG_ROW_PACK", 0) ? (off + 15) & ~15u : (off + 127) & ~127u;
    P.peer_bits = 0;
    while ((1u << P.peer_bits) < a->max_peers) ++P.peer_bits;
    {
        uint32_t bits = 28 + P.peer_bits;  // window/60 + flow type + peer entry
        bool ok = true;
        for (uint32_t k = 0; k < P.n_keys; ++k) {
            ok = ok && P.key_pw[k] != 0;
            bits += 1 + 8 * P.key_pw[k];
        }
        P.packed = ok && bits <= 63 && !ngz_knob("NGZ_AGG_NO_PACK", 0);
    }
    P.lds_ok = 1;
    for (uint32_t v = 0; v < P.n_vals; ++v)
        if (P.val_vc[v] == VC_BYTES) P.lds_ok = 0;
    // hashed keys of at most 8 words: key words in registers (KeyVal)
    {
        uint32_t nw = 0;
        for (uint32_t k = 0; k < P.n_keys; ++k) nw += P.key_slot[k] / 4;
        P.kw_n = 0;
        if (!P.packed && nw <= 8 && !ngz_knob("NGZ_AGG_NO_KW", 0)) {
            uint32_t j = 0;
            for (uint32_t k = 0; k < P.n_keys; ++k)
                for (uint32_t i = 0; i < P.key_slot[k] / 4; ++i, ++j) {
                    P.kw_key[j] = (uint8_t)k;
                    P.kw_idx[j] = (uint8_t)i;
                }
            P.kw_n = nw;
        }
    }
    // owner path: rows of up to 256 bytes, no byte-wise ORs, aggregated fields 0-7
    P.own = P.lds_ok && P.row_bytes <= 256 && P.n_vals <= 8;  // NGZ_AGG_OPT_OWNER 0 turns it off per push
    {
        uint8_t op[32] = {}, src[32] = {};
        op[1] = U_VP;                                   // val_present (high word of key_present's unit)
        op[2] = U_ADD, src[2] = U_SRC_ONE;              // record_count
        op[3] = U_TS;                                   // min / max export time
        op[4] = U_SYS;                                  // max sys-up time, push marker
        op[5] = U_MIN, src[5] = U_SRC_COLL;             // min / max collection time (flipped)
        op[6] = U_MAX, src[6] = U_SRC_COLL;
        op[7] = U_OR, src[7] = U_SRC_TPL;               // template, peer port, domain sets
        op[8] = U_OR, src[8] = U_SRC_PORT;
        op[9] = U_OR, src[9] = U_SRC_DOM0;
        op[10] = U_OR, src[10] = U_SRC_DOM1;
        for (uint32_t v = 0; v < P.n_vals && v < 8; ++v) {
            if (vc_ordered(P.val_vc[v])) continue;      // k_agg_ordered
            const uint32_t u = P.val_off[v] / 8;
            op[u] = P.val_op[v] == NGZ_AGG_ADD ? U_ADD : P.val_op[v] == NGZ_AGG_MIN ? U_MIN
                  : P.val_op[v] == NGZ_AGG_MAX ? U_MAX : U_OR;
            src[u] = (uint8_t)v;
        }
        P.unit_op[0] = P.unit_op[1] = P.unit_src[0] = P.unit_src[1] = 0;
        for (uint32_t u = 0; u < 32; ++u) {
            P.unit_op[u >> 4] |= (uint64_t)op[u] << (4 * (u & 15));
            P.unit_src[u >> 4] |= (uint64_t)src[u] << (4 * (u & 15));
        }
    }
    P.hash_mask = ~0ull;
    if (capacity > (1ull << 30)) { delete a; return NGZ_E_LIMIT; }  // slot indexes stay below OWN_BIT
    uint64_t slots = 1024;
    while (slots < 2 * std::max<uint64_t>(capacity, 1)) slots <<= 1;
    a->slots = slots;
    a->limit = std::max<uint64_t>(capacity, 1);
    P.mask = slots - 1;
    // identity row: min fields at their maximum
    std::vector<uint32_t> ident(P.row_bytes / 4, 0);
    ident[24 / 4] = 0xFFFFFFFFu;                      // min_export_time
    ident[40 / 4] = ident[44 / 4] = 0xFFFFFFFFu;      // min_collection (flipped order)
    for (uint32_t v = 0; v < P.n_vals; ++v)
        if (P.val_op[v] == NGZ_AGG_MIN && !vc_ordered(P.val_vc[v]))
            ident[P.val_off[v] / 4] = ident[P.val_off[v] / 4 + 1] = 0xFFFFFFFFu;
    auto bail = [&](int r, const char *what) {
        a->last_error = what;
        ngz_agg_destroy(a);
        return r;
    };
    if (hipSetDevice(device) != hipSuccess) return bail(NGZ_E_DEVICE, "hipSetDevice");
    if (hipStreamCreateWithFlags(&a->stream, hipStreamNonBlocking) != hipSuccess) return bail(NGZ_E_DEVICE, "stream");
    hipEventCreate(&a->ev0);
    hipEventCreate(&a->ev1);
    if (hipMalloc(&a->tags, slots * 8) != hipSuccess || hipMalloc(&a->rows, slots * P.row_bytes) != hipSuccess ||
        hipMalloc(&a->ident, P.row_bytes) != hipSuccess || hipMalloc(&a->dom_dict, DOM_SLOTS * 8) != hipSuccess ||
        hipMalloc(&a->newdom, NEWDOM_SLOTS * 8) != hipSuccess || hipMalloc(&a->err, 4) != hipSuccess ||
        hipMalloc(&a->late, 8) != hipSuccess || hipMalloc(&a->cursor, 8) != hipSuccess ||
        hipMalloc(&a->n_claims, 8) != hipSuccess || hipMalloc(&a->n_coll, 4) != hipSuccess ||
        hipMalloc(&a->used, 32) != hipSuccess || hipMalloc(&a->arena_used, 24) != hipSuccess)
        return bail(NGZ_E_NOMEM, "hipMalloc (group table)");
    hipMemset(a->arena_used, 0, 24);
    P.arena_used = a->arena_used;
    if (ranks) {
        // sub-registry ranks: which values are registered variants (known bitmap per value)
        if (hipMalloc(&a->rank_maps, (size_t)P.n_vals * 8192) != hipSuccess) return bail(NGZ_E_NOMEM, "hipMalloc (ranks)");
        std::vector<uint32_t> map(2048);
        for (uint32_t v = 0; v < P.n_vals; ++v) {
            if (P.val_vc[v] != VC_RANK || P.val_tcp[v]) continue;
            uint64_t nested[257];
            if (ngzh::subreg_nested_ranks(a->vals[v].pen, a->vals[v].ie_id, nested)) {
                // the 8 KB map slot holds the 257 ranks of a nested sub-registry instead
                unsigned long long *dst = (unsigned long long *)(a->rank_maps + (size_t)v * 2048);
                hipMemcpy(dst, nested, sizeof nested, hipMemcpyHostToDevice);
                P.rank_nested[v] = dst;
                continue;
            }
            std::fill(map.begin(), map.end(), 0u);
            for (uint32_t x = 0; x < 65536; ++x)
                if (ngzh::subreg_known(a->vals[v].pen, a->vals[v].ie_id, x)) map[x >> 5] |= 1u << (x & 31);
            uint32_t *dst = a->rank_maps + (size_t)v * 2048;
            hipMemcpy(dst, map.data(), 8192, hipMemcpyHostToDevice);
            P.rank_known[v] = dst;
        }
    }
    hipMemcpy(a->ident, ident.data(), P.row_bytes, hipMemcpyHostToDevice);
    hipMemset(a->dom_dict, 0, DOM_SLOTS * 8);
    hipMemset(a->err, 0, 4);
    int rc = reset_rows(a, a->tags, a->rows);
    if (rc == NGZ_OK && hipStreamSynchronize(a->stream) != hipSuccess) rc = NGZ_E_DEVICE;
    if (rc != NGZ_OK) return bail(rc, "table init");
    *out = a;
    return NGZ_OK;
}

void ngz_agg_destroy(ngz_agg *a) {
    if (!a) return;
    if (a->stream) hipStreamSynchronize(a->stream);
    hipFree(a->tags);
    hipFree(a->rows);
    hipFree(a->ident);
    hipFree(a->dom_dict);
    hipFree(a->newdom);
    hipFree(a->err);
    hipFree(a->late);
    hipFree(a->cursor);
    hipFree(a->n_claims);
    hipFree(a->n_coll);
    hipFree(a->used);
    hipFree(a->arena);
    hipFree(a->arena_used);
    hipFree(a->cut);
    hipFree(a->rank_maps);
    hipFree(a->plans);
    hipFree(a->scratch);
    hipFree(a->rec_buf);
    hipFree(a->part_buf);
    hipFree(a->lc);
    hipFree(a->lc_cnt);
    hipFree(a->lc_sets);
    if (a->ev0) hipEventDestroy(a->ev0);
    if (a->ev1) hipEventDestroy(a->ev1);
    if (a->stream) hipStreamDestroy(a->stream);
    delete a;
}

const char *ngz_agg_last_error(ngz_agg *a) { return a ? a->last_error.c_str() : "null aggregator"; }

int ngz_agg_layout(ngz_agg *a, uint32_t *row_bytes, uint32_t *key_off, uint16_t *key_width, uint32_t *val_off,
                   uint16_t *val_width) {
    if (!a) return NGZ_E_INVALID;
    if (row_bytes) *row_bytes = a->P.row_bytes;
    for (uint32_t k = 0; k < a->P.n_keys; ++k) {
        if (key_off) key_off[k] = a->P.key_off[k];
        if (key_width) key_width[k] = (uint16_t)std::max(a->key_w[k], 0);
    }
    for (uint32_t v = 0; v < a->P.n_vals; ++v) {
        if (val_off) val_off[v] = a->P.val_off[v];
        if (val_width) {
            const int vc = a->P.val_vc[v];
            val_width[v] = (uint16_t)(vc == VC_IPV6 ? 16 : std::max(a->val_w[v], 0));
        }
    }
    return NGZ_OK;
}

int ngz_agg_push(ngz_agg *a, ngz_ctx *ctx, const ngz_batch_out *out, const ngz_peer *peer,
                 int64_t collection_time_ms, uint64_t *late_records, void *hip_stream) {
    if (!a || !ctx || !out || !peer || (peer->family != 4 && peer->family != 6)) return NGZ_E_INVALID;
    if (late_records) *late_records = 0;
    a->last_path = "none";  // no record to reduce (set below otherwise)
    if (a->poisoned) return fail(a, NGZ_AGG_E_POISONED, "aggregator failed earlier: ngz_agg_reset it");
    AGG_HIP(a, hipSetDevice(a->device));
    if (hip_stream) AGG_HIP(a, hipStreamSynchronize((hipStream_t)hip_stream));
    const uint16_t peer_port = peer->port;
    // the peer IP's entry (a new IP gets the next one; taken back if the push fails)
    const std::string pk = peer_key(*peer);
    bool new_peer = false;
    uint32_t pi;
    {
        auto it = a->peer_index.find(pk);
        if (it != a->peer_index.end()) {
            pi = it->second;
        } else {
            if (a->peers.size() >= a->max_peers)
                return fail(a, NGZ_AGG_E_OVERFLOW,
                            ("a new peer IP beyond max_peers (" + std::to_string(a->max_peers) +
                             " distinct peer IPs since the last flush; entries are kept until ngz_agg_flush / "
                             "ngz_agg_reset, as each peer's event time is)"));
            pi = (uint32_t)a->peers.size();
            ngz_peer p = *peer;
            if (p.family == 4) memset(p.addr + 4, 0, 12);
            p.reserved = 0;
            a->peers.push_back(p);
            a->peer_time.push_back(0);
            a->peer_index.emplace(pk, pi);
            new_peer = true;
        }
    }
    // tombstones of emitted windows are not reused by the probes: rebuild the table first when
    // they and the most groups this push can add would crowd it
    if (a->tombs && a->live + a->tombs + std::min<uint64_t>(out->n_records, a->limit - std::min(a->live, a->limit)) >
                        a->slots / 4 * 3) {
        if (int r = rehash(a)) {
            if (new_peer) { a->peers.pop_back(); a->peer_time.pop_back(); a->peer_index.erase(pk); }
            return r;
        }
    }
    // dictionaries as they were: a failed push puts them back
    const std::vector<int64_t> keep_t = a->templates, keep_p = a->ports, keep_d = a->domains;
    const std::vector<int> keep_vw = a->val_w, keep_kw = a->key_w, keep_kk = a->key_kind_seen, keep_vk = a->val_kind_seen;
    bool gc_done = false;
    auto restore = [&]() {
        if (new_peer) {
            a->peers.pop_back();
            a->peer_time.pop_back();
            a->peer_index.erase(pk);
            new_peer = false;
        }
        a->templates = keep_t;
        a->ports = keep_p;
        a->domains = keep_d;
        a->val_w = keep_vw;
        a->key_w = keep_kw;
        a->key_kind_seen = keep_kk;
        a->val_kind_seen = keep_vk;
    };
    auto put = [&](std::vector<int64_t> &d, int64_t x, uint32_t cap, int &bit) -> int {
        bit = dict_put(d, x, cap);
        if (bit < 0 && !gc_done) {  // full: free the entries no live group uses, then retry
            const int r = dict_gc(a);
            if (r) return r;
            gc_done = true;
            bit = dict_put(d, x, cap);
        }
        return NGZ_OK;
    };
    int port_bit;
    if (int r = put(a->ports, peer_port, SET_BITS, port_bit)) { restore(); return r; }
    if (port_bit < 0) { restore(); return fail(a, NGZ_AGG_E_OVERFLOW, "more than 64 peer ports in live windows"); }
    // per-slot plans: FieldRef lookup (IE, occurrence among non-scope fields), types fixed at first sight
    const uint32_t S = out->n_slots;
    std::vector<AggSlotPlan> plans(std::max<uint32_t>(S, 1));
    std::vector<ngz_field_info> fi;
    for (uint32_t s = 0; s < S; ++s) {
        AggSlotPlan &sp = plans[s];
        memset(&sp, 0, sizeof sp);
        const ngz_slot_info &si = out->slots[s];
        sp.proto = si.proto;
        sp.bytes = ctx->last_in.bytes;
        if (!si.n_records || !si.columns) continue;
        const int nf = ngz_slot_fields(ctx, s, nullptr, 0);
        if (nf < 0) { restore(); return fail(a, NGZ_E_INVALID, "ngz_slot_fields"); }
        fi.resize(std::max(nf, 1));
        ngz_slot_fields(ctx, s, fi.data(), (uint32_t)nf);
        int tbit;
        if (int r = put(a->templates, ((int64_t)si.proto << 16) | si.template_id, SET_BITS, tbit)) { restore(); return r; }
        if (tbit < 0) { restore(); return fail(a, NGZ_AGG_E_OVERFLOW, "more than 64 template ids in live windows"); }
        sp.tpl_bit = 1ull << tbit;
        auto find_field = [&](const ngz_agg_field &f) -> int {
            uint32_t seen = 0;
            for (int i = 0; i < nf; ++i) {
                if (fi[i].is_scope) continue;
                if (fi[i].pen == f.pen && fi[i].ie_id == f.ie_id) {
                    if (seen == f.index) return i;
                    ++seen;
                }
            }
            return -1;
        };
        for (uint32_t k = 0; k < a->P.n_keys; ++k) {
            const int i = find_field(a->keys[k]);
            if (i < 0) continue;
            const ngz_field_info &f = fi[i];
            if (a->P.key_kind[k] == KK_BYTES) {
                // any length, fixed or variable-length (a record's text / bytes, BVAL)
                if (f.kind == NGZ_K_FAIL) { restore(); return fail(a, NGZ_E_LIMIT, "key field of a failing template"); }
                if (f.kind == NGZ_K_VLEN) sp.key_vlen |= 1u << k;
                sp.key_col[k] = si.columns + (uint64_t)si.capacity * f.col_off;
                sp.key_w[k] = f.width;
                if (a->key_w[k] < 0) a->key_w[k] = f.width;
                if (a->key_kind_seen[k] < 0) a->key_kind_seen[k] = f.kind;
                continue;
            }
            if (f.kind == NGZ_K_VLEN || f.kind == NGZ_K_FAIL) {
                restore();
                return fail(a, NGZ_E_LIMIT, "fixed-size key field sent variable-length (its records fail to decode)");
            }
            if (f.width > a->P.key_slot[k]) { restore(); return fail(a, NGZ_E_LIMIT, "key field wider than its row slot"); }
            if (a->P.packed && f.width != a->P.key_pw[k]) {
                restore();
                return fail(a, NGZ_E_LIMIT, "key column width differs from the IE's width");
            }
            sp.key_col[k] = si.columns + (uint64_t)si.capacity * f.col_off;
            sp.key_w[k] = f.width;
            if (a->key_w[k] < 0) a->key_w[k] = f.width;
            if (a->key_kind_seen[k] < 0) a->key_kind_seen[k] = f.kind;
        }
        for (uint32_t v = 0; v < a->P.n_vals; ++v) {
            const int i = find_field(a->vals[v]);
            if (i < 0) continue;
            const ngz_field_info &f = fi[i];
            const int vc = a->P.val_vc[v];
            if ((vc == VC_VBYTES || vc == VC_VLIST) && f.kind != NGZ_K_FAIL) {
                // Box<[u8]> values: any length, fixed or variable-length (BVAL)
                if (f.kind == NGZ_K_VLEN) sp.val_vlen |= 1u << v;
                if (a->val_w[v] < 0) a->val_w[v] = f.width;
                if (a->val_kind_seen[v] < 0) a->val_kind_seen[v] = f.kind;
                sp.val_col[v] = si.columns + (uint64_t)si.capacity * f.col_off;
                sp.val_w[v] = f.width;
                continue;
            }
            if (f.kind == NGZ_K_VLEN || f.kind == NGZ_K_FAIL || (vc == VC_BYTES && f.width > 32)) {
                restore();
                return fail(a, NGZ_E_LIMIT, "fixed-size aggregated field sent variable-length (its records fail to decode)");
            }
            const bool int_like = vc == VC_UINT || vc == VC_SINT || vc == VC_RANK;
            if ((int_like && f.width != 1 && f.width != 2 && f.width != 4 && f.width != 8) ||
                (vc == VC_F32 && f.width != 4) || (vc == VC_F64 && f.width != 8) || (vc == VC_IPV6 && f.width != 16) ||
                (vc == VC_DTFRAC && f.width != 8)) {
                restore();
                return fail(a, NGZ_E_LIMIT, "aggregated field of an unexpected column width");
            }
            if (a->val_w[v] >= 0 && a->val_w[v] != f.width) {
                restore();
                return fail(a, NGZ_E_LIMIT, "aggregated field width differs between templates");
            }
            a->val_w[v] = f.width;
            if (a->val_kind_seen[v] < 0) a->val_kind_seen[v] = f.kind;
            sp.val_col[v] = si.columns + (uint64_t)si.capacity * f.col_off;
            sp.val_w[v] = f.width;
        }
        sp.usable = 1;
    }
    const uint32_t D = out->n_dgrams, NS = out->n_sets;
    if (!D || !NS) return NGZ_OK;
    // scratch: has_rec[D], ts[D], pm[D], dginfo[D], cnt/rstart[NS+1], cub temp
    size_t cub_max = 0, cub_sum = 0;
    hipcub::DeviceScan::InclusiveScan(nullptr, cub_max, (uint32_t *)nullptr, (uint32_t *)nullptr, hipcub::Max(), D,
                                      a->stream);
    hipcub::DeviceScan::ExclusiveSum(nullptr, cub_sum, (uint32_t *)nullptr, (uint32_t *)nullptr, NS + 1, a->stream);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_has = 0, o_ts = o_has + al(4ull * D), o_pm = o_ts + al(4ull * D), o_dg = o_pm + al(4ull * D),
                 o_cnt = o_dg + al(2ull * D), o_rs = o_cnt + al(4ull * (NS + 1)), o_cub = o_rs + al(4ull * (NS + 1)),
                 need = o_cub + al(std::max(cub_max, cub_sum));
    if (need > a->scratch_cap) {
        hipFree(a->scratch);
        a->scratch = nullptr;
        if (hipMalloc(&a->scratch, need) != hipSuccess) { a->scratch_cap = 0; restore(); return fail(a, NGZ_E_NOMEM, "scratch"); }
        a->scratch_cap = need;
    }
    uint8_t *sc = (uint8_t *)a->scratch;
    uint32_t *has_rec = (uint32_t *)(sc + o_has), *ts = (uint32_t *)(sc + o_ts), *pm = (uint32_t *)(sc + o_pm);
    uint16_t *dginfo = (uint16_t *)(sc + o_dg);
    uint32_t *cnt = (uint32_t *)(sc + o_cnt), *rstart = (uint32_t *)(sc + o_rs);
    void *cub_tmp = sc + o_cub;
    if (S > a->plans_cap) {
        hipFree(a->plans);
        a->plans = nullptr;
        if (hipMalloc(&a->plans, sizeof(AggSlotPlan) * S) != hipSuccess) {
            a->plans_cap = 0;
            restore();
            return fail(a, NGZ_E_NOMEM, "plans");
        }
        a->plans_cap = S;
    }
    hipStream_t st = a->stream;
    AGG_HIP(a, hipMemcpyAsync(a->plans, plans.data(), sizeof(AggSlotPlan) * S, hipMemcpyHostToDevice, st));
    AggParams P = a->P;
    P.push_id = ++a->push_id;
    P.port_bit = (uint32_t)port_bit;
    P.peer = pi;
    P.coll_flip = (uint64_t)collection_time_ms ^ (1ull << 63);
    // owner path only where groups get few records per push (many groups per record): with
    // few, hot groups the wave / workgroup pre-aggregation of k_agg_apply serves them better
    // and the owner stores and checks would only add traffic.  Decided from the groups held
    // before the push (an empty table: the first push of any key).
    P.own = P.own && a->opt_owner && (a->live == 0 || a->live * 8 > (uint64_t)out->n_records);
    AGG_HIP(a, hipEventRecord(a->ev0, st));
    AGG_HIP(a, hipMemsetAsync(has_rec, 0, 4ull * D, st));
    AGG_HIP(a, hipMemsetAsync(a->late, 0, 8, st));
    AGG_HIP(a, hipMemsetAsync(a->err, 0, 4, st));
    AGG_HIP(a, hipMemsetAsync(a->newdom, 0, NEWDOM_SLOTS * 8, st));
    AGG_HIP(a, hipMemsetAsync(a->n_claims, 0, 8, st));
    const ngz_dgram_hdr *hdr = out->dgrams;
    const ngz_set_info *sets = out->sets;
    hipLaunchKernelGGL(k_agg_dgram, dim3(grid_for(NS)), dim3(256), 0, st, sets, NS, D, has_rec);
    hipLaunchKernelGGL(k_agg_ts, dim3(grid_for(D)), dim3(256), 0, st, hdr, has_rec, D, ts);
    size_t tmp = cub_max;
    AGG_HIP(a, hipcub::DeviceScan::InclusiveScan(cub_tmp, tmp, ts, pm, hipcub::Max(), D, st));
    hipLaunchKernelGGL(k_agg_late, dim3(grid_for(D)), dim3(256), 0, st, hdr, has_rec, pm, D, a->peer_time[pi],
                       a->lateness_ms, a->dom_dict, dginfo, a->newdom, a->err);
    // record starts of every set: n copied out of the set table (stride 16 B) then scanned
    AGG_HIP(a, hipMemsetAsync(cnt + NS, 0, 4, st));
    AGG_HIP(a, hipMemcpy2DAsync(cnt, 4, (const uint8_t *)sets + offsetof(ngz_set_info, n), sizeof(ngz_set_info), 4, NS,
                                hipMemcpyDeviceToDevice, st));
    tmp = cub_sum;
    AGG_HIP(a, hipcub::DeviceScan::ExclusiveSum(cub_tmp, tmp, cnt, rstart, NS + 1, st));
    // one synchronisation: the record count sizes the record kernels, new domains need entries
    uint32_t n_rec = 0;
    unsigned long long newdom[NEWDOM_SLOTS];
    unsigned int errv = 0;
    AGG_HIP(a, hipMemcpyAsync(&n_rec, rstart + NS, 4, hipMemcpyDeviceToHost, st));
    AGG_HIP(a, hipMemcpyAsync(newdom, a->newdom, sizeof newdom, hipMemcpyDeviceToHost, st));
    AGG_HIP(a, hipMemcpyAsync(&errv, a->err, 4, hipMemcpyDeviceToHost, st));
    AGG_HIP(a, hipStreamSynchronize(st));
    if (errv & 1) { restore(); return fail(a, NGZ_AGG_E_OVERFLOW, "more than 256 new observation domains in one push"); }
    bool fix = false;
    for (uint32_t i = 0; i < NEWDOM_SLOTS; ++i) {
        if (!newdom[i]) continue;
        int bit;
        if (int r = put(a->domains, (int64_t)(uint32_t)newdom[i], DOM_SLOTS, bit)) { restore(); return r; }
        if (bit < 0) {
            restore();
            upload_domains(a);
            return fail(a, NGZ_AGG_E_OVERFLOW, "more than 128 observation domains in live windows");
        }
        fix = true;
    }
    if (fix) {
        if (int r = upload_domains(a)) { restore(); return r; }
        hipLaunchKernelGGL(k_agg_domfix, dim3(grid_for(D)), dim3(256), 0, st, hdr, a->dom_dict, dginfo, D, a->err);
    }
    // per-record buffers: contexts (16 B), rec_g, claims, two record lists, sort keys / values (x2)
    const uint64_t R4 = al(4ull * std::max<uint32_t>(n_rec, 1));
    const bool ordered = [&] {
        for (uint32_t v = 0; v < P.n_vals; ++v)
            if (vc_ordered(P.val_vc[v])) return true;
        return false;
    }();
    size_t sort_tmp = 0;
    if (ordered)
        hipcub::DeviceRadixSort::SortPairs(nullptr, sort_tmp, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                           (uint32_t *)nullptr, (uint32_t *)nullptr, (int)std::max<uint32_t>(n_rec, 1),
                                           0, 32, st);
    const uint64_t n_blk = ((uint64_t)n_rec + 255) / 256;
    const size_t B0 = al(16ull * NS) + al(4 * (n_blk + 1));  // set contexts, block sets
    const size_t rec_need = B0 + 4 * R4 + (ordered ? 4 * R4 + al(sort_tmp) : 0);
    if (rec_need > a->rec_cap) {
        hipFree(a->rec_buf);
        a->rec_buf = nullptr;
        a->rec_cap = 0;
        if (hipMalloc(&a->rec_buf, rec_need) != hipSuccess) { restore(); upload_domains(a); return fail(a, NGZ_E_NOMEM, "record buffers"); }
        a->rec_cap = rec_need;
    }
    uint4 *sctx = (uint4 *)a->rec_buf;
    uint32_t *bset = (uint32_t *)(a->rec_buf + al(16ull * NS));
    uint32_t *rec_g = (uint32_t *)(a->rec_buf + B0), *claims = (uint32_t *)(a->rec_buf + B0 + R4),
             *list_a = (uint32_t *)(a->rec_buf + B0 + 2 * R4), *list_b = (uint32_t *)(a->rec_buf + B0 + 3 * R4);
    const RecCtx C{sctx, rstart, bset, NS, (uint64_t)n_rec, a->plans};
    const uint32_t blocks = (uint32_t)((n_rec + 255) / 256);
    static const uint32_t grid_cap = (uint32_t)std::max<int64_t>(1, ngz_knob("NGZ_AGG_GRID", 4096));
    const uint32_t ig = std::max<uint32_t>(1, std::min<uint32_t>(blocks, grid_cap));
    unsigned long long n_claims = 0;
    auto rollback = [&](int rc, const std::string &why) {
        if (n_claims)
            hipLaunchKernelGGL(k_agg_unclaim, dim3(grid_for(n_claims)), dim3(256), 0, st, a->tags, claims, (uint64_t)n_claims);
        if (P.has_bytes)  // the released claims' key tails: the arena as after the last push
            hipMemcpyAsync(a->arena_used, &a->arena_mark, 8, hipMemcpyHostToDevice, st);
        restore();
        upload_domains(a);
        if (hipStreamSynchronize(st) != hipSuccess) a->poisoned = true;
        return fail(a, rc, why);
    };
    // Low-cardinality path (packed keys, no byte-wise / ordered values): k_agg_lc_part reduces
    // every record in one pass into per-wave partial groups, k_agg_lc_merge combines them
    // per tag, claims and applies.  A wave with more than LC_NK key tuples in one window
    // context, or more than LC_MAX_TAGS tags in the push, sends the push to the general
    // path below, with nothing claimed or applied (NGZ_AGG_OPT_LOWCARD: 0 never, 1 at any size;
    // default from 2^16 records).
    const int lc_now = a->opt_lowcard;  // NGZ_AGG_OPT_LOWCARD
    // a push that found too many key tuples sends the next 15 pushes of the aggregator
    // straight to the general path (high-cardinality keys pay for one try in 16)
    const bool lc_try = lc_now == 1 || (lc_now != 0 && n_rec >= (1u << 16) && (a->lc_skip == 0 || --a->lc_skip == 0));
    if (n_rec && P.packed && P.lds_ok && P.n_vals <= (uint32_t)LC_MAXV && P.n_keys <= (uint32_t)LC_MAXK &&
        !ordered && lc_try) {
        // one-wave workgroups; the lane-private LDS cells of LC_NK tuples bound the residency
        // (160 KB per CU): a grid of that many workgroups, a multiple of the 8 XCDs
        const size_t lds = lc_lds_bytes(P.n_vals);
        const uint32_t per_cu = (uint32_t)std::max<size_t>(1, std::min<size_t>(16, (160u * 1024 - 1024) / (lds + 256)));
        const uint32_t rg = std::max<uint32_t>(8, std::min<uint32_t>(256 * per_cu, (NS + 7) & ~7u));
        const uint32_t cap = rg * LC_NK * 4;  // 4 window contexts per wave; more: the general path
        if (cap > a->lc_cap || !a->lc_cnt) {
            hipFree(a->lc);
            a->lc = nullptr;
            a->lc_cap = 0;
            if (!a->lc_cnt && hipMalloc(&a->lc_cnt, 16) != hipSuccess) a->lc_cnt = nullptr;
            // the waves' entries, then the merge workgroups' slices
            if (!a->lc_cnt ||
                hipMalloc(&a->lc, sizeof(LcEntry) * ((size_t)cap + LCM_BLOCKS * LC_MAX_TAGS)) != hipSuccess) {
                a->lc = nullptr;
                restore();
                upload_domains(a);
                return fail(a, NGZ_E_NOMEM, "low-cardinality buffers");
            }
            a->lc_cap = cap;
        }
        if (NS > a->lc_sets_cap) {
            hipFree(a->lc_sets);
            a->lc_sets_cap = 0;
            if (hipMalloc(&a->lc_sets, sizeof(LcSet) * (size_t)NS) != hipSuccess) {
                a->lc_sets = nullptr;
                restore();
                upload_domains(a);
                return fail(a, NGZ_E_NOMEM, "low-cardinality set descriptors");
            }
            a->lc_sets_cap = NS;
        }
        uint32_t kb = 0;
        for (uint32_t k = 0; k < P.n_keys; ++k) kb += 1 + 8 * P.key_pw[k];
        AGG_HIP(a, hipMemsetAsync(a->lc_cnt, 0, 16, st));
        hipLaunchKernelGGL(k_agg_lc_sets, dim3(grid_for(NS)), dim3(256), 0, st, sets, NS, hdr, dginfo, a->plans, D, S,
                           a->lc_sets, a->late, a->err);
        hipLaunchKernelGGL(k_agg_lc_part, dim3(rg), dim3(64), lds, st, a->lc_sets, NS, a->plans, P, kb, a->lc,
                           a->lc_cnt, cap, a->lc_cnt + 1);
        AGG_HIP(a, hipGetLastError());
        const uint64_t room = a->limit - std::min(a->live, a->limit);
        hipLaunchKernelGGL(k_agg_lc_merge, dim3(LCM_BLOCKS), dim3(LCM_THREADS), 0, st, a->lc, cap, a->lc + cap,
                           a->lc_cnt, P, a->tags, a->rows, room, claims, a->n_claims, a->err);
        AGG_HIP(a, hipGetLastError());
        unsigned int lcc[2] = {0, 0};
        AGG_HIP(a, hipMemcpyAsync(lcc, a->lc_cnt, 8, hipMemcpyDeviceToHost, st));
        AGG_HIP(a, hipMemcpyAsync(&n_claims, a->n_claims, 8, hipMemcpyDeviceToHost, st));
        AGG_HIP(a, hipMemcpyAsync(&errv, a->err, 4, hipMemcpyDeviceToHost, st));
        AGG_HIP(a, hipStreamSynchronize(st));
        if (errv & 16) { a->poisoned = true; return rollback(NGZ_E_DEVICE, "set table entry out of range"); }
        if (!lcc[1]) {
            // the merge released its claims when the push did not fit: nothing to undo
            if (errv & 2) return rollback(NGZ_AGG_E_OVERFLOW, "group table full");
            if (errv & 32) return rollback(NGZ_AGG_E_OVERFLOW, "more groups than the aggregator's capacity");
            a->last_path = "lowcard";
            goto done;
        }
        // too many key tuples / distinct tags: the general path from the start (nothing was
        // claimed or applied; its claim pass counts the late records again)
        AGG_HIP(a, hipMemsetAsync(a->late, 0, 8, st));
        a->lc_skip = 16;  // the next 15 pushes take the general path, the 16th tries this one again
    }
    a->last_path = "general";
    {
    hipLaunchKernelGGL(k_agg_recinfo, dim3(grid_for(NS, 256, 4096)), dim3(256), 0, st, sets, NS, hdr, dginfo, a->plans, D,
                       S, sctx, a->err);
    if (n_blk) hipLaunchKernelGGL(k_agg_bset, dim3(grid_for(n_blk, 256, 4096)), dim3(256), 0, st, rstart, NS, n_blk, bset);
    AGG_HIP(a, hipGetLastError());
    if (P.has_bytes && n_rec) {
        // byte values longer than 32 bytes: room in the arena for every tail this push can write.
        // Key claims and ordered folds write at most one tail per group and field, and a push
        // touches at most every slot of the table: the bound is the smaller of the records' tails
        // and slots x byte fields x the longest tail (10^8 records of a 64-byte key over a few
        // groups reserve 2 slots per group's worth, not 3 GB)
        unsigned long long nd[2] = {0, 0};
        AGG_HIP(a, hipMemsetAsync(a->arena_used + 1, 0, 16, st));
        hipLaunchKernelGGL(k_agg_tail_need, dim3(grid_for(n_rec, 256, 4096)), dim3(256), 0, st, C, P, a->arena_used + 1);
        AGG_HIP(a, hipMemcpyAsync(nd, a->arena_used + 1, 16, hipMemcpyDeviceToHost, st));
        AGG_HIP(a, hipStreamSynchronize(st));
        uint32_t n_bval = 0;
        for (uint32_t k = 0; k < P.n_keys; ++k) n_bval += P.key_kind[k] == KK_BYTES;
        for (uint32_t v = 0; v < P.n_vals; ++v) n_bval += P.val_vc[v] == VC_VBYTES || P.val_vc[v] == VC_VLIST;
        const uint64_t need = std::min<uint64_t>(nd[0], a->slots * n_bval * nd[1]);
        if (int r = arena_reserve(a, need)) { restore(); upload_domains(a); return r; }
        P.arena = a->P.arena;
        P.arena_cap = a->P.arena_cap;
    }
    // claim / check keep no state across tiles: one record per thread, all of them in flight
    const uint32_t fg = std::max<uint32_t>(1, std::min<uint32_t>(blocks, 1u << 20));
    if (n_rec) {
        AGG_HIP(a, hipMemsetAsync(a->n_coll, 0, 4, st));
        hipLaunchKernelGGL(k_agg_claim, dim3(fg), dim3(256), 0, st, C, P, a->tags, a->rows, rec_g, claims, a->n_claims,
                           a->late, list_b, a->n_coll, a->err);
        if (!P.packed) {
            // hashed keys: the records that took a slot another record of this pass claimed are
            // compared now that every key is written; the records of collided keys re-probe
            // comparing keys
            unsigned int nt = 0;
            AGG_HIP(a, hipMemcpyAsync(&nt, a->n_coll, 4, hipMemcpyDeviceToHost, st));
            AGG_HIP(a, hipStreamSynchronize(st));
            AGG_HIP(a, hipMemsetAsync(a->n_coll, 0, 4, st));
            if (nt)
                hipLaunchKernelGGL(k_agg_check, dim3(grid_for(nt, 256, 1u << 20)), dim3(256), 0, st, C, P, a->rows, rec_g,
                                   list_b, nt, list_a, a->n_coll, a->err);
            for (int round = 0;; ++round) {
                unsigned int nc = 0;
                AGG_HIP(a, hipMemcpyAsync(&nc, a->n_coll, 4, hipMemcpyDeviceToHost, st));
                AGG_HIP(a, hipStreamSynchronize(st));
                if (!nc) break;
                if (round == 64) {
                    AGG_HIP(a, hipMemcpyAsync(&n_claims, a->n_claims, 8, hipMemcpyDeviceToHost, st));
                    AGG_HIP(a, hipStreamSynchronize(st));
                    return rollback(NGZ_E_DEVICE, "key collision resolution did not converge");
                }
                hipLaunchKernelGGL(k_agg_reprobe, dim3(grid_for(nc)), dim3(256), 0, st, C, P, a->tags, a->rows, rec_g,
                                   list_a, nc, claims, a->n_claims, a->err);
                AGG_HIP(a, hipMemsetAsync(a->n_coll, 0, 4, st));
                hipLaunchKernelGGL(k_agg_check, dim3(grid_for(nc)), dim3(256), 0, st, C, P, a->rows, rec_g, list_a, nc,
                                   list_b, a->n_coll, a->err);
                std::swap(list_a, list_b);
            }
        }
    }
    AGG_HIP(a, hipGetLastError());
    AGG_HIP(a, hipMemcpyAsync(&n_claims, a->n_claims, 8, hipMemcpyDeviceToHost, st));
    AGG_HIP(a, hipMemcpyAsync(&errv, a->err, 4, hipMemcpyDeviceToHost, st));
    AGG_HIP(a, hipStreamSynchronize(st));
    if (errv & 16) { a->poisoned = true; return rollback(NGZ_E_DEVICE, "set table entry out of range"); }
    if (errv & 2) return rollback(NGZ_AGG_E_OVERFLOW, "group table full");
    if (a->live + n_claims > a->limit) return rollback(NGZ_AGG_E_OVERFLOW, "more groups than the aggregator's capacity");
    // commit: every record has its group; reduce.  Few groups: a bounded grid whose workgroups
    // walk many tiles, so the LDS combine table collects each group's records across them; many
    // groups (about one record per group and push): one tile per workgroup, all records in flight
    if (n_rec) {
        const uint32_t ag = (a->live + n_claims) * 8 > n_rec ? fg : ig;
        // fused owner test (k_agg_apply_own first) only when the table holds many groups per
        // record after the claims: then nearly every record is its group's owner.  Few, hot
        // groups (a first push of a low-cardinality key included) would list almost every record
        // for k_agg_apply, one counter atomic per wave on a single word (142 ms for 12 groups
        // and 10^8 records), so the owner test stays in k_agg_apply there.
        static const bool split = ngz_knob("NGZ_AGG_OWN_SPLIT", 0) != 0;  // A/B: the owner test in k_agg_apply
        // partitioned reduction: more groups than LDS tables hold, at least 8 records per group
        // (NGZ_AGG_OPT_PARTITION: 0 never, 1 whenever the config allows it)
        const int part_env = a->opt_partition;  // NGZ_AGG_OPT_PARTITION
        const uint64_t groups = a->live + n_claims, n_part = a->slots / PART_SLOTS;
        const bool part_ok = P.lds_ok && P.n_vals <= 8 && a->slots >= PART_SLOTS && n_part <= 8192;
        const bool part = part_ok && (part_env == 1 || (part_env != 0 && n_rec >= (1u << 20) && groups > 4096 &&
                                                         groups * 8 <= (uint64_t)n_rec));
        if (part) {
            const uint32_t nt = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n_rec + PART_TILE - 1) / PART_TILE, 2048)),
                           np = (uint32_t)n_part;
            // operand layout of the payloads (k_agg_part_scatter): widest first, from byte 16
            uint32_t at = 16;
            for (uint32_t wd = 8; wd; wd >>= 1)
                for (uint32_t v = 0; v < 8; ++v) {
                    uint32_t ow = 0;
                    if (v < P.n_vals && !vc_ordered(P.val_vc[v]) && a->val_w[v] > 0)
                        ow = P.val_vc[v] == VC_UINT ? (uint32_t)a->val_w[v] : 8u;
                    if (ow != wd) continue;
                    P.op_off[v] = (uint8_t)at;
                    P.op_w[v] = (uint8_t)ow;
                    at += ow;
                }
            const uint32_t pb = (at + 31) & ~31u;
            const uint64_t nc = (uint64_t)np * nt + 1;
            size_t stb = 0;
            hipcub::DeviceScan::ExclusiveSum(nullptr, stb, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)nc, st);
            const size_t need = 2 * al(4 * nc) + al(stb) + (size_t)n_rec * pb;
            if (need > a->part_cap) {
                hipFree(a->part_buf);
                a->part_buf = nullptr;
                a->part_cap = 0;
                if (hipMalloc(&a->part_buf, need) != hipSuccess) {
                    a->poisoned = true;  // the claims are committed: this push cannot be undone here
                    return fail(a, NGZ_E_NOMEM, "partition buffers");
                }
                a->part_cap = need;
            }
            uint32_t *counts = (uint32_t *)a->part_buf, *offs = (uint32_t *)(a->part_buf + al(4 * nc));
            void *stmp = a->part_buf + 2 * al(4 * nc);
            uint8_t *pay = a->part_buf + 2 * al(4 * nc) + al(stb);
            AGG_HIP(a, hipMemsetAsync(counts + nc - 1, 0, 4, st));
            hipLaunchKernelGGL(k_agg_part_hist, dim3(nt), dim3(256), 4 * np, st, C, rec_g, np, counts);
            AGG_HIP(a, hipcub::DeviceScan::ExclusiveSum(stmp, stb, counts, offs, (int)nc, st));
            switch (pb / 16) {
            case 2: hipLaunchKernelGGL(k_agg_part_scatter<2>, dim3(nt), dim3(256), 4 * np, st, C, P, rec_g, np, offs, pay); break;
            case 4: hipLaunchKernelGGL(k_agg_part_scatter<4>, dim3(nt), dim3(256), 4 * np, st, C, P, rec_g, np, offs, pay); break;
            default: hipLaunchKernelGGL(k_agg_part_scatter<6>, dim3(nt), dim3(256), 4 * np, st, C, P, rec_g, np, offs, pay); break;
            }
            // payloads per thread and round in the reduce (NGZ_AGG_RED_RPT 1 or 4; A/B knob)
            static const uint32_t red_rpt = ngz_knob("NGZ_AGG_RED_RPT", 4) == 1 ? 1u : 4u;
            // threads per partition workgroup (one LDS table per workgroup: more threads, more waves
            // per CU on the same LDS; dport push 11.9 -> 10.4 ms at 512, 10.7 at 1024; knob
            // NGZ_AGG_RED_THREADS)
            static const uint32_t red_thr = (uint32_t)std::max<int64_t>(64, std::min<int64_t>(1024, ngz_knob("NGZ_AGG_RED_THREADS", 512))) / 64 * 64;
            switch (pb / 16 * 8 + red_rpt) {
            case 17: hipLaunchKernelGGL((k_agg_part_reduce<2, 1>), dim3(np), dim3(red_thr), 0, st, P, a->plans, offs, nt, pay, a->rows); break;
            case 20: hipLaunchKernelGGL((k_agg_part_reduce<2, 4>), dim3(np), dim3(red_thr), 0, st, P, a->plans, offs, nt, pay, a->rows); break;
            case 33: hipLaunchKernelGGL((k_agg_part_reduce<4, 1>), dim3(np), dim3(red_thr), 0, st, P, a->plans, offs, nt, pay, a->rows); break;
            case 36: hipLaunchKernelGGL((k_agg_part_reduce<4, 4>), dim3(np), dim3(red_thr), 0, st, P, a->plans, offs, nt, pay, a->rows); break;
            case 49: hipLaunchKernelGGL((k_agg_part_reduce<6, 1>), dim3(np), dim3(red_thr), 0, st, P, a->plans, offs, nt, pay, a->rows); break;
            default: hipLaunchKernelGGL((k_agg_part_reduce<6, 4>), dim3(np), dim3(red_thr), 0, st, P, a->plans, offs, nt, pay, a->rows); break;
            }
        } else if (P.own && !split && groups * 8 > (uint64_t)n_rec) {

            // owners reduce their rows first, the records k_agg_apply_own lists apply atomics after
            AGG_HIP(a, hipMemsetAsync(a->n_coll, 0, 4, st));
            hipLaunchKernelGGL(k_agg_apply_own<true>, dim3(fg), dim3(256), 0, st, C, P, rec_g, a->rows, list_a, a->n_coll,
                               a->err);
            if (P.n_vals <= 8)
                hipLaunchKernelGGL(k_agg_apply<8>, dim3(ig), dim3(256), 0, st, C, P, rec_g, a->rows, list_a, a->n_coll, a->err);
            else
                hipLaunchKernelGGL(k_agg_apply<NGZ_AGG_MAX_VALUES>, dim3(ig), dim3(256), 0, st, C, P, rec_g, a->rows, list_a,
                                   a->n_coll, a->err);
        } else {
            // owner records (marked in rec_g) reduced after every other record
            if (P.n_vals <= 8)
                hipLaunchKernelGGL(k_agg_apply<8>, dim3(ag), dim3(256), 0, st, C, P, rec_g, a->rows, nullptr, nullptr, a->err);
            else
                hipLaunchKernelGGL(k_agg_apply<NGZ_AGG_MAX_VALUES>, dim3(ag), dim3(256), 0, st, C, P, rec_g, a->rows, nullptr,
                                   nullptr, a->err);
            if (P.own)
                hipLaunchKernelGGL(k_agg_apply_own<false>, dim3(fg), dim3(256), 0, st, C, P, rec_g, a->rows, nullptr, nullptr,
                                   a->err);
        }
        if (ordered) {
            uint32_t *sk = (uint32_t *)(a->rec_buf + B0 + 4 * R4), *sv = (uint32_t *)(a->rec_buf + B0 + 5 * R4),
                     *sk2 = (uint32_t *)(a->rec_buf + B0 + 6 * R4), *sv2 = (uint32_t *)(a->rec_buf + B0 + 7 * R4);
            void *stmp = a->rec_buf + B0 + 8 * R4;
            AGG_HIP(a, hipMemcpyAsync(sk, rec_g, 4ull * n_rec, hipMemcpyDeviceToDevice, st));
            hipLaunchKernelGGL(k_agg_iota, dim3(grid_for(n_rec)), dim3(256), 0, st, sv, (uint64_t)n_rec);
            int end_bit = 1;
            while (end_bit < 32 && (1ull << end_bit) <= a->slots) ++end_bit;
            end_bit = 32;  // NONE (all ones) must sort after every slot
            size_t tb = sort_tmp;
            AGG_HIP(a, hipcub::DeviceRadixSort::SortPairs(stmp, tb, sk, sk2, sv, sv2, (int)n_rec, 0, end_bit, st));
            hipLaunchKernelGGL(k_agg_ordered, dim3(grid_for(n_rec)), dim3(256), 0, st, C, P, sk2, sv2, (uint64_t)n_rec,
                               a->rows, a->err);
        }
    }
    AGG_HIP(a, hipGetLastError());
    }
done:
    AGG_HIP(a, hipEventRecord(a->ev1, st));
    uint32_t last_pm = 0;
    unsigned long long late = 0, arena_now = a->arena_mark;
    AGG_HIP(a, hipMemcpyAsync(&last_pm, pm + (D - 1), 4, hipMemcpyDeviceToHost, st));
    AGG_HIP(a, hipMemcpyAsync(&late, a->late, 8, hipMemcpyDeviceToHost, st));
    if (P.has_bytes) {
        AGG_HIP(a, hipMemcpyAsync(&arena_now, a->arena_used, 8, hipMemcpyDeviceToHost, st));
        AGG_HIP(a, hipMemcpyAsync(&errv, a->err, 4, hipMemcpyDeviceToHost, st));
    }
    AGG_HIP(a, hipStreamSynchronize(st));
    if (P.has_bytes) {
        a->arena_mark = arena_now;
        if (errv & 64) {  // cannot happen: the push reserved every tail it writes
            a->poisoned = true;
            return fail(a, NGZ_E_DEVICE, "byte arena overrun");
        }
    }
    hipEventElapsedTime(&a->t_push, a->ev0, a->ev1);
    a->live += n_claims;
    if (last_pm > a->peer_time[pi]) a->peer_time[pi] = last_pm;
    if (late_records) *late_records = late;
    return NGZ_OK;
}

int64_t ngz_agg_groups(ngz_agg *a) {
    if (!a) return NGZ_E_INVALID;
    return (int64_t)a->live;
}

int64_t ngz_agg_flush(ngz_agg *a, void *dst, uint64_t cap) {
    if (!a) return NGZ_E_INVALID;
    if (a->poisoned) return fail(a, NGZ_AGG_E_POISONED, "aggregator failed earlier: ngz_agg_reset it");
    const int64_t n = take_rows(a, dst, cap, nullptr, false);
    if (n < 0) return n;
    // WindowAggregator::flush: every window out, the event times forgotten; the set and
    // peer dictionaries start over (the rows just returned refer to out_*)
    forget_peers(a);
    a->templates.clear();
    a->ports.clear();
    a->domains.clear();
    a->live = a->tombs = 0;
    int rc = reset_rows(a, a->tags, a->rows);
    if (rc == NGZ_OK) rc = upload_domains(a);
    if (rc == NGZ_OK) rc = arena_clear(a);
    if (rc != NGZ_OK) return rc;
    AGG_HIP(a, hipStreamSynchronize(a->stream));
    return n;
}

int64_t ngz_agg_closed(ngz_agg *a) {
    if (!a) return NGZ_E_INVALID;
    if (a->poisoned) return fail(a, NGZ_AGG_E_POISONED, "aggregator failed earlier: ngz_agg_reset it");
    AGG_HIP(a, hipSetDevice(a->device));
    bool any = false;
    if (int r = upload_cutoffs(a, &any)) return r;
    if (!any) return 0;
    unsigned long long n = 0;
    AGG_HIP(a, hipMemsetAsync(a->cursor, 0, 8, a->stream));
    hipLaunchKernelGGL(k_agg_count, dim3(grid_for(a->slots)), dim3(256), 0, a->stream, a->tags, a->rows, a->slots,
                       a->P.row_bytes, a->cut, a->cursor);
    AGG_HIP(a, hipMemcpyAsync(&n, a->cursor, 8, hipMemcpyDeviceToHost, a->stream));
    AGG_HIP(a, hipStreamSynchronize(a->stream));
    return (int64_t)n;
}

int64_t ngz_agg_emit(ngz_agg *a, void *dst, uint64_t cap) {
    if (!a) return NGZ_E_INVALID;
    if (a->poisoned) return fail(a, NGZ_AGG_E_POISONED, "aggregator failed earlier: ngz_agg_reset it");
    AGG_HIP(a, hipSetDevice(a->device));
    bool any = false;
    if (int r = upload_cutoffs(a, &any)) return r;
    if (!any) {
        a->out_templates = a->templates;
        a->out_ports = a->ports;
        a->out_domains = a->domains;
        a->out_peers = a->peers;
        return 0;
    }
    const int64_t n = take_rows(a, dst, cap, a->cut, true);
    if (n <= 0) return n;
    a->live -= (uint64_t)n;
    a->tombs += (uint64_t)n;
    // the n groups are handed out and their slots freed whatever happens next: a failed
    // rebuild poisons the aggregator (reported by the next call), it does not lose them
    if (a->live + a->tombs > a->slots / 2) rehash(a);
    return n;
}

int ngz_agg_reset(ngz_agg *a) {
    if (!a) return NGZ_E_INVALID;
    AGG_HIP(a, hipSetDevice(a->device));
    a->poisoned = false;
    forget_peers(a);
    a->templates.clear();
    a->ports.clear();
    a->domains.clear();
    a->live = a->tombs = 0;
    int rc = reset_rows(a, a->tags, a->rows);
    if (rc == NGZ_OK) rc = upload_domains(a);
    if (rc == NGZ_OK) rc = arena_clear(a);
    if (rc != NGZ_OK) return rc;
    AGG_HIP(a, hipStreamSynchronize(a->stream));
    return NGZ_OK;
}

int ngz_agg_sets(ngz_agg *a, uint32_t *templates, uint32_t *n_templates, uint16_t *ports, uint32_t *n_ports,
                 uint32_t *domains, uint32_t *n_domains, uint32_t cap) {
    if (!a) return NGZ_E_INVALID;
    // entry i <-> bit i of the rows last returned by ngz_agg_flush / ngz_agg_emit; free entries read 0xFFFFFFFF
    auto out = [cap](const std::vector<int64_t> &d, auto *dst, uint32_t *n, auto none) {
        if (n) *n = (uint32_t)d.size();
        for (uint32_t i = 0; i < d.size() && i < cap; ++i)
            if (dst) dst[i] = d[i] < 0 ? none : (decltype(none))d[i];
    };
    out(a->out_templates, templates, n_templates, 0xFFFFFFFFu);
    out(a->out_ports, ports, n_ports, (uint16_t)0xFFFF);
    out(a->out_domains, domains, n_domains, 0xFFFFFFFFu);
    return NGZ_OK;
}

int ngz_agg_peer(ngz_agg *a, uint32_t index, ngz_peer *out) {
    if (!a || index >= a->out_peers.size()) return NGZ_E_INVALID;
    if (out) *out = a->out_peers[index];
    return (int)a->out_peers.size();
}

const char *ngz_agg_last_path(ngz_agg *a) { return a ? a->last_path : ""; }

int ngz_agg_set_option(ngz_agg *a, int opt, int64_t value) {
    if (!a) return NGZ_E_INVALID;
    switch (opt) {
    case NGZ_AGG_OPT_LOWCARD:
        if (value < -1 || value > 1) return fail(a, NGZ_E_INVALID, "NGZ_AGG_OPT_LOWCARD takes -1, 0 or 1");
        a->opt_lowcard = (int)value;
        a->lc_skip = 0;
        return NGZ_OK;
    case NGZ_AGG_OPT_PARTITION:
        if (value < -1 || value > 1) return fail(a, NGZ_E_INVALID, "NGZ_AGG_OPT_PARTITION takes -1, 0 or 1");
        a->opt_partition = (int)value;
        return NGZ_OK;
    case NGZ_AGG_OPT_OWNER:
        if (value < 0 || value > 1) return fail(a, NGZ_E_INVALID, "NGZ_AGG_OPT_OWNER takes 0 or 1");
        a->opt_owner = value != 0;
        return NGZ_OK;
    case NGZ_AGG_OPT_HASH_BITS:
        // groups sit at their hash's slot: only an empty table may change the hash
        if (value < 0 || value > 63) return fail(a, NGZ_E_INVALID, "NGZ_AGG_OPT_HASH_BITS takes 0..63");
        if (a->live || a->tombs) return fail(a, NGZ_E_INVALID, "NGZ_AGG_OPT_HASH_BITS: the aggregator holds groups");
        a->P.hash_mask = value ? (1ull << value) - 1 : ~0ull;
        return NGZ_OK;
    }
    return fail(a, NGZ_E_INVALID, "unknown option");
}

int ngz_agg_last_timing(ngz_agg *a, float *push_ms) {
    if (!a) return NGZ_E_INVALID;
    if (push_ms) *push_ms = a->t_push;
    return NGZ_OK;
}

int ngz_agg_value_info(ngz_agg *a, uint32_t v, ngz_agg_value_desc *out) {
    if (!a || !out || v >= a->P.n_vals) return NGZ_E_INVALID;
    memset(out, 0, sizeof *out);
    out->vclass = a->P.val_vc[v];
    out->width = (uint16_t)std::max(a->val_w[v], 0);
    out->kind = (uint8_t)std::max(a->val_kind_seen[v], 0);
    return NGZ_OK;
}

int64_t ngz_agg_row_bytes(ngz_agg *a, const void *row, int is_value, uint32_t index, uint8_t *dst, uint64_t cap) {
    if (!a || !row) return NGZ_E_INVALID;
    uint32_t off;
    if (is_value) {
        if (index >= a->P.n_vals || (a->P.val_vc[index] != VC_VBYTES && a->P.val_vc[index] != VC_VLIST))
            return NGZ_E_INVALID;
        off = a->P.val_off[index];
    } else {
        if (index >= a->P.n_keys || a->P.key_kind[index] != KK_BYTES) return NGZ_E_INVALID;
        off = a->P.key_off[index];
    }
    uint32_t take;
    memcpy(&take, (const uint8_t *)row + 36, 4);
    if (take == 0 || take != a->take_id) return NGZ_E_INVALID;  // a row of an earlier flush / emit
    const uint8_t *slot = (const uint8_t *)row + off;
    uint32_t n, toff8;
    memcpy(&n, slot, 4);
    memcpy(&toff8, slot + 4, 4);
    const uint64_t toff = (uint64_t)toff8 << 3;  // 8-byte units (tail_span)
    if (n > BVAL_INLINE && toff + (n - BVAL_INLINE) > a->out_tails.size()) return NGZ_E_INVALID;
    if (dst)
        for (uint64_t i = 0; i < n && i < cap; ++i)
            dst[i] = i < BVAL_INLINE ? slot[8 + i] : a->out_tails[toff + i - BVAL_INLINE];
    return (int64_t)n;
}

int ngz_agg_key_info(ngz_agg *a, uint32_t k, ngz_agg_key_desc *out) {
    if (!a || !out || k >= a->P.n_keys) return NGZ_E_INVALID;
    memset(out, 0, sizeof *out);
    out->kkind = a->P.key_kind[k];
    out->slot = (uint16_t)a->P.key_slot[k];
    out->width = (uint16_t)std::max(a->key_w[k], 0);
    out->kind = (uint8_t)std::max(a->key_kind_seen[k], 0);
    return NGZ_OK;
}

}  // extern "C"

// FlowInfo rendering of aggregated groups lives in ngz_agg_json.cpp (needs the IE registry
// and the JSON field writers); it reads the aggregator through these.
namespace ngzh {
const std::vector<ngz_agg_field> &agg_keys(const ngz_agg *a) { return a->keys; }
const std::vector<ngz_agg_field> &agg_vals(const ngz_agg *a) { return a->vals; }
void agg_out_dicts(const ngz_agg *a, const std::vector<int64_t> **t, const std::vector<int64_t> **p,
                   const std::vector<int64_t> **d) {
    *t = &a->out_templates;
    *p = &a->out_ports;
    *d = &a->out_domains;
}
const std::vector<ngz_peer> &agg_out_peers(const ngz_agg *a) { return a->out_peers; }
uint64_t agg_window_ms(const ngz_agg *a) { return a->window_ms; }
}  // namespace ngzh
