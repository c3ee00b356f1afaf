// Flow aggregation on the device: the collector's windowed FlowAggregator
// (crates/collector/src/flow/aggregation/aggregator.rs) over the columns the
// decode path leaves in HBM.  C ABI: include/ngz/flow_aggregate.h.
//
// Pipeline of one ngz_agg_push (all on one stream):
//   k_agg_dgram   per datagram: event time it contributes (OK status and >= 1
//                 data record, aggregator.rs:308 yields one item per record),
//                 observation-domain dictionary bit (device CAS table)
//   hipcub max-scan over event times -> k_agg_late: lateness flag per datagram
//                 (aggregation.rs:139-141: ts < current_time - lateness, with
//                 current_time the running max of earlier non-late items)
//   hipcub sum-scan over set record counts -> k_agg_setidx: set of every record
//   k_agg_insert  one lane per record: key hash over the key columns, open
//                 addressing insert into the HBM group table (64-bit CAS on the
//                 tag), then the reductions of FlowCacheRecord::reduce
//                 (aggregator.rs:159-198) as atomics on the group row
//   k_agg_verify  (after all inserts) re-hashes every record and compares its
//                 key bytes with the stored key of the group it landed in; a
//                 mismatch is a 64-bit hash collision -> NGZ_AGG_E_COLLISION
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ngz/flow_aggregate.h"
#include "ngz/flow_decode.h"
#include "ngz_host.h"

namespace {

constexpr uint32_t ROW_HDR = 88;  // sizeof(ngz_agg_row)
static_assert(sizeof(ngz_agg_row) == ROW_HDR, "ngz_agg_row layout");
constexpr uint32_t DOM_SLOTS = 128;

// value classes (how a column value becomes the 64-bit accumulator operand)
enum : uint8_t { VC_UINT = 0, VC_SINT = 1, VC_DTFRAC = 2, VC_BYTES = 3 };

struct AggSlotPlan {            // per batch slot, built on the host every push
    const uint8_t *key_col[NGZ_AGG_MAX_KEYS];   // null: the record has no such field (None)
    const uint8_t *val_col[NGZ_AGG_MAX_VALUES];
    uint16_t key_w[NGZ_AGG_MAX_KEYS];
    uint16_t val_w[NGZ_AGG_MAX_VALUES];
    uint8_t key_str[NGZ_AGG_MAX_KEYS];          // fixed string: bytes after the first NUL do not count
    uint8_t val_vc[NGZ_AGG_MAX_VALUES];
    uint64_t tpl_bit;
    uint32_t proto;
    uint32_t usable;                            // 0: slot not aggregated (no records / not device-decoded)
};

struct AggParams {
    uint32_t n_keys, n_vals;
    uint32_t key_off[NGZ_AGG_MAX_KEYS];
    uint32_t key_w[NGZ_AGG_MAX_KEYS];   // packed mode: the IE's fixed column width
    uint32_t val_off[NGZ_AGG_MAX_VALUES];
    uint8_t val_op[NGZ_AGG_MAX_VALUES];
    uint32_t row_bytes;
    uint64_t mask;              // capacity - 1
    uint32_t push_id;
    uint32_t port_bit;
    uint64_t coll_flip;         // collection time ms, sign bit flipped (unsigned order == signed order)
    uint32_t lds_ok;            // 1: no byte-wise OR values (wave results may be combined in LDS)
    uint32_t packed;            // 1: the whole group key packs into 63 bits (exact tag, no verify pass)
};

// dginfo: bit 0 usable (OK + has records + not late), bits 1..7 domain bit
__device__ __forceinline__ uint64_t mix64(uint64_t h, uint64_t v) {
    h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h *= 0xBF58476D1CE4E5B9ull;
    return h ^ (h >> 31);
}

__device__ __forceinline__ uint64_t slot_of(uint64_t h) {  // table position of a tag (tags may be packed keys)
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    return h ^ (h >> 33);
}

__device__ __forceinline__ uint32_t load_word(const uint8_t *p, uint32_t w, uint32_t j, bool str, bool &nul) {
    // word j (4 bytes, zero padded past w) of a w-byte value at p
    if ((w & 3) == 0 && !str) return *(const uint32_t *)(p + 4 * j);
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

__device__ __forceinline__ uint64_t key_hash(const AggSlotPlan &sp, const AggParams &P, uint64_t row, uint32_t win,
                                             uint32_t &present) {
    if (P.packed) {  // exact tag: bit 63 | window/60 (27 bits) | flow type | presence bits | key bits
        uint64_t x = ((uint64_t)(win / 60) << 1) | (sp.proto == 9);
        present = 0;
        for (uint32_t k = 0; k < P.n_keys; ++k) {
            const uint8_t *c = sp.key_col[k];
            const uint32_t w = sp.key_w[k];
            uint64_t v = 0;
            if (c) {
                present |= 1u << k;
                const uint8_t *q = c + row * w;
                v = w == 4 ? *(const uint32_t *)q : w == 2 ? *(const uint16_t *)q : w == 8 ? *(const uint64_t *)q : *q;
            }
            x = (((x << 1) | (c != nullptr)) << (8 * P.key_w[k])) | v;
        }
        return x | (1ull << 63);
    }
    uint64_t h = mix64(0x4E475A41474731ull, ((uint64_t)win << 8) | sp.proto);
    present = 0;
    for (uint32_t k = 0; k < P.n_keys; ++k) {
        const uint8_t *c = sp.key_col[k];
        const uint32_t w = sp.key_w[k];
        h = mix64(h, c ? (0x10000u | w) : 0u);
        if (!c) continue;
        present |= 1u << k;
        const uint8_t *p = c + row * w;
        bool nul = false;
        for (uint32_t j = 0; j < (w + 3) / 4; ++j) h = mix64(h, load_word(p, w, j, sp.key_str[k], nul));
    }
    return h ? h : 1;
}

__device__ __forceinline__ uint64_t load_value(const uint8_t *p, uint32_t w, uint8_t vc) {
    uint64_t v = 0;
    if (vc == VC_DTFRAC) {  // {u32 secs, u32 nanos} -> ordered (secs, nanos)
        const uint32_t s = *(const uint32_t *)p, ns = *(const uint32_t *)(p + 4);
        return ((uint64_t)s << 32) | ns;
    }
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

__global__ void k_agg_dgram(const ngz_dgram_hdr *__restrict__ hdr, const ngz_set_info *__restrict__ sets,
                            uint32_t n_sets, uint32_t n_dgrams, uint32_t *__restrict__ has_rec) {
    // has_rec[d] = 1 if the datagram carries >= 1 data record (in any set)
    for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < n_sets; s += gridDim.x * blockDim.x)
        if (sets[s].n && sets[s].dgram < n_dgrams) has_rec[sets[s].dgram] = 1;
}

__global__ void k_agg_ts(const ngz_dgram_hdr *__restrict__ hdr, const uint32_t *__restrict__ has_rec, uint32_t n,
                         uint32_t *__restrict__ ts) {
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < n; d += gridDim.x * blockDim.x)
        ts[d] = (hdr[d].status == NGZ_DG_OK && has_rec[d]) ? hdr[d].time : 0u;
}

__global__ void k_agg_late(const ngz_dgram_hdr *__restrict__ hdr, const uint32_t *__restrict__ has_rec,
                           const uint32_t *__restrict__ pmax, uint32_t n, uint32_t state_ct, uint64_t lateness_ms,
                           unsigned long long *__restrict__ dom_tab, uint8_t *__restrict__ dginfo,
                           unsigned int *__restrict__ err) {
    for (uint32_t d = blockIdx.x * blockDim.x + threadIdx.x; d < n; d += gridDim.x * blockDim.x) {
        uint8_t info = 0;
        if (hdr[d].status == NGZ_DG_OK && has_rec[d]) {
            uint32_t ct = state_ct;
            if (d > 0 && pmax[d - 1] > ct) ct = pmax[d - 1];
            const bool late = ct != 0 && (int64_t)hdr[d].time * 1000 < (int64_t)ct * 1000 - (int64_t)lateness_ms;
            if (!late) {
                // observation domain dictionary: linear probing over DOM_SLOTS entries (1<<32 | id)
                const unsigned long long key = (1ull << 32) | hdr[d].domain;
                uint32_t i = (hdr[d].domain * 2654435761u) % DOM_SLOTS, probes = 0;
                for (;;) {
                    unsigned long long cur = dom_tab[i];
                    if (cur == 0) {
                        cur = atomicCAS(&dom_tab[i], 0ull, key);
                        if (cur == 0) break;
                    }
                    if (cur == key) break;
                    i = (i + 1) % DOM_SLOTS;
                    if (++probes == DOM_SLOTS) { atomicOr(err, 1u); i = 0xFF; break; }
                }
                if (i != 0xFF) info = (uint8_t)(1u | (i << 1));
            } else {
                info = 0x80;  // late marker (bit 0 clear)
            }
        }
        dginfo[d] = info;
    }
}

__global__ void k_agg_setidx(const ngz_set_info *__restrict__ sets, const uint32_t *__restrict__ rstart,
                             uint32_t n_sets, uint32_t *__restrict__ setidx) {
    // one wave per set writes the set index of each of its records
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t n_waves = (gridDim.x * blockDim.x) >> 6;
    for (uint32_t s = wave; s < n_sets; s += n_waves) {
        const uint32_t n = sets[s].n, r0 = rstart[s];
        for (uint32_t i = lane; i < n; i += 64) setidx[r0 + i] = s;
    }
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

// Open-addressing insert of hash h: returns the group's row, the key written by the
// record that claimed the slot (64-bit CAS on the tag).
__device__ __forceinline__ uint8_t *group_row(const AggSlotPlan &sp, const AggParams &P, uint64_t row, uint32_t win,
                                              uint32_t kp, uint64_t h, unsigned long long *__restrict__ tags,
                                              uint8_t *__restrict__ rows, unsigned int *__restrict__ err,
                                              bool *claimed = nullptr) {
    uint64_t g = slot_of(h) & P.mask;
    bool won = false;
    if (claimed) *claimed = false;
    for (uint64_t probes = 0;; ++probes) {
        unsigned long long cur = tags[g];
        if (cur == 0) {
            cur = atomicCAS(&tags[g], 0ull, (unsigned long long)h);
            if (cur == 0) { won = true; break; }
        }
        if (cur == h) break;
        g = (g + 1) & P.mask;
        if (probes > P.mask) { atomicOr(err, 2u); return nullptr; }
    }
    uint8_t *R = rows + g * P.row_bytes;
    if (claimed) *claimed = won;
    if (won) {  // plain stores; read by later kernels only (flush, verify)
        *(uint32_t *)(R + 0) = win;
        *(uint32_t *)(R + 4) = sp.proto;
        *(uint32_t *)(R + 8) = kp;
        for (uint32_t k = 0; k < P.n_keys; ++k) {
            const uint8_t *c = sp.key_col[k];
            const uint32_t w = sp.key_w[k];
            uint32_t *dst = (uint32_t *)(R + P.key_off[k]);
            bool nul = false;
            if (c)
                for (uint32_t j = 0; j < (w + 3) / 4; ++j) dst[j] = load_word(c + row * w, w, j, sp.key_str[k], nul);
        }
    }
    return R;
}

// Operand of value v for the accumulator (signed min/max: sign bit flipped so unsigned order holds).
__device__ __forceinline__ uint64_t value_operand(const AggSlotPlan &sp, const AggParams &P, uint32_t v, uint64_t row) {
    const uint8_t vc = sp.val_vc[v];
    uint64_t x = load_value(sp.val_col[v] + row * sp.val_w[v], sp.val_w[v], vc);
    if (vc == VC_SINT && (P.val_op[v] == NGZ_AGG_MIN || P.val_op[v] == NGZ_AGG_MAX)) x ^= 1ull << 63;
    return x;
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

template <bool HOT = false>
__device__ __forceinline__ void apply_push_constants(uint8_t *R, const AggParams &P) {
    // per-push constants once per (group, push): collection time bounds, peer port
    if ((HOT || peek32(R + 36) != P.push_id) && atomicExch((unsigned int *)(R + 36), P.push_id) != P.push_id) {
        atomicMin((unsigned long long *)(R + 40), (unsigned long long)P.coll_flip);
        atomicMax((unsigned long long *)(R + 48), (unsigned long long)P.coll_flip);
        atomicOr((unsigned long long *)(R + 64), 1ull << P.port_bit);
    }
}

// One lane per record.  Lanes of a wave that share a group (same key hash) are first
// reduced across the wave and applied by one lane (wave pre-aggregation: low-cardinality
// keys would otherwise serialise on a few hot rows); once the largest remaining group of
// the wave has fewer than 4 records, every remaining lane applies its own record.  Wave
// results are combined further in a per-workgroup LDS table (CN entries) across all the
// tiles the workgroup walks, and applied to HBM once per workgroup: hot rows then see one
// set of atomics per workgroup instead of one per wave.
constexpr int CN = 64;
// (256, 4): 4 waves per SIMD (<= 128 VGPRs, no spills); the kernel is latency-bound
template <int MAXV>  // aggregated fields held in registers (value loads issued together, before any atomic)
__global__ __launch_bounds__(256, 4) void k_agg_insert(const ngz_dgram_hdr *__restrict__ hdr,
                                                    const ngz_set_info *__restrict__ sets,
                                                    const uint32_t *__restrict__ rstart,
                                                    const uint32_t *__restrict__ setidx, uint64_t n_rec,
                                                    uint32_t n_dgrams, uint32_t n_slots,
                                                    const uint8_t *__restrict__ dginfo,
                                                    const AggSlotPlan *__restrict__ plans, const AggParams P,
                                                    unsigned long long *__restrict__ tags, uint8_t *__restrict__ rows,
                                                    unsigned long long *__restrict__ late_count,
                                                    unsigned int *__restrict__ err) {
    __shared__ unsigned long long c_tag[CN], c_cnt[CN], c_tpl[CN], c_d0[CN], c_d1[CN];
    __shared__ unsigned long long c_val[CN][NGZ_AGG_MAX_VALUES];
    __shared__ uint32_t c_slot[CN], c_row[CN], c_win[CN], c_kp[CN], c_tmin[CN], c_tmax[CN], c_smax[CN], c_vp[CN];
    for (int e = threadIdx.x; e < CN; e += blockDim.x) {
        c_tag[e] = c_cnt[e] = c_tpl[e] = c_d0[e] = c_d1[e] = 0;
        c_tmin[e] = 0xFFFFFFFFu;
        c_tmax[e] = c_smax[e] = c_vp[e] = 0;
        for (uint32_t v = 0; v < P.n_vals; ++v) c_val[e][v] = P.val_op[v] == NGZ_AGG_MIN ? ~0ull : 0ull;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    for (uint64_t tile = blockIdx.x; tile * blockDim.x < n_rec; tile += gridDim.x) {
    const uint64_t t = tile * blockDim.x + threadIdx.x;
    bool valid = false, late = false;
    ngz_set_info si{};
    uint8_t info = 0;
    if (t < n_rec) {
        const uint32_t s = setidx[t];
        si = sets[s];
        if (si.dgram >= n_dgrams || si.slot >= n_slots) atomicOr(err, 16u);
        else {
            info = dginfo[si.dgram];
            late = info == 0x80;
            valid = (info & 1) && plans[si.slot].usable;
            if (valid) si.rec0 += (uint32_t)(t - rstart[s]);  // the record's row
        }
    }
    const uint64_t late_mask = __ballot(late);
    if (lane == 0 && late_mask) atomicAdd(late_count, (unsigned long long)__popcll(late_mask));
    const AggSlotPlan &sp = plans[valid ? si.slot : 0];
    const uint64_t row = si.rec0;
    uint32_t ts = 0, win = 0, kp = 0, sysup = 0;
    uint64_t h = 0, tpl = 0, dom0 = 0, dom1 = 0;
    if (valid) {
        ts = hdr[si.dgram].time;
        win = ts - ts % 60;  // get_window_start: minute floor
        h = key_hash(sp, P, row, win, kp);
        sysup = hdr[si.dgram].version == 9 ? hdr[si.dgram].sys_up_time : 0u;
        tpl = sp.tpl_bit;
        const uint32_t db = info >> 1;
        (db < 64 ? dom0 : dom1) = 1ull << (db & 63);
    }
    uint64_t xv[MAXV];
    uint32_t hv = 0, hb = 0;  // aggregated fields present: numeric (in xv) / byte-wise OR
#pragma unroll
    for (int v = 0; v < MAXV; ++v) {
        xv[v] = 0;
        if (valid && v < (int)P.n_vals && sp.val_col[v]) {
            if (sp.val_vc[v] == VC_BYTES) hb |= 1u << v;
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
    while (todo) {
        const int leader = __ffsll((unsigned long long)todo) - 1;
        const uint64_t lh = readlane64(h, leader);
        const bool mine = valid && ((todo >> lane) & 1) && h == lh;
        const uint64_t match = __ballot(mine);
        if (__popcll(match) < 4) break;
        todo &= ~match;
        const uint64_t cnt = __popcll(match);
        if (P.lds_ok) {
            // combine-table path: the leader claims the group's LDS entry and every matching
            // lane applies its own record with LDS atomics (no cross-lane reductions)
            int e0 = -1;
            if (lane == leader) {
                int i = (int)(slot_of(h) & (CN - 1));
                for (int probes = 0; probes < CN; ++probes, i = (i + 1) & (CN - 1)) {
                    unsigned long long cur = c_tag[i];
                    if (cur == 0) {
                        cur = atomicCAS(&c_tag[i], 0ull, (unsigned long long)h);
                        if (cur == 0) {
                            c_slot[i] = si.slot;
                            c_row[i] = (uint32_t)row;
                            c_win[i] = win;
                            c_kp[i] = kp;
                            e0 = i;
                            break;
                        }
                    }
                    if (cur == h) { e0 = i; break; }
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
        uint8_t *R = nullptr;
        int e = -1;
        if (lane == leader && P.lds_ok) {  // workgroup combine table (linear probing, CAS on the tag)
            int i = (int)(slot_of(h) & (CN - 1));
            for (int probes = 0; probes < CN; ++probes, i = (i + 1) & (CN - 1)) {
                unsigned long long cur = c_tag[i];
                if (cur == 0) {
                    cur = atomicCAS(&c_tag[i], 0ull, (unsigned long long)h);
                    if (cur == 0) {
                        c_slot[i] = si.slot;
                        c_row[i] = (uint32_t)row;
                        c_win[i] = win;
                        c_kp[i] = kp;
                        e = i;
                        break;
                    }
                }
                if (cur == h) { e = i; break; }
            }
            if (e >= 0) {
                atomicAdd(&c_cnt[e], (unsigned long long)cnt);
                atomicMin(&c_tmin[e], (uint32_t)tmin);
                atomicMax(&c_tmax[e], (uint32_t)tmax);
                atomicMax(&c_smax[e], (uint32_t)smax);
                atomicOr(&c_tpl[e], (unsigned long long)tpls);
                atomicOr(&c_d0[e], (unsigned long long)d0);
                atomicOr(&c_d1[e], (unsigned long long)d1);
            }
        }
        if (lane == leader && e < 0) {
            R = group_row(sp, P, row, win, kp, h, tags, rows, err);
            if (R) {
                atomicAdd((unsigned long long *)(R + 16), (unsigned long long)cnt);
                // hot rows: fire-and-forget atomics (a load of a contended line costs more)
                atomicMin((unsigned int *)(R + 24), (uint32_t)tmin);
                atomicMax((unsigned int *)(R + 28), (uint32_t)tmax);
                if (smax) atomicMax((unsigned int *)(R + 32), (uint32_t)smax);
                atomicOr((unsigned long long *)(R + 56), (unsigned long long)tpls);
                if (d0) atomicOr((unsigned long long *)(R + 72), (unsigned long long)d0);
                if (d1) atomicOr((unsigned long long *)(R + 80), (unsigned long long)d1);
                apply_push_constants<true>(R, P);
            }
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
            uint64_t r = 0;
            if (any_num) switch (op) {
            case NGZ_AGG_ADD: r = wave_reduce<R_ADD>(x); break;
            case NGZ_AGG_MIN: r = wave_reduce<R_MIN>(x); break;
            case NGZ_AGG_MAX: r = wave_reduce<R_MAX>(x); break;
            default: r = wave_reduce<R_OR>(x); break;
            }
            if (lane == leader && any_num) {
                if (e >= 0) {
                    unsigned long long *c = &c_val[e][v];
                    switch (op) {
                    case NGZ_AGG_ADD: atomicAdd(c, (unsigned long long)r); break;
                    case NGZ_AGG_MIN: atomicMin(c, (unsigned long long)r); break;
                    case NGZ_AGG_MAX: atomicMax(c, (unsigned long long)r); break;
                    default: atomicOr(c, (unsigned long long)r); break;
                    }
                } else if (R) {
                    apply_value_hot(R + P.val_off[v], op, r);
                }
            }
            if (any_bytes) {  // byte ORs: each matching lane ORs its words into the leader's row
                const uint64_t Rl = readlane64((uint64_t)R, leader);
                if (bytes && Rl) {
                    const uint32_t w = sp.val_w[v];
                    bool nul = false;
                    for (uint32_t j = 0; j < (w + 3) / 4; ++j) {
                        const uint32_t y = load_word(sp.val_col[v] + row * w, w, j, false, nul);
                        or32((uint8_t *)Rl + P.val_off[v] + 4 * j, y);
                    }
                }
            }
        }
        if (lane == leader && e >= 0 && vp) atomicOr(&c_vp[e], vp);
        if (lane == leader && R && vp) atomicOr((unsigned int *)(R + 12), vp);
    }
    if (!(valid && ((todo >> lane) & 1))) continue;
    // per-record path
    bool claimed;
    uint8_t *R = group_row(sp, P, row, win, kp, h, tags, rows, err, &claimed);
    if (!R) continue;
    atomicAdd((unsigned long long *)(R + 16), 1ull);
    if (claimed) {  // a row this record just claimed: a pre-load would only read the identities back
        atomicMin((unsigned int *)(R + 24), ts);
        atomicMax((unsigned int *)(R + 28), ts);
        if (sysup) atomicMax((unsigned int *)(R + 32), sysup);
        atomicOr((unsigned long long *)(R + 56), (unsigned long long)tpl);
        atomicOr((unsigned long long *)(R + (dom0 ? 72 : 80)), (unsigned long long)(dom0 | dom1));
        apply_push_constants<true>(R, P);
    } else {
        min32(R + 24, ts);
        max32(R + 28, ts);
        max32(R + 32, sysup);
        or64(R + 56, tpl);
        or64(R + (dom0 ? 72 : 80), dom0 | dom1);
        apply_push_constants(R, P);
    }
#pragma unroll
    for (int v = 0; v < MAXV; ++v) {
        if (v >= (int)P.n_vals) break;
        uint8_t *dst = R + P.val_off[v];
        if ((hv >> v) & 1) {
            if (claimed) apply_value_hot(dst, P.val_op[v], xv[v]);
            else apply_value(dst, P.val_op[v], xv[v]);
        } else if ((hb >> v) & 1) {  // BoolMapOr over bytes (mac, mpls label, octetArray, u256)
            const uint32_t w = sp.val_w[v];
            bool nul = false;
            for (uint32_t j = 0; j < (w + 3) / 4; ++j) or32(dst + 4 * j, load_word(sp.val_col[v] + row * w, w, j, false, nul));
        }
    }
    if (claimed) atomicOr((unsigned int *)(R + 12), hv | hb);
    else or32(R + 12, hv | hb);
    }  // tiles
    __syncthreads();
    for (int e = threadIdx.x; e < CN; e += blockDim.x) {  // the workgroup's combined groups -> HBM
        const unsigned long long h = c_tag[e];
        if (!h) continue;
        uint8_t *R = group_row(plans[c_slot[e]], P, c_row[e], c_win[e], c_kp[e], h, tags, rows, err);
        if (!R) continue;
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

__global__ __launch_bounds__(256) void k_agg_verify(const ngz_dgram_hdr *__restrict__ hdr,
                                                    const ngz_set_info *__restrict__ sets,
                                                    const uint32_t *__restrict__ rstart,
                                                    const uint32_t *__restrict__ setidx, uint64_t n_rec,
                                                    uint32_t n_dgrams, uint32_t n_slots,
                                                    const uint8_t *__restrict__ dginfo,
                                                    const AggSlotPlan *__restrict__ plans, const AggParams P,
                                                    const unsigned long long *__restrict__ tags,
                                                    const uint8_t *__restrict__ rows, unsigned int *__restrict__ err) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n_rec) return;
    const uint32_t s = setidx[t];
    const ngz_set_info si = sets[s];
    if (si.dgram >= n_dgrams || si.slot >= n_slots) return;
    if (!(dginfo[si.dgram] & 1)) return;
    const AggSlotPlan &sp = plans[si.slot];
    if (!sp.usable) return;
    const uint64_t row = si.rec0 + (uint32_t)(t - rstart[s]);
    const uint32_t ts = hdr[si.dgram].time;
    const uint32_t win = ts - ts % 60;
    uint32_t kp;
    const uint64_t h = key_hash(sp, P, row, win, kp);
    uint64_t g = slot_of(h) & P.mask;
    for (uint64_t probes = 0; tags[g] != h; ++probes) {
        g = (g + 1) & P.mask;
        if (probes > P.mask) { atomicOr(err, 4u); return; }
    }
    const uint8_t *R = rows + g * P.row_bytes;
    bool same = *(const uint32_t *)(R + 0) == win && *(const uint32_t *)(R + 4) == sp.proto &&
                *(const uint32_t *)(R + 8) == kp;
    for (uint32_t k = 0; k < P.n_keys && same; ++k) {
        const uint8_t *c = sp.key_col[k];
        if (!c) continue;
        const uint32_t w = sp.key_w[k];
        bool nul = false;
        for (uint32_t j = 0; j < (w + 3) / 4; ++j)
            same = same && ((const uint32_t *)(R + P.key_off[k]))[j] == load_word(c + row * w, w, j, sp.key_str[k], nul);
    }
    if (!same) atomicOr(err, 8u);
}

__global__ void k_agg_init(uint8_t *__restrict__ rows, uint64_t n_groups, uint32_t row_bytes,
                           const uint32_t *__restrict__ ident, uint32_t ident_words) {
    // every row <- the identity row (min fields at their maximum)
    const uint64_t n_words = n_groups * (row_bytes / 4);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_words;
         i += (uint64_t)gridDim.x * blockDim.x)
        ((uint32_t *)rows)[i] = ident[i % ident_words];
}

__global__ void k_agg_count(const unsigned long long *__restrict__ tags, uint64_t n_groups,
                            unsigned long long *__restrict__ cursor) {
    uint32_t c = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n_groups;
         g += (uint64_t)gridDim.x * blockDim.x)
        c += tags[g] != 0;
    if (c) atomicAdd(cursor, (unsigned long long)c);
}

__global__ void k_agg_compact(const unsigned long long *__restrict__ tags, const uint8_t *__restrict__ rows,
                              uint64_t n_groups, uint32_t row_bytes, uint8_t *__restrict__ out,
                              unsigned long long *__restrict__ cursor) {
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        if (!tags[g]) continue;
        const uint64_t o = atomicAdd(cursor, 1ull);
        const uint32_t *src = (const uint32_t *)(rows + g * row_bytes);
        uint32_t *dst = (uint32_t *)(out + o * row_bytes);
        for (uint32_t i = 0; i < row_bytes / 4; ++i) dst[i] = src[i];
    }
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
    std::vector<ngz_agg_field> keys, vals;
    uint64_t window_ms = 0, lateness_ms = 0;
    uint64_t cap = 0;
    AggParams P{};
    // per-value state fixed at first sight: column width and value class
    std::vector<int> val_w, val_vc, key_w;
    std::vector<uint8_t> val_dtype;
    // dictionaries (host) for template ids and peer ports
    std::vector<uint32_t> templates;
    std::vector<uint16_t> ports;
    uint32_t current_time = 0;  // the peer's event time (seconds), 0 = none yet
    uint32_t push_id = 0;
    float t_push = 0;
    // device
    unsigned long long *tags = nullptr;
    uint8_t *rows = nullptr;
    uint32_t *ident = nullptr;
    unsigned long long *dom_tab = nullptr;
    unsigned int *err = nullptr;
    unsigned long long *late = nullptr;
    unsigned long long *cursor = nullptr;
    AggSlotPlan *plans = nullptr;
    uint32_t plans_cap = 0;
    // scratch, grown on demand
    void *scratch = nullptr;
    size_t scratch_cap = 0;
    uint32_t *setidx = nullptr;
    uint64_t setidx_cap = 0;
};

namespace {

int fail(ngz_agg *a, int rc, const std::string &msg) {
    if (a) a->last_error = msg;
    return rc;
}

#define AGG_HIP(a, x)                                                                     \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) return fail(a, NGZ_E_DEVICE, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

uint32_t grid_for(uint64_t n, uint32_t block = 256, uint32_t max_blocks = 8192) {
    uint64_t g = (n + block - 1) / block;
    if (g == 0) g = 1;
    return (uint32_t)std::min<uint64_t>(g, max_blocks);
}

int reset_table(ngz_agg *a) {
    AGG_HIP(a, hipMemsetAsync(a->tags, 0, a->cap * 8, a->stream));
    hipLaunchKernelGGL(k_agg_init, dim3(8192), dim3(256), 0, a->stream, a->rows, a->cap, a->P.row_bytes, a->ident,
                       a->P.row_bytes / 4);
    AGG_HIP(a, hipGetLastError());
    return NGZ_OK;
}

// Which reductions the device runs for an IE data type (generator.rs:580-629,
// config.rs:212-250).  Returns the value class or -1 with a reason.
int value_class(const ngzh::IeRow *r, uint8_t op, std::string &why) {
    using namespace ngzh;
    const uint8_t dt = r ? r->dtype : DT_octetArray;
    const bool subreg = r && (r->flags & 4);
    const bool tcp = r && (r->flags & 2);
    const bool integer = dt == DT_unsigned8 || dt == DT_unsigned16 || dt == DT_unsigned32 || dt == DT_unsigned64 ||
                         dt == DT_signed8 || dt == DT_signed16 || dt == DT_signed32 || dt == DT_signed64;
    const bool sgn = dt == DT_signed8 || dt == DT_signed16 || dt == DT_signed32 || dt == DT_signed64;
    switch (op) {
    case NGZ_AGG_ADD:
        if (dt == DT_float32 || dt == DT_float64) { why = "float addition is order dependent (not on device)"; return -1; }
        if (!integer || subreg || tcp) { why = "field does not support arithmetic operations"; return -1; }
        return sgn ? VC_SINT : VC_UINT;
    case NGZ_AGG_MIN:
    case NGZ_AGG_MAX:
        if (dt == DT_float32 || dt == DT_float64 || dt == DT_macAddress || dt == DT_ipv6Address || subreg || tcp ||
            dt == DT_boolean) {
            why = "comparison of this type is not on the device yet";
            return -1;
        }
        if (integer || dt == DT_ipv4Address || dt == DT_dateTimeSeconds) return sgn ? VC_SINT : VC_UINT;
        if (dt == DT_dateTimeMilliseconds) return VC_SINT;
        if (dt == DT_dateTimeMicroseconds || dt == DT_dateTimeNanoseconds) return VC_DTFRAC;
        why = "field does not support comparison operations";
        return -1;
    case NGZ_AGG_OR:
        if (dt == DT_float32 || dt == DT_float64 || dt == DT_string || dt == DT_basicList ||
            dt == DT_subTemplateList || dt == DT_subTemplateMultiList || dt == DT_dateTimeSeconds ||
            dt == DT_dateTimeMilliseconds || dt == DT_dateTimeMicroseconds || dt == DT_dateTimeNanoseconds) {
            why = "field does not support bitwise operations";
            return -1;
        }
        if (subreg && !tcp) { why = "bitwise OR of sub-registry values is not on the device yet"; return -1; }
        if (integer || dt == DT_boolean || dt == DT_ipv4Address) return VC_UINT;
        return VC_BYTES;  // octetArray, macAddress, ipv6Address, unsigned256
    }
    why = "unknown op";
    return -1;
}

}  // namespace

extern "C" {

int ngz_agg_create(int device, const ngz_agg_field *fields, uint32_t n_fields, uint64_t window_ms,
                   uint64_t lateness_ms, uint64_t capacity, ngz_agg **out) {
    if (!out || (n_fields && !fields)) return NGZ_E_INVALID;
    *out = nullptr;
    if (window_ms == 0 || lateness_ms > window_ms) return NGZ_E_INVALID;  // AggregationConfig::validate
    ngz_agg *a = new ngz_agg();
    a->device = device;
    a->window_ms = window_ms;
    a->lateness_ms = lateness_ms;
    for (uint32_t i = 0; i < n_fields; ++i) {
        const ngz_agg_field &f = fields[i];
        if (f.op > NGZ_AGG_OR) { delete a; return NGZ_E_INVALID; }
        if (f.op == NGZ_AGG_KEY) a->keys.push_back(f);
        else {
            std::string why;
            if (value_class(ngzh::ie_find(f.pen, f.ie_id), f.op, why) < 0) { delete a; return NGZ_E_INVALID; }
            a->vals.push_back(f);
        }
    }
    if (a->keys.size() > NGZ_AGG_MAX_KEYS || a->vals.size() > NGZ_AGG_MAX_VALUES) { delete a; return NGZ_E_LIMIT; }
    a->key_w.assign(a->keys.size(), -1);
    a->val_w.assign(a->vals.size(), -1);
    a->val_vc.assign(a->vals.size(), -1);
    // row layout: header, keys (IE width rounded to 4; the width is fixed by the IE's Rust type except
    // for octet arrays, whose width is fixed at first sight), values (8 B; byte ORs up to 32 B)
    uint32_t off = ROW_HDR;
    AggParams &P = a->P;
    P.n_keys = (uint32_t)a->keys.size();
    P.n_vals = (uint32_t)a->vals.size();
    for (uint32_t k = 0; k < P.n_keys; ++k) {
        const ngzh::IeRow *r = ngzh::ie_find(a->keys[k].pen, a->keys[k].ie_id);
        uint32_t w = 32;  // octetArray / string keys: up to 32 bytes on the device
        if (r) {
            switch (r->dtype) {
            case ngzh::DT_unsigned8: case ngzh::DT_signed8: case ngzh::DT_boolean: w = 4; break;
            case ngzh::DT_unsigned16: case ngzh::DT_signed16: w = 4; break;
            case ngzh::DT_unsigned32: case ngzh::DT_signed32: case ngzh::DT_float32: case ngzh::DT_ipv4Address:
            case ngzh::DT_dateTimeSeconds: w = 4; break;
            case ngzh::DT_unsigned64: case ngzh::DT_signed64: case ngzh::DT_float64:
            case ngzh::DT_dateTimeMilliseconds: case ngzh::DT_dateTimeMicroseconds:
            case ngzh::DT_dateTimeNanoseconds: w = 8; break;
            case ngzh::DT_macAddress: w = 8; break;
            case ngzh::DT_ipv6Address: w = 16; break;
            default: w = 32; break;
            }
        }
        P.key_off[k] = off;
        off += w;
        // packed-key eligibility: IEs whose column width is fixed by the Rust type (1/2/4/8 bytes)
        int fw = 0;
        if (r) switch (r->dtype) {
            case ngzh::DT_unsigned8: case ngzh::DT_signed8: case ngzh::DT_boolean: fw = 1; break;
            case ngzh::DT_unsigned16: fw = (r->flags & 2) ? 1 : 2; break;  // tcpControlBits column is u8
            case ngzh::DT_signed16: fw = 2; break;
            case ngzh::DT_unsigned32: case ngzh::DT_signed32: case ngzh::DT_ipv4Address:
            case ngzh::DT_dateTimeSeconds: case ngzh::DT_float32: fw = 4; break;
            default: fw = 0; break;
        }
        P.key_w[k] = (uint32_t)fw;
    }
    if (off - ROW_HDR > NGZ_AGG_MAX_KEY_BYTES + 64) { delete a; return NGZ_E_LIMIT; }
    off = (off + 7) & ~7u;
    for (uint32_t v = 0; v < P.n_vals; ++v) {
        std::string why;
        const int vc = value_class(ngzh::ie_find(a->vals[v].pen, a->vals[v].ie_id), a->vals[v].op, why);
        P.val_off[v] = off;
        P.val_op[v] = a->vals[v].op;
        off += vc == VC_BYTES ? 32 : 8;
    }
    P.row_bytes = (off + 7) & ~7u;
    {
        uint32_t bits = 28;  // window/60 + flow type
        bool ok = true;
        for (uint32_t k = 0; k < P.n_keys; ++k) {
            ok = ok && P.key_w[k] != 0;
            bits += 1 + 8 * P.key_w[k];
        }
        P.packed = ok && bits <= 63 && getenv("NGZ_AGG_NO_PACK") == nullptr;
    }
    P.lds_ok = 1;
    for (uint32_t v = 0; v < P.n_vals; ++v) {
        std::string why;
        if (value_class(ngzh::ie_find(a->vals[v].pen, a->vals[v].ie_id), a->vals[v].op, why) == VC_BYTES) P.lds_ok = 0;
    }
    uint64_t cap = 1024;
    while (cap < 2 * std::max<uint64_t>(capacity, 1)) cap <<= 1;
    a->cap = cap;
    P.mask = cap - 1;
    // identity row: min fields at their maximum
    std::vector<uint32_t> ident(P.row_bytes / 4, 0);
    ident[24 / 4] = 0xFFFFFFFFu;                      // min_export_time
    ident[40 / 4] = ident[44 / 4] = 0xFFFFFFFFu;      // min_collection (flipped order)
    for (uint32_t v = 0; v < P.n_vals; ++v)
        if (P.val_op[v] == NGZ_AGG_MIN) ident[P.val_off[v] / 4] = ident[P.val_off[v] / 4 + 1] = 0xFFFFFFFFu;
    int rc = NGZ_OK;
    auto bail = [&](int r, const char *what) {
        a->last_error = what;
        ngz_agg_destroy(a);
        return r;
    };
    if (hipSetDevice(device) != hipSuccess) return bail(NGZ_E_DEVICE, "hipSetDevice");
    if (hipStreamCreateWithFlags(&a->stream, hipStreamNonBlocking) != hipSuccess) return bail(NGZ_E_DEVICE, "stream");
    hipEventCreate(&a->ev0);
    hipEventCreate(&a->ev1);
    if (hipMalloc(&a->tags, cap * 8) != hipSuccess || hipMalloc(&a->rows, cap * P.row_bytes) != hipSuccess ||
        hipMalloc(&a->ident, P.row_bytes) != hipSuccess || hipMalloc(&a->dom_tab, DOM_SLOTS * 8) != hipSuccess ||
        hipMalloc(&a->err, 4) != hipSuccess || hipMalloc(&a->late, 8) != hipSuccess ||
        hipMalloc(&a->cursor, 8) != hipSuccess)
        return bail(NGZ_E_NOMEM, "hipMalloc (group table)");
    hipMemcpy(a->ident, ident.data(), P.row_bytes, hipMemcpyHostToDevice);
    hipMemset(a->dom_tab, 0, DOM_SLOTS * 8);
    hipMemset(a->err, 0, 4);
    rc = reset_table(a);
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
    hipFree(a->dom_tab);
    hipFree(a->err);
    hipFree(a->late);
    hipFree(a->cursor);
    hipFree(a->plans);
    hipFree(a->scratch);
    hipFree(a->setidx);
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
        if (val_width) val_width[v] = (uint16_t)std::max(a->val_w[v], 0);
    }
    return NGZ_OK;
}

int ngz_agg_push(ngz_agg *a, ngz_ctx *ctx, const ngz_batch_out *out, uint16_t peer_port, int64_t collection_time_ms,
                 uint64_t *late_records, void *hip_stream) {
    if (!a || !ctx || !out) return NGZ_E_INVALID;
    if (late_records) *late_records = 0;
    AGG_HIP(a, hipSetDevice(a->device));
    if (hip_stream) AGG_HIP(a, hipStreamSynchronize((hipStream_t)hip_stream));
    // port dictionary
    uint32_t port_bit = 0;
    {
        auto it = std::find(a->ports.begin(), a->ports.end(), peer_port);
        if (it == a->ports.end()) {
            if (a->ports.size() >= NGZ_AGG_SET_BITS) return fail(a, NGZ_AGG_E_OVERFLOW, "more than 64 peer ports");
            a->ports.push_back(peer_port);
            it = a->ports.end() - 1;
        }
        port_bit = (uint32_t)(it - a->ports.begin());
    }
    // per-slot plans: FieldRef lookup (IE, occurrence among non-scope fields), types fixed at first sight
    const uint32_t S = out->n_slots;
    std::vector<AggSlotPlan> plans(std::max<uint32_t>(S, 1));
    std::vector<ngz_field_info> fi;
    for (uint32_t s = 0; s < S; ++s) {
        AggSlotPlan &sp = plans[s];
        memset(&sp, 0, sizeof sp);
        const ngz_slot_info &si = out->slots[s];
        sp.proto = si.proto;
        if (!si.n_records || !si.columns) continue;
        const int nf = ngz_slot_fields(ctx, s, nullptr, 0);
        if (nf < 0) return fail(a, NGZ_E_INVALID, "ngz_slot_fields");
        fi.resize(std::max(nf, 1));
        ngz_slot_fields(ctx, s, fi.data(), (uint32_t)nf);
        const uint32_t tkey = ((uint32_t)si.proto << 16) | si.template_id;
        auto it = std::find(a->templates.begin(), a->templates.end(), tkey);
        if (it == a->templates.end()) {
            if (a->templates.size() >= NGZ_AGG_SET_BITS) return fail(a, NGZ_AGG_E_OVERFLOW, "more than 64 template ids");
            a->templates.push_back(tkey);
            it = a->templates.end() - 1;
        }
        sp.tpl_bit = 1ull << (it - a->templates.begin());
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
            if (f.kind == NGZ_K_VLEN || f.kind == NGZ_K_FAIL)
                return fail(a, NGZ_E_LIMIT, "variable-length key field (not on the device yet)");
            const uint32_t room = (k + 1 < a->P.n_keys ? a->P.key_off[k + 1] : ((a->P.n_vals ? a->P.val_off[0] : a->P.row_bytes))) - a->P.key_off[k];
            if (f.width > room) return fail(a, NGZ_E_LIMIT, "key field wider than its row slot");
            if (a->P.packed && f.width != a->P.key_w[k])
                return fail(a, NGZ_E_LIMIT, "key column width differs from the IE's width");
            sp.key_col[k] = si.columns + (uint64_t)si.capacity * f.col_off;
            sp.key_w[k] = f.width;
            sp.key_str[k] = f.kind == NGZ_K_STR;
            if (a->key_w[k] < 0) a->key_w[k] = f.width;
        }
        for (uint32_t v = 0; v < a->P.n_vals; ++v) {
            const int i = find_field(a->vals[v]);
            if (i < 0) continue;
            const ngz_field_info &f = fi[i];
            std::string why;
            const int vc = value_class(ngzh::ie_find(a->vals[v].pen, a->vals[v].ie_id), a->vals[v].op, why);
            if (f.kind == NGZ_K_VLEN || f.kind == NGZ_K_FAIL || (vc == VC_BYTES && f.width > 32))
                return fail(a, NGZ_E_LIMIT, "aggregated field is variable-length or wider than 32 bytes");
            if (vc != VC_BYTES && vc != VC_DTFRAC && f.width != 1 && f.width != 2 && f.width != 4 && f.width != 8)
                return fail(a, NGZ_E_LIMIT, "aggregated integer field of odd width");
            if (a->val_w[v] >= 0 && a->val_w[v] != f.width)
                return fail(a, NGZ_E_LIMIT, "aggregated field width differs between templates");
            a->val_w[v] = f.width;
            a->val_vc[v] = vc;
            sp.val_col[v] = si.columns + (uint64_t)si.capacity * f.col_off;
            sp.val_w[v] = f.width;
            sp.val_vc[v] = (uint8_t)vc;
        }
        sp.usable = 1;
    }
    const uint32_t D = out->n_dgrams, NS = out->n_sets;
    if (!D || !NS) return NGZ_OK;
    // scratch: has_rec[D], ts[D], pm[D], dginfo[D], cnt/rstart[NS+1], cub temp; then setidx[R]
    size_t cub_max = 0, cub_sum = 0;
    hipcub::DeviceScan::InclusiveScan(nullptr, cub_max, (uint32_t *)nullptr, (uint32_t *)nullptr, hipcub::Max(), D,
                                      a->stream);
    hipcub::DeviceScan::ExclusiveSum(nullptr, cub_sum, (uint32_t *)nullptr, (uint32_t *)nullptr, NS + 1, a->stream);
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t o_has = 0, o_ts = o_has + al(4ull * D), o_pm = o_ts + al(4ull * D), o_dg = o_pm + al(4ull * D),
                 o_cnt = o_dg + al(D), o_rs = o_cnt + al(4ull * (NS + 1)), o_cub = o_rs + al(4ull * (NS + 1)),
                 need = o_cub + al(std::max(cub_max, cub_sum));
    if (need > a->scratch_cap) {
        hipFree(a->scratch);
        a->scratch = nullptr;
        if (hipMalloc(&a->scratch, need) != hipSuccess) { a->scratch_cap = 0; return fail(a, NGZ_E_NOMEM, "scratch"); }
        a->scratch_cap = need;
    }
    uint8_t *sc = (uint8_t *)a->scratch;
    uint32_t *has_rec = (uint32_t *)(sc + o_has), *ts = (uint32_t *)(sc + o_ts), *pm = (uint32_t *)(sc + o_pm);
    uint8_t *dginfo = sc + o_dg;
    uint32_t *cnt = (uint32_t *)(sc + o_cnt), *rstart = (uint32_t *)(sc + o_rs);
    void *cub_tmp = sc + o_cub;
    if (S > a->plans_cap) {
        hipFree(a->plans);
        a->plans = nullptr;
        if (hipMalloc(&a->plans, sizeof(AggSlotPlan) * S) != hipSuccess) { a->plans_cap = 0; return fail(a, NGZ_E_NOMEM, "plans"); }
        a->plans_cap = S;
    }
    hipStream_t st = a->stream;
    AGG_HIP(a, hipMemcpyAsync(a->plans, plans.data(), sizeof(AggSlotPlan) * S, hipMemcpyHostToDevice, st));
    AggParams P = a->P;
    P.push_id = ++a->push_id;
    P.port_bit = port_bit;
    P.coll_flip = (uint64_t)collection_time_ms ^ (1ull << 63);
    AGG_HIP(a, hipEventRecord(a->ev0, st));
    AGG_HIP(a, hipMemsetAsync(has_rec, 0, 4ull * D, st));
    AGG_HIP(a, hipMemsetAsync(a->late, 0, 8, st));
    AGG_HIP(a, hipMemsetAsync(a->err, 0, 4, st));
    const ngz_dgram_hdr *hdr = out->dgrams;
    const ngz_set_info *sets = out->sets;
    hipLaunchKernelGGL(k_agg_dgram, dim3(grid_for(NS)), dim3(256), 0, st, hdr, sets, NS, D, has_rec);
    hipLaunchKernelGGL(k_agg_ts, dim3(grid_for(D)), dim3(256), 0, st, hdr, has_rec, D, ts);
    size_t tmp = cub_max;
    AGG_HIP(a, hipcub::DeviceScan::InclusiveScan(cub_tmp, tmp, ts, pm, hipcub::Max(), D, st));
    hipLaunchKernelGGL(k_agg_late, dim3(grid_for(D)), dim3(256), 0, st, hdr, has_rec, pm, D, a->current_time,
                       a->lateness_ms, a->dom_tab, dginfo, a->err);
    // record starts of every set: n copied out of the set table (stride 16 B) then scanned
    AGG_HIP(a, hipMemsetAsync(cnt + NS, 0, 4, st));
    AGG_HIP(a, hipMemcpy2DAsync(cnt, 4, (const uint8_t *)sets + offsetof(ngz_set_info, n), sizeof(ngz_set_info), 4, NS,
                                hipMemcpyDeviceToDevice, st));
    tmp = cub_sum;
    AGG_HIP(a, hipcub::DeviceScan::ExclusiveSum(cub_tmp, tmp, cnt, rstart, NS + 1, st));
    // records of the set table (synchronises once: the grid of the record kernels depends on it)
    uint32_t n_rec = 0;
    AGG_HIP(a, hipMemcpyAsync(&n_rec, rstart + NS, 4, hipMemcpyDeviceToHost, st));
    AGG_HIP(a, hipStreamSynchronize(st));
    if ((uint64_t)n_rec * 4 > a->setidx_cap) {
        hipFree(a->setidx);
        a->setidx = nullptr;
        a->setidx_cap = 0;
        if (hipMalloc(&a->setidx, std::max<uint64_t>(n_rec, 1) * 4) != hipSuccess) return fail(a, NGZ_E_NOMEM, "setidx");
        a->setidx_cap = std::max<uint64_t>(n_rec, 1) * 4;
    }
    uint32_t *setidx = a->setidx;
    hipLaunchKernelGGL(k_agg_setidx, dim3(grid_for(64ull * NS, 256, 4096)), dim3(256), 0, st, sets, rstart, NS, setidx);
    AGG_HIP(a, hipGetLastError());
    const uint32_t blocks = (uint32_t)((n_rec + 255) / 256);
    // insert grid: workgroups walk tiles of 256 records (NGZ_AGG_GRID overrides the default 4096)
    static const uint32_t grid_cap = getenv("NGZ_AGG_GRID") ? (uint32_t)std::max(1, atoi(getenv("NGZ_AGG_GRID"))) : 4096u;
    const uint32_t ig = std::min<uint32_t>(blocks, grid_cap);
    if (n_rec) {
        if (P.n_vals <= 8)
            hipLaunchKernelGGL(k_agg_insert<8>, dim3(ig), dim3(256), 0, st, hdr, sets,
                               rstart, setidx, (uint64_t)n_rec, D, S, dginfo, a->plans, P, a->tags, a->rows, a->late,
                               a->err);
        else
            hipLaunchKernelGGL(k_agg_insert<NGZ_AGG_MAX_VALUES>, dim3(ig), dim3(256), 0,
                               st, hdr, sets, rstart, setidx, (uint64_t)n_rec, D, S, dginfo, a->plans, P, a->tags,
                               a->rows, a->late, a->err);
        if (!P.packed) hipLaunchKernelGGL(k_agg_verify, dim3(blocks), dim3(256), 0, st, hdr, sets, rstart, setidx, (uint64_t)n_rec,
                           D, S, dginfo, a->plans, P, a->tags, a->rows, a->err);
    }
    AGG_HIP(a, hipGetLastError());
    AGG_HIP(a, hipEventRecord(a->ev1, st));
    uint32_t last_pm = 0, errv = 0;
    unsigned long long late = 0;
    AGG_HIP(a, hipMemcpyAsync(&last_pm, pm + (D - 1), 4, hipMemcpyDeviceToHost, st));
    AGG_HIP(a, hipMemcpyAsync(&errv, a->err, 4, hipMemcpyDeviceToHost, st));
    AGG_HIP(a, hipMemcpyAsync(&late, a->late, 8, hipMemcpyDeviceToHost, st));
    AGG_HIP(a, hipStreamSynchronize(st));
    hipEventElapsedTime(&a->t_push, a->ev0, a->ev1);
    if (last_pm > a->current_time) a->current_time = last_pm;
    if (late_records) *late_records = late;
    if (errv & 1) return fail(a, NGZ_AGG_E_OVERFLOW, "more than 128 observation domains");
    if (errv & 6) return fail(a, NGZ_AGG_E_OVERFLOW, "group table full");
    if (errv & 8) return fail(a, NGZ_AGG_E_COLLISION, "64-bit key hash collision");
    if (errv & 16) return fail(a, NGZ_E_INVALID, "set table entry out of range");
    return NGZ_OK;
}

int64_t ngz_agg_groups(ngz_agg *a) {
    if (!a) return NGZ_E_INVALID;
    AGG_HIP(a, hipSetDevice(a->device));
    unsigned long long n = 0;
    AGG_HIP(a, hipMemsetAsync(a->cursor, 0, 8, a->stream));
    hipLaunchKernelGGL(k_agg_count, dim3(grid_for(a->cap)), dim3(256), 0, a->stream, a->tags, a->cap, a->cursor);
    AGG_HIP(a, hipMemcpyAsync(&n, a->cursor, 8, hipMemcpyDeviceToHost, a->stream));
    AGG_HIP(a, hipStreamSynchronize(a->stream));
    return (int64_t)n;
}

int64_t ngz_agg_flush(ngz_agg *a, void *dst, uint64_t cap) {
    if (!a) return NGZ_E_INVALID;
    const int64_t n = ngz_agg_groups(a);
    if (n < 0) return n;
    const uint32_t RB = a->P.row_bytes;
    if ((uint64_t)n * RB > cap || (n && !dst)) return fail(a, NGZ_E_INVALID, "flush buffer too small");
    if (n) {
        uint8_t *tmp = nullptr;
        if (hipMalloc(&tmp, (uint64_t)n * RB) != hipSuccess) return fail(a, NGZ_E_NOMEM, "flush staging");
        AGG_HIP(a, hipMemsetAsync(a->cursor, 0, 8, a->stream));
        hipLaunchKernelGGL(k_agg_compact, dim3(grid_for(a->cap)), dim3(256), 0, a->stream, a->tags, a->rows, a->cap, RB,
                           tmp, a->cursor);
        hipError_t e = hipMemcpyAsync(dst, tmp, (uint64_t)n * RB, hipMemcpyDeviceToHost, a->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(a->stream);
        hipFree(tmp);
        if (e != hipSuccess) return fail(a, NGZ_E_DEVICE, hipGetErrorString(e));
        // host finish: collection times back to signed, per-push marker cleared, values at the IE width
        for (int64_t g = 0; g < n; ++g) {
            uint8_t *R = (uint8_t *)dst + (uint64_t)g * RB;
            uint64_t c;
            memcpy(&c, R + 40, 8); c ^= 1ull << 63; memcpy(R + 40, &c, 8);
            memcpy(&c, R + 48, 8); c ^= 1ull << 63; memcpy(R + 48, &c, 8);
            memset(R + 36, 0, 4);
            uint32_t vp;
            memcpy(&vp, R + 12, 4);
            for (uint32_t v = 0; v < a->P.n_vals; ++v) {
                if (a->val_vc[v] == VC_BYTES || a->val_vc[v] < 0) continue;
                uint8_t *p = R + a->P.val_off[v];
                uint64_t x;
                memcpy(&x, p, 8);
                if (!(vp >> v & 1)) x = 0;
                else {
                    const int vc = a->val_vc[v];
                    const uint8_t op = a->P.val_op[v];
                    if (vc == VC_SINT && (op == NGZ_AGG_MIN || op == NGZ_AGG_MAX)) x ^= 1ull << 63;
                    const int w = a->val_w[v];
                    if (vc != VC_DTFRAC && w < 8) {  // wrap at the Rust width (release-mode +=), then extend
                        const uint32_t sh = 64 - 8 * w;
                        x = vc == VC_SINT ? (uint64_t)(((int64_t)(x << sh)) >> sh) : (x << sh) >> sh;
                    }
                }
                memcpy(p, &x, 8);
            }
        }
    }
    a->current_time = 0;  // WindowAggregator::flush clears current_time
    int rc = reset_table(a);
    if (rc != NGZ_OK) return rc;
    AGG_HIP(a, hipStreamSynchronize(a->stream));
    return n;
}

int ngz_agg_sets(ngz_agg *a, uint32_t *templates, uint32_t *n_templates, uint16_t *ports, uint32_t *n_ports,
                 uint32_t *domains, uint32_t *n_domains, uint32_t cap) {
    if (!a) return NGZ_E_INVALID;
    if (n_templates) *n_templates = (uint32_t)a->templates.size();
    if (n_ports) *n_ports = (uint32_t)a->ports.size();
    for (uint32_t i = 0; i < a->templates.size() && i < cap; ++i)
        if (templates) templates[i] = a->templates[i];
    for (uint32_t i = 0; i < a->ports.size() && i < cap; ++i)
        if (ports) ports[i] = a->ports[i];
    unsigned long long tab[DOM_SLOTS];
    AGG_HIP(a, hipMemcpy(tab, a->dom_tab, sizeof tab, hipMemcpyDeviceToHost));
    if (n_domains) *n_domains = DOM_SLOTS;
    for (uint32_t i = 0; i < DOM_SLOTS && i < cap; ++i)  // bit i <-> slot i; absent slots read 0xFFFFFFFF
        if (domains) domains[i] = tab[i] ? (uint32_t)tab[i] : 0xFFFFFFFFu;
    return NGZ_OK;
}

int ngz_agg_last_timing(ngz_agg *a, float *push_ms) {
    if (!a) return NGZ_E_INVALID;
    if (push_ms) *push_ms = a->t_push;
    return NGZ_OK;
}

}  // extern "C"
