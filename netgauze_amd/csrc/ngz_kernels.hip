// HIP kernels for gfx950 (CDNA4): datagram framing, record counting/layout,
// the generic (field-table driven) columnar record decode and the
// processed-count bookkeeping.  Per-template specialised decode kernels are
// generated and compiled at run time (ngz_rtc.cpp) from the same primitives
// (ngz_dev.h).
//
// Reference behaviour restated (file:line relative to the NetGauze checkout):
//   framing   crates/flow-pkt/src/codec.rs:189-220 (decode gate),
//             wire/deserializer/ipfix.rs:54-104,133-238 (IPFIX message/sets),
//             wire/deserializer/netflow.rs:56-114,143-235 (NFv9 message/sets)
//   records   ipfix.rs:335-370, netflow.rs:399-475, generated Field::parse
//             (ipfix-code-generator/src/generator.rs:1439-1807)
//   reader    crates/parse-utils/src/reader.rs:214-295 (reduced-size ints)
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "ngz/flow_decode.h"
#include "ngz_dev.h"
#include "ngz_internal.h"

namespace {
using namespace ngzdev;

__device__ __forceinline__ uint32_t ld8(const uint8_t *p) { return p[0]; }
__device__ __forceinline__ uint32_t be16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }
__device__ __forceinline__ uint32_t be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// The first 32 bytes of a datagram in registers (W[0..7], wire order, little-endian dwords):
// three aligned 16-byte loads and a per-lane shift, instead of one byte load per header byte
// (each such load a separate scattered line request across the wave).  Only when the 48
// aligned bytes lie inside the batch.
struct HdrWin {
    uint32_t w[8];
    bool ok;
};
__device__ __forceinline__ void hdr_window(const BatchDev &B, const uint8_t *p, HdrWin &H) {
    const uint64_t pa = (uint64_t)(uintptr_t)p, a16 = pa & ~15ull;
    H.ok = a16 + 48 <= (uint64_t)(uintptr_t)B.bytes + B.bytes_size;
#pragma unroll
    for (int j = 0; j < 8; ++j) H.w[j] = 0;
    if (!H.ok) return;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 *q = (const u32x4 *)(uintptr_t)a16;
    const u32x4 v0 = q[0], v1 = q[1], v2 = q[2];
    const uint32_t T[12] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3], v2[0], v2[1], v2[2], v2[3]};
    // dword shift by (pa >> 2) & 3 with bitwise selects (no dynamically indexed array), then
    // the byte shift
    const uint32_t m0 = 0u - (uint32_t)((pa >> 2) & 1), m1 = 0u - (uint32_t)((pa >> 3) & 1), sh = (uint32_t)(pa & 3);
    uint32_t U[11], R[9];
#pragma unroll
    for (int j = 0; j < 11; ++j) U[j] = (T[j + 1] & m0) | (T[j] & ~m0);
#pragma unroll
    for (int j = 0; j < 9; ++j) R[j] = (U[j + 2] & m1) | (U[j] & ~m1);
#pragma unroll
    for (int j = 0; j < 8; ++j) H.w[j] = __builtin_amdgcn_alignbyte(R[j + 1], R[j], sh);
}
// big-endian reads at constant window offsets
__device__ __forceinline__ uint32_t hw_be32(const HdrWin &H, int o) { return __builtin_bswap32(H.w[o >> 2]); }
__device__ __forceinline__ uint32_t hw_be16(const HdrWin &H, int o) {
    return (o & 2) ? __builtin_bswap32(H.w[o >> 2]) & 0xFFFFu : __builtin_bswap32(H.w[o >> 2]) >> 16;
}

struct WalkOut {
    uint32_t status, version, length, time, seq, domain, sysup, nsets;
    uint64_t err;
};

__device__ __forceinline__ uint16_t resolve_slot(const BatchDev &B, uint32_t pidx, uint32_t id, uint32_t d) {
    uint32_t key = (pidx << 16) | id;
    if (B.tl_n) {
        // last timeline entry with (key, dgram < d)
        uint32_t lo = 0, hi = B.tl_n;
        while (lo < hi) {
            uint32_t mid = (lo + hi) >> 1;
            uint32_t k = B.tl_key[mid];
            bool less = (k < key) || (k == key && B.tl_dgram[mid] < d);
            if (less)
                lo = mid + 1;
            else
                hi = mid;
        }
        if (lo > 0 && B.tl_key[lo - 1] == key) return B.tl_slot[lo - 1];
    }
    return B.cur_slot[pidx * 65536u + id];
}

// Walk one datagram as FlowInfoCodec::decode + {Ipfix,NetFlowV9}Packet::parse
// would, without decoding records.  For every data set reached, vis.on_set()
// gets the set header position, the template slot, the record count and the
// position of the first record.  Template sets end the walk with NGZ_FR_HOST.
template <class V>
__device__ void walk_datagram(const BatchDev &B, const uint32_t *__restrict__ hf_flag, const uint32_t *__restrict__ hf_first,
                              uint32_t d, WalkOut &o, V &vis) {
    o.status = NGZ_FR_OK;
    o.version = o.length = o.time = o.seq = o.domain = o.sysup = o.nsets = 0;
    o.err = NGZ_NO_ERR;
    if (hf_flag != nullptr && hf_flag[d]) {
        o.status = NGZ_FR_HOST;
        const uint8_t *p = B.bytes + B.offsets[d];
        for (uint32_t i = hf_first[d]; i < hf_first[d + 1]; ++i) {
            const HostSet &h = B.hf_sets[i];
            const DevPlan &pl = B.plans[h.slot];
            if (pl.has_vlen && h.n) {  // record offsets (the host walk counted the same records)
                uint64_t e = NGZ_NO_ERR;
                vis.vlen(p, h.payload_pos, h.set_pos + be16(p + h.set_pos + 2), h.slot, pl, &e);
            }
            vis.on_set(h.set_pos, h.slot, h.n, h.payload_pos, pl.rec_len);
        }
        return;
    }
    const uint8_t *p = B.bytes + B.offsets[d];
    const uint32_t dl = B.lengths[d];
    HdrWin H;
    hdr_window(B, p, H);
    // codec.rs:197-209: need the 16-byte header and buf.len() >= u16 at [2..4]
    if (dl < 16) { o.status = NGZ_FR_NEED_MORE; return; }
    const uint32_t ver = H.ok ? hw_be16(H, 0) : be16(p), len = H.ok ? hw_be16(H, 2) : be16(p + 2);
    if (dl < len) { o.status = NGZ_FR_NEED_MORE; return; }
    o.version = ver;
    o.length = len;
    if (ver == 10) {
        if (len < 16) {  // ipfix.rs:69-75
            o.status = NGZ_FR_ERROR;
            o.err = ngz_err_key(2, E_IPFIX_INVALID_LENGTH, 0, len);
            return;
        }
        o.time = H.ok ? hw_be32(H, 4) : be32(p + 4);
        o.seq = H.ok ? hw_be32(H, 8) : be32(p + 8);
        o.domain = H.ok ? hw_be32(H, 12) : be32(p + 12);
        uint32_t pos = 16;
        while (pos < len) {  // ipfix.rs:94-96
            const uint32_t rem = len - pos;
            if (rem < 2) { o.status = NGZ_FR_ERROR; o.err = ngz_err_key(pos, E_SET_EOF_ID, 2, rem); return; }
            const bool first = H.ok && pos == 16;  // the first set header is in the window
            const uint32_t id = first ? hw_be16(H, 16) : be16(p + pos);
            if (id != 2 && id != 3 && id < 256) {  // ipfix.rs:142-150
                o.status = NGZ_FR_ERROR; o.err = ngz_err_key(pos, E_SET_INVALID_ID, id, 0); return;
            }
            if (rem < 4) { o.status = NGZ_FR_ERROR; o.err = ngz_err_key(pos + 2, E_SET_EOF_LEN, 2, rem - 2); return; }
            const uint32_t sl = first ? hw_be16(H, 18) : be16(p + pos + 2);
            if (sl < 4) { o.status = NGZ_FR_ERROR; o.err = ngz_err_key(pos + 2, E_SET_INVALID_LENGTH, 0, sl); return; }
            if (sl - 4 > rem - 4) {  // take_slice (reader.rs:157-161)
                o.status = NGZ_FR_ERROR; o.err = ngz_err_key(pos + 4, E_SET_EOF_BODY, sl - 4, rem - 4); return;
            }
            if (id == 2 || id == 3) { o.status = NGZ_FR_HOST; return; }
            const uint16_t slot = resolve_slot(B, 0, id, d);
            if (slot == NGZ_NO_SLOT) {  // ipfix.rs:184-191
                o.status = NGZ_FR_ERROR; o.err = ngz_err_key(pos, E_SET_NO_TEMPLATE, id, 0); return;
            }
            const DevPlan &pl = B.plans[slot];
            const uint32_t minlen = pl.rec_len;  // ipfix.rs:193-214 (vlen counted as 1)
            uint64_t verr = NGZ_NO_ERR;
            uint32_t n;
            if (pl.has_vlen && pl.rpl)  // :219-222 record by record: lengths come from the data
                n = vis.vlen(p, pos + 4, pos + sl, slot, pl, &verr);
            else
                n = minlen ? (sl - 4) / minlen : 0;  // :219 loop bound
            if (n && !pl.rpl) { o.status = NGZ_FR_UNSUPPORTED; return; }
            o.nsets++;
            vis.on_set(pos, slot, n, pos + 4, minlen);
            if (verr != NGZ_NO_ERR) { o.status = NGZ_FR_ERROR; o.err = verr; return; }  // first error aborts
            pos += sl;  // leftover (padding or garbage) ignored: ipfix.rs:224-227
        }
        return;
    }
    if (ver == 9) {
        if (dl < 20) {  // header read_u32 of source_id (netflow.rs:86)
            o.status = NGZ_FR_ERROR; o.err = ngz_err_key(16, E_HDR_EOF, 4, dl - 16); return;
        }
        o.sysup = H.ok ? hw_be32(H, 4) : be32(p + 4);
        o.time = H.ok ? hw_be32(H, 8) : be32(p + 8);
        o.seq = H.ok ? hw_be32(H, 12) : be32(p + 12);
        o.domain = H.ok ? hw_be32(H, 16) : be32(p + 16);
        const uint32_t count = len;
        uint32_t i = count, pos = 20;
        while (i > 0 && dl - pos > 3) {  // netflow.rs:89
            const uint32_t rem = dl - pos;
            const bool first = H.ok && pos == 20;
            const uint32_t id = first ? hw_be16(H, 20) : be16(p + pos);
            if (id != 0 && id != 1 && id < 256) {
                o.status = NGZ_FR_ERROR; o.err = ngz_err_key(pos, E_SET_INVALID_ID, id, 0); return;
            }
            const uint32_t sl = first ? hw_be16(H, 22) : be16(p + pos + 2);
            if (sl < 4) { o.status = NGZ_FR_ERROR; o.err = ngz_err_key(pos + 2, E_SET_INVALID_LENGTH, 0, sl); return; }
            if (sl - 4 > rem - 4) {
                o.status = NGZ_FR_ERROR; o.err = ngz_err_key(pos + 4, E_SET_EOF_BODY, sl - 4, rem - 4); return;
            }
            if (id <= 1) { o.status = NGZ_FR_HOST; return; }
            const uint16_t slot = resolve_slot(B, 1, id, d);
            if (slot == NGZ_NO_SLOT) {
                o.status = NGZ_FR_ERROR; o.err = ngz_err_key(pos, E_SET_NO_TEMPLATE, id, 0); return;
            }
            const DevPlan &pl = B.plans[slot];
            const uint32_t rl = pl.rec_len;  // exact, 65535 literal (netflow.rs:201-210)
            const uint32_t n = rl ? (sl - 4) / rl : 0;
            if (n && !pl.rpl) { o.status = NGZ_FR_UNSUPPORTED; return; }
            o.nsets++;
            vis.on_set(pos, slot, n, pos + 4, rl);
            // check_padding_value (netflow.rs:225,237-248)
            for (uint32_t b = pos + 4 + n * rl; b < pos + sl; ++b) {
                const uint32_t v = ld8(p + b);
                if (v) { o.status = NGZ_FR_ERROR; o.err = ngz_err_key(b, E_SET_PADDING, 0, v); return; }
            }
            if (n > i) {  // InvalidCount (netflow.rs:95-100), raised after the set parsed
                o.status = NGZ_FR_ERROR; o.err = ngz_err_key(pos + sl, E_NF_INVALID_COUNT, 0, count); return;
            }
            i -= n;
            pos += sl;
        }
        return;
    }
    o.status = NGZ_FR_ERROR;  // codec.rs:214-217
    o.err = ngz_err_key(0, E_CODEC_UNSUPPORTED_VERSION, ver, 0);
}

// Does the datagram's set chain contain a (options) template set anywhere?
// Structural only (independent of template state and of NFv9 record counts),
// so it over-approximates which datagrams must be framed on the host.
__device__ bool has_template_sets(const BatchDev &B, uint32_t d) {
    const uint8_t *p = B.bytes + B.offsets[d];
    const uint32_t dl = B.lengths[d];
    if (dl < 16) return false;
    const uint32_t ver = be16(p), len = be16(p + 2);
    if (dl < len) return false;
    uint32_t pos, end;
    if (ver == 10) { pos = 16; end = len; }
    else if (ver == 9) { pos = 20; end = dl; }
    else return false;
    while (pos + 4 <= end) {
        const uint32_t id = be16(p + pos), sl = be16(p + pos + 2);
        if (ver == 10 ? (id == 2 || id == 3) : (id <= 1)) return true;
        if (sl < 4 || sl > end - pos) return false;
        pos += sl;
    }
    return false;
}

constexpr uint32_t kFrameBlock = 256;

// 64 bytes of a datagram for the record walk, in this thread's 16 LDS dwords (the window starts
// at a 16-byte aligned address): the length prefixes of a variable-length record lie 20-40 bytes
// apart, so most of them come out of the window already loaded instead of from a byte load of their
// own.  Each byte load was a round trip on the walk's dependent chain (k_frame spent 86 % of its wave
// cycles waiting); a window is four independent 16-byte loads, one round trip.  LDS, not registers:
// k_frame has no VGPRs to spare for 16 more.  The slots are transposed -- dword j of thread t at
// col[j * kFrameBlock + t] -- so a wave's window stores and its byte reads (every lane its own
// dword) touch 64 different banks: thread-contiguous 64-byte slots put the lanes 16 banks apart
// (4-16-way conflicts, 3.6e7 conflict cycles per config-4 k_frame, profiles/r5/cfg4).
#ifndef NGZ_FRAME_ATTRIB
#define NGZ_FRAME_ATTRIB 0  // 1: k_frame skips the record walk (experiment builds; timing only: every
                            // variable-length set then counts no records, so nothing reads its offsets)
#endif
#ifndef NGZ_WALKWIN_BYTES
#define NGZ_WALKWIN_BYTES 64  // window bytes (a multiple of 16; the experiment variants try others)
#endif
struct WalkWin {
    static constexpr uint32_t kBytes = NGZ_WALKWIN_BYTES, kLoads = kBytes / 16;
    uint32_t *col;       // this thread's column of the transposed window table
    uintptr_t base = 0;  // address the window starts at; 0 = empty
    // the byte at address q; lim: end of the batch buffer (no window reaches past it)
    __device__ __forceinline__ uint32_t byte(const uint8_t *q, const uint8_t *lim) {
        const uintptr_t a = (uintptr_t)q;
        if (!col) return *q;
        if (!base || a < base || a >= base + kBytes) {
            const uintptr_t b0 = a & ~(uintptr_t)15;
            if (b0 + kBytes > (uintptr_t)lim) return *q;
            const uint4 *v = (const uint4 *)b0;
            uint4 x[kLoads];
#pragma unroll
            for (uint32_t j = 0; j < kLoads; ++j) x[j] = v[j];
#pragma unroll
            for (uint32_t j = 0; j < kLoads; ++j) {
                col[(4 * j + 0) * kFrameBlock] = x[j].x;
                col[(4 * j + 1) * kFrameBlock] = x[j].y;
                col[(4 * j + 2) * kFrameBlock] = x[j].z;
                col[(4 * j + 3) * kFrameBlock] = x[j].w;
            }
            base = b0;
        }
        const uint32_t o = (uint32_t)(a - base);
        return (col[(o >> 2) * kFrameBlock] >> (8 * (o & 3))) & 0xFFu;
    }
};

// ngz_vlen_walk's fast form (ngz_internal.h) with the length prefixes read through a WalkWin; a
// record the fast steps cannot complete goes to the exact form from its start, as there
template <class F>
__device__ uint32_t vlen_walk_win(const uint8_t *p, uint32_t pos, uint32_t end, const DevPlan &pl, uint64_t *err,
                                  const uint8_t *lim, uint32_t *slot, F &&on_rec) {
    if (pl.walk_nv > NGZ_WALK_MAX) return ngz_vlen_walk_exact(p, pos, end, pl, err, on_rec);
    const uint32_t minlen = pl.rec_len, nv = pl.walk_nv;
    // the fixed runs, two 16-bit ones per register (indexed by unrolled loop counters only)
    uint32_t fx2[(NGZ_WALK_MAX + 2) / 2];
#pragma unroll
    for (uint32_t k = 0; k < (NGZ_WALK_MAX + 2) / 2; ++k)
        fx2[k] = (uint32_t)pl.walk_fixed[2 * k] | ((uint32_t)pl.walk_fixed[2 * k + 1] << 16);
    auto fx = [&](uint32_t k) { return (fx2[k >> 1] >> (16 * (k & 1))) & 0xFFFFu; };
    WalkWin W{slot};
    uint32_t n = 0;
    while (minlen > 0 && end - pos >= minlen) {
        const uint32_t start = pos;
        bool ok = end - pos >= fx(0);
        pos += fx(0);
#pragma unroll
        for (uint32_t k = 0; k < NGZ_WALK_MAX; ++k) {
            if (k < nv && ok) {
                uint32_t len = 0, hdr = 1;
                ok = end - pos >= 1;
                if (ok) {
                    len = W.byte(p + pos, lim);
                    if (len == 255) {
                        ok = end - pos >= 4;
                        if (ok) len = ((uint32_t)p[pos + 1] << 16) | ((uint32_t)p[pos + 2] << 8) | p[pos + 3];
                        hdr = 4;
                    }
                }
                ok = ok && end - pos - hdr >= len && end - pos - hdr - len >= fx(k + 1);
                pos += hdr + len + fx(k + 1);
            }
        }
        if (!ok) return n + ngz_vlen_walk_exact(p, start, end, pl, err, on_rec, n);
        on_rec(n, start);
        ++n;
    }
    return n;
}

// Datagram d's record-offset list: 16-byte aligned, at entry ceil8(offsets[d] / div + 8 d).  A
// datagram of L bytes has at most L / div records (+ the terminator), so the lists of datagrams
// whose bytes do not overlap do not overlap either, whole 16-byte pieces included
__device__ __forceinline__ uint16_t *ngz_ro_list(const BatchDev &B, uint64_t dg_off, uint32_t d) {
    return B.recoff + ((dg_off / B.recoff_div + 8ull * d + 7) & ~7ull);
}

// Count matrix, slot-major rows of N datagrams (scanned in one pass):
//   rows [0, S)      records of slot s in datagram d
//   rows [S, 2S)     decode chunks of slot s in datagram d
//   row  2S          data sets in datagram d
struct CountVis {
    uint32_t *counts;
    uint32_t N, A, d;  // A: count-matrix rows (slots with a row)
    uint32_t sets;
    const DevPlan *plans;
    uint32_t *recmap;
    uint64_t dg_off;
    uint16_t *ro = nullptr;  // this datagram's record-offset list (BatchDev::recoff), or null
    // the list goes out 8 entries (16 bytes) at a time from two registers: stored entry by entry,
    // 64 lanes' 2-byte stores to 64 lists were 64 partial-line writes each (0.5 GB of WRITE_SIZE
    // per config-4 step for 20 MB of offsets)
    uint64_t q0 = 0, q1 = 0;
    uint32_t qn = 0;  // entries held
    __device__ void ro_push(uint32_t at) {
        const uint64_t e = (uint64_t)(at & 0xFFFFu);
        if (qn < 4) q0 |= e << (16 * qn);
        else q1 |= e << (16 * (qn - 4));
        if (++qn == 8) {
            *(uint4 *)ro = make_uint4((uint32_t)q0, (uint32_t)(q0 >> 32), (uint32_t)q1, (uint32_t)(q1 >> 32));
            ro += 8;
            q0 = q1 = 0;
            qn = 0;
        }
    }
    __device__ void ro_finish() {  // the 0xFFFF terminator, and the last (partial) 16 bytes
        ro_push(0xFFFFu);
        if (qn) *(uint4 *)ro = make_uint4((uint32_t)q0, (uint32_t)(q0 >> 32), (uint32_t)q1, (uint32_t)(q1 >> 32));
    }
    uint64_t sum = 0;  // the first data set: set_pos | slot << 16 | n << 32 | (end - set_pos, or 1) << 48
    uint64_t dg_end = 0;  // batch offset past the datagram
    uint32_t split = 0;    // BatchDev::split
    bool deferred = false;  // phase A: a variable-length set was left to phase B
    bool vlen_err = false;  // phase B: a variable-length set's record walk failed
    // record-start marks of the word being filled (record starts only ever move forward)
    uint64_t mw = ~0ull;
    uint32_t mbits = 0;
    __device__ void mark_flush() {
        if (mw == ~0ull) return;
        // a word wholly inside this datagram is this thread's alone: a plain store (the map
        // is zeroed per batch); a word shared with a neighbouring datagram takes an atomicOr
        if (32 * mw >= dg_off && 32 * mw + 32 <= dg_end) recmap[mw] = mbits;
        else atomicOr(&recmap[mw], mbits);
    }
    __device__ uint32_t vlen(const uint8_t *p, uint32_t pos, uint32_t end, uint32_t, const DevPlan &pl, uint64_t *err) {
        if (split == 1) {  // phase B walks it
            deferred = true;
            return 0;
        }
        if (!sets) sum = (uint64_t)(end - (pos - 4)) << 48;
        if (NGZ_FRAME_ATTRIB & 1) return 0;  // timing attribution (experiment variants): no record walk
        const uint64_t e0 = *err;
        const uint32_t n = walk_records(p, pos, end, pl, err);
        vlen_err = vlen_err || *err != e0;
        return n;
    }
    const uint8_t *lim = nullptr;  // end of the batch buffer (WalkWin loads stay inside it)
    uint32_t *win = nullptr;       // this thread's WalkWin column in LDS
    __device__ uint32_t walk_records(const uint8_t *p, uint32_t pos, uint32_t end, const DevPlan &pl, uint64_t *err) {
        return vlen_walk_win(p, pos, end, pl, err, lim, win, [this](uint32_t, uint32_t at) {
            if (ro) {  // the record's offset in the datagram, appended to the datagram's list
                ro_push(at);
                return;
            }
            if (!recmap) return;
            const uint64_t b = dg_off + at;
            if ((b >> 5) != mw) {
                mark_flush();
                mw = b >> 5;
                mbits = 0;
            }
            mbits |= 1u << (b & 31);
        });
    }
    const uint16_t *row;
    BatchSummary *summary;
    __device__ void on_set(uint32_t set_pos, uint32_t slot, uint32_t n, uint32_t, uint32_t) {
        if (split) {
            // phase A counts the records of fixed-length sets only, phase B of variable-length ones;
            // both count every set (the set table's order)
            const bool v = plans[slot].has_vlen && plans[slot].rpl;
            if (v == (split == 1)) {
                sets += 1;
                return;
            }
        }
        if (!sets) sum = (sum ? sum : 1ull << 48) | set_pos | ((uint64_t)slot << 16) | ((uint64_t)(n & 0xFFFF) << 32);
        const uint32_t r = row[slot];
        if (r == NGZ_NO_ROW) {
            atomicOr(&summary->overflow, 8u);  // the batch runs again with a row for every slot
        } else {
            counts[(uint64_t)r * N + d] += n;
            if (n) counts[(uint64_t)(A + r) * N + d] += (n + plans[slot].window - 1) / plans[slot].window + 1;
        }
        sets += 1;
    }
};

#ifdef NGZ_FRAME_WPE  // experiment variants: a waves-per-SIMD floor for k_frame's register allocation
#define NGZ_FRAME_ATTR __attribute__((amdgpu_waves_per_eu(NGZ_FRAME_WPE)))
#else
#define NGZ_FRAME_ATTR
#endif
__global__ void __launch_bounds__(kFrameBlock) NGZ_FRAME_ATTR k_frame(BatchDev B, const uint32_t *hf_flag, const uint32_t *hf_first) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= B.n) return;
    // this datagram's column of the count matrix starts at zero (no memset pass)
    for (uint32_t r = 0; r < 2 * B.n_rows; ++r) B.counts[(uint64_t)r * B.n + d] = 0;
    if (d == 0) B.counts[(uint64_t)(2 * B.n_rows + 1) * B.n] = 0;  // the scan's trailing element
    CountVis vis{B.counts, B.n, B.n_rows, d, 0, B.plans, B.recmap, B.offsets[d]};
    vis.row = B.slot_row;
    vis.summary = B.summary;
    vis.dg_end = vis.dg_off + B.lengths[d];
    vis.split = B.split;
    vis.lim = B.bytes + B.bytes_size;
    __shared__ uint32_t wwin[WalkWin::kBytes / 4 * kFrameBlock];
    vis.win = &wwin[threadIdx.x];
    if (B.recoff) vis.ro = ngz_ro_list(B, vis.dg_off, d);
    WalkOut o;
    walk_datagram(B, hf_flag, hf_first, d, o, vis);
    vis.mark_flush();
    if (vis.ro) vis.ro_finish();  // end of the list
    // a walk that ended OK visited every set (template sets end it with HOST)
    if (o.status != NGZ_FR_HOST && o.status != NGZ_FR_OK && !(hf_flag && hf_flag[d]) && has_template_sets(B, d))
        o.status = NGZ_FR_HOST;
    const uint64_t N = B.n;
    B.counts[(uint64_t)(2 * B.n_rows) * N + d] = vis.sets;
    // one data set, parsed cleanly: k_emit takes it from here instead of walking the datagram again
    if (B.dsum)
        B.dsum[d] = (o.status == NGZ_FR_OK && o.err == NGZ_NO_ERR && vis.sets == 1 && !(hf_flag && hf_flag[d]) &&
                     ((vis.sum >> 32) & 0xFFFF) < 0xFFFF && !vis.deferred)
                        ? vis.sum
                        : 0ull;
    ngz_dgram_hdr h;
    h.status = (uint8_t)o.status;
    h.version = (uint8_t)o.version;
    h.length = (uint16_t)o.length;
    h.time = o.time;
    h.sequence = o.seq;
    h.domain = o.domain;
    h.sys_up_time = o.sysup;
    h.n_sets = o.nsets;
    h.err_key = o.err;
    if (hf_flag && hf_flag[d]) h = ((const ngz_dgram_hdr *)B.hf_hdr)[hf_flag[d] - 1];
    ((ngz_dgram_hdr *)B.hdr)[d] = h;
    if (o.status == NGZ_FR_HOST && !(hf_flag && hf_flag[d])) atomicAdd(&B.summary->n_host, 1u);
    if (o.status == NGZ_FR_UNSUPPORTED) atomicAdd(&B.summary->n_unsupported, 1u);
}

// Split framing, phase B (BatchDev::split 2, on its own stream beside phase A's fixed-length
// decode): the record walk of the variable-length sets, into phase B's own count matrix (rows of
// the variable-length slots, every set counted for the set order) and the record-offset lists.
// Phase A (k_frame with split 1) wrote the headers; a record error here, which phase A did not
// see, sends the batch round again unsplit (overflow bit 16).
__global__ void __launch_bounds__(kFrameBlock) k_frame_vlen(BatchDev B) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= B.n) return;
    for (uint32_t r = 0; r < 2 * B.n_rows; ++r) B.counts[(uint64_t)r * B.n + d] = 0;
    if (d == 0) B.counts[(uint64_t)(2 * B.n_rows + 1) * B.n] = 0;
    CountVis vis{B.counts, B.n, B.n_rows, d, 0, B.plans, nullptr, B.offsets[d]};
    vis.row = B.slot_row;
    vis.summary = B.summary;
    vis.dg_end = vis.dg_off + B.lengths[d];
    vis.split = 2;
    vis.lim = B.bytes + B.bytes_size;
    __shared__ uint32_t wwin[WalkWin::kBytes / 4 * kFrameBlock];
    vis.win = &wwin[threadIdx.x];
    vis.ro = ngz_ro_list(B, vis.dg_off, d);
    WalkOut o;
    walk_datagram(B, nullptr, nullptr, d, o, vis);
    vis.ro_finish();
    B.counts[(uint64_t)(2 * B.n_rows) * B.n + d] = vis.sets;
    if (vis.vlen_err) atomicOr(&B.summary->overflow, 16u);
}

// Column layout: slot-major rows of the scanned count matrix give each slot a
// dense, stream-ordered row range; columns of a slot are laid out
// column-major inside one 256-byte aligned block of cap*row_bytes bytes.
__global__ void k_layout(BatchDev B) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint64_t N = B.n;
    const uint32_t S = B.n_slots, A = B.n_rows;
    const uint32_t chunk_base = B.scan[(uint64_t)A * N];
    // split framing: phase A lays out the fixed-length slots from the arena start, phase B the
    // variable-length ones after them (it runs once phase A's layout is done)
    uint64_t off = B.split == 2 ? B.summary->arena_used : 0;
    for (uint32_t s = 0; s < S; ++s) {
        if (B.split && (B.plans[s].has_vlen && B.plans[s].rpl) != (B.split == 2)) continue;  // the other phase's
        const uint32_t r = B.slot_row[s];
        const bool has = r != NGZ_NO_ROW;
        // a slot without a row has no records in this batch (else the batch runs again)
        const uint32_t base = has ? B.scan[(uint64_t)r * N] : chunk_base;
        const uint32_t next = has ? B.scan[(uint64_t)(r + 1) * N] : chunk_base;
        const uint32_t total = next - base;
        const uint32_t w = B.plans[s].window ? B.plans[s].window : 64;
        // LDS-staged kernels store whole workgroup windows: capacity in those
        const uint32_t wa = B.plans[s].lds_waves ? w * B.plans[s].lds_waves : w;
        const uint32_t cap = total ? ((total + wa - 1) / wa + B.cap_pad_windows) * wa : 0;
        SlotRT rt;
        rt.block = off;
        rt.cap = cap;
        rt.total = total;
        rt.base = base;
        rt.chunk_scan0 = has ? B.scan[(uint64_t)(A + r) * N] : B.scan[(uint64_t)(2 * A) * N];
        rt.chunk0 = rt.chunk_scan0 - chunk_base;
        rt.nchunks = has ? B.scan[(uint64_t)(A + r + 1) * N] - rt.chunk_scan0 : 0;
        // row mode for variable-length records and for sets so small that
        // set-relative chunks would leave most lanes idle (< 25 % of rows used).
        // A specialised LDS-staged kernel gathers the rows of a window across
        // its chunks (ChunkGatherSrc, up to 64 chunk entries per 256-row
        // sub-window), so small sets stay in chunk mode there: two 32-byte
        // chunk entries per set instead of a 12-byte row entry per record.
        const bool gather = B.plans[s].spec && B.plans[s].lds_waves && 256ull * rt.nchunks <= 48ull * total;
        rt.mode = (B.plans[s].has_vlen || (!gather && 4ull * total < (uint64_t)rt.nchunks * w)) ? NGZ_MODE_ROW
                                                                                                  : NGZ_MODE_CHUNK;
        rt.reserved = 0;
        const uint64_t col_bytes = ((uint64_t)cap * B.plans[s].row_bytes + 7) & ~7ull;
        rt.rows = rt.mode == NGZ_MODE_ROW ? off + col_bytes : 0;
        rt.wtab = rt.mode == NGZ_MODE_CHUNK ? off + col_bytes : 0;
        if (rt.mode == NGZ_MODE_ROW) rt.nchunks = 0;
        B.slots[s] = rt;
        // row mode: rowsrc + rowdg; chunk mode: first chunk per window
        const uint64_t row_bytes_extra = rt.mode == NGZ_MODE_ROW ? 12ull * cap : 4ull * (cap / w + 1);
        off += (col_bytes + row_bytes_extra + 255) & ~255ull;
    }
    const uint32_t rec_total = chunk_base;
    const uint32_t chunks = B.scan[(uint64_t)(2 * A) * N] - chunk_base;
    const uint32_t sets = B.scan[(uint64_t)(2 * A + 1) * N] - B.scan[(uint64_t)(2 * A) * N];
    if (B.split == 2) {  // phase A's summary plus the variable-length slots
        B.summary->n_records_total += rec_total;
    } else {
        B.summary->n_records_total = rec_total;
        B.summary->n_chunks = chunks;
        B.summary->n_sets = sets;
    }
    B.summary->arena_used = off;
    // bits only ever set (the summary starts the batch zeroed): the other framing phase and
    // k_frame (bit 8) may be setting theirs
    uint32_t ov = 0;
    if (off > B.arena_cap) ov |= 1;
    if (B.split != 2 && chunks > B.chunk_cap) ov |= 2;  // phase B's rows only count records
    if (B.split != 2 && sets > B.set_cap) ov |= 4;
    if (ov) atomicOr(&B.summary->overflow, ov);
}

#ifndef NGZ_EMIT_STAGE_ROWS
#define NGZ_EMIT_STAGE_ROWS 3072  // rows a k_emit workgroup stages (12 B each in LDS)
#endif
// Row-mode record tables (variable-length slots, and fixed-length ones decoded by the staged-row
// kernel: config 4's NetFlow v9 template) are staged per workgroup:
// the workgroup's datagrams are consecutive, so their records of one slot are
// one contiguous row range; each thread writes its records' rows to LDS and
// the workgroup stores the range coalesced.  (Written per thread straight to
// HBM, 8- and 4-byte entries 64 lanes apart, they went out as partial-line
// writes: 1.1 GB of WRITE_SIZE for 0.12 GB of rows on config 4.)
constexpr uint32_t kEmitStageRows = NGZ_EMIT_STAGE_ROWS;
constexpr uint32_t kEmitStageSlots = 4;

struct EmitVis {
    const BatchDev *B;
    uint32_t d;
    uint64_t dg_off;
    uint32_t set_at;
    bool ok;
    const uint32_t (*tab)[4];  // staged slots: {slot, first row, LDS row, rows}
    uint32_t ntab;
    const uint16_t *ro;        // the datagram's record-offset list (k_frame), at its next set's first record
    uint64_t *lrs;             // LDS row tables
    uint32_t *lrd;
    uint32_t split;            // BatchDev::split: phase A emits the fixed-length sets, phase B the others
    // row mode: every record's batch offset and datagram, rows rec0.. of this set
    __device__ uint64_t *rowsrc(uint32_t slot) const { return (uint64_t *)(B->arena + B->slots[slot].rows); }
    __device__ uint32_t *rowdg(uint32_t slot) const {
        return (uint32_t *)(B->arena + B->slots[slot].rows + 8ull * B->slots[slot].cap);
    }
    __device__ uint32_t vlen(const uint8_t *p, uint32_t pos, uint32_t end, uint32_t slot, const DevPlan &pl,
                             uint64_t *err) {
        if (split == 1) return 0;  // phase B's
        const uint32_t rec0 = B->scan[(uint64_t)B->slot_row[slot] * B->n + d] - B->slots[slot].base;
        uint64_t *rs = rowsrc(slot) + rec0;
        uint32_t *rd = rowdg(slot) + rec0;
        for (uint32_t k = 0; k < ntab; ++k)
            if (tab[k][0] == slot) {
                rs = lrs + tab[k][2] + (rec0 - tab[k][1]);
                rd = lrd + tab[k][2] + (rec0 - tab[k][1]);
            }
        if (ro) {
            // k_frame's walk listed every complete record's offset: the set's are the next
            // entries below its end (the list ends with 0xFFFF)
            uint32_t k = 0;
            uint64_t prev = 0;
            for (uint32_t at = *ro; at < end; at = *++ro) {
                const uint64_t b = dg_off + at;
                if (k) rs[k - 1] = ngz_row_entry(prev, b - prev);
                prev = b;
                rd[k] = d;
                ++k;
            }
            if (k) rs[k - 1] = ngz_row_entry(prev, dg_off + end - prev);  // the last record: up to the set's end
            const uint64_t ek = ((const ngz_dgram_hdr *)B->hdr)[d].err_key;
            const uint32_t stop = (uint32_t)(ek >> 48);
            if (ek != NGZ_NO_ERR && stop >= pos && stop <= end) *err = ek;
            return k;
        }
        if (B->recmap) {
            // k_frame's walk marked every complete record start: read the marks
            // instead of walking the records again (independent loads, no
            // dependent length-prefix chain)
            const uint64_t g0 = dg_off + pos, g1 = dg_off + end;
            uint32_t k = 0;
            uint64_t prev = 0;  // the previous record's start: its span ends at this one
            if (g0 < g1) {
                const uint64_t w0 = g0 >> 5, w1 = (g1 - 1) >> 5;
                // 16-byte loads of the map (4 words = 128 batch bytes each; the map has slack past its end)
                for (uint64_t wq = w0 & ~3ull; wq <= w1; wq += 4) {
                    const uint4 q = *(const uint4 *)&B->recmap[wq];
                    const uint32_t words[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                    for (uint32_t j = 0; j < 4; ++j) {
                        const uint64_t w = wq + j;
                        if (w < w0 || w > w1) continue;
                        uint32_t bits = words[j];
                        if ((w << 5) < g0) bits &= 0xFFFFFFFFu << (g0 & 31);
                        if (((w + 1) << 5) > g1) bits &= 0xFFFFFFFFu >> (32 - (g1 & 31));
                        while (bits) {
                            const uint32_t bit = (uint32_t)__builtin_ctz(bits);
                            const uint64_t at = (w << 5) + bit;
                            if (k) rs[k - 1] = ngz_row_entry(prev, at - prev);
                            prev = at;
                            rd[k] = d;
                            ++k;
                            bits &= bits - 1;
                        }
                    }
                }
            }
            if (k) rs[k - 1] = ngz_row_entry(prev, g1 - prev);  // the last record: up to the set's end
            // the walk stopped inside (or right at the end of) this set: k_frame
            // recorded that framing error in the datagram header
            const uint64_t ek = ((const ngz_dgram_hdr *)B->hdr)[d].err_key;
            const uint32_t stop = (uint32_t)(ek >> 48);
            if (ek != NGZ_NO_ERR && stop >= pos && stop <= end) *err = ek;
            return k;
        }
        const uint32_t n = ngz_vlen_walk(p, pos, end, pl, err, [&](uint32_t k, uint32_t at) {
            rs[k] = dg_off + at;
            rd[k] = d;
        });
        for (uint32_t k = 0; k < n; ++k) {
            const uint64_t next = k + 1 < n ? rs[k + 1] : dg_off + end;
            rs[k] = ngz_row_entry(rs[k], next - rs[k]);
        }
        return n;
    }
    __device__ void on_set(uint32_t set_pos, uint32_t slot, uint32_t n, uint32_t payload_pos, uint32_t rl) {
        const uint64_t N = B->n;
        if (split && (B->plans[slot].has_vlen && B->plans[slot].rpl) != (split == 2)) {
            ++set_at;  // the other phase writes this set's entry
            return;
        }
        const uint32_t row = B->slot_row[slot];
        uint32_t *cell = &B->scan[(uint64_t)row * N + d];
        const uint32_t rec0 = *cell - B->slots[slot].base;
        *cell += n;
        if (!ok) return;
        ngz_set_info si;
        si.dgram = d;
        si.set_pos = (uint16_t)set_pos;
        si.slot = (uint16_t)slot;
        si.rec0 = rec0;
        si.n = n;
        ((ngz_set_info *)B->sets)[set_at++] = si;
        if (!n) return;
        if (B->slots[slot].mode == NGZ_MODE_ROW) {
            if (B->plans[slot].has_vlen) return;  // the walk (vlen) wrote the rows
            uint64_t *rs = rowsrc(slot) + rec0;
            uint32_t *rd = rowdg(slot) + rec0;
            for (uint32_t k = 0; k < ntab; ++k)  // staged: the workgroup stores the range coalesced
                if (tab[k][0] == slot) {
                    rs = lrs + tab[k][2] + (rec0 - tab[k][1]);
                    rd = lrd + tab[k][2] + (rec0 - tab[k][1]);
                }
            for (uint32_t k = 0; k < n; ++k) {
                rs[k] = ngz_row_entry(dg_off + payload_pos + (uint64_t)k * rl, rl);
                rd[k] = d;
            }
            return;
        }
        const uint32_t W = B->plans[slot].window;
        const uint32_t reserved = (n + W - 1) / W + 1;
        // this slot's chunk cursor; the scan row's own first cell is another
        // thread's cursor, so the row base comes from SlotRT (k_layout)
        uint32_t *ccell = &B->scan[(uint64_t)(B->n_rows + row) * N + d];
        const uint32_t chunk_at = *ccell - B->slots[slot].chunk_scan0 + B->slots[slot].chunk0;
        *ccell += reserved;
        uint32_t r = 0, used = 0;
        while (r < n) {
            const uint32_t cstart = rec0 + r;
            const uint32_t wend = (cstart / W + 1) * W;
            const uint32_t take = min(n - r, wend - cstart);
            const uint32_t at = payload_pos + r * rl;  // first record's offset in the datagram
            Chunk c;
            c.src = dg_off + at;
            c.rec0 = cstart;
            c.dgram = d;
            c.n = (uint16_t)take;
            c.slot = (uint16_t)slot;
            c.pos0 = (uint16_t)at;
            c.cls = 0;
            c.reserved2 = 0;
            B->chunks[chunk_at + used] = c;
            // every window starts with a chunk (sets are cut at window boundaries)
            if (cstart % W == 0) ((uint32_t *)(B->arena + B->slots[slot].wtab))[cstart / W] = chunk_at + used;
            ++used;
            r += take;
        }
        for (; used < reserved; ++used) {
            Chunk c = {};
            B->chunks[chunk_at + used] = c;
        }
    }
};

__global__ void __launch_bounds__(256) k_emit(BatchDev B, const uint32_t *hf_flag, const uint32_t *hf_first) {
    __shared__ uint64_t st_rs[kEmitStageRows];
    __shared__ uint32_t st_rd[kEmitStageRows];
    __shared__ uint32_t st_tab[kEmitStageSlots][4];
    __shared__ uint32_t st_cnt, st_used;
    if (B.summary->overflow) return;
    const uint32_t t = threadIdx.x;
    const uint32_t d0 = blockIdx.x * blockDim.x;
    const uint32_t d = d0 + t;
    const uint64_t N = B.n;
    const uint32_t S = B.n_slots, A = B.n_rows;
    const uint32_t dl = min(d0 + blockDim.x, B.n) - 1;  // the workgroup's last datagram
    if (t == 0) st_cnt = st_used = 0;
    __syncthreads();
    // the workgroup's row range of every variable-length row-mode slot, read
    // before any thread moves its scan cursors
    for (uint32_t s = t; s < S; s += blockDim.x) {
        if (B.slots[s].mode != NGZ_MODE_ROW || B.slot_row[s] == NGZ_NO_ROW) continue;
        const uint32_t base = B.slots[s].base, sr = B.slot_row[s];
        const uint32_t r0 = B.scan[(uint64_t)sr * N + d0] - base;
        const uint32_t r1 = B.scan[(uint64_t)sr * N + dl] - base + B.counts[(uint64_t)sr * N + dl];
        const uint32_t n = r1 - r0;
        if (!n) continue;
        const uint32_t off = atomicAdd(&st_used, n);
        if (off + n > kEmitStageRows) continue;  // direct stores for this slot
        const uint32_t k = atomicAdd(&st_cnt, 1u);
        if (k >= kEmitStageSlots) continue;
        st_tab[k][0] = s;
        st_tab[k][1] = r0;
        st_tab[k][2] = off;
        st_tab[k][3] = n;
    }
    __syncthreads();
    const uint32_t ntab = min(st_cnt, kEmitStageSlots);
    if (ntab) {
        // every staged row is written below (k_frame counted exactly the rows this walk emits);
        // zeroed first all the same, so no row could ever reach the decode as a stale LDS value
        const uint32_t used = min(st_used, kEmitStageRows);
        for (uint32_t i = t; i < used; i += blockDim.x) {
            st_rs[i] = 0;
            st_rd[i] = 0;
        }
        __syncthreads();
    }
    if (d < B.n) {
        EmitVis vis;
        vis.B = &B;
        vis.d = d;
        vis.dg_off = B.offsets[d];
        vis.set_at = B.scan[(uint64_t)(2 * A) * N + d] - B.scan[(uint64_t)(2 * A) * N];
        vis.ok = true;
        vis.tab = st_tab;
        vis.ntab = ntab;
        vis.lrs = st_rs;
        vis.lrd = st_rd;
        vis.split = B.split;
        vis.ro = B.recoff ? ngz_ro_list(B, vis.dg_off, d) : nullptr;
        const unsigned long long sm = B.dsum ? B.dsum[d] : 0ull;
        if (sm) {
            // k_frame's summary of the datagram's one data set (same calls as walk_datagram)
            const uint32_t set_pos = (uint32_t)(sm & 0xFFFF), slot = (uint32_t)(sm >> 16) & 0xFFFF;
            const uint32_t n = (uint32_t)(sm >> 32) & 0xFFFF, sl = (uint32_t)(sm >> 48);
            const DevPlan &pl = B.plans[slot];
            if (pl.has_vlen && pl.rpl) {
                uint64_t e = NGZ_NO_ERR;
                vis.vlen(B.bytes + vis.dg_off, set_pos + 4, set_pos + sl, slot, pl, &e);
            }
            vis.on_set(set_pos, slot, n, set_pos + 4, pl.rec_len);
        } else {
            WalkOut o;
            walk_datagram(B, hf_flag, hf_first, d, o, vis);
        }
    }
    if (!ntab) return;
    __syncthreads();
    for (uint32_t k = 0; k < ntab; ++k) {
        const uint32_t s = st_tab[k][0], r0 = st_tab[k][1], off = st_tab[k][2], n = st_tab[k][3];
        uint64_t *rs = (uint64_t *)(B.arena + B.slots[s].rows) + r0;
        uint32_t *rd = (uint32_t *)(B.arena + B.slots[s].rows + 8ull * B.slots[s].cap) + r0;
        for (uint32_t i = t; i < n; i += blockDim.x) {
            rs[i] = st_rs[off + i];
            rd[i] = st_rd[off + i];
        }
    }
}

// ---------------------------------------------------------------------------
// Generic record decode (any fixed-length template; the fallback for slots
// without a specialised run-time-compiled kernel).  One wave per chunk
// (<= NGZ_REG_WINDOW rows of one output window), 64 rows per pass, one record
// per lane (ngz_dev.h).  The template's field table is held one descriptor per
// lane and fetched with v_readlane into SGPRs, so every field's offset,
// length and kind is wave-uniform; the 80-byte register window slides along
// the record as fields require (fields are in record order).  Every lane runs
// the whole field walk (uniform control flow: the register-indexing
// sequences assume it); only lanes whose row belongs to the chunk store.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_decode_generic(BatchDev B) {
    if (sload(&B.summary->overflow)) return;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t cached = 0xFFFFFFFFu, rl = 0, nf = 0, skip = 0, row_bytes = 0, has_vlen = 0;
    uint4 fA = make_uint4(0, 0, 0, 0), fB = make_uint4(0, 0, 0, 0);  // field descriptors f = lane, lane + 64
    const uint4 *ft = nullptr;  // the slot's field table (descriptors past NGZ_LANE_FIELDS: scalar loads)
    auto want = [&](uint32_t slot) {
        if (slot != cached) {
            const DevPlan *pl = &B.plans[slot];
            const uint4 h0 = sload((const uint4 *)pl);
            rl = h0.x;
            row_bytes = h0.y;
            nf = h0.z & 0xFFFF;
            has_vlen = (h0.w >> 8) & 0xFF;
            skip = (h0.w >> 24) & 0xFF;  // DevPlan::spec: decoded by its own kernel
            ft = (const uint4 *)sload(&pl->f);
            fA = lane < nf ? ft[lane] : make_uint4(0, 0, 0, 0);
            fB = lane + 64 < nf ? ft[lane + 64] : make_uint4(0, 0, 0, 0);
            cached = slot;
        }
        return skip == 0;
    };
    auto shape = [&](uint32_t) { return RecShape{rl, row_bytes, has_vlen != 0}; };
    auto pass = [&](const Pass (&PP)[1]) {
        const Pass &P0 = PP[0];
        Pass P = P0;               // window loads are relative to the current segment
        const uint32_t rel0 = P0.rbase + P0.sh;  // record start, relative to the resource
        uint32_t seg = 0;          // per lane: record offset of the current segment (after the last vlen field)
        uint32_t so = 0;           // uniform: offset of the next field inside the segment
        uint32_t R[WIN_DW];
        uint32_t wb = 0xFFFFFFFFu;  // segment offset of the window held in R (uniform)
        auto window = [&](uint32_t lo, uint32_t hi) {  // make segment bytes [lo, hi) available
            if (wb == 0xFFFFFFFFu || lo < wb || hi > wb + WIN_B) {
                wb = lo & ~3u;
                win_load<WIN_DW - 1>(R, P, wb);
            }
        };
        for (uint32_t f = 0; f < nf; ++f) {
            uint32_t dx, dy, col_off;
            if (f < NGZ_LANE_FIELDS) {
                const uint4 &fs = f < 64 ? fA : fB;
                const uint32_t fl = f & 63;
                dx = lane_u32(fs.x, fl);
                dy = lane_u32(fs.y, fl);
                col_off = lane_u32(fs.z, fl);
            } else {  // wide template: wave-uniform descriptor through the scalar cache
                const uint4 fs = sload(ft + f);
                dx = fs.x;
                dy = fs.y;
                col_off = fs.z;
            }
            const uint32_t len = dx >> 16, width = dy & 0xFFFF, kind = (dy >> 16) & 0xFF;
            const uint32_t off = seg + so;  // record offset of the field (per lane after a vlen field)
            if (kind == NGZ_K_FAIL) {
                // template-constant failure: only the chunk's first record matters
                // (vlen templates never get here: the framing walk stops at it)
                fail_field(P0, off, f);
                so += len;
                continue;
            }
            if (kind == NGZ_K_VLEN) {
                // u8 length, 255 -> 3-byte length (generator.rs:1775-1793); column = {u64 batch offset, u32 len, 0}
                window(so, so + 4);
                uint32_t L = rbyte(R, so - wb), hdr = 1;
                if (L == 255) {
                    L = (uint32_t)rbe(R, so + 1 - wb, 3);
                    hdr = 4;
                }
                const uint32_t data = off + hdr;  // record offset of the value
                if (P.valid) {
                    const uint64_t at = P0.a0 + rel0 + data;
                    ColSt(P, col_off, 16).b128(P.lrow * 16, (uint32_t)at, (uint32_t)(at >> 32), L, 0);
                    if ((dy >> 31) && !utf8_valid_global(P.rsrc, rel0 + data, L, false))  // vlen string
                        rec_error(P0, data, E_REC_UTF8, f, L);
                }
                seg = data + L;  // the next segment starts after the value
                so = 0;
                P.rbase = (rel0 + seg) & ~3u;
                P.sh = (rel0 + seg) & 3u;
                P.any_sh = __builtin_amdgcn_ballot_w64(P.sh != 0) != 0;
                wb = 0xFFFFFFFFu;
                continue;
            }
            if (kind == 0) { so += len; continue; }
            const bool raw = kind == NGZ_K_STR || kind == NGZ_K_BYTES || kind == NGZ_K_U256;
            if (kind == NGZ_K_STR && len > 64) check_str(R, P0, 0, off, f, len, false);
            // one window per field, or per 64-byte piece of a raw field
            for (uint32_t j = 0;; j += 64) {
                const uint32_t piece = raw ? min(64u, len - j) : 8u;
                const uint32_t lo = so + j;
                window(lo, lo + ((piece + 3) & ~3u));
                const uint32_t o = lo - wb;
                if (!raw) {
                    dec_num(R, P0, o, off, f, len, width, kind, col_off);
                    break;
                }
                if (kind == NGZ_K_STR && len <= 64) check_str(R, P0, o, off, f, len, true);
                const bool last = j + 64 >= len;
                dec_raw(R, P0, o, j, piece, width, col_off, last ? width : 0);
                if (last) break;
            }
            so += len;
        }
    };
    // slot by slot: chunk-mode slots through their chunk range, row-mode
    // slots through their row windows (specialised slots are skipped by want)
    for (uint32_t s = 0; s < B.n_slots; ++s) {
        const SlotRT rt = sload(&B.slots[s]);
        if (rt.total == 0 || !want(s)) continue;
        if (rt.mode == NGZ_MODE_ROW)
            run_windows<1, false>(B, s, shape, pass);
        else
            run_chunks<1, false>(B, rt.chunk0, rt.chunk0 + rt.nchunks, want, shape, pass);
    }
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

__global__ void __launch_bounds__(256) k_counts(BatchDev B) {
    __shared__ unsigned long long acc[NGZ_MAX_SLOTS];  // this block's processed_count increments
    if (B.summary->overflow) return;
    const uint32_t nsets = B.summary->n_sets;
    const uint32_t S = B.n_slots;
    for (uint32_t k = threadIdx.x; k < S; k += blockDim.x) acc[k] = 0;
    __syncthreads();
    const uint32_t lim = max(nsets, B.n);
    // grid-stride over sets and datagrams; the loop bound is uniform per block
    for (uint32_t base = blockIdx.x * blockDim.x; base < lim; base += gridDim.x * blockDim.x) {
        const uint32_t i = base + threadIdx.x;
        // final datagram status.  The status byte only moves OK -> ERROR, which
        // the count rule below treats alike, so threads reading this header
        // concurrently are unaffected.  NGZ_FR_HOST survives only in the
        // speculative pass, whose results the host discards and redoes with
        // the template-bearing datagrams host-framed.
        if (i < B.n) {
            ngz_dgram_hdr *h = &((ngz_dgram_hdr *)B.hdr)[i];
            if (h->err_key != NGZ_NO_ERR && h->status != NGZ_FR_UNSUPPORTED && h->status != NGZ_FR_HOST)
                h->status = NGZ_DG_ERROR;
        }
        uint32_t slot = 0;
        uint64_t inc = 0;
        if (i < nsets) {
            const ngz_set_info s = ((const ngz_set_info *)B.sets)[i];
            const ngz_dgram_hdr h = ((const ngz_dgram_hdr *)B.hdr)[s.dgram];
            slot = s.slot;
            const DevPlan &pl = B.plans[s.slot];
            if (h.status == NGZ_FR_NEED_MORE || h.status == NGZ_FR_UNSUPPORTED ||
                (((uint64_t)s.dgram << 16) | s.set_pos) <= pl.count_from) {  // before a re-announcement
                inc = 0;
            } else if (h.err_key == NGZ_NO_ERR) {
                // the whole message parsed: +1 per IPFIX set (ipfix.rs:223), +1 per NFv9 record (netflow.rs:218)
                inc = pl.proto == 10 ? 1 : s.n;
            } else {
                const uint32_t stop = (uint32_t)(h.err_key >> 48);
                const uint8_t *p = B.bytes + B.offsets[s.dgram];
                const uint32_t set_len = be16(p + s.set_pos + 2);
                if (pl.proto == 10) {
                    // the set's records all parsed (ipfix.rs:219-223); an UnexpectedEof at
                    // exactly the set end (available 0) is this set's failing record
                    const uint32_t code = (uint32_t)(h.err_key >> 40) & 0xFF;
                    const uint32_t end = s.set_pos + set_len;
                    inc = (stop > end || (stop == end && code != E_REC_EOF)) ? 1 : 0;
                } else {
                    // records fully parsed before the stop position
                    const uint32_t first = s.set_pos + 4, rl = pl.rec_len;
                    if (rl && stop > first) {
                        inc = (stop - first) / rl;
                        if (inc > s.n) inc = s.n;
                    }
                }
            }
        }
        // one LDS atomic per (wave, slot): consecutive sets mostly share a template
        uint64_t pending = __ballot(inc != 0);
        while (pending) {
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)pending) - 1;
            const uint32_t s0 = __builtin_amdgcn_readlane(slot, leader);
            const bool mine = inc != 0 && slot == s0;
            const uint64_t sum = wave_sum(mine ? inc : 0);
            if ((threadIdx.x & 63) == leader) atomicAdd(&acc[s0], (unsigned long long)sum);
            pending &= ~__ballot(mine);
        }
    }
    __syncthreads();
    // one global atomic per (block, slot with increments)
    for (uint32_t k = threadIdx.x; k < S; k += blockDim.x)
        if (acc[k]) atomicAdd(&B.proc_counts[k], acc[k]);
}

// End of a batch: the summary, the slot table and the processed_count
// increments go straight into the context's pinned host export buffers
// (device writes over the fabric, no copy commands), and the other parity's
// summary / increments are zeroed for the next batch.
__global__ void __launch_bounds__(256) k_export(BatchDev B, BatchSummary *h_summary, SlotRT *h_slots,
                                                unsigned long long *h_proc, BatchSummary *next_summary,
                                                unsigned long long *next_proc, unsigned long long *h_done,
                                                unsigned long long seq) {
    const uint32_t t = threadIdx.x, S = B.n_slots;
    if (t == 0) {
        *h_summary = *B.summary;
        *next_summary = BatchSummary{};
    }
    for (uint32_t i = t; i < S; i += blockDim.x) {
        h_slots[i] = B.slots[i];
        h_proc[i] = B.proc_counts[i];
    }
    for (uint32_t i = t; i < NGZ_MAX_SLOTS; i += blockDim.x) next_proc[i] = 0;  // the next batch may have more slots
    __threadfence_system();
    __syncthreads();
    // completion word last: the host may spin on it instead of a stream synchronisation
    if (t == 0) __hip_atomic_store(h_done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Column blocks to pinned host memory by the CUs (ngz_columns_to_host_async, NGZ_D2H_KERNEL): the
// stores cross PCIe as posted writes, so a copy engine stays free for the next batch's H2D and the
// link carries both directions at once (copy engine + copy engine measured 57 GB/s both ways
// together on MI355X, copy-engine H2D + this D2H 85 GB/s: tools/pcie_kernel_probe.hip).  Four
// independent 16-byte loads in flight per lane before their stores.
__global__ void __launch_bounds__(256) k_to_host(const uint4 *__restrict__ src, uint4 *__restrict__ dst, uint64_t n16) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (; i + 3 * step < n16; i += 4 * step) {
        const uint4 a = src[i], b = src[i + step], c = src[i + 2 * step], e = src[i + 3 * step];
        dst[i] = a;
        dst[i + step] = b;
        dst[i + 2 * step] = c;
        dst[i + 3 * step] = e;
    }
    for (; i < n16; i += step) dst[i] = src[i];
}

__global__ void __launch_bounds__(256) k_to_host_bytes(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                       uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

}  // namespace

// ---------------------------------------------------------------------------
// launch wrappers (C linkage, used by ngz_host.cpp)
// ---------------------------------------------------------------------------
// Arena placement probe (ngz_host.cpp place_arena, NGZ_OPT_PLACE_PROBE): the memory pattern of a
// slot's LDS-staged decode without the parse -- 1024-row windows dealt XCD-aware as win_seq deals
// them, each reading its record bytes with 16-byte loads and writing every column's run of the
// window with 16-byte nontemporal stores at the slot's column stride -- over the first `frac16`
// sixteenths of each XCD's stretch of windows.  The slow placement mode is DRAM contention among
// those concurrent streams, set by the arena's pages and the stride, so a short
// probe of the same streams ranks arenas without decoding the batch on each.
struct ProbeCols {
    uint32_t n;
    uint32_t w[32];    // column widths (the probe takes the slot's first 32 columns)
    uint32_t off[32];  // column offset factors (bytes per row before the column)
};
__global__ void __launch_bounds__(256) k_place_probe(const uint8_t *__restrict__ in, uint64_t in_bytes,
                                                     uint8_t *__restrict__ blk, uint32_t cap, uint32_t total,
                                                     uint32_t rec_len, uint32_t frac16, ProbeCols C) {
    constexpr uint32_t ROWS = 1024;
    const uint32_t nwin = (total + ROWS - 1) / ROWS;
    // win_seq's dealing (ngz_dev.h): block b works through the (b % 8)-th contiguous eighth of the windows
    const uint32_t G = gridDim.x, X = (G % 8 == 0 && G >= 8) ? 8u : 1u;
    const uint32_t x = blockIdx.x % X, l = blockIdx.x / X;
    const uint32_t per = (nwin + X - 1) / X;
    const uint32_t start = min(nwin, x * per), end = min(nwin, start + per);
    const uint32_t lim = start + ((end - start) * frac16 + 15) / 16;
    const uint64_t n16 = in_bytes >> 4;
    const __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void *)in, (short)0, 0x7FFFFFF0, 0x00020000);
    for (uint32_t W = start + l; W < end && W < lim; W += G / X) {
        // the window's record bytes: ROWS * rec_len from the batch (wrapping), 16 B per thread per step
        const uint64_t b0 = ((uint64_t)W * ROWS * rec_len >> 4) % (n16 ? n16 : 1);
        const uint32_t pieces = ROWS * rec_len / 16;
        uint32_t acc = 0;
        for (uint32_t p = threadIdx.x; p < pieces; p += blockDim.x) {
            const uint64_t q = (b0 + p) % (n16 ? n16 : 1);
            const v4u v = __builtin_amdgcn_raw_buffer_load_b128(ri, (uint32_t)(q << 4) & 0x7FFFFFF0u, 0, 0);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
        const uint32_t rows = min(ROWS, total - W * ROWS);
        for (uint32_t c = 0; c < C.n; ++c) {
            const uint32_t w = C.w[c];
            uint8_t *dst = blk + (uint64_t)cap * C.off[c] + (uint64_t)W * ROWS * w;
            const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, 0x7FFFFFF0, 0x00020000);
            const uint32_t n = rows * w / 16;
            for (uint32_t p = threadIdx.x; p < n; p += blockDim.x) {
                const v4u x = {acc, acc ^ p, acc + p, acc};
                __builtin_amdgcn_raw_buffer_store_b128(x, ro, 16 * p, 0, NGZ_ST_AUX);
            }
        }
    }
}

extern "C" int ngz_launch_place_probe(const uint8_t *in, uint64_t in_bytes, uint8_t *blk, uint32_t cap, uint32_t total,
                                      uint32_t rec_len, uint32_t frac16, const uint32_t *w, const uint32_t *off,
                                      uint32_t ncol, uint32_t grid, hipStream_t st) {
    ProbeCols C{};
    C.n = ncol < 32 ? ncol : 32;
    for (uint32_t i = 0; i < C.n; ++i) {
        C.w[i] = w[i];
        C.off[i] = off[i];
    }
    hipLaunchKernelGGL(k_place_probe, dim3(grid), dim3(256), 0, st, in, in_bytes, blk, cap, total, rec_len, frac16, C);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

#ifdef NGZ_EXPERIMENTS
// Experiment builds only ("walk the variable-length records next to the data they
// decode"): how fast can the record walk run once the sets' bytes sit in LDS?  Over the last batch's
// set table, the variable-length sets only:
//   mode 0: one lane per set walks it from HBM (the walk of k_frame, alone);
//   mode 1: each wave stages up to 64 consecutive sets (as many as fit its kWaveLds bytes) with
//           coalesced 16-byte loads, 8 in flight per lane, then one lane per staged set walks it in LDS;
//   mode 2: mode 1's staging without the walk.
// out[0] += records walked, out[1] += sets whose count differs from the framing's.  kWaveLds sets the
// waves per CU (four waves per workgroup): 8 KB 20, 12 KB 12, 16 KB 8, 36 KB 4.
template <uint32_t kWaveLds>
__global__ void __launch_bounds__(256) k_walk_probe(const uint8_t *__restrict__ bytes, uint64_t bytes_size,
                                                    const uint64_t *__restrict__ offsets,
                                                    const ngz_set_info *__restrict__ sets, uint32_t nsets,
                                                    const DevPlan *__restrict__ plans, uint32_t mode,
                                                    uint32_t *__restrict__ out) {
    constexpr uint32_t kPieces = kWaveLds / 16;
    __shared__ uint4 stage[4][kPieces];
    __shared__ uint32_t tab[4][65];
    __shared__ uint64_t atab[4][64];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t gw = blockIdx.x * 4 + wv, nw = gridDim.x * 4;
    uint32_t recs = 0, bad = 0;
    if (mode == 0) {
        for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < nsets; j += gridDim.x * blockDim.x) {
            const ngz_set_info si = sets[j];
            const DevPlan &pl = plans[si.slot];
            if (!pl.has_vlen) continue;
            const uint8_t *p = bytes + offsets[si.dgram];
            const uint32_t len = ((uint32_t)p[si.set_pos + 2] << 8) | p[si.set_pos + 3];
            uint64_t err = NGZ_NO_ERR;
            const uint32_t n = ngz_vlen_walk(p, si.set_pos + 4u, si.set_pos + len, pl, &err, [](uint32_t, uint32_t) {});
            recs += n;
            bad += n != si.n;
        }
    } else {
        const uint32_t per = (nsets + nw - 1) / nw;
        uint32_t s = min(nsets, gw * per);
        const uint32_t se = min(nsets, s + per);
        while (s < se) {
            const uint32_t j = s + lane;
            ngz_set_info si{};
            bool v = false;
            uint32_t len = 0, pieces = 0;
            uint64_t a = 0, a0 = 0;
            if (j < se) {
                si = sets[j];
                v = plans[si.slot].has_vlen;
                a = offsets[si.dgram] + si.set_pos;
                len = ((uint32_t)bytes[a + 2] << 8) | bytes[a + 3];
                a0 = a & ~15ull;
                if (v) pieces = (uint32_t)((a + len + 15 - a0) >> 4);
            }
            uint32_t inc = pieces;
#pragma unroll
            for (uint32_t o = 1; o < 64; o <<= 1) {
                const uint32_t t = __shfl_up(inc, o);
                if (lane >= o) inc += t;
            }
            const uint64_t take = __ballot(j < se && inc <= kPieces);
            const uint32_t k = take == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~take);
            if (k == 0) {  // one set larger than the wave's stage: walk it from HBM
                if (lane == 0 && v) {
                    uint64_t err = NGZ_NO_ERR;
                    const uint8_t *p = bytes + offsets[si.dgram];
                    const uint32_t n = ngz_vlen_walk(p, si.set_pos + 4u, si.set_pos + len, plans[si.slot], &err,
                                                     [](uint32_t, uint32_t) {});
                    recs += n;
                    bad += n != si.n;
                }
                s += 1;
                continue;
            }
            if (lane < k) {
                tab[wv][lane] = inc - pieces;
                atab[wv][lane] = a0;
            }
            if (lane == k - 1) tab[wv][k] = inc;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t total = tab[wv][k];
            for (uint32_t b = 0; b < total; b += 8 * 64) {
                uint4 x[8];
                uint32_t at[8];
#pragma unroll
                for (uint32_t i = 0; i < 8; ++i) {
                    const uint32_t q = b + 64 * i + lane;
                    at[i] = q;
                    x[i] = make_uint4(0, 0, 0, 0);
                    if (q < total) {
                        uint32_t lo = 0, hi = k;  // owner: the last set whose first piece is <= q
                        while (hi - lo > 1) {
                            const uint32_t m = (lo + hi) >> 1;
                            if (tab[wv][m] <= q) lo = m; else hi = m;
                        }
                        const uint64_t g = atab[wv][lo] + 16ull * (q - tab[wv][lo]);
                        if (g + 16 <= bytes_size) x[i] = *(const uint4 *)(bytes + g);
                    }
                }
#pragma unroll
                for (uint32_t i = 0; i < 8; ++i)
                    if (at[i] < total) stage[wv][at[i]] = x[i];
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (mode == 1 && lane < k && v) {
                const uint8_t *ps = (const uint8_t *)&stage[wv][tab[wv][lane]] + (uint32_t)(a - a0);
                uint64_t err = NGZ_NO_ERR;
                const uint32_t n = ngz_vlen_walk(ps, 4u, len, plans[si.slot], &err, [](uint32_t, uint32_t) {});
                recs += n;
                bad += n != si.n;
            } else if (mode == 2 && lane < k && v) {
                recs += ((const uint8_t *)&stage[wv][tab[wv][lane]])[(uint32_t)(a - a0) + 3] != 0xEEu;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            s += k;
        }
    }
    if (recs) atomicAdd(&out[0], recs);
    if (bad) atomicAdd(&out[1], bad);
}

extern "C" int ngz_launch_walk_probe(const uint8_t *bytes, uint64_t bytes_size, const uint64_t *offsets,
                                     const ngz_set_info *sets, uint32_t nsets, const DevPlan *plans, uint32_t mode,
                                     uint32_t lds_kb, uint32_t grid, uint32_t *out, hipStream_t st) {
    if (lds_kb == 8)
        hipLaunchKernelGGL(k_walk_probe<8192>, dim3(grid), dim3(256), 0, st, bytes, bytes_size, offsets, sets, nsets, plans, mode, out);
    else if (lds_kb == 12)
        hipLaunchKernelGGL(k_walk_probe<12288>, dim3(grid), dim3(256), 0, st, bytes, bytes_size, offsets, sets, nsets, plans, mode, out);
    else if (lds_kb == 16)
        hipLaunchKernelGGL(k_walk_probe<16384>, dim3(grid), dim3(256), 0, st, bytes, bytes_size, offsets, sets, nsets, plans, mode, out);
    else if (lds_kb == 36)
        hipLaunchKernelGGL(k_walk_probe<36864>, dim3(grid), dim3(256), 0, st, bytes, bytes_size, offsets, sets, nsets, plans, mode, out);
    else
        return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
#endif

extern "C" int ngz_launch_frame(const BatchDev *B, const uint32_t *hf_flag, const uint32_t *hf_first, hipStream_t st) {
    const uint32_t nb = (B->n + kFrameBlock - 1) / kFrameBlock;
    if (nb) hipLaunchKernelGGL(k_frame, dim3(nb), dim3(kFrameBlock), 0, st, *B, hf_flag, hf_first);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int ngz_launch_frame_vlen(const BatchDev *B, hipStream_t st) {
    const uint32_t nb = (B->n + kFrameBlock - 1) / kFrameBlock;
    if (nb) hipLaunchKernelGGL(k_frame_vlen, dim3(nb), dim3(kFrameBlock), 0, st, *B);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int ngz_scan_temp_bytes(uint64_t n_items, size_t *bytes) {
    *bytes = 0;
    return hipcub::DeviceScan::ExclusiveSum(nullptr, *bytes, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)n_items) ==
                   hipSuccess
               ? 0
               : -1;
}

extern "C" int ngz_launch_scan(void *temp, size_t temp_bytes, const uint32_t *in, uint32_t *out, uint64_t n_items,
                               hipStream_t st) {
    return hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, in, out, (int)n_items, st) == hipSuccess ? 0 : -1;
}

extern "C" int ngz_launch_layout_emit(const BatchDev *B, const uint32_t *hf_flag, const uint32_t *hf_first,
                                      hipStream_t st) {
    hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, st, *B);
    const uint32_t nb = (B->n + 255) / 256;
    if (nb) hipLaunchKernelGGL(k_emit, dim3(nb), dim3(256), 0, st, *B, hf_flag, hf_first);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int ngz_launch_layout(const BatchDev *B, hipStream_t st) {
    hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, st, *B);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int ngz_launch_emit(const BatchDev *B, hipStream_t st) {
    const uint32_t nb = (B->n + 255) / 256;
    if (nb) hipLaunchKernelGGL(k_emit, dim3(nb), dim3(256), 0, st, *B, nullptr, nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int ngz_launch_decode_generic(const BatchDev *B, uint32_t grid, hipStream_t st) {
    if (grid) hipLaunchKernelGGL(k_decode_generic, dim3(grid), dim3(256), 0, st, *B);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

#ifndef NGZ_COUNTS_BLOCKS
#define NGZ_COUNTS_BLOCKS 1024  // config 4: 128 / 256 / 512 / 1024 / 8192 blocks took 134 / 71 / 48 / 43 / 110 us
#endif
extern "C" int ngz_launch_counts(const BatchDev *B, uint64_t set_cap, hipStream_t st) {
    // n_sets is known on device only; the grid also covers every datagram (finalize).  At most
    // NGZ_COUNTS_BLOCKS blocks striding (profiles/r5/cfg4_counts_grid.txt)
    const uint64_t nb = std::min<uint64_t>((std::max<uint64_t>(set_cap, B->n) + 255) / 256, NGZ_COUNTS_BLOCKS);
    if (nb) hipLaunchKernelGGL(k_counts, dim3((uint32_t)nb), dim3(256), 0, st, *B);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// dst: a device-visible address of pinned host memory
extern "C" int ngz_launch_to_host(const void *src, void *dst, uint64_t bytes, hipStream_t st) {
    if (!bytes) return 0;
    const uint64_t n16 = ((uintptr_t)src | (uintptr_t)dst) & 15 ? 0 : bytes / 16;
    if (n16) {
        const uint32_t nb = (uint32_t)std::min<uint64_t>((n16 + 255) / 256, 512);
        hipLaunchKernelGGL(k_to_host, dim3(nb), dim3(256), 0, st, (const uint4 *)src, (uint4 *)dst, n16);
    }
    const uint64_t rest = bytes - 16 * n16;
    if (rest) {
        const uint32_t nb = (uint32_t)std::min<uint64_t>((rest + 255) / 256, 512);
        hipLaunchKernelGGL(k_to_host_bytes, dim3(nb), dim3(256), 0, st, (const uint8_t *)src + 16 * n16,
                           (uint8_t *)dst + 16 * n16, rest);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int ngz_launch_export(const BatchDev *B, BatchSummary *h_summary, SlotRT *h_slots,
                                 unsigned long long *h_proc, BatchSummary *next_summary,
                                 unsigned long long *next_proc, unsigned long long *h_done, unsigned long long seq,
                                 hipStream_t st) {
    hipLaunchKernelGGL(k_export, dim3(1), dim3(256), 0, st, *B, h_summary, h_slots, h_proc, next_summary, next_proc,
                       h_done, seq);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
