// HIP kernels for gfx950 (CDNA4): datagram framing, record counting/layout
// and the LDS-staged columnar record decode.
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

#include "ngz/flow_decode.h"
#include "ngz_internal.h"

namespace {

__device__ __forceinline__ uint32_t ld8(const uint8_t *p) { return p[0]; }
__device__ __forceinline__ uint32_t be16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }
__device__ __forceinline__ uint32_t be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
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
        for (uint32_t i = hf_first[d]; i < hf_first[d + 1]; ++i) {
            const HostSet &h = B.hf_sets[i];
            vis.on_set(h.set_pos, h.slot, h.n, h.payload_pos, B.plans[h.slot].rec_len);
        }
        return;
    }
    const uint8_t *p = B.bytes + B.offsets[d];
    const uint32_t dl = B.lengths[d];
    // codec.rs:197-209: need the 16-byte header and buf.len() >= u16 at [2..4]
    if (dl < 16) { o.status = NGZ_FR_NEED_MORE; return; }
    const uint32_t ver = be16(p), len = be16(p + 2);
    if (dl < len) { o.status = NGZ_FR_NEED_MORE; return; }
    o.version = ver;
    o.length = len;
    if (ver == 10) {
        if (len < 16) {  // ipfix.rs:69-75
            o.status = NGZ_FR_ERROR;
            o.err = ngz_err_key(2, E_IPFIX_INVALID_LENGTH, 0, len);
            return;
        }
        o.time = be32(p + 4);
        o.seq = be32(p + 8);
        o.domain = be32(p + 12);
        uint32_t pos = 16;
        while (pos < len) {  // ipfix.rs:94-96
            const uint32_t rem = len - pos;
            if (rem < 2) { o.status = NGZ_FR_ERROR; o.err = ngz_err_key(pos, E_SET_EOF_ID, 2, rem); return; }
            const uint32_t id = be16(p + pos);
            if (id != 2 && id != 3 && id < 256) {  // ipfix.rs:142-150
                o.status = NGZ_FR_ERROR; o.err = ngz_err_key(pos, E_SET_INVALID_ID, id, 0); return;
            }
            if (rem < 4) { o.status = NGZ_FR_ERROR; o.err = ngz_err_key(pos + 2, E_SET_EOF_LEN, 2, rem - 2); return; }
            const uint32_t sl = be16(p + pos + 2);
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
            const uint32_t minlen = pl.rec_len;  // ipfix.rs:193-214
            const uint32_t n = minlen ? (sl - 4) / minlen : 0;  // :219 loop bound
            if (n && !pl.rpl) { o.status = NGZ_FR_UNSUPPORTED; return; }
            o.nsets++;
            vis.on_set(pos, slot, n, pos + 4, minlen);
            pos += sl;  // leftover (padding or garbage) ignored: ipfix.rs:224-227
        }
        return;
    }
    if (ver == 9) {
        if (dl < 20) {  // header read_u32 of source_id (netflow.rs:86)
            o.status = NGZ_FR_ERROR; o.err = ngz_err_key(16, E_HDR_EOF, 4, dl - 16); return;
        }
        o.sysup = be32(p + 4);
        o.time = be32(p + 8);
        o.seq = be32(p + 12);
        o.domain = be32(p + 16);
        const uint32_t count = len;
        uint32_t i = count, pos = 20;
        while (i > 0 && dl - pos > 3) {  // netflow.rs:89
            const uint32_t rem = dl - pos;
            const uint32_t id = be16(p + pos);
            if (id != 0 && id != 1 && id < 256) {
                o.status = NGZ_FR_ERROR; o.err = ngz_err_key(pos, E_SET_INVALID_ID, id, 0); return;
            }
            const uint32_t sl = be16(p + pos + 2);
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

struct CountVis {
    uint32_t *counts;
    uint32_t N, S, d;
    uint32_t chunks, sets;
    const DevPlan *plans;
    __device__ void on_set(uint32_t, uint32_t slot, uint32_t n, uint32_t, uint32_t) {
        counts[(uint64_t)slot * N + d] += n;
        if (n) chunks += (n + plans[slot].window - 1) / plans[slot].window + 1;
        sets += 1;
    }
};

__global__ void k_frame(BatchDev B, const uint32_t *hf_flag, const uint32_t *hf_first) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= B.n) return;
    CountVis vis{B.counts, B.n, B.n_slots, d, 0, 0, B.plans};
    WalkOut o;
    walk_datagram(B, hf_flag, hf_first, d, o, vis);
    if (o.status != NGZ_FR_HOST && !(hf_flag && hf_flag[d]) && has_template_sets(B, d)) o.status = NGZ_FR_HOST;
    const uint64_t N = B.n;
    B.counts[(uint64_t)B.n_slots * N + d] = vis.chunks;
    B.counts[(uint64_t)(B.n_slots + 1) * N + d] = vis.sets;
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

// Column layout: slot-major rows of the scanned count matrix give each slot a
// dense, stream-ordered row range; columns of a slot are laid out
// column-major inside one 256-byte aligned block of cap*row_bytes bytes.
__global__ void k_layout(BatchDev B) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint64_t N = B.n;
    const uint32_t S = B.n_slots;
    uint64_t off = 0;
    for (uint32_t s = 0; s < S; ++s) {
        const uint32_t base = B.scan[(uint64_t)s * N];
        const uint32_t next = B.scan[(uint64_t)(s + 1) * N];
        const uint32_t total = next - base;
        const uint32_t w = B.plans[s].window ? B.plans[s].window : 64;
        const uint32_t cap = total ? ((total + w - 1) / w) * w : 0;
        SlotRT rt;
        rt.block = off;
        rt.cap = cap;
        rt.total = total;
        rt.base = base;
        rt.reserved = 0;
        B.slots[s] = rt;
        off += ((uint64_t)cap * B.plans[s].row_bytes + 255) & ~255ull;
    }
    const uint64_t last = (uint64_t)(S + 2) * N;
    const uint32_t grand = B.scan[last];
    const uint32_t rec_total = B.scan[(uint64_t)S * N];
    const uint32_t chunks = B.scan[(uint64_t)(S + 1) * N] - rec_total;
    const uint32_t sets = grand - B.scan[(uint64_t)(S + 1) * N];
    B.summary->n_records_total = rec_total;
    B.summary->n_chunks = chunks;
    B.summary->n_sets = sets;
    B.summary->arena_used = off;
    uint32_t ov = 0;
    if (off > B.arena_cap) ov |= 1;
    if (chunks > B.chunk_cap) ov |= 2;
    if (sets > B.set_cap) ov |= 4;
    B.summary->overflow = ov;
}

struct EmitVis {
    const BatchDev *B;
    uint32_t d;
    uint64_t dg_off;
    uint32_t chunk_at, set_at;
    bool ok;
    __device__ void on_set(uint32_t set_pos, uint32_t slot, uint32_t n, uint32_t payload_pos, uint32_t rl) {
        const uint64_t N = B->n;
        uint32_t *cell = &B->scan[(uint64_t)slot * N + d];
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
        const uint32_t W = B->plans[slot].window;
        const uint32_t reserved = (n + W - 1) / W + 1;
        uint32_t r = 0, used = 0;
        while (r < n) {
            const uint32_t cstart = rec0 + r;
            const uint32_t wend = (cstart / W + 1) * W;
            const uint32_t take = min(n - r, wend - cstart);
            Chunk c;
            c.src = dg_off + payload_pos + (uint64_t)r * rl;
            c.rec0 = cstart;
            c.dgram = d;
            c.n = (uint16_t)take;
            c.slot = (uint16_t)slot;
            c.pos0 = (uint16_t)(payload_pos + r * rl);
            c.reserved = 0;
            c.reserved2 = 0;
            B->chunks[chunk_at + used] = c;
            ++used;
            r += take;
        }
        for (; used < reserved; ++used) {
            Chunk c = {};
            B->chunks[chunk_at + used] = c;
        }
        chunk_at += reserved;
    }
};

__global__ void k_emit(BatchDev B, const uint32_t *hf_flag, const uint32_t *hf_first) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= B.n) return;
    if (B.summary->overflow) return;
    const uint64_t N = B.n;
    const uint32_t S = B.n_slots;
    EmitVis vis;
    vis.B = &B;
    vis.d = d;
    vis.dg_off = B.offsets[d];
    vis.chunk_at = B.scan[(uint64_t)S * N + d] - B.scan[(uint64_t)S * N];
    vis.set_at = B.scan[(uint64_t)(S + 1) * N + d] - B.scan[(uint64_t)(S + 1) * N];
    vis.ok = true;
    WalkOut o;
    walk_datagram(B, hf_flag, hf_first, d, o, vis);
}

// ---------------------------------------------------------------------------
// Record decode: one wave (workgroup of 64) per chunk of <= 64*RPL records.
// 1) the chunk's bytes are staged HBM -> LDS with 16-byte buffer loads (one
//    pad dword per 2^pad_shift dwords to spread the strided reads over banks);
// 2) lane l owns RPL consecutive rows of every column: it reads each field of
//    its records from LDS, byte-swaps/widens in VGPRs and writes RPL*width
//    contiguous bytes per column, so a wave stores 64*RPL*width contiguous bytes.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t pidx(uint32_t q, uint32_t ps) { return q + (q >> ps); }

__device__ __forceinline__ uint32_t lds_dw(const uint32_t *lds, uint32_t q, uint32_t ps) { return lds[pidx(q, ps)]; }

// big-endian unsigned of `len` (0..8) bytes starting at staged byte x
__device__ __forceinline__ uint64_t read_be(const uint32_t *lds, uint32_t x, uint32_t len, uint32_t ps) {
    const uint32_t q = x >> 2, s = x & 3;
    const uint32_t d0 = lds_dw(lds, q, ps), d1 = lds_dw(lds, q + 1, ps);
    const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, s);
    if (len <= 4) {
        if (len == 0) return 0;
        return __builtin_bswap32(lo) >> (32 - 8 * len);
    }
    const uint32_t d2 = lds_dw(lds, q + 2, ps);
    const uint32_t hi = __builtin_amdgcn_alignbyte(d2, d1, s);
    const uint64_t v = ((uint64_t)__builtin_bswap32(lo) << 32) | __builtin_bswap32(hi);
    return v >> (64 - 8 * len);
}

__device__ __forceinline__ uint32_t read_byte(const uint32_t *lds, uint32_t x, uint32_t ps) {
    return (lds_dw(lds, x >> 2, ps) >> (8 * (x & 3))) & 0xFF;
}

// 4 raw bytes at staged byte x as a little-endian dword (wire order)
__device__ __forceinline__ uint32_t read_raw4(const uint32_t *lds, uint32_t x, uint32_t ps) {
    const uint32_t q = x >> 2;
    return __builtin_amdgcn_alignbyte(lds_dw(lds, q + 1, ps), lds_dw(lds, q, ps), x & 3);
}

// chrono NaiveDate range (0.4.45): -262143-01-01 .. +262142-12-31, in ms
__device__ constexpr int64_t kMinMillis = -8334601315200000LL;  // days_from_civil(-262143,1,1)*86400000
__device__ constexpr int64_t kMaxMillis = 8210266876799999LL;   // (days_from_civil(262142,12,31)+1)*86400000-1

template <int RPL>
__device__ __forceinline__ void store_num(uint8_t *col, uint32_t row0, uint32_t width, const uint64_t (&v)[RPL], uint32_t vmask) {
    constexpr uint32_t full = (1u << RPL) - 1;
    if (vmask == full) {
        if (width == 1) {
            if constexpr (RPL == 4) {
                *(uint32_t *)(col + row0) = (uint32_t)(v[0] & 0xFF) | ((uint32_t)(v[1] & 0xFF) << 8) |
                                            ((uint32_t)(v[2] & 0xFF) << 16) | ((uint32_t)(v[3] & 0xFF) << 24);
            } else if constexpr (RPL == 2) {
                *(uint16_t *)(col + row0) = (uint16_t)((v[0] & 0xFF) | ((v[1] & 0xFF) << 8));
            } else {
                col[row0] = (uint8_t)v[0];
            }
        } else if (width == 2) {
            if constexpr (RPL == 4) {
                uint2 w;
                w.x = (uint32_t)(v[0] & 0xFFFF) | ((uint32_t)(v[1] & 0xFFFF) << 16);
                w.y = (uint32_t)(v[2] & 0xFFFF) | ((uint32_t)(v[3] & 0xFFFF) << 16);
                *(uint2 *)(col + 2 * row0) = w;
            } else if constexpr (RPL == 2) {
                *(uint32_t *)(col + 2 * row0) = (uint32_t)(v[0] & 0xFFFF) | ((uint32_t)(v[1] & 0xFFFF) << 16);
            } else {
                *(uint16_t *)(col + 2 * row0) = (uint16_t)v[0];
            }
        } else if (width == 4) {
            if constexpr (RPL == 4) {
                uint4 w = make_uint4((uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3]);
                *(uint4 *)(col + 4 * row0) = w;
            } else if constexpr (RPL == 2) {
                *(uint2 *)(col + 4 * row0) = make_uint2((uint32_t)v[0], (uint32_t)v[1]);
            } else {
                *(uint32_t *)(col + 4 * row0) = (uint32_t)v[0];
            }
        } else {  // 8
            if constexpr (RPL == 4) {
                uint4 a = make_uint4((uint32_t)v[0], (uint32_t)(v[0] >> 32), (uint32_t)v[1], (uint32_t)(v[1] >> 32));
                uint4 b = make_uint4((uint32_t)v[2], (uint32_t)(v[2] >> 32), (uint32_t)v[3], (uint32_t)(v[3] >> 32));
                *(uint4 *)(col + 8 * row0) = a;
                *(uint4 *)(col + 8 * row0 + 16) = b;
            } else if constexpr (RPL == 2) {
                *(uint4 *)(col + 8 * row0) =
                    make_uint4((uint32_t)v[0], (uint32_t)(v[0] >> 32), (uint32_t)v[1], (uint32_t)(v[1] >> 32));
            } else {
                *(uint2 *)(col + 8 * row0) = make_uint2((uint32_t)v[0], (uint32_t)(v[0] >> 32));
            }
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
        if (!(vmask >> k & 1)) continue;
        uint8_t *dst = col + (uint64_t)(row0 + k) * width;
        if (width == 1) *dst = (uint8_t)v[k];
        else if (width == 2) *(uint16_t *)dst = (uint16_t)v[k];
        else if (width == 4) *(uint32_t *)dst = (uint32_t)v[k];
        else *(uint64_t *)dst = v[k];
    }
}

// raw byte columns (mac, mpls, ipv6, octets, strings, u256): `len` wire bytes
// copied to `width` column bytes (zero padded when width > len)
template <int RPL>
__device__ __forceinline__ void store_bytes(uint8_t *col, uint32_t row0, uint32_t width, uint32_t len,
                                            const uint32_t *lds, const uint32_t (&x)[RPL], uint32_t vmask,
                                            uint32_t ps) {
    constexpr uint32_t full = (1u << RPL) - 1;
    if (vmask == full && (width & 3) == 0 && len == width) {
        // every output dword lies inside one record
        uint32_t *dst = (uint32_t *)(col + (uint64_t)row0 * width);
        const uint32_t wd = width >> 2;
#pragma unroll
        for (int k = 0; k < RPL; ++k)
            for (uint32_t j = 0; j < wd; ++j) dst[k * wd + j] = read_raw4(lds, x[k] + 4 * j, ps);
        return;
    }
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
        if (!(vmask >> k & 1)) continue;
        uint8_t *dst = col + (uint64_t)(row0 + k) * width;
        uint32_t j = 0;
        if ((width & 3) == 0 && (((uintptr_t)dst) & 3) == 0) {
            for (; j + 4 <= len; j += 4) *(uint32_t *)(dst + j) = read_raw4(lds, x[k] + j, ps);
        }
        for (; j < len; ++j) dst[j] = (uint8_t)read_byte(lds, x[k] + j, ps);
        for (; j < width; ++j) dst[j] = 0;
    }
}

__device__ bool utf8_valid_prefix(const uint32_t *lds, uint32_t x, uint32_t len, uint32_t ps) {
    // validate bytes up to the first NUL (generator.rs:1651-1668)
    uint32_t i = 0;
    while (i < len) {
        const uint32_t c = read_byte(lds, x + i, ps);
        if (c == 0) return true;
        if (c < 0x80) { ++i; continue; }
        uint32_t need, lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) need = 1;
        else if (c >= 0xE0 && c <= 0xEF) { need = 2; if (c == 0xE0) lo = 0xA0; if (c == 0xED) hi = 0x9F; }
        else if (c >= 0xF0 && c <= 0xF4) { need = 3; if (c == 0xF0) lo = 0x90; if (c == 0xF4) hi = 0x8F; }
        else return false;
        for (uint32_t t = 1; t <= need; ++t) {
            if (i + t >= len) return false;
            const uint32_t b = read_byte(lds, x + i + t, ps);
            const uint32_t l2 = (t == 1) ? lo : 0x80, h2 = (t == 1) ? hi : 0xBF;
            if (b < l2 || b > h2) return false;
        }
        i += need + 1;
    }
    return true;
}

__device__ __forceinline__ uint32_t sgpr(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

typedef uint32_t v4u __attribute__((ext_vector_type(4)));
constexpr int STAGE_BATCH = 16;  // 16 x 1 KiB per wave in flight

struct ChunkS {  // chunk descriptor in SGPRs
    uint64_t src;
    uint32_t rec0, dgram, n, slot, pos0;
};

struct PlanS {  // plan header in SGPRs
    uint32_t rec_len, n_fields, rpl, ps;
};

template <int RPL>
__device__ void decode_chunk(const BatchDev &B, const ChunkS &c, const PlanS &P, const uint4 *ftab, uint32_t *lds) {
    const uint32_t lane = threadIdx.x;
    const uint32_t n = c.n;
    const uint32_t rl = P.rec_len;
    const uint32_t ps = P.ps;
    // ---- stage the chunk's bytes into LDS (16-byte buffer loads) ----
    const uint64_t a0 = c.src & ~15ull;
    const uint32_t sh = (uint32_t)(c.src - a0);
    const uint32_t total = sh + n * rl;
    const uint64_t avail64 = B.bytes_size - a0;
    const uint32_t avail = avail64 > 0x7FFFFFF0ull ? 0x7FFFFFF0u : (uint32_t)avail64;
    __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)(B.bytes + a0), (short)0, (int)avail, 0x00020000);
    const uint32_t nq = (total + 15) >> 4;
    // issue up to 16 x 16-byte loads per lane before the first LDS write, so a
    // 16 KB chunk costs one HBM round trip (not one per load)
    for (uint32_t q0 = 0; q0 < nq; q0 += 64 * STAGE_BATCH) {
        v4u v[STAGE_BATCH];
#pragma unroll
        for (int j = 0; j < STAGE_BATCH; ++j) {
            const uint32_t q = q0 + j * 64 + lane;
            v[j] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, q * 16, 0, 0);  // OOB -> 0
        }
#pragma unroll
        for (int j = 0; j < STAGE_BATCH; ++j) {
            const uint32_t q = q0 + j * 64 + lane;
            if (q < nq) {
                const uint32_t b = 4 * q;
                lds[pidx(b, ps)] = v[j][0];
                lds[pidx(b + 1, ps)] = v[j][1];
                lds[pidx(b + 2, ps)] = v[j][2];
                lds[pidx(b + 3, ps)] = v[j][3];
            }
        }
    }
    __syncthreads();
    // ---- this lane's rows ----
    const uint32_t W = 64 * RPL;
    const uint32_t wbase = c.rec0 & ~(W - 1);
    const uint32_t row0 = wbase + lane * RPL;  // first row this lane owns
    uint32_t vmask = 0;
    uint32_t xr[RPL];  // staged byte of each record
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
        const int32_t r = (int32_t)(row0 + k) - (int32_t)c.rec0;
        const bool ok = r >= 0 && (uint32_t)r < n;
        vmask |= (ok ? 1u : 0u) << k;
        xr[k] = ok ? sh + (uint32_t)r * rl : sh;
    }
    if (vmask) {
        const SlotRT rt = B.slots[c.slot];
        uint8_t *blk = B.arena + sgpr((uint32_t)rt.block) + ((uint64_t)sgpr((uint32_t)(rt.block >> 32)) << 32);
        const uint32_t cap = sgpr(rt.cap);
        const uint32_t nf = P.n_fields;
        for (uint32_t f = 0; f < nf; ++f) {
            const uint4 fdv = ftab[f];  // LDS broadcast read of the field descriptor
            const uint32_t off = sgpr(fdv.x & 0xFFFF), len = sgpr(fdv.x >> 16);
            const uint32_t width = sgpr(fdv.y & 0xFFFF), kind = sgpr((fdv.y >> 16) & 0xFF);
            const uint32_t col_off = sgpr(fdv.z);
            uint8_t *col = blk + (uint64_t)cap * col_off;
            uint32_t x[RPL];
#pragma unroll
            for (int k = 0; k < RPL; ++k) x[k] = xr[k] + off;
            switch (kind) {
            case NGZ_K_UINT:
            case NGZ_K_SCOPE32: {
                uint64_t v[RPL];
#pragma unroll
                for (int k = 0; k < RPL; ++k) v[k] = read_be(lds, x[k], len, ps);
                store_num<RPL>(col, row0, width, v, vmask);
                break;
            }
            case NGZ_K_TCPFLAGS: {
                uint64_t v[RPL];
#pragma unroll
                for (int k = 0; k < RPL; ++k) v[k] = read_be(lds, x[k], len, ps) & 0xFF;
                store_num<RPL>(col, row0, width, v, vmask);
                break;
            }
            case NGZ_K_SINT: {
                uint64_t v[RPL];
#pragma unroll
                for (int k = 0; k < RPL; ++k) {
                    const uint64_t u = read_be(lds, x[k], len, ps);
                    const uint32_t sh2 = len ? 64 - 8 * len : 0;
                    v[k] = (uint64_t)(((int64_t)(u << sh2)) >> sh2);
                }
                store_num<RPL>(col, row0, width, v, vmask);
                break;
            }
            case NGZ_K_BOOL: {
                uint64_t v[RPL];
#pragma unroll
                for (int k = 0; k < RPL; ++k) v[k] = read_byte(lds, x[k], ps) != 0;
                store_num<RPL>(col, row0, width, v, vmask);
                break;
            }
            case NGZ_K_DTMS: {
                uint64_t v[RPL];
#pragma unroll
                for (int k = 0; k < RPL; ++k) {
                    v[k] = read_be(lds, x[k], 8, ps);
                    const int64_t ms = (int64_t)v[k];
                    if ((vmask >> k & 1) && (ms < kMinMillis || ms > kMaxMillis)) {
                        const uint32_t pos = c.pos0 + (row0 + k - c.rec0) * rl + off;
                        atomicMin((unsigned long long *)&((ngz_dgram_hdr *)B.hdr)[c.dgram].err_key,
                                  (unsigned long long)ngz_err_key(pos, E_REC_DTMS, f, 0));
                    }
                }
                store_num<RPL>(col, row0, width, v, vmask);
                break;
            }
            case NGZ_K_DTFRAC: {
                uint64_t v[RPL];
#pragma unroll
                for (int k = 0; k < RPL; ++k) {
                    const uint32_t secs = (uint32_t)read_be(lds, x[k], 4, ps);
                    const uint32_t frac = (uint32_t)read_be(lds, x[k] + 4, 4, ps);
                    // (1_000_000_000f64 * (fraction as f64 / u32::MAX as f64)) as u32 (generator.rs:1764)
                    const double q = (double)frac / 4294967295.0;
                    const uint32_t ns = (uint32_t)(1000000000.0 * q);
                    v[k] = (uint64_t)secs | ((uint64_t)ns << 32);
                    if ((vmask >> k & 1) && ns >= 1000000000u && (secs % 60u) != 59u) {
                        const uint32_t pos = c.pos0 + (row0 + k - c.rec0) * rl + off;
                        atomicMin((unsigned long long *)&((ngz_dgram_hdr *)B.hdr)[c.dgram].err_key,
                                  (unsigned long long)ngz_err_key(pos, E_REC_DTFRAC, f, 0));
                    }
                }
                store_num<RPL>(col, row0, 8, v, vmask);
                break;
            }
            case NGZ_K_STR: {
#pragma unroll
                for (int k = 0; k < RPL; ++k) {
                    if ((vmask >> k & 1) && !utf8_valid_prefix(lds, x[k], len, ps)) {
                        const uint32_t pos = c.pos0 + (row0 + k - c.rec0) * rl + off;
                        atomicMin((unsigned long long *)&((ngz_dgram_hdr *)B.hdr)[c.dgram].err_key,
                                  (unsigned long long)ngz_err_key(pos, E_REC_UTF8, f, 0));
                    }
                }
                store_bytes<RPL>(col, row0, width, len, lds, x, vmask, ps);
                break;
            }
            case NGZ_K_BYTES:
            case NGZ_K_U256:
                store_bytes<RPL>(col, row0, width, len, lds, x, vmask, ps);
                break;
            case NGZ_K_FAIL: {
                // template-constant failure: only the chunk's first record matters
                if ((vmask & 1) && row0 == c.rec0) {
                    const uint32_t pos = c.pos0 + off;
                    atomicMin((unsigned long long *)&((ngz_dgram_hdr *)B.hdr)[c.dgram].err_key,
                              (unsigned long long)ngz_err_key(pos, E_REC_FAIL, f, 0));
                }
                break;
            }
            default:
                break;
            }
        }
    }
    __syncthreads();  // LDS reused by the next chunk
}

// one wave per workgroup; LDS = [field table of the current slot][staged chunk]
__global__ void __launch_bounds__(64) k_decode(BatchDev B) {
    extern __shared__ uint32_t lds_all[];
    uint4 *ftab = (uint4 *)lds_all;
    uint32_t *lds = lds_all + 4 * NGZ_MAXF;
    const uint32_t nchunks = sgpr(B.summary->n_chunks);
    if (sgpr(B.summary->overflow)) return;
    uint32_t cached = 0xFFFFFFFFu;
    PlanS P{};
    for (uint32_t ci = blockIdx.x; ci < nchunks; ci += gridDim.x) {
        const uint4 *cp = (const uint4 *)&B.chunks[ci];
        const uint4 c0 = cp[0], c1 = cp[1];
        ChunkS c;
        c.src = (uint64_t)sgpr(c0.x) | ((uint64_t)sgpr(c0.y) << 32);
        c.rec0 = sgpr(c0.z);
        c.dgram = sgpr(c0.w);
        c.n = sgpr(c1.x & 0xFFFF);
        c.slot = sgpr(c1.x >> 16);
        c.pos0 = sgpr(c1.y & 0xFFFF);
        if (c.n == 0) continue;
        if (c.slot != cached) {
            const DevPlan *pl = &B.plans[c.slot];
            const uint4 h0 = ((const uint4 *)pl)[0], h1 = ((const uint4 *)pl)[1];
            P.rec_len = sgpr(h0.x);
            P.n_fields = sgpr(h0.z & 0xFFFF);
            P.rpl = sgpr((h0.z >> 24) & 0xFF);
            P.ps = sgpr(h0.w & 0xFF);
            (void)h1;
            for (uint32_t i = threadIdx.x; i < P.n_fields; i += 64) ftab[i] = ((const uint4 *)pl->f)[i];
            cached = c.slot;
        }
        if (P.rpl == 4) decode_chunk<4>(B, c, P, ftab, lds);
        else if (P.rpl == 2) decode_chunk<2>(B, c, P, ftab, lds);
        else decode_chunk<1>(B, c, P, ftab, lds);
    }
}

// processed_count increments (ipfix.rs:223 once per set; netflow.rs:218 once
// per record), honouring where each message's parse stopped.
__global__ void k_counts(BatchDev B) {
    const uint32_t nsets = B.summary->n_sets;
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (B.summary->overflow || i >= nsets) return;
    const ngz_set_info s = ((const ngz_set_info *)B.sets)[i];
    const ngz_dgram_hdr h = ((const ngz_dgram_hdr *)B.hdr)[s.dgram];
    if (h.status == NGZ_FR_NEED_MORE || h.status == NGZ_FR_UNSUPPORTED) return;
    const uint32_t stop = h.err_key == NGZ_NO_ERR ? 0x10000u : (uint32_t)(h.err_key >> 48);
    const DevPlan &pl = B.plans[s.slot];
    const uint8_t *p = B.bytes + B.offsets[s.dgram];
    const uint32_t set_len = be16(p + s.set_pos + 2);
    if (pl.proto == 10) {
        if (stop >= s.set_pos + set_len) atomicAdd(&B.proc_counts[s.slot], 1ull);
    } else {
        // records fully parsed before the stop position
        const uint32_t first = s.set_pos + 4, rl = pl.rec_len;
        uint64_t k = 0;
        if (rl && stop > first) {
            k = (stop - first) / rl;
            if (k > s.n) k = s.n;
        }
        if (k) atomicAdd(&B.proc_counts[s.slot], (unsigned long long)k);
    }
}

__global__ void k_finalize(BatchDev B) {
    const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= B.n) return;
    ngz_dgram_hdr *h = &((ngz_dgram_hdr *)B.hdr)[d];
    // NGZ_FR_HOST survives only in the speculative pass, whose results the
    // host discards and redoes with the template-bearing datagrams host-framed
    if (h->err_key != NGZ_NO_ERR && h->status != NGZ_FR_UNSUPPORTED && h->status != NGZ_FR_HOST)
        h->status = NGZ_DG_ERROR;
}

}  // namespace

// ---------------------------------------------------------------------------
// launch wrappers (C linkage, used by ngz_host.cpp)
// ---------------------------------------------------------------------------
extern "C" int ngz_launch_frame(const BatchDev *B, const uint32_t *hf_flag, const uint32_t *hf_first, hipStream_t st) {
    const uint32_t nb = (B->n + 255) / 256;
    if (nb) hipLaunchKernelGGL(k_frame, dim3(nb), dim3(256), 0, st, *B, hf_flag, hf_first);
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

extern "C" int ngz_launch_decode(const BatchDev *B, uint32_t grid, uint32_t lds_bytes, hipStream_t st) {
    if (grid) hipLaunchKernelGGL(k_decode, dim3(grid), dim3(64), lds_bytes, st, *B);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int ngz_launch_counts(const BatchDev *B, uint64_t set_cap, hipStream_t st) {
    const uint64_t nb = (set_cap + 255) / 256;
    if (nb) hipLaunchKernelGGL(k_counts, dim3((uint32_t)nb), dim3(256), 0, st, *B);
    const uint32_t nd = (B->n + 255) / 256;
    if (nd) hipLaunchKernelGGL(k_finalize, dim3(nd), dim3(256), 0, st, *B);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
