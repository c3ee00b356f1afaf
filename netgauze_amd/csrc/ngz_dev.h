// Device-side record decode primitives, shared by the ahead-of-time generic
// decode kernel (ngz_kernels.hip) and the per-template kernels generated and
// compiled at run time with hiprtc (ngz_rtc.cpp embeds this file's text).
//
// Reference behaviour restated (file:line relative to the NetGauze checkout):
//   crates/flow-pkt/src/wire/deserializer/ipfix.rs:335-370 (DataRecord::parse),
//   netflow.rs:399-475 (NFv9 DataRecord / ScopeField), and the generated
//   Field::parse rules in crates/flow-pkt/ipfix-code-generator/src/generator.rs:
//   reduced-size unsigned/signed reads :1468-1562 via parse-utils/src/reader.rs:214-295,
//   tcpControlBits :1416-1417 (iana/src/tcp.rs:165-168), bool :1607-1619,
//   fixed strings :1635-1672, dateTimeMilliseconds :1725-1746,
//   dateTimeMicro/Nanoseconds :1748-1773, u256 :1498-1518.
//
// Record model: one lane decodes one record.  A lane holds an 80-byte window
// of its record in 20 VGPRs (five 16-byte buffer loads), re-aligned so that
// window byte 0 is record byte `wb`.  All field offsets are wave-uniform, so
// extraction is register selection (constant-folded in generated kernels,
// s_set_gpr_idx-indexed in the generic kernel), v_perm/v_alignbyte and shifts.
#pragma once
#include <stdint.h>

#include "ngz/flow_decode.h"
#include "ngz_internal.h"

// Cache policy (buffer instruction aux bits) of the generated kernels' record loads and column
// stores.  Column stores are nontemporal (2 = nt on gfx950): the columns are written once and not
// read back by the decode, and streaming them past the caches measured 1-2 % faster (T20 2.138 ->
// 2.098 ms, config 3 4.27 -> 4.22 ms, same box); nt record loads were 1.4-2x slower, so loads keep the
// default.  The generator overrides either from NGZ_LD_AUX / NGZ_ST_AUX (experiments), and an
// override is part of the kernel's cache signature.
#ifndef NGZ_LD_AUX
#define NGZ_LD_AUX 0
#endif
#ifndef NGZ_ST_AUX
#define NGZ_ST_AUX 2
#endif

namespace ngzdev {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr int WIN_DW = 20;      // dwords loaded per window (5 x 16 B)
constexpr uint32_t WIN_B = 76;  // record bytes usable in a window after re-alignment (19 dwords)

// chrono NaiveDate range (0.4.45): -262143-01-01 .. +262142-12-31, in ms
constexpr int64_t kMinMillis = -8334601315200000LL;  // days_from_civil(-262143,1,1)*86400000
constexpr int64_t kMaxMillis = 8210266876799999LL;   // (days_from_civil(262142,12,31)+1)*86400000-1

__device__ __forceinline__ uint32_t sgpr(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t sgpr64(uint64_t v) {
    return (uint64_t)sgpr((uint32_t)v) | ((uint64_t)sgpr((uint32_t)(v >> 32)) << 32);
}

// v_readlane as an unsigned value (the builtin returns int: widening it
// directly to 64 bits would sign-extend)
__device__ __forceinline__ uint32_t lane_u32(uint32_t v, uint32_t lane) {
    return (uint32_t)__builtin_amdgcn_readlane(v, lane);
}

// Wave-uniform load through the scalar cache (s_load_*): the pointer is cast to
// the constant address space, which is sound for tables no kernel writes while
// the reader runs (chunk descriptors, slot table, plans).  Scalar loads count
// on lgkmcnt, so they overlap the vector loads instead of queueing behind them.
template <class T>
__device__ __forceinline__ T sload(const T *p) {
    static_assert(sizeof(T) % 4 == 0, "dword-sized tables only");
    typedef const __attribute__((address_space(4))) uint32_t *cptr;
    const cptr q = (cptr)p;
    uint32_t w[sizeof(T) / 4];
#pragma unroll
    for (uint32_t i = 0; i < sizeof(T) / 4; ++i) w[i] = q[i];
    T out;
    __builtin_memcpy(&out, w, sizeof(T));
    return out;
}

// 4 wire bytes at uniform window byte offset o, as a little-endian dword
__device__ __forceinline__ uint32_t rdw(const uint32_t (&R)[WIN_DW], uint32_t o) {
    uint32_t q = o >> 2;
    q = q < WIN_DW - 2 ? q : WIN_DW - 2;
    if ((o & 3) == 0) return R[q];
    return __builtin_amdgcn_alignbyte(R[q + 1], R[q], o & 3);
}

__device__ __forceinline__ uint32_t rbyte(const uint32_t (&R)[WIN_DW], uint32_t o) {
    uint32_t q = o >> 2;
    q = q < WIN_DW - 1 ? q : WIN_DW - 1;
    return (R[q] >> (8 * (o & 3))) & 0xFF;
}

// big-endian unsigned of `len` (0..8) bytes at window byte offset o
// (read_unsigned32_be / read_unsigned64_be: right-aligned reduced size)
// Touches exactly window dwords [o/4, (o+len-1)/4].
__device__ __forceinline__ uint64_t rbe(const uint32_t (&R)[WIN_DW], uint32_t o, uint32_t len) {
    if (len == 0) return 0;
    if ((o & 3) + len <= 4) {  // inside one dword
        uint32_t q = o >> 2;
        q = q < WIN_DW - 1 ? q : WIN_DW - 1;
        return __builtin_bswap32(R[q] >> (8 * (o & 3))) >> (32 - 8 * len);
    }
    const uint32_t a = __builtin_bswap32(rdw(R, o));
    if (len <= 4) return a >> (32 - 8 * len);
    const uint32_t b = __builtin_bswap32(rdw(R, o + 4));
    return (((uint64_t)a << 32) | b) >> (64 - 8 * len);
}

// Everything one pass (64 rows, one per lane) needs; uniform except the
// per-lane row / record position / alignment.
struct Pass {
    __amdgpu_buffer_rsrc_t rsrc;  // the chunk's bytes (OOB reads return 0)
    uint8_t *blk;                 // slot's column block
    uint32_t cap;                 // rows per column
    uint32_t rbase;               // this lane's record start, dword aligned, relative to rsrc
    uint32_t sh;                  // this lane's record misalignment (0..3)
    bool any_sh;                  // some lane misaligned (uniform)
    bool valid;                   // this lane's row belongs to the chunk
    uint32_t row;                 // this lane's output row
    uint32_t prow;                // first row of the pass (uniform; row = prow + lrow)
    uint32_t wrow;                // LDS-staged kernels: prow relative to the workgroup window (uniform)
    uint32_t lrow;                // this lane's row within the pass
    uint32_t lane;
    uint32_t rec0;                // first row of the chunk
    uint32_t dgram;               // datagram of the chunk
    uint32_t recpos;              // this lane's record offset in the datagram (~0: row mode, derive from rabs)
    uint32_t pos0;                // chunk's first record offset in the datagram
    uint64_t a0;                  // batch byte offset of the resource base
    uint64_t rabs;                // row mode: this lane's record batch offset
    const uint64_t *offsets;      // datagram offsets (row-mode error positions)
    void *hdr;                    // ngz_dgram_hdr[] (errors)
    uint32_t img;                 // staged row mode: dword index of the group's bytes in ngz_vstage
                                  // (rbase/sh then relative to it); ~0: read through rsrc
};

// Load record dwords [wb/4, wb/4 + ND) of this lane's record into R[0, ND)
// (ND <= WIN_DW - 1).  Every load is a 16-byte aligned buffer_load_dwordx4
// (the resource base is 16-byte aligned): misaligned 16-byte loads cost ~11 %
// of HBM throughput on gfx950 (tools/hbm_probe2.hip).  The lane's window
// starts dsh = 0..3 dwords into its first aligned block, so ceil((ND+3)/4)
// blocks cover it (plus one dword when some lane's record is not
// dword-aligned and the last block has no spare dword); two v_bfi steps per
// dword shift the blocks down by dsh (per lane), then v_alignbyte by the
// record's byte misalignment sh when any lane has one.
template <int ND>
__device__ __forceinline__ void win_load(uint32_t (&R)[WIN_DW], const Pass &P, uint32_t wb) {
    constexpr int NB = (ND + 3 + 3) / 4;
    constexpr int NT = 4 * NB + 1;
    const uint32_t o = P.rbase + wb;  // dword aligned
    const uint32_t o16 = o & ~15u;
    uint32_t T[NT];
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(P.rsrc, o16 + 16 * i, 0, NGZ_LD_AUX);
        T[4 * i] = v[0];
        T[4 * i + 1] = v[1];
        T[4 * i + 2] = v[2];
        T[4 * i + 3] = v[3];
    }
    T[NT - 1] = 0;
    // the byte shift reads dword ND; with dsh = 3 it is block dword ND + 3
    if (P.any_sh && ND + 3 >= 4 * NB) T[NT - 1] = __builtin_amdgcn_raw_buffer_load_b32(P.rsrc, o16 + 16 * NB, 0, NGZ_LD_AUX);
    // per-lane dword shift by dsh (bitwise selects: a ternary on array
    // elements would become a dynamically indexed, scratch-allocated array)
    const uint32_t m0 = 0u - ((o >> 2) & 1u), m1 = 0u - ((o >> 3) & 1u);
    uint32_t U[NT - 1];
#pragma unroll
    for (int j = 0; j < NT - 1; ++j) U[j] = (T[j + 1] & m0) | (T[j] & ~m0);
    constexpr int NR = ND + 1 < WIN_DW ? ND + 1 : WIN_DW;
#pragma unroll
    for (int j = 0; j < NR; ++j) R[j] = (j + 2 < NT - 1 ? (U[j + 2] & m1) : 0u) | (U[j] & ~m1);
#pragma unroll
    for (int j = NR; j < WIN_DW; ++j) R[j] = 0;
    if (P.any_sh) {  // records not dword-aligned: shift the window to the record start
#pragma unroll
        for (int j = 0; j < ND; ++j) R[j] = __builtin_amdgcn_alignbyte(R[j + 1], R[j], P.sh);
    }
}

// Report a record error at byte `rec_off` of this lane's record (the datagram
// keeps the smallest key = the first error in parse order).
__device__ __forceinline__ void rec_error(const Pass &P, uint32_t rec_off, uint32_t code, uint32_t f, uint32_t b = 0) {
    const uint32_t recpos = P.recpos != 0xFFFFFFFFu ? P.recpos : (uint32_t)(P.rabs - P.offsets[P.dgram]);
    atomicMin((unsigned long long *)&((ngz_dgram_hdr *)P.hdr)[P.dgram].err_key,
              (unsigned long long)ngz_err_key(recpos + rec_off, code, f, b));
}

// Template-constant field failure (InvalidLength etc.): the first record of
// each set fails there; chunk mode reports it from the chunk's first row,
// row mode from every row (the smallest position per datagram wins).
__device__ __forceinline__ void fail_field(const Pass &P, uint32_t rec_off, uint32_t f) {
    if (P.valid && (P.recpos == 0xFFFFFFFFu || P.row == P.rec0)) rec_error(P, rec_off, E_REC_FAIL, f);
}

// Column `col_off` rows of a pass start at a uniform address: stores go
// through a buffer resource built from it in SGPRs, lanes add a small 32-bit
// offset (lrow*width + byte) -- no per-lane 64-bit column addresses, which
// would otherwise cost 2 VGPRs per column for the whole chunk loop.
typedef uint32_t v2u __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint8_t *pass_col(const Pass &P, uint32_t col_off, uint32_t width) {
    return P.blk + (uint64_t)P.cap * col_off + (uint64_t)P.prow * width;
}

// Direct column stores (buffer resource on the column's pass address)
struct ColGlb {
    __amdgpu_buffer_rsrc_t r;
    __device__ __forceinline__ ColGlb(const Pass &P, uint32_t col_off, uint32_t width)
        : r(__builtin_amdgcn_make_buffer_rsrc(pass_col(P, col_off, width), (short)0, 0x7FFFFFF0, 0x00020000)) {}
    __device__ __forceinline__ void b8(uint32_t off, uint32_t v) const {
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, r, off, 0, NGZ_ST_AUX);
    }
    __device__ __forceinline__ void b16(uint32_t off, uint32_t v) const {
        __builtin_amdgcn_raw_buffer_store_b16((uint16_t)v, r, off, 0, NGZ_ST_AUX);
    }
    __device__ __forceinline__ void b32(uint32_t off, uint32_t v) const {
        __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, NGZ_ST_AUX);
    }
    __device__ __forceinline__ void b64(uint32_t off, uint32_t lo, uint32_t hi) const {
        v2u x = {lo, hi};
        __builtin_amdgcn_raw_buffer_store_b64(x, r, off, 0, NGZ_ST_AUX);
    }
    __device__ __forceinline__ void b128(uint32_t off, uint32_t a, uint32_t b, uint32_t c, uint32_t d) const {
        v4u x = {a, b, c, d};
        __builtin_amdgcn_raw_buffer_store_b128(x, r, off, 0, NGZ_ST_AUX);
    }
    // one value of `width` bytes (1/2/4/8) at row lrow
    __device__ __forceinline__ void w(uint32_t lrow, uint32_t width, uint64_t v) const {
        if (width == 1) b8(lrow, (uint32_t)v);
        else if (width == 2) b16(2 * lrow, (uint32_t)v);
        else if (width == 4) b32(4 * lrow, (uint32_t)v);
        else b64(8 * lrow, (uint32_t)v, (uint32_t)(v >> 32));
    }
};

#if defined(NGZ_LDS_WAVES) || defined(NGZ_LDS_BYTES)
// LDS-staged generated kernels: the decode writes a workgroup window of ROWS
// rows into LDS, column-major (column f at ROWS*col_off, row r at + r*width),
// and the generated store step writes each column's run to HBM with 16-byte
// stores.  A per-template kernel is generated with NGZ_LDS_WAVES / NGZ_LDS_ROWB
// (ColSt = its LDS column); a multi-template kernel with NGZ_LDS_BYTES (the
// largest window image of its templates), each template body naming its own
// ColLds<ROWS>.
#ifndef NGZ_LDS_BYTES
#define NGZ_LDS_BYTES (NGZ_REG_WINDOW * NGZ_LDS_WAVES * NGZ_LDS_ROWB)
#endif
__shared__ __attribute__((aligned(16))) uint8_t ngz_lds[NGZ_LDS_BYTES];

template <uint32_t ROWS>
struct ColLds {
    uint32_t base;  // LDS byte offset of this pass's first row in the column
    __device__ __forceinline__ ColLds(const Pass &P, uint32_t col_off, uint32_t width)
        : base(ROWS * col_off + P.wrow * width) {}
    __device__ __forceinline__ void b8(uint32_t off, uint32_t v) const { ngz_lds[base + off] = (uint8_t)v; }
    __device__ __forceinline__ void b16(uint32_t off, uint32_t v) const {
        *(uint16_t *)&ngz_lds[base + off] = (uint16_t)v;
    }
    __device__ __forceinline__ void b32(uint32_t off, uint32_t v) const { *(uint32_t *)&ngz_lds[base + off] = v; }
    __device__ __forceinline__ void b64(uint32_t off, uint32_t lo, uint32_t hi) const {
        v2u x = {lo, hi};
        *(v2u *)&ngz_lds[base + off] = x;
    }
    __device__ __forceinline__ void b128(uint32_t off, uint32_t a, uint32_t b, uint32_t c, uint32_t d) const {
        v4u x = {a, b, c, d};
        *(v4u *)&ngz_lds[base + off] = x;
    }
    __device__ __forceinline__ void w(uint32_t lrow, uint32_t width, uint64_t v) const {
        if (width == 1) b8(lrow, (uint32_t)v);
        else if (width == 2) b16(2 * lrow, (uint32_t)v);
        else if (width == 4) b32(4 * lrow, (uint32_t)v);
        else b64(8 * lrow, (uint32_t)v, (uint32_t)(v >> 32));
    }
};

// Store step: `lanes` x 16 B of LDS at lds_off to the column whose run of
// this window starts at `dst` (uniform), byte `at` of the run.
__device__ __forceinline__ void lds_flush(uint8_t *dst, uint32_t at, uint32_t lds_off, uint32_t lanes) {
    const uint32_t lane = threadIdx.x & 63;
    if (lane < lanes) {
        const v4u x = *(const v4u *)&ngz_lds[lds_off + 16 * lane];
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, 0x7FFFFFF0, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(x, r, at + 16 * lane, 0, NGZ_ST_AUX);
    }
}
#endif
#ifdef NGZ_LDS_WAVES
constexpr uint32_t LDS_ROWS = NGZ_REG_WINDOW * NGZ_LDS_WAVES;
typedef ColLds<LDS_ROWS> ColSt;
#else
typedef ColGlb ColSt;
#endif

// Value of a numeric field (UINT/SCOPE32/TCPFLAGS/SINT/BOOL/DTMS/DTFRAC) at
// window offset o, in its column encoding; reports the field's errors.
__device__ __forceinline__ uint64_t num_value(const uint32_t (&R)[WIN_DW], const Pass &P, uint32_t o, uint32_t off,
                                              uint32_t f, uint32_t len, uint32_t kind) {
    uint64_t v;
    if (kind == NGZ_K_BOOL) {
        v = rbyte(R, o) != 0;
    } else if (kind == NGZ_K_DTFRAC) {
        const uint32_t secs = (uint32_t)rbe(R, o, 4);
        const uint32_t frac = (uint32_t)rbe(R, o + 4, 4);
        // (1_000_000_000f64 * (fraction as f64 / u32::MAX as f64)) as u32 (generator.rs:1764)
        const double q = (double)frac / 4294967295.0;
        const uint32_t ns = (uint32_t)(1000000000.0 * q);
        // chrono timestamp_opt: ns >= 1e9 only as a leap second (secs % 60 == 59)
        if (P.valid && ns >= 1000000000u && (secs % 60u) != 59u) rec_error(P, off, E_REC_DTFRAC, f);
        v = (uint64_t)secs | ((uint64_t)ns << 32);
    } else {
        v = rbe(R, o, kind == NGZ_K_DTMS ? 8 : len);
        if (kind == NGZ_K_TCPFLAGS) v &= 0xFF;  // TCPHeaderFlags::from(u16) keeps the low byte
        if (kind == NGZ_K_SINT) {
            const uint32_t s2 = len ? 64 - 8 * len : 0;
            v = (uint64_t)(((int64_t)(v << s2)) >> s2);
        }
        if (P.valid && kind == NGZ_K_DTMS && ((int64_t)v < kMinMillis || (int64_t)v > kMaxMillis))
            rec_error(P, off, E_REC_DTMS, f);
    }
    return v;
}

// Numeric field of one record per lane: one store of `width` bytes per lane
// (Col = ColSt: the kernel's column store, LDS in staged kernels; ColGlb: a
// direct HBM store, for the wide columns of a staged kernel).
template <class Col = ColSt>
__device__ __forceinline__ void dec_num(const uint32_t (&R)[WIN_DW], const Pass &P, uint32_t o, uint32_t off,
                                        uint32_t f, uint32_t len, uint32_t width, uint32_t kind, uint32_t col_off) {
    const uint64_t v = num_value(R, P, o, off, f, len, kind);
    if (P.valid) Col(P, col_off, width).w(P.lrow, width, v);
}

// Numeric field of C consecutive rows per lane (run_chunks<C, true>): the C
// values are packed into one C*width-byte store per lane when all C rows
// belong to the chunk (a wave writes 64*C*width contiguous bytes).
template <int C, class Col = ColSt>
__device__ __forceinline__ void dec_num_c(const uint32_t (&R)[C][WIN_DW], const Pass (&P)[C], uint32_t o, uint32_t off,
                                          uint32_t f, uint32_t len, uint32_t width, uint32_t kind, uint32_t col_off) {
    uint64_t v[C];
    bool full = true;
#pragma unroll
    for (int k = 0; k < C; ++k) {
        v[k] = num_value(R[k], P[k], o, off, f, len, kind);
        full = full && P[k].valid;
    }
    const Col cs(P[0], col_off, width);
    if (full) {
        const uint32_t at = P[0].lrow * width;  // lrow of record 0 = C*lane
        if (width == 1) {
            uint32_t w = 0;
#pragma unroll
            for (int k = 0; k < C; ++k) w |= (uint32_t)(v[k] & 0xFF) << (8 * k);
            if (C == 4) cs.b32(at, w);
            else if (C == 2) cs.b16(at, w);
            else cs.b8(at, w);
        } else if (width == 2) {
            uint32_t w[2] = {0, 0};
#pragma unroll
            for (int k = 0; k < C; ++k) w[k >> 1] |= (uint32_t)(v[k] & 0xFFFF) << (16 * (k & 1));
            if (C == 4) cs.b64(at, w[0], w[1]);
            else if (C == 2) cs.b32(at, w[0]);
            else cs.b16(at, w[0]);
        } else if (width == 4) {
            if (C == 4) cs.b128(at, (uint32_t)v[0], (uint32_t)v[1 % C], (uint32_t)v[2 % C], (uint32_t)v[3 % C]);
            else if (C == 2) cs.b64(at, (uint32_t)v[0], (uint32_t)v[1 % C]);
            else cs.b32(at, (uint32_t)v[0]);
        } else {
#pragma unroll
            for (int k = 0; k + 1 < C; k += 2)
                cs.b128(at + 8 * k, (uint32_t)v[k], (uint32_t)(v[k] >> 32), (uint32_t)v[k + 1], (uint32_t)(v[k + 1] >> 32));
            if (C == 1) cs.b64(at, (uint32_t)v[0], (uint32_t)(v[0] >> 32));
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < C; ++k)
        if (P[k].valid) cs.w(P[k].lrow, width, v[k]);
}

struct WindowBytes {
    const uint32_t (&R)[WIN_DW];
    uint32_t o;
    __device__ uint32_t operator()(uint32_t i) const { return rbyte(R, o + i); }
};

struct GlobalBytes {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t base;  // this lane's byte, relative to the resource
    __device__ uint32_t operator()(uint32_t i) const { return __builtin_amdgcn_raw_buffer_load_b8(rsrc, base + i, 0, 0); }
};

// std::str::from_utf8 of `len` bytes; with stop_at_nul only the bytes up to
// the first NUL (fixed-length strings, generator.rs:1651-1668)
template <class F>
__device__ bool utf8_valid_prefix(const F &byte_at, uint32_t len, bool stop_at_nul = true) {
    uint32_t i = 0;
    while (i < len) {
        const uint32_t c = byte_at(i);
        if (c == 0 && stop_at_nul) return true;
        if (c < 0x80) { ++i; continue; }
        uint32_t need, lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) need = 1;
        else if (c >= 0xE0 && c <= 0xEF) { need = 2; if (c == 0xE0) lo = 0xA0; if (c == 0xED) hi = 0x9F; }
        else if (c >= 0xF0 && c <= 0xF4) { need = 3; if (c == 0xF0) lo = 0x90; if (c == 0xF4) hi = 0x8F; }
        else return false;
        for (uint32_t t = 1; t <= need; ++t) {
            if (i + t >= len) return false;
            const uint32_t b = byte_at(i + t);
            const uint32_t l2 = (t == 1) ? lo : 0x80, h2 = (t == 1) ? hi : 0xBF;
            if (b < l2 || b > h2) return false;
        }
        i += need + 1;
    }
    return true;
}

// UTF-8 check of bytes [base, base+len) of a buffer resource: an ASCII fast
// path reads the bytes 16 at a time (any byte >= 0x80 in them -> the exact
// byte-wise check).  Strings made of ASCII are valid with or without the
// stop-at-NUL rule, so the fast path answers for both.
__device__ __forceinline__ bool utf8_valid_global(__amdgpu_buffer_rsrc_t r, uint32_t base, uint32_t len,
                                                  bool stop_at_nul) {
    const uint32_t end = base + len;
    uint32_t acc = 0;
    for (uint32_t a = base & ~3u; a < end; a += 16) {
        const v4u x = __builtin_amdgcn_raw_buffer_load_b128(r, a, 0, 0);
        const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int lo = (int)base - (int)(a + 4 * j), hi = (int)end - (int)(a + 4 * j);
            if (hi <= 0) break;
            uint32_t m = 0xFFFFFFFFu;
            if (lo > 0) m = lo >= 4 ? 0u : (m << (8 * lo));
            if (hi < 4) m &= 0xFFFFFFFFu >> (8 * (4 - hi));
            acc |= w[j] & m;
        }
    }
    if (!(acc & 0x80808080u)) return true;
    return utf8_valid_prefix(GlobalBytes{r, base}, len, stop_at_nul);
}

// UTF-8 check of a fixed string field (errors only; the bytes go through dec_raw)
__device__ __forceinline__ void check_str(const uint32_t (&R)[WIN_DW], const Pass &P, uint32_t o, uint32_t off,
                                          uint32_t f, uint32_t len, bool in_window) {
    if (!P.valid) return;
    const bool ok = in_window ? utf8_valid_prefix(WindowBytes{R, o}, len)
                              : utf8_valid_global(P.rsrc, P.rbase + P.sh + off, len, true);
    if (!ok) rec_error(P, off, E_REC_UTF8, f);
}

// Copy `piece` (<= 64) raw wire bytes at window offset o to column bytes
// [j, j+piece) of this lane's row; `pad_to` > 0 zero-fills [j+piece, pad_to)
// (u256: left-aligned, zero padded).
template <class Col = ColSt>
__device__ __forceinline__ void dec_raw(const uint32_t (&R)[WIN_DW], const Pass &P, uint32_t o, uint32_t j,
                                        uint32_t piece, uint32_t width, uint32_t col_off, uint32_t pad_to) {
    if (!P.valid) return;
    const Col cs(P, col_off, width);
    const uint32_t at = P.lrow * width + j;
    const bool dw = (width & 3) == 0 && (j & 3) == 0;
    uint32_t t = 0;
    if (dw && (width & 15) == 0 && (j & 15) == 0) {
        for (; t + 16 <= piece; t += 16) cs.b128(at + t, rdw(R, o + t), rdw(R, o + t + 4), rdw(R, o + t + 8), rdw(R, o + t + 12));
    }
    if (dw)
        for (; t + 4 <= piece; t += 4) cs.b32(at + t, rdw(R, o + t));
    for (; t < piece; ++t) cs.b8(at + t, rbyte(R, o + t));
    for (uint32_t z = j + piece; z < pad_to; ++z) cs.b8(at + z - j, 0);
}

// Raw field of C consecutive rows per lane (run_chunks<C, true>), whole field
// in the window and len == width (ipv6, mac, MPLS labels, short octet arrays):
// the C records' bytes are concatenated in registers and written as
// C*width/4 dwords (C*width contiguous bytes per lane), instead of per-record
// byte stores.  Other cases go record by record through dec_raw.
template <int C, class Col = ColSt>
__device__ __forceinline__ void dec_raw_c(const uint32_t (&R)[C][WIN_DW], const Pass (&P)[C], uint32_t o,
                                          uint32_t width, uint32_t col_off) {
    bool full = true;
#pragma unroll
    for (int k = 0; k < C; ++k) full = full && P[k].valid;
    if (full && C == 4 && width <= 16) {
        const Col cs(P[0], col_off, width);
        const uint32_t at = P[0].lrow * width;
        // dword m of the lane's 4*width bytes: byte i comes from record (4m+i)/width,
        // field byte (4m+i)%width -- constants once width is
        for (uint32_t m = 0; m < width; ++m) {
            uint32_t w = 0;
#pragma unroll
            for (uint32_t i = 0; i < 4; ++i) {
                const uint32_t b = 4 * m + i;
                w |= rbyte(R[b / width], o + b % width) << (8 * i);
            }
            cs.b32(at + 4 * m, w);
        }
        return;
    }
#pragma unroll
    for (int k = 0; k < C; ++k) dec_raw<Col>(R[k], P[k], o, 0, width, width, col_off, 0);
}

// Walk chunks [c_begin, c_end) of the batch's chunk array, one wave per chunk
// (wave-strided).  A chunk's window of NGZ_REG_WINDOW rows is covered in
// groups of 64*RPL rows, RPL records per lane (all their loads in flight at
// once): with CONSEC lane l owns the RPL consecutive rows prow + RPL*l + k
// (so narrow columns pack into wide stores), otherwise rows prow + 64*k + l.
// want(slot) decides (and may load per-slot state) whether a chunk's slot is
// handled here; shape(slot) gives its record shape; pass(P) decodes one group.
struct RecShape {
    uint32_t rl;         // record length (fixed templates)
    uint32_t row_bytes;  // column bytes per row (locates the record-offset array of vlen slots)
    bool vlen;           // variable-length records: per-row offsets from the record-offset array
};

// Chunk descriptor j of the 64 a wave fetched (lane j holds it; v_readlane)
__device__ __forceinline__ Chunk chunk_at_lane(const uint4 &e0, const uint4 &e1, uint32_t j) {
    Chunk cur;
    const uint32_t w1x = lane_u32(e1.x, j);
    cur.n = (uint16_t)(w1x & 0xFFFF);
    cur.slot = (uint16_t)(w1x >> 16);
    cur.src = (uint64_t)lane_u32(e0.x, j) | ((uint64_t)lane_u32(e0.y, j) << 32);
    cur.rec0 = lane_u32(e0.z, j);
    cur.dgram = lane_u32(e0.w, j);
    cur.pos0 = (uint16_t)(lane_u32(e1.y, j) & 0xFFFF);
    return cur;
}

// The passes of one chunk (its rows of one NGZ_REG_WINDOW window); row0 is
// the first row of the LDS workgroup window (0 for direct stores).
template <int RPL, bool CONSEC, class PassFn>
__device__ __forceinline__ void chunk_passes(const BatchDev &B, const Chunk &cur, uint32_t rl, uint8_t *blk,
                                             uint32_t cap, uint32_t lane, uint32_t row0, PassFn &&pass) {
    const uint32_t n = cur.n;
    const uint64_t src = cur.src;
    Pass P[RPL];
    P[0].rec0 = cur.rec0;
    P[0].dgram = cur.dgram;
    P[0].pos0 = cur.pos0;
    P[0].hdr = B.hdr;
    P[0].blk = blk;
    P[0].cap = cap;
    P[0].img = 0xFFFFFFFFu;  // record bytes through the resource (no staged image)
    const uint64_t a0 = src & ~15ull;  // 16-byte aligned resource base (win_load)
    // buffer range checks are per dword (a dword straddling num_records reads 0),
    // so round up: the <= 3 bytes past bytes_size share the last valid byte's
    // 4-byte word, hence its page; those bytes are never used
    const uint64_t avail64 = (B.bytes_size - a0 + 3) & ~3ull;
    const uint32_t avail = avail64 > 0x7FFFFFF0ull ? 0x7FFFFFF0u : (uint32_t)avail64;
    P[0].rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)(B.bytes + a0), (short)0, (int)avail, 0x00020000);
    P[0].a0 = a0;
    P[0].rabs = 0;
    P[0].offsets = B.offsets;
    P[0].lane = lane;
#pragma unroll
    for (int k = 1; k < RPL; ++k) P[k] = P[0];
    const uint32_t rec0 = P[0].rec0;
    const uint32_t wbase = rec0 & ~(uint32_t)(NGZ_REG_WINDOW - 1);
    for (uint32_t p = 0; p < NGZ_REG_WINDOW; p += 64 * RPL) {
        const uint32_t pr0 = wbase + p;
        if (pr0 + 64 * RPL <= rec0 || pr0 >= rec0 + n) continue;  // no row of this group in the chunk
#pragma unroll
        for (int k = 0; k < RPL; ++k) {
            Pass &Q = P[k];
            Q.prow = CONSEC ? pr0 : pr0 + 64 * k;
            Q.wrow = Q.prow - row0;
            Q.lrow = CONSEC ? RPL * lane + k : lane;
            Q.row = Q.prow + Q.lrow;
            Q.valid = Q.row >= rec0 && Q.row < rec0 + n;
            const uint32_t r = Q.valid ? Q.row - rec0 : 0;
            const uint32_t d = r * rl;  // record offset from the chunk's first record
            const uint32_t rel = d + (uint32_t)(src & 15);
            Q.rbase = rel & ~3u;
            Q.sh = rel & 3u;
            Q.any_sh = __builtin_amdgcn_ballot_w64(Q.sh != 0) != 0;
            Q.recpos = Q.pos0 + d;
        }
        pass(P);
    }
}

template <int RPL, bool CONSEC, class Want, class Shape, class PassFn>
__device__ __forceinline__ void run_chunks(const BatchDev &B, uint32_t c_begin, uint32_t c_end, Want &&want,
                                           Shape &&shape, PassFn &&pass) {
    static_assert(RPL == 1 || RPL == 2 || RPL == 4, "RPL");
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wpb = blockDim.x >> 6;
    const uint32_t wid = sgpr(blockIdx.x * wpb + (threadIdx.x >> 6));
    const uint32_t nw = gridDim.x * wpb;
    uint32_t rt_slot = 0xFFFFFFFFu, cap = 0;
    uint8_t *blk = nullptr;
    // Chunk descriptors are fetched 64 at a time, one per lane (lane j holds
    // the wave's j-th next chunk), and read with v_readlane: one descriptor
    // round trip per 64 chunks instead of one per chunk.  (vmcnt counts loads
    // and stores in order, so a per-chunk descriptor load would also wait for
    // the previous chunk's column stores.)
    for (uint32_t cb = c_begin + wid; cb < c_end; cb += 64 * nw) {
        const uint32_t mine = cb + lane * nw;
        uint4 e0 = make_uint4(0, 0, 0, 0), e1 = make_uint4(0, 0, 0, 0);
        if (mine < c_end) {
            e0 = ((const uint4 *)&B.chunks[mine])[0];
            e1 = ((const uint4 *)&B.chunks[mine])[1];
        }
        const uint32_t cnt = min(64u, (c_end - cb + nw - 1) / nw);
        for (uint32_t j = 0; j < cnt; ++j) {
            const Chunk cur = chunk_at_lane(e0, e1, j);
            if (cur.n == 0) continue;  // padding chunk
            const uint32_t slot = cur.slot;
            if (!want(slot)) continue;
            const RecShape rs = shape(slot);
            if (slot != rt_slot) {
                const SlotRT rt = sload(&B.slots[slot]);
                blk = B.arena + rt.block;
                cap = rt.cap;
                rt_slot = slot;
            }
            chunk_passes<RPL, CONSEC>(B, cur, rs.rl, blk, cap, lane, 0u, pass);
        }
    }
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint64_t o = __shfl_xor(v, m, 64);
        v = o < v ? o : v;
    }
    return sgpr64(v);  // every lane holds it: scalar (a buffer resource built from it needs no waterfall loop)
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint64_t o = __shfl_xor(v, m, 64);
        v = o > v ? o : v;
    }
    return sgpr64(v);  // every lane holds it: scalar (a buffer resource built from it needs no waterfall loop)
}

// exclusive prefix sum over the wave's lanes (total: the sum over all 64)
__device__ __forceinline__ uint32_t wave_excl_sum(uint32_t v, uint32_t lane, uint32_t &total) {
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    total = __shfl(x, 63, 64);
    return x - v;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint32_t o = __shfl_xor(v, m, 64);
        v = o > v ? o : v;
    }
    return v;
}

// Row mode: walk the slot's output in windows of NGZ_REG_WINDOW rows (wave
// strided), groups of 64*RPL rows as in run_chunks, every row's record found
// through rowsrc/rowdg (k_emit).  A group's records are read through one
// buffer resource based at their smallest address; a group whose records
// span more than the 31-bit offset range (only with far-apart datagram
// offsets) is decoded one record at a time.
// Row source of row mode: the record table k_emit wrote (batch offset and
// datagram of every row; error positions derived from the batch offset).
struct RowTableSrc {
    const uint64_t *rs;
    const uint32_t *rd;
    __device__ __forceinline__ bool operator()(Pass &Q, uint64_t &src) const {
        src = rs[Q.row] & NGZ_ROW_OFF_MASK;
        Q.dgram = rd[Q.row];
        Q.recpos = 0xFFFFFFFFu;
        Q.rec0 = Q.row;
        return true;
    }
    // smallest / largest record address of the group: from the lanes' rows
    static constexpr bool kRange = false;
    __device__ __forceinline__ void range(uint64_t &, uint64_t &) const {}
};

// One NGZ_REG_WINDOW window w of a slot whose every row's record is found by
// `srcfn(Q, src)` (sets src, Q.dgram, Q.recpos, Q.rec0 for row Q.row; false =
// no record), so a group's lanes may read records of different sets and
// datagrams.  P[] is preset by the caller; row0 as in chunk_passes.
template <int RPL, bool CONSEC, class SrcFn, class PassFn>
__device__ __forceinline__ void row_group(const BatchDev &B, const SrcFn &srcfn, uint32_t total, uint32_t pr0, uint32_t row0,
                                          Pass (&P)[RPL], PassFn &&pass) {
    const uint32_t lane = threadIdx.x & 63;
    {
        uint64_t src[RPL];
        uint64_t lo = ~0ull, hi = 0;
#pragma unroll
        for (int k = 0; k < RPL; ++k) {
            Pass &Q = P[k];
            Q.prow = CONSEC ? pr0 : pr0 + 64 * k;
            Q.wrow = Q.prow - row0;
            Q.lrow = CONSEC ? RPL * lane + k : lane;
            Q.row = Q.prow + Q.lrow;
            src[k] = 0;
            Q.valid = Q.row < total && srcfn(Q, src[k]);
            if (!Q.valid) {
                src[k] = 0;
                Q.dgram = 0;
            }
            Q.rabs = src[k];
            if (Q.valid) {
                lo = src[k] < lo ? src[k] : lo;
                hi = src[k] > hi ? src[k] : hi;
            }
        }
        uint64_t base, top;
        if constexpr (SrcFn::kRange) {
            srcfn.range(base, top);  // uniform, without cross-lane reductions
            base &= ~15ull;
        } else {
            base = wave_min_u64(lo) & ~15ull;
            top = wave_max_u64(hi);
        }
        if (top - base < 0x7FFF0000ull) {
            const uint64_t avail64 = (B.bytes_size - base + 3) & ~3ull;
            const uint32_t avail = avail64 > 0x7FFFFFF0ull ? 0x7FFFFFF0u : (uint32_t)avail64;
            const __amdgpu_buffer_rsrc_t r =
                __builtin_amdgcn_make_buffer_rsrc((void *)(B.bytes + base), (short)0, (int)avail, 0x00020000);
#pragma unroll
            for (int k = 0; k < RPL; ++k) {
                Pass &Q = P[k];
                const uint32_t rel = Q.valid ? (uint32_t)(src[k] - base) : 0;
                Q.rsrc = r;
                Q.a0 = base;
                Q.rbase = rel & ~3u;
                Q.sh = rel & 3u;
                Q.any_sh = __builtin_amdgcn_ballot_w64(Q.sh != 0) != 0;
            }
            pass(P);
        } else {
            // records too far apart for one resource: one record per pass
            bool keep[RPL];
#pragma unroll
            for (int k = 0; k < RPL; ++k) keep[k] = P[k].valid;
            for (uint32_t L = 0; L < 64; ++L) {
#pragma unroll
                for (int k0 = 0; k0 < RPL; ++k0) {
                    if (!__builtin_amdgcn_readlane((int)keep[k0], L)) continue;
                    const uint64_t b1 = ((uint64_t)lane_u32((uint32_t)src[k0], L) |
                                         ((uint64_t)lane_u32((uint32_t)(src[k0] >> 32), L) << 32)) & ~15ull;
                    const uint64_t avail64 = (B.bytes_size - b1 + 3) & ~3ull;
                    const uint32_t avail = avail64 > 0x7FFFFFF0ull ? 0x7FFFFFF0u : (uint32_t)avail64;
                    const __amdgpu_buffer_rsrc_t r =
                        __builtin_amdgcn_make_buffer_rsrc((void *)(B.bytes + b1), (short)0, (int)avail, 0x00020000);
#pragma unroll
                    for (int k = 0; k < RPL; ++k) {
                        Pass &Q = P[k];
                        Q.valid = k == k0 && lane == L && keep[k];
                        const uint32_t rel = Q.valid ? (uint32_t)(src[k] - b1) : 0;
                        Q.rsrc = r;
                        Q.a0 = b1;
                        Q.rbase = rel & ~3u;
                        Q.sh = rel & 3u;
                        Q.any_sh = __builtin_amdgcn_ballot_w64(Q.sh != 0) != 0;
                    }
                    pass(P);
                }
            }
        }
    }
}

template <int RPL, bool CONSEC, class SrcFn, class PassFn>
__device__ __forceinline__ void row_window(const BatchDev &B, const SrcFn &srcfn, uint32_t total, uint32_t w, uint32_t row0,
                                           Pass (&P)[RPL], PassFn &&pass) {
    for (uint32_t p = 0; p < NGZ_REG_WINDOW; p += 64 * RPL) {
        const uint32_t pr0 = w * NGZ_REG_WINDOW + p;
        if (pr0 >= total) break;
        row_group<RPL, CONSEC>(B, srcfn, total, pr0, row0, P, pass);
    }
}

// P[] fields of a row-mode slot that do not change per window
template <int RPL>
__device__ __forceinline__ void row_preset(const BatchDev &B, const SlotRT &rt, Pass (&P)[RPL]) {
    P[0].blk = B.arena + rt.block;
    P[0].cap = rt.cap;
    P[0].hdr = B.hdr;
    P[0].offsets = B.offsets;
    P[0].lane = threadIdx.x & 63;
    P[0].recpos = 0xFFFFFFFFu;
    P[0].pos0 = 0;
    P[0].dgram = 0;
    P[0].img = 0xFFFFFFFFu;
#pragma unroll
    for (int k = 1; k < RPL; ++k) P[k] = P[0];
}

template <int RPL, bool CONSEC, class Shape, class PassFn>
__device__ __forceinline__ void run_windows(const BatchDev &B, uint32_t slot, Shape &&shape, PassFn &&pass) {
    const uint32_t wpb = blockDim.x >> 6;
    const uint32_t wid = sgpr(blockIdx.x * wpb + (threadIdx.x >> 6));
    const uint32_t nw = gridDim.x * wpb;
    const SlotRT rt = sload(&B.slots[slot]);
    const uint64_t *rs = (const uint64_t *)(B.arena + rt.rows);
    const uint32_t *rd = (const uint32_t *)(B.arena + rt.rows + 8ull * rt.cap);
    (void)shape;
    Pass P[RPL];
    row_preset<RPL>(B, rt, P);
    const uint32_t nwin = (rt.total + NGZ_REG_WINDOW - 1) / NGZ_REG_WINDOW;
    for (uint32_t w = wid; w < nwin; w += nw) row_window<RPL, CONSEC>(B, RowTableSrc{rs, rd}, rt.total, w, 0u, P, pass);
}

#ifdef NGZ_VSTAGE
// ---------------------------------------------------------------------------
// Row mode with each group's record bytes staged in LDS (variable-length
// templates, generate_vlen).  The rows of a 64-row group are consecutive
// records of the slot, so their bytes are a few contiguous runs (one per set:
// a run ends where a record's end is not the next row's start).  The wave
// copies the runs' 16-byte blocks into its LDS image -- every lane its own
// record's blocks, all loads in flight at once -- and the generated decode
// then reads its register windows, length prefixes and string bytes from LDS.
// Without staging each lane walks its record with a chain of dependent global
// loads (a window load per variable-length field), and the wave's records are
// re-fetched from HBM between them (FETCH_SIZE 2x the record bytes on
// config 4).  A record's bytes run to the next record of its set, or to the
// set's end (the span k_emit stores with the offset, ngz_row_entry), so the
// image never holds bytes of another set.  Groups whose image exceeds
// NGZ_VSTAGE_BYTES per wave decode through global loads as before (row_group).
// ---------------------------------------------------------------------------
#ifndef NGZ_VSTAGE_BYTES
#define NGZ_VSTAGE_BYTES NGZ_VSTAGE_IMAGE
#endif
constexpr uint32_t kVStageDw = NGZ_VSTAGE_BYTES / 4;
constexpr uint32_t kVStageWaves = 4;  // the generated kernels run 256-thread workgroups
__shared__ uint32_t ngz_vstage[kVStageWaves * kVStageDw];

// win_load<ND> for the generated variable-length kernels: from the LDS image when the group is staged
template <int ND>
__device__ __forceinline__ void win_load_v(uint32_t (&R)[WIN_DW], const Pass &P, uint32_t wb) {
    if (P.img == 0xFFFFFFFFu) {
        win_load<ND>(R, P, wb);
        return;
    }
    const uint32_t q = P.img + ((P.rbase + wb) >> 2);
    constexpr int NR = ND + 1 < WIN_DW ? ND + 1 : WIN_DW;
#pragma unroll
    for (int j = 0; j < NR; ++j) R[j] = (j < ND || P.any_sh) ? ngz_vstage[q + j] : 0u;
#pragma unroll
    for (int j = NR; j < WIN_DW; ++j) R[j] = 0;
    if (P.any_sh) {
#pragma unroll
        for (int j = 0; j < ND; ++j) R[j] = __builtin_amdgcn_alignbyte(R[j + 1], R[j], P.sh);
    }
}

struct StageBytes {
    uint32_t base;  // this lane's byte, relative to the wave's image
    uint32_t img;
    __device__ uint32_t operator()(uint32_t i) const {
        const uint32_t b = base + i;
        return (ngz_vstage[img + (b >> 2)] >> (8 * (b & 3))) & 0xFF;
    }
};

// utf8_valid_global for the generated variable-length kernels; rel is
// relative to the lane's rsrc / image base as P.rbase is
__device__ __forceinline__ bool utf8_valid_v(const Pass &P, uint32_t rel, uint32_t len, bool stop_at_nul) {
    if (P.img == 0xFFFFFFFFu) return utf8_valid_global(P.rsrc, rel, len, stop_at_nul);
    if (len == 0) return true;
    // ASCII fast path: no byte of [rel, rel + len) has its high bit set.  Only the first and the
    // last dword need masks; the ones between are ORed whole (two LDS dwords per read), so the
    // loop body is a read and an OR (the per-dword mask version cost ~15 VALU per dword).
    const uint32_t end = rel + len, d0 = rel >> 2, d1 = (end - 1) >> 2;
    const uint32_t mf = 0xFFFFFFFFu << (8 * (rel & 3)), ml = 0xFFFFFFFFu >> (8 * (3 - ((end - 1) & 3)));
    const uint32_t *img = &ngz_vstage[P.img];
    uint32_t acc = d0 == d1 ? img[d0] & mf & ml : (img[d0] & mf) | (img[d1] & ml);
    for (uint32_t d = d0 + 1; d < d1; ++d) acc |= img[d];
    if (!(acc & 0x80808080u)) return true;
    return utf8_valid_prefix(StageBytes{rel, P.img}, len, stop_at_nul);
}

template <class PassFn>
__device__ __forceinline__ void run_windows_staged(const BatchDev &B, uint32_t slot, PassFn &&pass) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t wpb = blockDim.x >> 6;
    const uint32_t wid = sgpr(blockIdx.x * wpb + wv);
    const uint32_t nw = gridDim.x * wpb;
    const SlotRT rt = sload(&B.slots[slot]);
    const uint64_t *rs = (const uint64_t *)(B.arena + rt.rows);
    const uint32_t *rd = (const uint32_t *)(B.arena + rt.rows + 8ull * rt.cap);
    const RowTableSrc srcfn{rs, rd};
    Pass P[1];
    row_preset<1>(B, rt, P);
    const uint32_t img0 = sgpr(wv * kVStageDw);
    const uint32_t total = rt.total;
    const uint32_t ngroups = (total + 63) / 64;
    // the row entries of the wave's next group are loaded one group ahead (their round trip
    // overlaps this group's copy and decode instead of starting each group)
    uint64_t ent_n = 0;
    uint32_t dg_n = 0;
    if (wid * 64 + lane < total) {
        ent_n = rs[wid * 64 + lane];
        dg_n = rd[wid * 64 + lane];
    }
    for (uint32_t g = wid; g < ngroups; g += nw) {
        Pass &Q = P[0];
        Q.img = 0xFFFFFFFFu;
        const uint32_t pr0 = g * 64;
        Q.prow = pr0;
        Q.wrow = pr0;
        Q.lrow = lane;
        Q.row = pr0 + lane;
        Q.valid = Q.row < total;
        const uint64_t ent = ent_n;
        Q.dgram = dg_n;
        {
            const uint32_t r2 = (g + nw) * 64 + lane;
            const bool v2 = g + nw < ngroups && r2 < total;
            ent_n = v2 ? rs[r2] : 0;
            dg_n = v2 ? rd[r2] : 0;
        }
        Q.recpos = 0xFFFFFFFFu;
        Q.rec0 = Q.row;
        const uint64_t src = ent & NGZ_ROW_OFF_MASK;
        Q.rabs = src;
        // the record's bytes: up to the next record of its set, or to the set's end (ngz_row_entry)
        const uint64_t bound = Q.valid ? src + (ent >> 48) : 0;
        const uint64_t pb = __shfl_up(bound, 1, 64);
        const bool cont = lane > 0 && Q.valid && pb == src;  // the previous row's record ends where this one starts
        const uint64_t blo = cont ? (src + 15) >> 4 : src >> 4;
        const uint64_t bhi = (bound + 15) >> 4;
        const uint32_t c = Q.valid && bhi > blo ? (uint32_t)(bhi - blo) : 0u;
        uint32_t T;
        const uint32_t pc = wave_excl_sum(c, lane, T);
        const uint64_t base = wave_min_u64(Q.valid ? src : ~0ull) & ~15ull;
        const uint64_t top = wave_max_u64(bound);
        if (T == 0 || 16 * T > NGZ_VSTAGE_BYTES || top - base >= 0x7FFF0000ull) {
            row_group<1, false>(B, srcfn, total, pr0, 0u, P, pass);
            continue;
        }
        const uint64_t avail64 = (B.bytes_size - base + 3) & ~3ull;
        const uint32_t avail = avail64 > 0x7FFFFFF0ull ? 0x7FFFFFF0u : (uint32_t)avail64;
        const __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc((void *)(B.bytes + base), (short)0, (int)avail, 0x00020000);
        // copy: lane l's blocks [blo, bhi) are image pieces [pc, pc + c).  Consecutive lanes whose
        // records follow each other in the batch (cont) have consecutive blocks, so the image is a few
        // runs of consecutive batch blocks, one per lane that does not continue its predecessor (a
        // run head: the group's first record of each set).  The wave copies the image piece by piece
        // -- lane l takes pieces l, l + 64, ... -- so every load instruction reads 1 KiB of
        // consecutive blocks (a few lines; one record per lane was 64 blocks ~150 B apart, 64 lines
        // an instruction) and every LDS store writes 1 KiB of consecutive pieces (no bank conflicts).
        uint64_t hm = __builtin_amdgcn_ballot_w64(c != 0 && !cont);
        const uint32_t gb = (uint32_t)(((blo << 4) - base) >> 4);  // this lane's first block, resource-relative
        uint32_t hp[8], hb[8];  // the first 8 runs: first piece (~0: none) and first block, uniform
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) {
            const uint32_t h = hm ? (uint32_t)__builtin_ctzll(hm) : 0u;
            hp[i] = hm ? sgpr(lane_u32(pc, h)) : 0xFFFFFFFFu;
            hb[i] = hm ? sgpr(lane_u32(gb, h)) : 0u;
            hm &= hm - 1;
        }
        if (hm == 0) {
            // rounds of 64 pieces, 5 loads in flight (the image of 64 records of ~150 B is ~10 rounds).
            // Copying by buffer_load ... lds instead (every round in flight, no VGPRs) measured the same
            // (config 4: 580 against 571 us per staged launch, profiles/r5/cfg4_glds/ab.txt)
            constexpr uint32_t kBatch = 5;
            for (uint32_t k0 = 0; 64 * k0 < T; k0 += kBatch) {
                v4u v[kBatch];
#pragma unroll
                for (uint32_t k = 0; k < kBatch; ++k) {
                    const uint32_t p = 64 * (k0 + k) + lane;
                    uint32_t blk = 0x08000000u;  // past the image: out of the resource's range, reads 0
                    if (p < T) {
#pragma unroll
                        for (uint32_t i = 0; i < 8; ++i)
                            if (p >= hp[i]) blk = hb[i] + (p - hp[i]);
                    }
                    v[k] = __builtin_amdgcn_raw_buffer_load_b128(r, blk << 4, 0, 0);
                }
#pragma unroll
                for (uint32_t k = 0; k < kBatch; ++k) {
                    const uint32_t p = 64 * (k0 + k) + lane;
                    if (p < T) *(v4u *)&ngz_vstage[img0 + 4 * p] = v[k];
                }
            }
        } else {
            // more than 8 runs (records of many short sets): each lane copies its own blocks
            const uint32_t g0 = gb << 4;
            const uint32_t cmax = wave_max_u32(c);
            for (uint32_t j0 = 0; j0 < cmax; j0 += 8) {
                v4u v[8];
#pragma unroll
                for (uint32_t k = 0; k < 8; ++k)
                    v[k] = __builtin_amdgcn_raw_buffer_load_b128(r, j0 + k < c ? g0 + 16 * (j0 + k) : 0x80000000u, 0, 0);
#pragma unroll
                for (uint32_t k = 0; k < 8; ++k)
                    if (j0 + k < c) *(v4u *)&ngz_vstage[img0 + 4 * (pc + j0 + k)] = v[k];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the record's first byte in the image: its block is this lane's first piece,
        // or the previous contribution's last one when a continuing record starts mid-block
        const uint32_t rel = Q.valid ? 16 * (pc - (cont && (src & 15) ? 1u : 0u)) + (uint32_t)(src & 15) : 0u;
        Q.img = img0;
        Q.rsrc = r;
        Q.a0 = base;
        Q.rbase = rel & ~3u;
        Q.sh = rel & 3u;
        Q.any_sh = __builtin_amdgcn_ballot_w64(Q.sh != 0) != 0;
        pass(P);
        // the next group's copy overwrites the image: every lane's reads of it are done
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}
#endif  // NGZ_VSTAGE

#if defined(NGZ_LDS_WAVES) || defined(NGZ_LDS_BYTES)
// Row source of a chunk-mode window: the window's chunk descriptors, one per
// lane (e0/e1 as fetched by the wave, cnt valid); a row's record is in the
// chunk whose row range holds it.
struct ChunkGatherSrc {
    uint4 e0, e1;
    uint32_t cnt;
    uint32_t rl;
    __device__ __forceinline__ bool operator()(Pass &Q, uint64_t &src) const {
        bool hit = false;
        for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t n = lane_u32(e1.x, j) & 0xFFFF;  // 0 = padding chunk
            const uint32_t r0 = lane_u32(e0.z, j);
            const uint32_t r = Q.row - r0;
            if (r < n) {
                const uint32_t d = r * rl;
                src = ((uint64_t)lane_u32(e0.x, j) | ((uint64_t)lane_u32(e0.y, j) << 32)) + d;
                Q.dgram = lane_u32(e0.w, j);
                Q.recpos = (lane_u32(e1.y, j) & 0xFFFF) + d;
                Q.rec0 = r0;
                hit = true;
            }
        }
        return hit;
    }
    // the window's record addresses span [first record of the lowest chunk,
    // last record of the highest]: scalar, over the descriptors
    static constexpr bool kRange = true;
    __device__ __forceinline__ void range(uint64_t &lo, uint64_t &hi) const {
        lo = ~0ull;
        hi = 0;
        for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t n = lane_u32(e1.x, j) & 0xFFFF;
            if (!n) continue;
            const uint64_t a = (uint64_t)lane_u32(e0.x, j) | ((uint64_t)lane_u32(e0.y, j) << 32);
            lo = a < lo ? a : lo;
            const uint64_t b = a + (uint64_t)(n - 1) * rl;
            hi = b > hi ? b : hi;
        }
        if (lo > hi) lo = hi = 0;
    }
};

// LDS-staged decode of one slot: workgroup window W = rows [W*ROWS,
// (W+1)*ROWS) with ROWS = NGZ_REG_WINDOW*LW; wave q decodes its NGZ_REG_WINDOW
// sub-window s into LDS, then the workgroup writes the window's column runs
// (store(W, blk, cap), generated per template).  The capacity is a multiple of
// the window (k_layout), so a window's runs never leave the slot's block; rows
// past the slot's total carry stale bytes nobody reads.
//
// Chunk mode: the chunks of sub-window s are [wt[s], wt[s+1]) (k_emit).  A
// wave holds the window-table entries of its next 64 sub-windows in two
// VGPRs and fetches the next sub-window's chunk descriptors (one per lane)
// while it decodes the current one, so the record loads are the only memory
// latency on a window's path.  Lanes gather their rows' records across the
// sub-window's chunks (ChunkGatherSrc): one pass per group of 64*RPL rows
// even where a set ends inside the window.  Sub-windows of more than 64
// chunks go chunk by chunk.
// XCD-aware window order: workgroups are dealt round-robin over the 8 XCDs
// (b and b+8 share one), so workgroup b takes the (b % 8)-th contiguous eighth
// of the windows and strides through it with its XCD's other workgroups.
// Every XCD then works on one contiguous stretch of the input and of every
// column: its L2 and its address translations cover an eighth of what they
// would with windows dealt across all XCDs (those runs were up to 15 %
// slower, depending on where the allocations landed).  A multi-template kernel
// deals each template's windows this way in turn.
// NGZ_WIN_ROT (experiment): each XCD walks its stretch from a pseudo-random phase, wrapping, so
// the XCDs' concurrent positions are not at one fixed spacing
#ifndef NGZ_WIN_ROT
#define NGZ_WIN_ROT 0
#endif
struct WinSeq {
    uint32_t first, step, end;
    uint32_t base, len, rot;
    __device__ __forceinline__ uint32_t at(uint32_t i) const { return first + i * step; }
    __device__ __forceinline__ uint32_t map(uint32_t W) const {
#if NGZ_WIN_ROT
        uint32_t r = W - base + rot;
        if (r >= len) r -= len;
        return base + r;
#else
        return W;
#endif
    }
};

__device__ __forceinline__ WinSeq win_seq(uint32_t nwin) {
    const uint32_t G = gridDim.x;
    const uint32_t X = (G % 8 == 0 && G >= 8) ? 8u : 1u;
    const uint32_t x = blockIdx.x % X, l = blockIdx.x / X;
    const uint32_t per = (nwin + X - 1) / X;
    const uint32_t start = min(nwin, x * per);
    const uint32_t end = min(nwin, start + per);
    const uint32_t len = end - start;
    const uint32_t rot = len ? (uint32_t)(((uint64_t)((x * (uint32_t)NGZ_WIN_ROT * 2654435761u) >> 8) & 0xFFFFFF) * len >> 24) : 0;
    return WinSeq{start + l, G / X, end, start, len, rot};
}

// NGZ_TRACE diagnostics: the constant-rate clock (100 MHz) at a window's start and end
__device__ __forceinline__ unsigned long long win_clock(const BatchDev &B) {
    return B.trace ? (unsigned long long)__builtin_amdgcn_s_memrealtime() : 0ull;
}
__device__ __forceinline__ void win_trace(const BatchDev &B, uint32_t slot, uint32_t W, unsigned long long t0) {
    if (B.trace && threadIdx.x == 0 && W < NGZ_TRACE_WINDOWS) {
        unsigned long long *t = B.trace + 2ull * ((uint64_t)slot * NGZ_TRACE_WINDOWS + W);
        t[0] = t0;
        t[1] = (unsigned long long)__builtin_amdgcn_s_memrealtime();
    }
}

template <int RPL, bool CONSEC, uint32_t LW, class Shape, class PassFn, class StoreFn>
__device__ __forceinline__ void run_lds(const BatchDev &B, uint32_t slot, Shape &&shape, PassFn &&pass,
                                        StoreFn &&store, const WinSeq ws) {
    constexpr uint32_t ROWS = NGZ_REG_WINDOW * LW;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t q = sgpr(threadIdx.x >> 6);
    const SlotRT rt = sload(&B.slots[slot]);
    const uint32_t total = rt.total;
    const uint32_t nsub = (total + NGZ_REG_WINDOW - 1) / NGZ_REG_WINDOW;
    const RecShape shp = shape(slot);
    uint8_t *blk = B.arena + rt.block;
    const uint32_t c_end = rt.chunk0 + rt.nchunks;
    const uint32_t *wt = (const uint32_t *)(B.arena + rt.wtab);
    Pass P[RPL];
    row_preset<RPL>(B, rt, P);
    if (rt.mode == NGZ_MODE_ROW) {
        const uint64_t *rs = (const uint64_t *)(B.arena + rt.rows);
        const uint32_t *rd = (const uint32_t *)(B.arena + rt.rows + 8ull * rt.cap);
        for (uint32_t W0 = ws.first; W0 < ws.end; W0 += ws.step) {
            const uint32_t W = ws.map(W0);
            const unsigned long long t0 = win_clock(B);
            const uint32_t s = W * LW + q;
            if (s < nsub) row_window<RPL, CONSEC>(B, RowTableSrc{rs, rd}, total, s, W * ROWS, P, pass);
            __syncthreads();
            store(W, blk, rt.cap);
            __syncthreads();
            win_trace(B, slot, W, t0);
        }
        return;
    }
    // window-table entries [cb, ce) of this wave's sub-windows i0 .. i0+63 (lane i)
    auto wt_fetch = [&](uint32_t i0, uint32_t &ta, uint32_t &tb) {
        const uint32_t Wl = ws.at(i0 + lane);
        const bool in = Wl < ws.end;
        const uint32_t sl = (in ? ws.map(Wl) : Wl) * LW + q;
        ta = in && sl < nsub ? wt[sl] : c_end;
        tb = in && sl + 1 < nsub ? wt[sl + 1] : c_end;
    };
    auto desc_fetch = [&](uint32_t cb, uint32_t ce, uint4 &e0, uint4 &e1) {
        const uint32_t mine = cb + lane;
        e0 = make_uint4(0, 0, 0, 0);
        e1 = make_uint4(0, 0, 0, 0);
        if (mine < ce) {
            e0 = ((const uint4 *)&B.chunks[mine])[0];
            e1 = ((const uint4 *)&B.chunks[mine])[1];
        }
    };
    uint32_t ta = 0, tb = 0;
    uint4 n0, n1;  // descriptors of the next sub-window
    wt_fetch(0, ta, tb);
    desc_fetch(lane_u32(ta, 0), lane_u32(tb, 0), n0, n1);
    uint32_t i = 0;
    for (uint32_t W0 = ws.first; W0 < ws.end; W0 += ws.step, ++i) {
        const uint32_t W = ws.map(W0);
        const unsigned long long t0 = win_clock(B);
        const uint32_t s = W * LW + q;
        const uint32_t cb = lane_u32(ta, i & 63), ce = lane_u32(tb, i & 63);
        const uint4 e0 = n0, e1 = n1;
        // prefetch: the next sub-window's descriptors (and table entries every 64)
        if (((i + 1) & 63) == 0) wt_fetch(i + 1, ta, tb);
        desc_fetch(lane_u32(ta, (i + 1) & 63), lane_u32(tb, (i + 1) & 63), n0, n1);
        if (s < nsub) {
            if (ce - cb <= 64) {
                row_window<RPL, CONSEC>(B, ChunkGatherSrc{e0, e1, ce - cb, shp.rl}, total, s, W * ROWS, P, pass);
            } else {
                for (uint32_t c0 = cb; c0 < ce; c0 += 64) {
                    uint4 f0, f1;
                    desc_fetch(c0, ce, f0, f1);
                    const uint32_t cnt = min(64u, ce - c0);
                    for (uint32_t j = 0; j < cnt; ++j) {
                        const Chunk cur = chunk_at_lane(f0, f1, j);
                        if (cur.n == 0) continue;  // padding chunk
                        chunk_passes<RPL, CONSEC>(B, cur, shp.rl, blk, rt.cap, lane, W * ROWS, pass);
                    }
                }
            }
        }
        __syncthreads();
        store(W, blk, rt.cap);
        __syncthreads();
        win_trace(B, slot, W, t0);
    }
}
#endif

}  // namespace ngzdev
