// Internal structures shared by the host orchestration (ngz_host.cpp) and the
// HIP kernels (ngz_kernels.hip).  Not part of the C ABI.
#pragma once
#include <stdint.h>

#include "ngz/flow_decode.h"

#define NGZ_LANE_FIELDS 128   // field descriptors the generic kernel keeps in VGPRs (two per lane); the
                              // rest of a wider template's table is read with scalar loads
#define NGZ_RTC_MAX_FIELDS 512  // widest template that gets a generated kernel (wider: generic kernel)
#define NGZ_RTC_GROUP_MAX 16    // templates one multi-template decode launch takes (ngz_rtc.cpp generate_group)
#define NGZ_WALK_MAX 15       // variable-length fields a walk program holds (more: the exact field walk)
#define NGZ_MAX_SLOTS 1024    // template versions live in one batch
#define NGZ_NO_SLOT 0xFFFFu
#define NGZ_NO_ERR (~0ull)
#define NGZ_MAX_REC_LEN 65535 // longest fixed record the device decode takes
#define NGZ_REG_WINDOW 256    // records per chunk window (4 passes of 64 lanes)
#define NGZ_LDS_BUDGET 65536  // LDS bytes one workgroup may stage columns in
#define NGZ_VSTAGE_REC_MAX 160 // longest fixed record of a staged-row kernel (64 records per 10 KiB image)
#define NGZ_VSTAGE_IMAGE 10240 // bytes of a wave's LDS record image in the staged-row kernels (ngz_dev.h)

#ifndef __HIPCC_RTC__
// Experiment knobs (ngz_knobs.cpp): `dflt` in the product library; NGZ_<name> from the
// environment only in a -DNGZ_EXPERIMENTS build.  ngz_debug(): NGZ_DEBUG stderr traces.
int64_t ngz_knob(const char *name, int64_t dflt);
const char *ngz_knob_str(const char *name, const char *dflt);
bool ngz_debug();
int ngz_debug_level();  // 0 off, 1 traces (NGZ_DEBUG set), 2 also generated kernel sources (NGZ_DEBUG=2)
extern "C" int ngz_experiments_build();  // 1 in a -DNGZ_EXPERIMENTS build (tests check the product is not)
#endif

// Workgroup window of the LDS-staged per-template kernels: a workgroup
// decodes lds_waves consecutive 256-row windows (one per wave) into LDS,
// column-major, then writes every column's 256*lds_waves rows as one
// contiguous run of 16-byte stores.  As many waves as the budget allows, at
// most 4; 0 (rows too wide) = direct stores.
static inline __host__ __device__ uint32_t ngz_lds_waves(uint32_t row_bytes, uint32_t budget = NGZ_LDS_BUDGET,
                                                         uint32_t max_waves = 4) {
    if (!row_bytes) return 0;
    const uint32_t w = budget / (NGZ_REG_WINDOW * row_bytes);
    return w > max_waves ? max_waves : w;
}

// datagram frame state (k_frame -> host)
#define NGZ_FR_OK 0
#define NGZ_FR_NEED_MORE 1
#define NGZ_FR_ERROR 2
#define NGZ_FR_UNSUPPORTED 3
#define NGZ_FR_HOST 4        // contains template sets: framed on the host

// Error codes packed into the 64-bit error key.  Key layout (min wins =
// first error in parse order):
//   [63:48] stop position in the datagram (cursor where parsing stopped)
//   [47:40] code
//   [39:24] a (field index / set id / ...)
//   [23:0]  b (length / count / value / ...)
enum NgzErr : uint32_t {
    E_NONE = 0,
    E_CODEC_UNSUPPORTED_VERSION = 1,  // a = version
    E_IPFIX_INVALID_LENGTH = 2,       // b = length
    E_HDR_EOF = 3,                    // packet-level UnexpectedEof, b = available
    E_SET_EOF_ID = 4,                 // peek set id, b = available
    E_SET_EOF_LEN = 5,                // peek set length, b = available
    E_SET_INVALID_ID = 6,             // a = id
    E_SET_INVALID_LENGTH = 7,         // b = length
    E_SET_EOF_BODY = 8,               // take_slice, a = needed, b = available
    E_SET_NO_TEMPLATE = 9,            // a = id
    E_SET_PADDING = 10,               // b = value
    E_NF_INVALID_COUNT = 11,          // b = count
    E_REC_DTMS = 12,                  // a = field index (value re-read by host)
    E_REC_DTFRAC = 13,                // a = field index
    E_REC_UTF8 = 14,                  // a = field index, b = value length (variable-length strings)
    E_REC_FAIL = 15,                  // a = field index (template-constant failure)
    E_HOST = 16,                      // host-framed datagram error: b = index in host error table
    E_REC_EOF = 17,                   // UnexpectedEof inside a variable-length data record: a = field, b = needed
};

static inline __host__ __device__ uint64_t ngz_err_key(uint32_t stop, uint32_t code, uint32_t a, uint32_t b) {
    return ((uint64_t)(stop & 0xFFFF) << 48) | ((uint64_t)(code & 0xFF) << 40) | ((uint64_t)(a & 0xFFFF) << 24) |
           (uint64_t)(b & 0xFFFFFF);
}

struct DevField {        // 16 B
    uint16_t off;        // offset inside the record
    uint16_t len;        // wire length
    uint16_t width;      // column width
    uint8_t kind;        // NGZ_K_*
    uint8_t flags;       // NGZ_K_FAIL: failure sub-code; NGZ_K_VLEN: 0x80 = string (UTF-8 checked)
    uint32_t col_off;    // bytes per row before this column
    uint32_t reserved;
};

struct DevPlan {
    uint32_t rec_len;    // exact wire bytes per record (0 = no records)
    uint32_t row_bytes;  // sum of column widths
    uint16_t n_fields;
    uint8_t proto;       // 10 / 9
    uint8_t rpl;         // 1 = device-decodable (fixed-length records), 0 = not
    uint8_t reserved0;
    uint8_t has_vlen;
    uint8_t has_err;
    uint8_t spec;        // 1 = decoded by a run-time specialised kernel (the generic kernel skips it)
    uint32_t window;     // records per chunk window (NGZ_REG_WINDOW)
    uint32_t template_id;
    uint32_t lds_waves;  // per-template kernel stages columns in LDS: waves (256-row sub-windows) per
                         // workgroup window, 0 = direct column stores (ngz_lds_waves)
    uint32_t reserved1;
    const DevField *f;   // n_fields descriptors (scope first): host memory in the host's copy of a plan,
                         // the context's device field table in the uploaded one.  No field cap: a
                         // template may carry as many fields as its set holds (ipfix.rs:384-413).
    // Walk program of a variable-length template (ngz_vlen_walk's fast path): a record is
    // walk_fixed[0] fixed bytes, then for each of walk_nv variable-length fields its length
    // prefix + value followed by walk_fixed[k+1] fixed bytes.  walk_nv = 0xFF: no program
    // (template-constant field failures, or more than NGZ_WALK_MAX variable-length fields).
    uint8_t walk_nv;
    uint8_t walk_pad[3];
    uint16_t walk_fixed[NGZ_WALK_MAX + 1];
    // processed_count restarts inside this batch (an identical re-announcement of the template
    // reuses its version, ngz_host.cpp define_template): only sets at (datagram << 16 | set
    // position) > count_from count (k_counts); 0 = every set of the slot
    uint64_t count_from;
};

// chrono's NaiveDateTime range in milliseconds (timestamp_millis_opt, generator.rs:1725-1746)
#define NGZ_MIN_MILLIS (-8334601315200000LL)  // days_from_civil(-262143,1,1)*86400000
#define NGZ_MAX_MILLIS 8210266876799999LL     // (days_from_civil(262142,12,31)+1)*86400000-1

// std::str::from_utf8 of p[0, len); with stop_at_nul only the bytes up to the first NUL
// (fixed-length strings, generator.rs:1651-1668).  The framing walk's form (host and device);
// the decode kernels have their own register / LDS forms (ngz_dev.h utf8_valid_prefix).
__host__ __device__ inline bool ngz_utf8_ok(const uint8_t *p, uint32_t len, bool stop_at_nul) {
    uint32_t i = 0;
    while (i < len) {
        const uint32_t c = p[i];
        if (c == 0 && stop_at_nul) return true;
        if (c < 0x80) { ++i; continue; }
        uint32_t need, lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) need = 1;
        else if (c >= 0xE0 && c <= 0xEF) { need = 2; if (c == 0xE0) lo = 0xA0; if (c == 0xED) hi = 0x9F; }
        else if (c >= 0xF0 && c <= 0xF4) { need = 3; if (c == 0xF0) lo = 0x90; if (c == 0xF4) hi = 0x8F; }
        else return false;
        for (uint32_t t = 1; t <= need; ++t) {
            if (i + t >= len) return false;
            const uint32_t b = p[i + t];
            if (b < (t == 1 ? lo : 0x80u) || b > (t == 1 ? hi : 0xBFu)) return false;
        }
        i += need + 1;
    }
    return true;
}

// The record a walk stops in (UnexpectedEof, or a template-constant failure, at field stop_f):
// DataRecord::parse read its fields before that one and Field::parse checked their values as it
// read them (ipfix.rs:335-370, generator.rs:1635-1773), so the first value error among them is the
// record's error -- a dateTime out of chrono's range, a nanosecond fraction of 1e9 outside a leap
// second, a string that is not UTF-8.  The decode kernels check complete records only.  The
// walk's key stays the failure (it decides nothing else: the set is not counted either way), and
// the host applies this check when it renders the error (ngz_host.cpp render_error): inlined into
// the framing kernel's walk it took k_frame from 118 to 178 VGPRs with scratch spills (half the
// occupancy, 0.65 -> 1.45 ms on config 4).  pos = the record's start.  Found by the differential
// fuzz corpus (tests/test_gpu_fuzz.py: an invalid vlen string before a later field's EOF).
inline uint64_t ngz_partial_record_err(const uint8_t *p, uint32_t pos, uint32_t stop_f, const DevPlan &pl) {
    for (uint32_t f = 0; f < stop_f; ++f) {
        const DevField &fd = pl.f[f];
        if (fd.kind == NGZ_K_VLEN) {
            uint32_t len = p[pos], hdr = 1;
            if (len == 255) {
                len = ((uint32_t)p[pos + 1] << 16) | ((uint32_t)p[pos + 2] << 8) | p[pos + 3];
                hdr = 4;
            }
            if ((fd.flags & 0x80) && !ngz_utf8_ok(p + pos + hdr, len, false))
                return ngz_err_key(pos + hdr, E_REC_UTF8, f, len);
            pos += hdr + len;
            continue;
        }
        if (fd.kind == NGZ_K_DTMS) {
            uint64_t v = 0;
            for (int i = 0; i < 8; ++i) v = (v << 8) | p[pos + i];
            if ((int64_t)v < NGZ_MIN_MILLIS || (int64_t)v > NGZ_MAX_MILLIS) return ngz_err_key(pos, E_REC_DTMS, f, 0);
        } else if (fd.kind == NGZ_K_DTFRAC) {
            const uint32_t secs = ((uint32_t)p[pos] << 24) | ((uint32_t)p[pos + 1] << 16) | ((uint32_t)p[pos + 2] << 8) | p[pos + 3];
            const uint32_t frac = ((uint32_t)p[pos + 4] << 24) | ((uint32_t)p[pos + 5] << 16) | ((uint32_t)p[pos + 6] << 8) | p[pos + 7];
            const uint32_t ns = (uint32_t)(1000000000.0 * ((double)frac / 4294967295.0));
            if (ns >= 1000000000u && (secs % 60u) != 59u) return ngz_err_key(pos, E_REC_DTFRAC, f, 0);
        } else if (fd.kind == NGZ_K_STR) {
            if (!ngz_utf8_ok(p + pos, fd.len, true)) return ngz_err_key(pos, E_REC_UTF8, f, 0);
        }
        pos += fd.len;
    }
    return NGZ_NO_ERR;
}

// Records of one IPFIX data set whose template has variable-length (65535)
// fields, walked as Set::parse + DataRecord::parse + Field::parse would
// (ipfix.rs:193-222, 335-370; vlen prefix generator.rs:1775-1793: u8, 255 ->
// 3-byte length).  p = datagram, [pos, end) = set payload.  Calls
// on_rec(n0 + k, record_offset) for each complete record only (a failing
// record has no row); returns the number of complete records; on
// UnexpectedEof / a template-constant field failure sets *err to the error
// key (parsing stops there).  Exact form: one step per field.  fail_start (host, error
// rendering): the start of the record the walk failed in.
template <class F>
__host__ __device__ inline uint32_t ngz_vlen_walk_exact(const uint8_t *p, uint32_t pos, uint32_t end, const DevPlan &pl,
                                                        uint64_t *err, F &&on_rec, uint32_t n0 = 0,
                                                        uint32_t *fail_start = nullptr) {
    const uint32_t minlen = pl.rec_len;  // vlen counted as 1
    uint32_t n = 0;
    while (minlen > 0 && end - pos >= minlen) {
        const uint32_t start = pos;
        if (fail_start) *fail_start = start;
        for (uint32_t f = 0; f < pl.n_fields; ++f) {
            const DevField &fd = pl.f[f];
            const uint32_t rem = end - pos;
            if (fd.kind == NGZ_K_FAIL) {  // fails before reading (InvalidLength, ...)
                *err = ngz_err_key(pos, E_REC_FAIL, f, 0);
                return n;
            }
            if (fd.kind == NGZ_K_VLEN) {
                if (rem < 1) { *err = ngz_err_key(pos, E_REC_EOF, f, 1); return n; }
                uint32_t len = p[pos];
                pos += 1;
                if (len == 255) {  // read_unsigned32_be(3)
                    if (end - pos < 3) { *err = ngz_err_key(pos, E_REC_EOF, f, 3); return n; }
                    len = ((uint32_t)p[pos] << 16) | ((uint32_t)p[pos + 1] << 8) | p[pos + 2];
                    pos += 3;
                }
                if (end - pos < len) { *err = ngz_err_key(pos, E_REC_EOF, f, len); return n; }
                pos += len;
                continue;
            }
            if (fd.kind == NGZ_K_DTFRAC) {  // two u32 reads (generator.rs:1748-1773)
                if (rem < 4) { *err = ngz_err_key(pos, E_REC_EOF, f, 4); return n; }
                if (rem < 8) { *err = ngz_err_key(pos + 4, E_REC_EOF, f, 4); return n; }
                pos += 8;
                continue;
            }
            if (rem < fd.len) { *err = ngz_err_key(pos, E_REC_EOF, f, fd.len); return n; }
            pos += fd.len;
        }
        on_rec(n0 + n, start);
        ++n;
    }
    return n;
}

// The same walk through the plan's walk program: per record only the length
// prefixes are read (no per-field descriptor loads, the program sits in
// registers), each step checking that the bytes it skips are there.  Any
// record the fast steps cannot complete is re-walked from its start by the
// exact form, which reports the reference's error for it (a record fails
// exactly when some field runs past the set: both forms agree on that).
template <class F>
__host__ __device__ inline uint32_t ngz_vlen_walk(const uint8_t *p, uint32_t pos, uint32_t end, const DevPlan &pl,
                                                  uint64_t *err, F &&on_rec) {
    if (pl.walk_nv > NGZ_WALK_MAX) return ngz_vlen_walk_exact(p, pos, end, pl, err, on_rec);
    const uint32_t minlen = pl.rec_len, nv = pl.walk_nv;
    uint32_t fx[NGZ_WALK_MAX + 1];
#pragma unroll
    for (uint32_t k = 0; k <= NGZ_WALK_MAX; ++k) fx[k] = pl.walk_fixed[k];
    uint32_t n = 0;
    while (minlen > 0 && end - pos >= minlen) {
        const uint32_t start = pos;
        bool ok = end - pos >= fx[0];
        pos += fx[0];
#pragma unroll
        for (uint32_t k = 0; k < NGZ_WALK_MAX; ++k) {
            if (k < nv && ok) {
                uint32_t len = 0, hdr = 1;
                ok = end - pos >= 1;
                if (ok) {
                    len = p[pos];
                    if (len == 255) {
                        ok = end - pos >= 4;
                        if (ok) len = ((uint32_t)p[pos + 1] << 16) | ((uint32_t)p[pos + 2] << 8) | p[pos + 3];
                        hdr = 4;
                    }
                }
                ok = ok && end - pos - hdr >= len && end - pos - hdr - len >= fx[k + 1];
                pos += hdr + len + fx[k + 1];
            }
        }
        if (!ok) return n + ngz_vlen_walk_exact(p, start, end, pl, err, on_rec, n);
        on_rec(n, start);
        ++n;
    }
    return n;
}

// Row-mode record table entry (rowsrc): the record's batch offset in the low
// 48 bits, the bytes from it to the next record of its set (or to the set's
// end; at most 65535) in the high 16 -- the staged decode copies exactly
// those bytes to LDS without looking up the datagram's extent.
__host__ __device__ inline uint64_t ngz_row_entry(uint64_t off, uint64_t span) {
    return off | ((span < 0xFFFFu ? span : 0xFFFFull) << 48);
}
#define NGZ_ROW_OFF_MASK 0x0000FFFFFFFFFFFFull

struct SlotRT {          // per batch slot, computed on device by k_layout
    uint64_t block;      // byte offset of the slot's columns in the arena
    uint32_t cap;        // rows allocated
    uint32_t total;      // rows used
    uint32_t base;       // first element of the slot's row in the scanned count matrix
    uint32_t chunk0;     // first chunk of the slot (chunks are slot-major)
    uint32_t nchunks;    // chunks of the slot (incl. empty padding chunks); 0 in row mode
    uint32_t chunk_scan0;  // scanned count at the slot's first chunk cell (k_emit cursor base)
    uint32_t mode;       // NGZ_MODE_*
    uint32_t reserved;
    uint64_t rows;       // row mode: arena offset of u64 rowsrc[cap] (ngz_row_entry of each record),
                         // followed by u32 rowdg[cap] (its datagram)
    uint64_t wtab;       // chunk mode: arena offset of u32 wfirst[cap/window]: first chunk of
                         // every output window (k_emit), for the LDS-staged kernels
};

// Decode work of a slot: chunk mode walks set-relative chunks of <= 256 rows
// (large sets: records of a chunk are contiguous); row mode walks 256-row
// windows of the slot's output with a per-row source address, so small sets
// (MTU-sized IPFIX, NetFlow v9 packets of ~10 records) and variable-length
// records still fill every lane.
#define NGZ_MODE_CHUNK 0u
#define NGZ_MODE_ROW 1u

struct Chunk {           // 32 B, one wave of work
    uint64_t src;        // batch byte offset of the first record
    uint32_t rec0;       // first row in the slot's columns
    uint32_t dgram;
    uint16_t n;          // records (0 = empty slot)
    uint16_t slot;
    uint16_t pos0;       // first record's offset inside the datagram
    uint16_t cls;        // reserved (0)
    uint32_t reserved2;
};

// host-framed data set (template-bearing datagrams framed on the host)
struct HostSet {
    uint16_t set_pos;
    uint16_t slot;
    uint16_t payload_pos; // offset of the first record
    uint16_t reserved;
    uint32_t n;
    uint32_t reserved2;
};

struct BatchSummary {    // device -> host at the end of a batch
    uint32_t n_records_total;
    uint32_t n_chunks;
    uint32_t n_sets;
    uint32_t n_host;        // datagrams needing host framing (template sets)
    uint32_t overflow;      // 1: arena, 2: chunks, 4: sets, 8: a set of a slot without a count row,
                            // 16: split framing met a record error in a variable-length set (run again whole)
    uint32_t n_unsupported;
    uint64_t arena_used;
};

struct BatchDev {        // device pointers of one batch
    const uint8_t *bytes;
    uint64_t bytes_size;
    const uint64_t *offsets;
    const uint32_t *lengths;
    uint32_t n;
    uint32_t n_slots;
    const DevPlan *plans;      // [n_slots]
    const uint16_t *cur_slot;  // [2][65536]: proto index 0 = v10, 1 = v9
    // timeline of template definitions inside this batch (slow path)
    const uint32_t *tl_key;    // (proto_idx<<16)|id, sorted by (key, dgram)
    const uint32_t *tl_dgram;
    const uint16_t *tl_slot;
    uint32_t tl_n;
    // host-framed datagrams
    const uint32_t *hf_first;  // [n+1] CSR into hf_sets, or null
    const HostSet *hf_sets;
    const void *hf_hdr;        // [hosts] ngz_dgram_hdr of host-framed datagrams (hf_flag[d]-1 indexes)
    void *hdr;                 // ngz_dgram_hdr[n]
    uint32_t *counts;          // [(2*n_rows+1)*n + 1]
    uint32_t *scan;            // same length
    SlotRT *slots;             // [n_slots]
    Chunk *chunks;
    uint64_t chunk_cap;
    void *sets;                // ngz_set_info[set_cap]
    uint64_t set_cap;
    uint8_t *arena;
    uint64_t arena_cap;
    unsigned long long *proc_counts; // [n_slots] processed_count increments
    BatchSummary *summary;
    uint32_t cap_pad_windows;  // extra workgroup windows of capacity per slot (column placement tuning)
    uint32_t split;            // split framing (ngz_host.cpp run_pipeline): 0 off; 1 phase A, the sets of
                               // variable-length templates deferred (counted as sets, no records walked);
                               // 2 phase B, only those sets (record walk, row tables), on another stream
    uint32_t *recmap;          // variable-length slots: 1 bit per batch byte, set at every complete record
                               // (used when recoff is null)
    uint16_t *recoff;          // variable-length slots: per datagram, the offsets of its complete records
                               // in datagram order then 0xFFFF, from entry ceil8(offsets[d] / recoff_div + 8 d)
    uint32_t recoff_div;       // the smallest min_record_length of the batch's variable-length templates
    uint32_t reserved_c;
    unsigned long long *dsum;  // per datagram: its one data set (k_frame -> k_emit), 0 = walk it again
                               // start by k_frame's walk, read by k_emit instead of walking again (or null)
    // count-matrix rows: only the template slots expected to carry records in this batch have
    // one (the slots that did in the previous batch, or every slot); a set of another slot makes
    // k_frame raise overflow bit 8 and the batch runs again with every slot
    const uint16_t *slot_row;  // [n_slots]: the slot's row, or NGZ_NO_ROW
    uint32_t n_rows;           // rows A: counts / scan are [(2A + 1) n + 1]
    uint32_t reserved_d;
    unsigned long long *trace;  // NGZ_TRACE (diagnostics): per slot and window, start / end clock of the
                                // window in the generated LDS-staged kernels (ngz_dev.h run_lds), or null
};
#define NGZ_TRACE_WINDOWS (1u << 17)  // windows traced per slot
#define NGZ_NO_ROW 0xFFFFu
