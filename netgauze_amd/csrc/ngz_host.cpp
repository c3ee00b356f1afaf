// Host side of netgauze_amd: the C ABI (include/ngz/flow_decode.h), the
// per-peer template registry (≙ FlowInfoCodec's two TemplatesMap), host
// framing of the rare datagrams that carry (options) template sets, and the
// batch pipeline that drives the HIP kernels in ngz_kernels.hip.
//
// Reference (NetGauze v0.13.0, paths relative to the checkout):
//   crates/flow-pkt/src/codec.rs:68-220            FlowInfoCodec
//   crates/flow-pkt/src/wire/deserializer/mod.rs:50-67   FieldSpecifier::parse
//   crates/flow-pkt/src/wire/deserializer/ipfix.rs:133-413  sets / templates
//   crates/flow-pkt/src/wire/deserializer/netflow.rs:143-388 NFv9 sets / templates
//   crates/flow-pkt/src/lib.rs:147-154, ie.rs:114-149    length_range checks
//   crates/ipfix-code-generator/src/generator.rs:390-430,1439-1807  IE lookup, decode rules
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <tuple>
#include <string>
#include <unordered_map>
#include <set>
#include <vector>

#include "ngz/flow_decode.h"
#include "ngz_internal.h"
#include "ngz_host.h"

using namespace ngzh;

extern "C" int ngz_launch_frame(const BatchDev *B, const uint32_t *hf_flag, const uint32_t *hf_first, hipStream_t st);
extern "C" int ngz_scan_temp_bytes(uint64_t n_items, size_t *bytes);
extern "C" int ngz_launch_scan(void *temp, size_t temp_bytes, const uint32_t *in, uint32_t *out, uint64_t n_items,
                               hipStream_t st);
extern "C" int ngz_launch_layout_emit(const BatchDev *B, const uint32_t *hf_flag, const uint32_t *hf_first,
                                      hipStream_t st);
extern "C" int ngz_launch_decode_generic(const BatchDev *B, uint32_t grid, hipStream_t st);
extern "C" int ngz_launch_frame_vlen(const BatchDev *B, hipStream_t st);
extern "C" int ngz_launch_layout(const BatchDev *B, hipStream_t st);
extern "C" int ngz_launch_emit(const BatchDev *B, hipStream_t st);
void *ngz_rtc_kernel(int device, const DevPlan &P);
int ngz_rtc_kernel_async(int device, const DevPlan &P, void **fn, void **entry);
int ngz_rtc_poll(void *entry, void **fn);
int ngz_rtc_join(void *const *entries, size_t n);
void *ngz_rtc_group(int device, const DevPlan *const *plans, uint32_t n);
int ngz_rtc_group_async(int device, const DevPlan *const *plans, uint32_t n, void **fn, void **entry);
int ngz_rtc_launch_group(void *fn, const BatchDev *B, const uint32_t *slots, uint32_t n, uint32_t grid, uint32_t block,
                         hipStream_t st);
std::string ngz_rtc_group_source(const DevPlan *const *plans, uint32_t n);
std::string ngz_rtc_source(const DevPlan &P);
int ngz_rtc_compile_only(const DevPlan &P, std::string *log_out);
int ngz_rtc_compile_source(const std::string &src, std::string *log_out);
int ngz_rtc_launch(void *fn, const BatchDev *B, uint32_t slot, uint32_t grid, uint32_t block, hipStream_t st);
extern "C" int ngz_launch_counts(const BatchDev *B, uint64_t set_cap, hipStream_t st);
extern "C" int ngz_launch_to_host(const void *src, void *dst, uint64_t bytes, hipStream_t st);
extern "C" int ngz_launch_place_probe(const uint8_t *in, uint64_t in_bytes, uint8_t *blk, uint32_t cap, uint32_t total,
                                      uint32_t rec_len, uint32_t frac16, const uint32_t *w, const uint32_t *off,
                                      uint32_t ncol, uint32_t grid, hipStream_t st);
extern "C" int ngz_launch_export(const BatchDev *B, BatchSummary *h_summary, SlotRT *h_slots,
                                 unsigned long long *h_proc, BatchSummary *next_summary,
                                 unsigned long long *next_proc, unsigned long long *h_done, unsigned long long seq,
                                 hipStream_t st);

namespace {

// ------------------------------------------------------------------------
// IE registry (generated from the reference XML, tools/gen_ie_registry.py)
// ------------------------------------------------------------------------
#define NGZ_IE(pen, id, dt, fl, nm) {pen, (uint16_t)(id), (uint8_t)(dt), (uint8_t)(fl), nm},
#define NGZ_VENDOR(pen, nm)
const IeRow kIes[] = {
#include "ie_table.inc"
};
#undef NGZ_IE
#undef NGZ_VENDOR
#define NGZ_IE(pen, id, dt, fl, nm)
#define NGZ_VENDOR(pen, nm) {pen, nm},
const VendorRow kVendors[] = {
#include "ie_table.inc"
};
#undef NGZ_IE
#undef NGZ_VENDOR

struct IeIndex {
    std::unordered_map<uint64_t, const IeRow *> by_key;
    IeIndex() {
        for (const auto &r : kIes) by_key[((uint64_t)r.pen << 16) | r.id] = &r;
    }
    const IeRow *find(uint32_t pen, uint16_t id) const {
        auto it = by_key.find(((uint64_t)pen << 16) | id);
        return it == by_key.end() ? nullptr : it->second;
    }
    const char *vendor(uint32_t pen) const {
        for (const auto &v : kVendors)
            if (v.pen == pen) return v.name;
        return nullptr;
    }
};
const IeIndex &ies() {
    static IeIndex idx;
    return idx;
}

// length_range per data type (crates/flow-pkt/src/ie.rs:114-149), half open; {0,0} = unchecked
void length_range(uint8_t dt, int &lo, int &hi) {
    static const int r[24][2] = {{0, 0}, {1, 2}, {1, 3}, {1, 5}, {1, 9}, {1, 2}, {1, 3}, {1, 5}, {1, 9}, {4, 5},
                                 {8, 9}, {1, 2}, {6, 7}, {0, 0}, {4, 5}, {8, 9}, {8, 9}, {8, 9}, {4, 5}, {16, 17},
                                 {0, 0}, {0, 0}, {0, 0}, {1, 33}};
    lo = r[dt][0];
    hi = r[dt][1];
}

// ------------------------------------------------------------------------
// Template model
// ------------------------------------------------------------------------
}  // namespace

namespace ngzh {

std::string json_str(const char *s) {
    std::string o = "\"";
    for (const unsigned char *p = (const unsigned char *)s; *p; ++p) {
        unsigned c = *p;
        if (c == '"') o += "\\\"";
        else if (c == '\\') o += "\\\\";
        else if (c == '\n') o += "\\n";
        else if (c == '\r') o += "\\r";
        else if (c == '\t') o += "\\t";
        else if (c == '\b') o += "\\b";
        else if (c == '\f') o += "\\f";
        else if (c < 0x20) {
            char b[8];
            snprintf(b, sizeof b, "\\u%04x", c);
            o += b;
        } else
            o += (char)c;
    }
    return o + "\"";
}

std::string ie_json(const Spec &s) {
    char b[96];
    switch (s.kind) {
    case IK_IANA: return json_str(s.name);
    case IK_VENDOR: return std::string("{") + json_str(s.vendor) + ":" + json_str(s.name) + "}";
    case IK_VENDOR_UNKNOWN:
        snprintf(b, sizeof b, ":{\"Unknown\":{\"id\":%u}}}", s.id);
        return std::string("{") + json_str(s.vendor) + b;
    case IK_UNKNOWN: snprintf(b, sizeof b, "{\"Unknown\":{\"pen\":%u,\"id\":%u}}", s.pen, s.id); return b;
    case IK_SCOPE: {
        static const char *nm[] = {nullptr, "System", "Interface", "LineCard", "Cache", "Template"};
        if (s.pen == 0 && s.id >= 1 && s.id <= 5) return json_str(nm[s.id]);
        snprintf(b, sizeof b, "{\"Unknown\":{\"pen\":%u,\"id\":%u}}", s.pen, s.id);
        return b;
    }
    }
    return "null";
}

std::string spec_json(const Spec &s) {
    char b[32];
    snprintf(b, sizeof b, ",\"length\":%u}", s.length);
    return "{\"element_id\":" + ie_json(s) + b;
}

std::string wrap(const char *tag, const std::string &inner) { return std::string("{\"") + tag + "\":" + inner + "}"; }

const IeRow *ie_find(uint32_t pen, uint16_t id) { return ies().find(pen, id); }

const IeRow *ie_find_name(const char *vendor, const std::string &name) {
    const uint32_t pen = vendor ? vendor_pen(vendor) : 0;
    if (vendor && !pen) return nullptr;
    for (const auto &r : kIes)
        if (r.pen == pen && name == r.name) return &r;
    return nullptr;
}

const char *vendor_name(uint32_t pen) { return ies().vendor(pen); }

uint32_t vendor_pen(const std::string &vendor) {
    for (const auto &v : kVendors)
        if (vendor == v.name) return v.pen;
    return 0;
}

}  // namespace ngzh

namespace {

// Decode rule of one field (generator.rs:1439-1807 by data type;
// netflow.rs:443-475 for NFv9 scope fields) -> device kind and column width.
void field_rule(const Spec &s, uint8_t &kind, uint16_t &width, uint8_t &fail) {
    const uint32_t L = s.length;
    fail = 0;
    auto failk = [&](uint8_t sub) { kind = NGZ_K_FAIL; width = 0; fail = sub; };
    if (s.kind == IK_SCOPE) {
        if (s.pen == 0 && s.id >= 1 && s.id <= 3) {
            if (L > 4) failk(3);
            else { kind = NGZ_K_SCOPE32; width = 4; }
        } else { kind = NGZ_K_BYTES; width = (uint16_t)L; }
        return;
    }
    if (s.kind == IK_UNKNOWN || s.kind == IK_VENDOR_UNKNOWN) {
        // IE::Unknown reads 65535 fixed bytes (generator.rs:2971-2974); vendor Unknown is vlen-aware
        if (L == 0xFFFF && s.kind == IK_VENDOR_UNKNOWN) { kind = NGZ_K_VLEN; width = 16; }
        else { kind = NGZ_K_BYTES; width = (uint16_t)L; }
        return;
    }
    switch (s.dtype) {
    case DT_octetArray:
        if (s.flags & 1) { if (L != 3) failk(1); else { kind = NGZ_K_BYTES; width = 3; } return; }
        [[fallthrough]];
    case DT_basicList:
    case DT_subTemplateList:
    case DT_subTemplateMultiList:
        if (L == 0xFFFF) { kind = NGZ_K_VLEN; width = 16; }
        else { kind = NGZ_K_BYTES; width = (uint16_t)L; }
        return;
    case DT_string:
        if (L == 0xFFFF) { kind = NGZ_K_VLEN; width = 16; fail = 0x80; }
        else { kind = NGZ_K_STR; width = (uint16_t)L; }
        return;
    case DT_unsigned8: if (L != 1) failk(1); else { kind = NGZ_K_UINT; width = 1; } return;
    case DT_unsigned16:
        if (L != 1 && L != 2) failk(1);
        else if (s.flags & 2) { kind = NGZ_K_TCPFLAGS; width = 1; }
        else { kind = NGZ_K_UINT; width = 2; }
        return;
    case DT_unsigned32: if (L > 4) failk(1); else { kind = NGZ_K_UINT; width = 4; } return;
    case DT_unsigned64: if (L > 8) failk(1); else { kind = NGZ_K_UINT; width = 8; } return;
    case DT_unsigned256: if (L > 32) failk(1); else { kind = NGZ_K_U256; width = 32; } return;
    case DT_signed8: if (L != 1) failk(1); else { kind = NGZ_K_SINT; width = 1; } return;
    case DT_signed16: if (L != 1 && L != 2) failk(1); else { kind = NGZ_K_SINT; width = 2; } return;
    case DT_signed32:
        if (L > 8) failk(1);
        else if (L > 4) failk(2);
        else { kind = NGZ_K_SINT; width = 4; }
        return;
    case DT_signed64: if (L > 8) failk(1); else { kind = NGZ_K_SINT; width = 8; } return;
    case DT_float32: if (L != 4) failk(1); else { kind = NGZ_K_UINT; width = 4; } return;
    case DT_float64: if (L != 8) failk(1); else { kind = NGZ_K_UINT; width = 8; } return;
    case DT_boolean: if (L != 1) failk(1); else { kind = NGZ_K_BOOL; width = 1; } return;
    case DT_macAddress: if (L != 6) failk(1); else { kind = NGZ_K_BYTES; width = 6; } return;
    case DT_ipv4Address: if (L != 4) failk(1); else { kind = NGZ_K_UINT; width = 4; } return;
    case DT_ipv6Address: if (L != 16) failk(1); else { kind = NGZ_K_BYTES; width = 16; } return;
    case DT_dateTimeSeconds: if (L != 4) failk(1); else { kind = NGZ_K_UINT; width = 4; } return;
    case DT_dateTimeMilliseconds: if (L != 8) failk(1); else { kind = NGZ_K_DTMS; width = 8; } return;
    case DT_dateTimeMicroseconds:
    case DT_dateTimeNanoseconds: if (L != 8) failk(1); else { kind = NGZ_K_DTFRAC; width = 8; } return;
    }
    failk(1);
}

// A plan gets a generated kernel when the device decodes it at all and no
// raw field is huge (IE::Unknown of length 65535 never yields a record).
bool rtc_eligible(const DevPlan &P) {
    if (!P.rpl || P.n_fields > NGZ_RTC_MAX_FIELDS) return false;
    for (uint32_t i = 0; i < P.n_fields; ++i)
        if (P.f[i].kind != NGZ_K_VLEN && P.f[i].len > 4096) return false;
    return true;
}

void build_plan(Version &v) {
    DevPlan &P = v.plan;
    memset(&P, 0, sizeof P);
    P.proto = v.proto;
    P.template_id = v.tid;
    v.fail_sub.assign(v.specs.size(), 0);
    v.fields.assign(v.specs.size(), DevField{});
    uint32_t off = 0, col = 0, rl = 0;
    bool vlen = false;
    for (size_t i = 0; i < v.specs.size(); ++i) {
        const Spec &s = v.specs[i];
        uint8_t kind, fail;
        uint16_t width;
        field_rule(s, kind, width, fail);
        // IPFIX 65535 = variable length; IE::Unknown reads 65535 fixed bytes instead
        // (generator.rs:2971-2974), which the record walk always reports as UnexpectedEof
        if (v.proto == 10 && s.length == 0xFFFF) vlen = true;
        // min_record_length counts a vlen field as 1 (ipfix.rs:193-214); NFv9 literal (netflow.rs:201-210)
        rl += (v.proto == 10 && s.length == 0xFFFF) ? 1 : s.length;
        DevField &fd = v.fields[i];
        fd.off = (uint16_t)(vlen ? 0xFFFF : off);
        fd.len = s.length;
        fd.width = width;
        fd.kind = kind;
        fd.flags = fail;
        fd.col_off = col;
        v.fail_sub[i] = fail;
        off += s.length;
        col += width;
    }
    P.f = v.fields.data();
    // walk program of variable-length records (ngz_vlen_walk fast path)
    P.walk_nv = 0;
    {
        uint32_t k = 0, acc = 0;
        bool usable = true;
        for (const DevField &fd : v.fields) {
            if (fd.kind == NGZ_K_FAIL) usable = false;
            if (fd.kind == NGZ_K_VLEN) {
                if (k >= NGZ_WALK_MAX) { usable = false; break; }
                P.walk_fixed[k++] = (uint16_t)acc;
                acc = 0;
            } else {
                acc += fd.len;
                if (acc > 0xFFFF) usable = false;
            }
        }
        if (usable) {
            P.walk_fixed[k] = (uint16_t)acc;
            P.walk_nv = (uint8_t)k;
        } else {
            P.walk_nv = 0xFF;
        }
    }
    P.n_fields = (uint16_t)v.specs.size();
    P.rec_len = rl;
    P.row_bytes = col;
    P.has_vlen = vlen;
    for (uint32_t i = 0; i < P.n_fields; ++i)
        if (P.f[i].kind == NGZ_K_DTMS || P.f[i].kind == NGZ_K_DTFRAC || P.f[i].kind == NGZ_K_STR ||
            P.f[i].kind == NGZ_K_FAIL)
            P.has_err = 1;
    // rpl != 0: device-decodable (fixed-length records, and IPFIX records with
    // variable-length fields through the framing walk + record-offset arrays)
    P.rpl = 0;
    P.window = NGZ_REG_WINDOW;
    if (rl <= NGZ_MAX_REC_LEN) P.rpl = 1;
    // per-template kernels stage the columns of 256*lds_waves rows in LDS
    // (NGZ_LDS=0: direct column stores, for A/B measurements)
    static const bool lds_on = ngz_knob("NGZ_LDS", 1) != 0;
    // LDS budget per workgroup (gfx950 allows up to 160 KiB) and waves per window
    static const uint32_t lds_budget = (uint32_t)ngz_knob("NGZ_LDS_BUDGET", NGZ_LDS_BUDGET);
    static const uint32_t lds_maxw = (uint32_t)ngz_knob("NGZ_LDS_MAXW", 4);
    // columns at least lds_direct bytes wide skip LDS (stored directly; 0 = stage every column).
    // Default: rows too wide for 4 staged waves in the budget send their 8- and 16-byte columns
    // direct (config 5: 4.35 -> 4.12 ms per 10^8 records); narrower rows stage everything
    // (T20 stays at its 1024-row windows).
    static const int lds_direct_env = (int)ngz_knob("NGZ_LDS_DIRECT_MIN", -1);
    const uint32_t lds_direct = lds_direct_env >= 0 ? (uint32_t)lds_direct_env
                                : (NGZ_REG_WINDOW * 4 * P.row_bytes > lds_budget ? 8u : 0u);
    uint32_t staged = 0;
    for (uint32_t i = 0; i < P.n_fields; ++i) {
        bool seen = false;
        for (uint32_t g = 0; g < i; ++g) seen = seen || (P.f[g].width && P.f[g].col_off == P.f[i].col_off);
        if (!seen && !(lds_direct && P.f[i].width >= lds_direct)) staged += P.f[i].width;
    }
    P.reserved0 = (uint8_t)std::min<uint32_t>(lds_direct, 255);
    P.lds_waves = (P.rpl && !vlen && lds_on && staged) ? ngz_lds_waves(staged, lds_budget, lds_maxw) : 0;
    // NetFlow v9 fixed templates: exporters send a few records per packet (MTU datagrams, ~10-30),
    // so their sets are row-mode sized; they get the staged-row kernel shape of variable-length
    // templates (each wave copies its 64 records' image into LDS with 1 KiB loads, columns stored
    // directly) instead of LDS column windows gathering rows across ~26 chunks: config 4's
    // template 313 decode 669 -> ~610 us (profiles/r5/cfg4_nf313_staged).  Records of up to 160 B
    // (64 of them fit the 10 KiB per-wave image).
    if (P.proto == 9 && !vlen && P.rpl && rl <= NGZ_VSTAGE_REC_MAX && ngz_knob("NGZ_NF9_STAGED", 1)) P.lds_waves = 0;
    if (!P.lds_waves) P.reserved0 = 0;
}

int fail(ngz_ctx *c, int code, const char *msg) {
    if (c) c->last_error = msg;
    return code;
}

#define HIPCHK(x)                                                                   \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            ctx->last_error = std::string(#x) + ": " + hipGetErrorString(e_);       \
            return NGZ_E_DEVICE;                                                    \
        }                                                                           \
    } while (0)


// ------------------------------------------------------------------------
// Host framing of a template-bearing datagram (stream order).  Restates
// Set::parse for template / options-template sets and the framing of data
// sets; records themselves are decoded on the device.
// ------------------------------------------------------------------------
struct HostFrameOut {
    ngz_dgram_hdr hdr{};
    std::vector<HostSet> sets;
    std::vector<std::pair<uint32_t, int32_t>> defs;  // (set position, version) defined here
    std::vector<std::pair<uint32_t, int32_t>> restarts;  // the defs that re-announced the current version
    std::vector<std::pair<uint32_t, std::string>> tsets;  // (set position, serde JSON) of template sets
};

// serde JSON of a parsed (options) template record (ipfix.rs:384-413 /
// :276-327, netflow.rs:265-353; TemplateRecord has no scope key)
std::string template_record_json(uint32_t tid, const std::vector<Spec> *scope, const std::vector<Spec> &fields) {
    std::string j = "{\"id\":" + std::to_string(tid);
    if (scope) {
        j += ",\"scope_field_specifiers\":[";
        for (size_t i = 0; i < scope->size(); ++i) j += (i ? "," : "") + spec_json((*scope)[i]);
        j += "]";
    }
    j += ",\"field_specifiers\":[";
    for (size_t i = 0; i < fields.size(); ++i) j += (i ? "," : "") + spec_json(fields[i]);
    return j + "]}";
}

struct Eof {
    uint32_t offset, needed, available;
};

std::string eof_json(const Eof &e) {
    char b[128];
    snprintf(b, sizeof b, "{\"Parse\":{\"UnexpectedEof\":{\"offset\":%u,\"needed\":%u,\"available\":%u}}}", e.offset,
             e.needed, e.available);
    return b;
}

struct Cur {
    const uint8_t *p;
    uint32_t pos, end;
    bool need(uint32_t n, Eof &e) const {
        if (end - pos < n) { e = {pos, n, end - pos}; return false; }
        return true;
    }
};

// FieldSpecifier::parse (deserializer/mod.rs:53-66) -> json error on failure
bool parse_field_spec(Cur &c, Spec &out, std::string &err) {
    Eof e;
    if (!c.need(2, e)) { err = eof_json(e); return false; }
    uint32_t code = rd16(c.p + c.pos); c.pos += 2;
    if (!c.need(2, e)) { err = eof_json(e); return false; }
    uint32_t len = rd16(c.p + c.pos); c.pos += 2;
    uint32_t pen = 0;
    if (code & 0x8000) {
        if (!c.need(4, e)) { err = eof_json(e); return false; }
        pen = rd32(c.p + c.pos); c.pos += 4;
        code &= 0x7FFF;
    }
    Spec s{};
    s.pen = pen;
    s.length = (uint16_t)len;
    s.scope = false;
    if (pen == 0) {
        const IeRow *r = ies().find(0, (uint16_t)code);
        if (!r) {
            char b[96];
            snprintf(b, sizeof b, "{\"IEError\":{\"UndefinedIANAIE\":%u}}", code);
            err = b;
            return false;
        }
        s.kind = IK_IANA; s.id = (uint16_t)code; s.dtype = r->dtype; s.flags = r->flags; s.name = r->name;
    } else if (const char *vn = ies().vendor(pen)) {
        const uint16_t id = (uint16_t)(code & 0x7FFF);
        const IeRow *r = ies().find(pen, id);
        s.vendor = vn; s.id = id;
        if (r) { s.kind = IK_VENDOR; s.dtype = r->dtype; s.flags = r->flags; s.name = r->name; }
        else { s.kind = IK_VENDOR_UNKNOWN; s.dtype = DT_octetArray; s.flags = 0; }
    } else {
        s.kind = IK_UNKNOWN; s.id = (uint16_t)code; s.dtype = DT_octetArray; s.flags = 0;
    }
    int lo, hi;
    length_range(s.dtype, lo, hi);
    if (hi && !((int)len >= lo && (int)len < hi)) {  // lib.rs:147-154
        char b[64];
        snprintf(b, sizeof b, "{\"FieldSpecifierError\":{\"InvalidLength\":[%u,", len);
        err = std::string(b) + ie_json(s) + "]}}";
        return false;
    }
    out = s;
    return true;
}

// ScopeFieldSpecifier::parse (netflow.rs:368-388)
bool parse_scope_spec(Cur &c, Spec &out, std::string &err) {
    Eof e;
    const uint32_t off = c.pos;
    if (!c.need(2, e)) { err = eof_json(e); return false; }
    uint32_t code = rd16(c.p + c.pos); c.pos += 2;
    if (!c.need(2, e)) { err = eof_json(e); return false; }
    uint32_t len = rd16(c.p + c.pos); c.pos += 2;
    uint32_t pen = 0;
    if (code & 0x8000) {
        if (!c.need(4, e)) { err = eof_json(e); return false; }
        pen = rd32(c.p + c.pos); c.pos += 4;
    }
    Spec s{};
    s.kind = IK_SCOPE; s.scope = true; s.pen = pen; s.id = (uint16_t)code; s.length = (uint16_t)len;
    s.dtype = DT_octetArray;
    if (pen == 0 && (code == 2 || code == 3) && !(len >= 1 && len < 5)) {
        char b[160];
        snprintf(b, sizeof b, "{\"InvalidLength\":{\"offset\":%u,\"ie\":%s,\"length\":%u}}", off,
                 ie_json(s).c_str(), len);
        err = b;
        return false;
    }
    out = s;
    return true;
}


bool same_specs(const Spec &a, const Spec &b) {
    return a.kind == b.kind && a.pen == b.pen && a.id == b.id && a.length == b.length && a.scope == b.scope;
}

// A template record (ipfix.rs:384-413, :276-327; netflow.rs:265-353): the id's new current version.
// An exporter re-announces its templates every few packets or seconds; a re-announcement with the
// same specifiers as the current version reuses that version (its slot, columns and kernel) instead
// of appending one per announcement -- a batch with many refreshes stays within NGZ_MAX_SLOTS and a
// long-lived peer's version list does not grow.  The reference replaces the map entry with a fresh
// DecodingTemplate, so processed_count restarts: `restart` reports that (define_at records the
// position; finish_batch resets the count and k_counts counts only later sets).
int32_t define_template(ngz_ctx *ctx, uint8_t proto, uint16_t tid, std::vector<Spec> &&scope, std::vector<Spec> &&fields,
                        bool *restart) {
    const int32_t cur = ctx->cur[proto == 10 ? 0 : 1][tid];
    if (cur >= 0) {
        const Version &c = ctx->versions[cur];
        bool same = c.n_scope == scope.size() && c.specs.size() == scope.size() + fields.size();
        for (size_t i = 0; same && i < c.specs.size(); ++i) {
            Spec s = i < scope.size() ? scope[i] : fields[i - scope.size()];
            s.scope = i < scope.size();
            same = same_specs(c.specs[i], s);
        }
        if (same) {
            *restart = true;
            return cur;
        }
    }
    *restart = false;
    Version v;
    v.proto = proto;
    v.tid = tid;
    v.n_scope = (uint32_t)scope.size();
    v.specs = std::move(scope);
    for (auto &f : fields) v.specs.push_back(f);
    for (uint32_t i = 0; i < v.n_scope; ++i) v.specs[i].scope = true;
    build_plan(v);
    ctx->versions.push_back(std::move(v));
    const int32_t vid = (int32_t)ctx->versions.size() - 1;
    ctx->cur[proto == 10 ? 0 : 1][tid] = vid;
    ctx->tmpl_gen++;
    return vid;
}

// frame one datagram on the host; `limit` = stop before any set at a position > limit
void host_frame(ngz_ctx *ctx, const uint8_t *p, uint32_t dl, uint32_t limit, HostFrameOut &o) {
    ngz_dgram_hdr &h = o.hdr;
    memset(&h, 0, sizeof h);
    h.err_key = NGZ_NO_ERR;
    auto set_err = [&](uint32_t stop, const std::string &json) {
        ctx->host_errors.push_back({json});
        h.err_key = ngz_err_key(stop, E_HOST, 0, (uint32_t)ctx->host_errors.size() - 1);
    };
    if (dl < 16) { h.status = NGZ_DG_NEED_MORE; return; }
    const uint32_t ver = rd16(p), len = rd16(p + 2);
    if (dl < len) { h.status = NGZ_DG_NEED_MORE; return; }
    h.version = (uint8_t)ver;
    h.length = (uint16_t)len;
    char b[256];
    if (ver == 10) {
        const char *W = "IpfixParsingError";
        if (len < 16) {
            snprintf(b, sizeof b, "{\"InvalidLength\":{\"offset\":2,\"length\":%u}}", len);
            set_err(2, wrap(W, b));
            return;
        }
        h.time = rd32(p + 4); h.sequence = rd32(p + 8); h.domain = rd32(p + 12);
        uint32_t pos = 16;
        while (pos < len) {
            if (pos > limit) return;
            const uint32_t rem = len - pos;
            auto serr = [&](uint32_t stop, const std::string &j) { set_err(stop, wrap(W, wrap("SetParsingError", j))); };
            if (rem < 2) { serr(pos, eof_json({pos, 2, rem})); return; }
            const uint32_t id = rd16(p + pos);
            if (id != 2 && id != 3 && id < 256) {
                snprintf(b, sizeof b, "{\"InvalidSetId\":{\"offset\":%u,\"id\":%u}}", pos, id);
                serr(pos, b); return;
            }
            if (rem < 4) { serr(pos + 2, eof_json({pos + 2, 2, rem - 2})); return; }
            const uint32_t sl = rd16(p + pos + 2);
            if (sl < 4) {
                snprintf(b, sizeof b, "{\"InvalidLength\":{\"offset\":%u,\"length\":%u}}", pos + 2, sl);
                serr(pos + 2, b); return;
            }
            if (sl - 4 > rem - 4) { serr(pos + 4, eof_json({pos + 4, sl - 4, rem - 4})); return; }
            h.n_sets++;
            Cur c{p, pos + 4, pos + sl};
            if (id == 2) {  // ipfix.rs:162-168, TemplateRecord::parse :384-413
                std::string recs;
                while (c.pos < c.end) {
                    const uint32_t toff = c.pos;
                    Eof e;
                    auto terr = [&](const std::string &j) { serr(c.pos, wrap("TemplateRecordError", j)); };
                    if (!c.need(2, e)) { terr(eof_json(e)); return; }
                    const uint32_t tid = rd16(p + c.pos);
                    if (tid < 256) {
                        snprintf(b, sizeof b, "{\"InvalidTemplateId\":{\"offset\":%u,\"template_id\":%u}}", toff, tid);
                        terr(b); return;
                    }
                    c.pos += 2;
                    if (!c.need(2, e)) { terr(eof_json(e)); return; }
                    const uint32_t cnt = rd16(p + c.pos); c.pos += 2;
                    std::vector<Spec> fields;
                    for (uint32_t i = 0; i < cnt; ++i) {
                        Spec s; std::string err;
                        if (!parse_field_spec(c, s, err)) { terr(wrap("FieldSpecifierError", err)); return; }
                        fields.push_back(s);
                    }
                    recs += (recs.empty() ? "" : ",") + template_record_json(tid, nullptr, fields);
                    bool rs;
                    o.defs.push_back({toff, define_template(ctx, 10, (uint16_t)tid, {}, std::move(fields), &rs)});
                    if (rs) o.restarts.push_back({toff, o.defs.back().second});
                }
                o.tsets.push_back({pos, "{\"Template\":[" + recs + "]}"});
            } else if (id == 3) {  // ipfix.rs:169-181, OptionsTemplateRecord::parse :276-327
                std::string recs;
                while (c.end - c.pos > 3) {
                    const uint32_t toff = c.pos;
                    Eof e;
                    auto terr = [&](const std::string &j) { serr(c.pos, wrap("OptionsTemplateRecordError", j)); };
                    const uint32_t tid = rd16(p + c.pos);
                    if (tid < 256) {
                        snprintf(b, sizeof b, "{\"InvalidTemplateId\":{\"offset\":%u,\"template_id\":%u}}", toff, tid);
                        terr(b); return;
                    }
                    c.pos += 2;
                    if (!c.need(2, e)) { terr(eof_json(e)); return; }
                    const uint32_t total = rd16(p + c.pos); c.pos += 2;
                    const uint32_t soff = c.pos;
                    if (!c.need(2, e)) { terr(eof_json(e)); return; }
                    const uint32_t scount = rd16(p + c.pos);
                    if (scount > total) {
                        snprintf(b, sizeof b,
                                 "{\"InvalidScopeFieldsCount\":{\"offset\":%u,\"scope_fields_count\":%u,\"total_fields_count\":%u}}",
                                 soff, scount, total);
                        terr(b); return;
                    }
                    c.pos += 2;
                    std::vector<Spec> scope, fields;
                    for (uint32_t i = 0; i < total; ++i) {
                        Spec s; std::string err;
                        if (!parse_field_spec(c, s, err)) { terr(wrap("FieldError", err)); return; }
                        (i < scount ? scope : fields).push_back(s);
                    }
                    recs += (recs.empty() ? "" : ",") + template_record_json(tid, &scope, fields);
                    bool rs;
                    o.defs.push_back({toff, define_template(ctx, 10, (uint16_t)tid, std::move(scope), std::move(fields), &rs)});
                    if (rs) o.restarts.push_back({toff, o.defs.back().second});
                }
                for (uint32_t q = c.pos; q < c.end; ++q)  // check_padding_value (ipfix.rs:240-251)
                    if (p[q]) {
                        snprintf(b, sizeof b, "{\"InvalidPaddingValue\":{\"offset\":%u,\"value\":%u}}", q, p[q]);
                        serr(q, b); return;
                    }
                o.tsets.push_back({pos, "{\"OptionsTemplate\":[" + recs + "]}"});
            } else {
                const int32_t vid = ctx->cur[0][id];
                if (vid < 0) {
                    snprintf(b, sizeof b, "{\"NoTemplateDefinedFor\":{\"offset\":%u,\"id\":%u}}", pos, id);
                    serr(pos, b); return;
                }
                const Version &v = ctx->versions[vid];
                const uint32_t ml = v.plan.rec_len;
                uint64_t verr = NGZ_NO_ERR;
                uint32_t n;
                if (v.plan.has_vlen && v.plan.rpl)  // record lengths come from the data (ipfix.rs:219-222)
                    n = ngz_vlen_walk(p, pos + 4, pos + sl, v.plan, &verr, [](uint32_t, uint32_t) {});
                else
                    n = ml ? (sl - 4) / ml : 0;
                if (n && !v.plan.rpl) { h.status = NGZ_DG_UNSUPPORTED; return; }
                HostSet hs{};
                hs.set_pos = (uint16_t)pos; hs.reserved2 = (uint32_t)vid; hs.payload_pos = (uint16_t)(pos + 4); hs.n = n;
                o.sets.push_back(hs);
                if (verr != NGZ_NO_ERR) { h.err_key = verr; return; }  // rendered like a device-found record error
            }
            pos += sl;
        }
        return;
    }
    if (ver == 9) {
        const char *W = "NetFlowV9ParingError";
        if (dl < 20) { set_err(16, wrap(W, eof_json({16, 4, dl - 16}))); return; }
        h.sys_up_time = rd32(p + 4); h.time = rd32(p + 8); h.sequence = rd32(p + 12); h.domain = rd32(p + 16);
        const uint32_t count = len;
        uint32_t i = count, pos = 20;
        while (i > 0 && dl - pos > 3) {
            if (pos > limit) return;
            const uint32_t rem = dl - pos;
            auto serr = [&](uint32_t stop, const std::string &j) { set_err(stop, wrap(W, wrap("SetError", j))); };
            const uint32_t id = rd16(p + pos);
            if (id != 0 && id != 1 && id < 256) {
                snprintf(b, sizeof b, "{\"InvalidSetId\":{\"offset\":%u,\"id\":%u}}", pos, id);
                serr(pos, b); return;
            }
            const uint32_t sl = rd16(p + pos + 2);
            if (sl < 4) {
                snprintf(b, sizeof b, "{\"InvalidLength\":{\"offset\":%u,\"length\":%u}}", pos + 2, sl);
                serr(pos + 2, b); return;
            }
            if (sl - 4 > rem - 4) { serr(pos + 4, eof_json({pos + 4, sl - 4, rem - 4})); return; }
            h.n_sets++;
            Cur c{p, pos + 4, pos + sl};
            if (id == 0) {  // netflow.rs:172-178, TemplateRecord :324-353
                std::string recs;
                while (c.pos < c.end) {
                    const uint32_t toff = c.pos;
                    Eof e;
                    auto terr = [&](const std::string &j) { serr(c.pos, wrap("TemplateRecordError", j)); };
                    if (!c.need(2, e)) { terr(eof_json(e)); return; }
                    const uint32_t tid = rd16(p + c.pos);
                    if (tid < 256) {
                        snprintf(b, sizeof b, "{\"InvalidTemplateId\":{\"offset\":%u,\"template_id\":%u}}", toff, tid);
                        terr(b); return;
                    }
                    c.pos += 2;
                    if (!c.need(2, e)) { terr(eof_json(e)); return; }
                    const uint32_t cnt = rd16(p + c.pos); c.pos += 2;
                    std::vector<Spec> fields;
                    for (uint32_t k = 0; k < cnt; ++k) {
                        Spec s; std::string err;
                        if (!parse_field_spec(c, s, err)) { terr(wrap("FieldSpecifierError", err)); return; }
                        fields.push_back(s);
                    }
                    recs += (recs.empty() ? "" : ",") + template_record_json(tid, nullptr, fields);
                    bool rs;
                    o.defs.push_back({toff, define_template(ctx, 9, (uint16_t)tid, {}, std::move(fields), &rs)});
                    if (rs) o.restarts.push_back({toff, o.defs.back().second});
                }
                o.tsets.push_back({pos, "{\"Template\":[" + recs + "]}"});
                i -= 1;
            } else if (id == 1) {  // netflow.rs:179-190, OptionsTemplateRecord :265-310
                std::string recs;
                while (c.end - c.pos > 3) {
                    const uint32_t toff = c.pos;
                    Eof e;
                    auto terr = [&](const std::string &j) { serr(c.pos, wrap("OptionsTemplateRecordError", j)); };
                    const uint32_t tid = rd16(p + c.pos);
                    if (tid < 256) {
                        snprintf(b, sizeof b, "{\"InvalidTemplateId\":{\"offset\":%u,\"template_id\":%u}}", toff, tid);
                        terr(b); return;
                    }
                    c.pos += 2;
                    if (!c.need(2, e)) { terr(eof_json(e)); return; }
                    const uint32_t slen = rd16(p + c.pos); c.pos += 2;
                    if (!c.need(2, e)) { terr(eof_json(e)); return; }
                    const uint32_t olen = rd16(p + c.pos); c.pos += 2;
                    if (!c.need(slen, e)) { terr(eof_json(e)); return; }
                    Cur sc{p, c.pos, c.pos + slen};
                    c.pos += slen;
                    if (!c.need(olen, e)) { terr(eof_json(e)); return; }
                    Cur oc{p, c.pos, c.pos + olen};
                    c.pos += olen;
                    std::vector<Spec> scope, fields;
                    while (sc.pos < sc.end) {
                        Spec s; std::string err;
                        if (!parse_scope_spec(sc, s, err)) { serr(sc.pos, wrap("OptionsTemplateRecordError", wrap("ScopeFieldSpecifierError", err))); return; }
                        scope.push_back(s);
                    }
                    while (oc.pos < oc.end) {
                        Spec s; std::string err;
                        if (!parse_field_spec(oc, s, err)) { serr(oc.pos, wrap("OptionsTemplateRecordError", wrap("FieldSpecifierError", err))); return; }
                        fields.push_back(s);
                    }
                    recs += (recs.empty() ? "" : ",") + template_record_json(tid, &scope, fields);
                    bool rs;
                    o.defs.push_back({toff, define_template(ctx, 9, (uint16_t)tid, std::move(scope), std::move(fields), &rs)});
                    if (rs) o.restarts.push_back({toff, o.defs.back().second});
                }
                for (uint32_t q = c.pos; q < c.end; ++q)
                    if (p[q]) {
                        snprintf(b, sizeof b, "{\"InvalidPaddingValue\":{\"offset\":%u,\"value\":%u}}", q, p[q]);
                        serr(q, b); return;
                    }
                o.tsets.push_back({pos, "{\"OptionsTemplate\":[" + recs + "]}"});
                i -= 1;
            } else {
                const int32_t vid = ctx->cur[1][id];
                if (vid < 0) {
                    snprintf(b, sizeof b, "{\"NoTemplateDefinedFor\":{\"offset\":%u,\"id\":%u}}", pos, id);
                    serr(pos, b); return;
                }
                const Version &v = ctx->versions[vid];
                const uint32_t rl = v.plan.rec_len;
                const uint32_t n = rl ? (sl - 4) / rl : 0;
                if (n && !v.plan.rpl) { h.status = NGZ_DG_UNSUPPORTED; return; }
                HostSet hs{};
                hs.set_pos = (uint16_t)pos; hs.reserved2 = (uint32_t)vid; hs.payload_pos = (uint16_t)(pos + 4); hs.n = n;
                o.sets.push_back(hs);
                for (uint32_t q = pos + 4 + n * rl; q < pos + sl; ++q)
                    if (p[q]) {
                        snprintf(b, sizeof b, "{\"InvalidPaddingValue\":{\"offset\":%u,\"value\":%u}}", q, p[q]);
                        serr(q, b); return;
                    }
                if (n > i) {
                    snprintf(b, sizeof b, "{\"InvalidCount\":{\"offset\":2,\"count\":%u}}", count);
                    set_err(pos + sl, wrap(W, b)); return;
                }
                i -= n;
            }
            pos += sl;
        }
        return;
    }
    snprintf(b, sizeof b, "{\"UnsupportedVersion\":%u}", ver);
    set_err(0, b);
}

// ------------------------------------------------------------------------
// Batch pipeline
// ------------------------------------------------------------------------
struct Timeline {
    std::vector<uint32_t> key, dgram;
    std::vector<uint16_t> slot;
};

int assign_slots(ngz_ctx *ctx, const std::vector<int32_t> &extra) {
    // slots = every current version of both protocols + versions defined in the batch
    std::vector<int32_t> sv;
    for (int pi = 0; pi < 2; ++pi)
        for (uint32_t id = 0; id < 65536; ++id)
            if (ctx->cur[pi][id] >= 0) sv.push_back(ctx->cur[pi][id]);
    for (int32_t v : extra) sv.push_back(v);
    std::sort(sv.begin(), sv.end());
    sv.erase(std::unique(sv.begin(), sv.end()), sv.end());
    if (sv.size() > NGZ_MAX_SLOTS) return fail(ctx, NGZ_E_LIMIT, "too many live template versions in one batch");
    if (sv != ctx->slot_version) {
        ctx->slot_version = sv;
        ctx->plans_dirty = true;
    }
    ctx->version_slot.assign(ctx->versions.size(), -1);
    for (size_t s = 0; s < sv.size(); ++s) ctx->version_slot[sv[s]] = (int32_t)s;
    ctx->assigned_gen = extra.empty() ? ctx->tmpl_gen : 0;  // reused until the template state changes
    return 0;
}

int upload_slots(ngz_ctx *ctx, const std::vector<int32_t> cur_start[2], hipStream_t st) {
    const size_t S = ctx->slot_version.size();
    if (ctx->d_plans.ensure(std::max<size_t>(S, 1)) || ctx->d_cur_slot.ensure(2 * 65536))
        return fail(ctx, NGZ_E_NOMEM, "device alloc (plans)");
    size_t nf_total = 0;
    for (size_t s = 0; s < S; ++s) nf_total += ctx->versions[ctx->slot_version[s]].fields.size();
    if (ctx->d_fields.ensure(std::max<size_t>(nf_total, 1))) return fail(ctx, NGZ_E_NOMEM, "device alloc (field tables)");
    std::vector<DevPlan> plans(S);
    std::vector<DevField> ftab;
    ftab.reserve(nf_total);
    for (size_t s = 0; s < S; ++s) {
        Version &v = ctx->versions[ctx->slot_version[s]];
        plans[s] = v.plan;
        plans[s].f = ctx->d_fields.p + ftab.size();  // the slot's descriptors in the device field table
        const auto cf = ctx->count_from.find(ctx->slot_version[s]);
        plans[s].count_from = cf == ctx->count_from.end() ? 0 : cf->second;
        ftab.insert(ftab.end(), v.fields.begin(), v.fields.end());
        plans[s].spec = 0;
        if (ctx->specialize && rtc_eligible(v.plan)) {
            // NGZ_OPT_SPECIALIZE 2: compile once the template has seen enough records to pay for it
            const bool want = ctx->specialize == 1 || v.seen_records >= NGZ_SPECIALIZE_MIN_RECORDS;
            if (want && (v.rtc_state == 0 || (v.rtc_state == 3 && ctx->rtc_sync))) {
                if (ctx->rtc_sync) {  // wait for the compile (NGZ_OPT_RTC_SYNC)
                    v.rtc_fn = ngz_rtc_kernel(ctx->device, v.plan);
                    v.rtc_state = v.rtc_fn ? 1 : 2;
                } else {  // compile in the background; the generic kernel decodes meanwhile
                    const int r = ngz_rtc_kernel_async(ctx->device, v.plan, &v.rtc_fn, &v.rtc_entry);
                    v.rtc_state = r == 1 ? 1 : r < 0 ? 2 : 3;
                }
            }
            plans[s].spec = v.rtc_state == 1;
        }
    }
    ctx->slot_spec.assign(S, 0);  // the kernel each slot's records go through (ngz_slot_kernel)
    for (size_t s = 0; s < S; ++s)
        ctx->slot_spec[s] = plans[s].spec ? 1 : ctx->versions[ctx->slot_version[s]].rtc_state == 3 ? 2 : 0;
    std::vector<uint16_t> cs(2 * 65536, NGZ_NO_SLOT);
    for (int pi = 0; pi < 2; ++pi)
        for (uint32_t id = 0; id < 65536; ++id)
            if (cur_start[pi][id] >= 0) cs[pi * 65536 + id] = (uint16_t)ctx->version_slot[cur_start[pi][id]];
    HIPCHK(hipMemcpyAsync(ctx->d_plans.p, plans.data(), S * sizeof(DevPlan), hipMemcpyHostToDevice, st));
    if (!ftab.empty())
        HIPCHK(hipMemcpyAsync(ctx->d_fields.p, ftab.data(), ftab.size() * sizeof(DevField), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(ctx->d_cur_slot.p, cs.data(), cs.size() * 2, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));  // host vectors go out of scope
    ctx->plans_dirty = false;
    return 0;
}

struct HostFramed {
    std::vector<uint32_t> flag;       // per datagram: 0, or 1 + index into hdrs
    std::vector<uint32_t> first;      // CSR
    std::vector<HostSet> sets;
    std::vector<ngz_dgram_hdr> hdrs;
    Timeline tl;
};

static void trace_report(ngz_ctx *ctx, uint32_t S, hipStream_t st);

int run_pipeline(ngz_ctx *ctx, const ngz_batch_in *in, hipStream_t st, const HostFramed *hf) {
    const uint32_t N = in->n;
    const uint32_t S = (uint32_t)ctx->slot_version.size();
    // count-matrix rows: steady state gives rows only to the slots that had records in the last
    // batch (config 4's context holds 18 template slots, 2 with data: 37 rows of 4 bytes per
    // datagram were zeroed, filled and scanned for 5); a set of another slot makes k_frame raise
    // overflow bit 8 and the batch runs again with a row for every slot
    const bool few_rows = ctx->pred_valid && ctx->pred_versions == ctx->slot_version && !hf && !ctx->rows_all &&
                          ctx->pred_active.size() == S;
    bool any_vlen = false;
    uint32_t min_vlen_rec = 0xFFFFFFFFu;
    std::vector<uint8_t> is_v(S, 0);  // a variable-length template (records walked one by one)
    for (uint32_t s = 0; s < S; ++s) {
        const DevPlan &P = ctx->versions[ctx->slot_version[s]].plan;
        if (P.has_vlen && P.rpl) {
            any_vlen = true;
            is_v[s] = 1;
            min_vlen_rec = std::min<uint32_t>(min_vlen_rec, P.rec_len);
        }
    }
    // Records of variable-length sets found by k_frame's walk reach k_emit as a list of
    // record offsets per datagram (2 bytes per record, written in order by the walking
    // thread; no per-batch zeroing).  Every such record spans at least min_record_length
    // bytes (ipfix.rs:193-214), so datagram d's list fits from entry offsets[d] / that + d.
    // Templates whose records may be shorter than 8 bytes use the record-start bitmap (one
    // bit per batch byte, zeroed per batch).  NGZ_RECMAP: 0 walk twice, 1 bitmap, 2 lists.
    static const int recmap_env = (int)ngz_knob("NGZ_RECMAP", -1);
    const bool lists = any_vlen && recmap_env != 0 && recmap_env != 1 && min_vlen_rec >= 8;
    // Split framing (steady state, every active template with its compiled kernel, record-offset
    // lists): the record walk of the variable-length sets -- one thread per datagram through a
    // chain of dependent length-prefix loads, latency-bound -- runs on a second stream (phase B)
    // beside the framing, layout and decode of the fixed-length sets (phase A, bandwidth-bound),
    // then lays out, emits and decodes its own templates there; the two join before the counts.
    // Measured on config 4 (NFv9 + variable-length IPFIX, r4b): 2.69 ms per step split against
    // 2.51 unsplit on the same box.  Phase A's framing without the walk took 0.72 ms beside phase
    // B's walk (0.66 ms) -- the whole k_frame took 0.61 alone --, both emits slowed, and the two
    // decodes side by side took 1.55 ms against 1.50 in turn: framing is bound by the memory
    // system's scattered line requests, as the decode is by bandwidth, not by load latency that
    // another stream could fill.  Off unless NGZ_SPLIT=1 (read per batch).
    const int split_env = ctx->split_framing;
    bool split = false;
    if (split_env && few_rows && lists && ctx->specialize) {
        bool any_v = false, any_f = false, all_spec = true;
        for (uint32_t s = 0; s < S; ++s) {
            if (!ctx->pred_active[s]) continue;
            (is_v[s] ? any_v : any_f) = true;
            all_spec = all_spec && ctx->versions[ctx->slot_version[s]].rtc_state == 1;
        }
        split = any_v && any_f && all_spec && ctx->split_skip == 0;
    }
    if (ctx->split_skip) --ctx->split_skip;
    if (ctx->pipeline_runs++) ctx->batch_info |= NGZ_BATCH_RERUN;
    if (split) ctx->batch_info |= NGZ_BATCH_SPLIT;
    else ctx->batch_info &= ~(uint32_t)NGZ_BATCH_SPLIT;
    std::vector<uint16_t> rows(S, (uint16_t)NGZ_NO_ROW), rows2(S, (uint16_t)NGZ_NO_ROW);
    uint32_t A = 0, A2 = 0;
    for (uint32_t s = 0; s < S; ++s)
        if (!few_rows || ctx->pred_active[s]) {
            if (split && is_v[s]) rows2[s] = (uint16_t)A2++;
            else rows[s] = (uint16_t)A++;
        }
    const uint64_t n_items = (uint64_t)(2 * A + 1) * N + 1, n_items2 = (uint64_t)(2 * A2 + 1) * N + 1;
    if (n_items > 0x7FFFFFF0ull || n_items2 > 0x7FFFFFF0ull)
        return fail(ctx, NGZ_E_LIMIT, "batch too large for the count matrix");
    size_t scan_tmp = 0, scan_tmp2 = 0;
    if (ngz_scan_temp_bytes(n_items, &scan_tmp)) return fail(ctx, NGZ_E_DEVICE, "scan temp size");
    if (split && ngz_scan_temp_bytes(n_items2, &scan_tmp2)) return fail(ctx, NGZ_E_DEVICE, "scan temp size");
    // capacities (overflow is detected on device and retried with more room)
    uint64_t chunk_cap = std::max<uint64_t>(ctx->d_chunks.cap, in->bytes_size / 4096 + 3ull * N + 1024);
    uint64_t set_cap = std::max<uint64_t>(ctx->d_sets.cap, 2ull * N + 1024);
    double ratio = 1.0;
    uint32_t maxwin_row = 0;
    for (uint32_t s = 0; s < S; ++s) {
        const DevPlan &P = ctx->versions[ctx->slot_version[s]].plan;
        // columns + row-mode record table (12 B/row) per wire byte
        if (P.rec_len) ratio = std::max(ratio, (double)(P.row_bytes + 12) / (double)P.rec_len);
        maxwin_row = std::max<uint32_t>(maxwin_row, P.window * std::max<uint32_t>(P.lds_waves, 1) * P.row_bytes);
    }
    uint64_t arena_cap = (uint64_t)(ratio * (double)in->bytes_size) +
                         (uint64_t)S * (1 + ctx->cap_pad_windows) * (maxwin_row + 256) + 4096;
    arena_cap = std::max<uint64_t>(arena_cap + ctx->arena_shift, ctx->d_arena.cap);
    static const uint64_t arena_min = (uint64_t)ngz_knob("NGZ_ARENA_MIN_MB", 0) << 20;
    arena_cap = std::max(arena_cap, arena_min);  // experiment: allocation size vs placement
    const uint16_t *old_rows = ctx->d_slot_row.p;
    if (ctx->d_hdr.ensure(std::max<uint32_t>(N, 1)) || ctx->d_counts.ensure(n_items) || ctx->d_scan.ensure(n_items) ||
        ctx->d_scan_tmp.ensure(scan_tmp + 1) || ctx->d_slots.ensure(std::max<uint32_t>(S, 1)) ||
        ctx->d_chunks.ensure(chunk_cap) || ctx->d_sets.ensure(set_cap) || ctx->d_arena.ensure(arena_cap) ||
        ctx->d_proc.ensure(2 * NGZ_MAX_SLOTS) || ctx->d_summary.ensure(2) ||
        ctx->d_slot_row.ensure(std::max<uint32_t>(S, 1)))
        return fail(ctx, NGZ_E_NOMEM, "device alloc (batch)");
    if (rows != ctx->slot_row_host || ctx->d_slot_row.p != old_rows) {  // changed, or a new buffer
        if (S) HIPCHK(hipMemcpy(ctx->d_slot_row.p, rows.data(), S * 2, hipMemcpyHostToDevice));
        ctx->slot_row_host = rows;
    }
    if (split) {
        const uint16_t *old2 = ctx->d_slot_row2.p;
        if (ctx->d_counts2.ensure(n_items2) || ctx->d_scan2.ensure(n_items2) || ctx->d_scan_tmp2.ensure(scan_tmp2 + 1) ||
            ctx->d_slot_row2.ensure(std::max<uint32_t>(S, 1)))
            return fail(ctx, NGZ_E_NOMEM, "device alloc (split framing)");
        if (rows2 != ctx->slot_row2_host || ctx->d_slot_row2.p != old2) {
            HIPCHK(hipMemcpy(ctx->d_slot_row2.p, rows2.data(), S * 2, hipMemcpyHostToDevice));
            ctx->slot_row2_host = rows2;
        }
        if (!ctx->split_stream) {
            HIPCHK(hipStreamCreateWithFlags(&ctx->split_stream, hipStreamNonBlocking));
            for (auto &e : ctx->split_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
    }
    const int par = ctx->parity;
    BatchSummary *d_sum = ctx->d_summary.p + par;
    unsigned long long *d_proc = ctx->d_proc.p + (size_t)par * NGZ_MAX_SLOTS;
    // host-framed inputs
    const uint32_t *hf_flag = nullptr;
    const uint32_t *hf_first = nullptr;
    BatchDev B{};
    if (hf) {
        if (ctx->d_hf_flag.ensure(N) || ctx->d_hf_first.ensure(N + 1) || ctx->d_hf_sets.ensure(hf->sets.size() + 1) ||
            ctx->d_hf_hdr.ensure(hf->hdrs.size() + 1) ||
            ctx->d_tl_key.ensure(hf->tl.key.size() + 1) || ctx->d_tl_dgram.ensure(hf->tl.key.size() + 1) ||
            ctx->d_tl_slot.ensure(hf->tl.key.size() + 1))
            return fail(ctx, NGZ_E_NOMEM, "device alloc (host framing)");
        HIPCHK(hipMemcpyAsync(ctx->d_hf_flag.p, hf->flag.data(), N * 4ull, hipMemcpyHostToDevice, st));
        if (!hf->hdrs.empty())
            HIPCHK(hipMemcpyAsync(ctx->d_hf_hdr.p, hf->hdrs.data(), hf->hdrs.size() * sizeof(ngz_dgram_hdr),
                                  hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(ctx->d_hf_first.p, hf->first.data(), (N + 1) * 4, hipMemcpyHostToDevice, st));
        if (!hf->sets.empty())
            HIPCHK(hipMemcpyAsync(ctx->d_hf_sets.p, hf->sets.data(), hf->sets.size() * sizeof(HostSet),
                                  hipMemcpyHostToDevice, st));
        if (!hf->tl.key.empty()) {
            HIPCHK(hipMemcpyAsync(ctx->d_tl_key.p, hf->tl.key.data(), hf->tl.key.size() * 4, hipMemcpyHostToDevice, st));
            HIPCHK(hipMemcpyAsync(ctx->d_tl_dgram.p, hf->tl.dgram.data(), hf->tl.dgram.size() * 4, hipMemcpyHostToDevice, st));
            HIPCHK(hipMemcpyAsync(ctx->d_tl_slot.p, hf->tl.slot.data(), hf->tl.slot.size() * 2, hipMemcpyHostToDevice, st));
        }
        hf_flag = ctx->d_hf_flag.p;
        hf_first = ctx->d_hf_first.p;
        B.tl_key = ctx->d_tl_key.p;
        B.tl_dgram = ctx->d_tl_dgram.p;
        B.tl_slot = ctx->d_tl_slot.p;
        B.tl_n = (uint32_t)hf->tl.key.size();
        B.hf_first = hf_first;
        B.hf_hdr = ctx->d_hf_hdr.p;
        B.hf_sets = ctx->d_hf_sets.p;
    }
    B.bytes = in->bytes;
    B.bytes_size = in->bytes_size;
    B.offsets = in->offsets;
    B.lengths = in->lengths;
    B.n = N;
    B.n_slots = S;
    B.slot_row = ctx->d_slot_row.p;
    B.n_rows = A;
    static const bool trace_on = ngz_knob("NGZ_TRACE", 0) != 0;
    if (trace_on) {
        const uint64_t n = 2ull * NGZ_TRACE_WINDOWS * std::max<uint32_t>(S, 1);
        if (ctx->d_trace.ensure(n)) return fail(ctx, NGZ_E_NOMEM, "trace buffer");
        HIPCHK(hipMemsetAsync(ctx->d_trace.p, 0, n * 8, st));
        B.trace = ctx->d_trace.p;
    }
    B.plans = ctx->d_plans.p;
    B.cur_slot = ctx->d_cur_slot.p;
    B.hdr = ctx->d_hdr.p;
    B.counts = ctx->d_counts.p;
    B.scan = ctx->d_scan.p;
    B.slots = ctx->d_slots.p;
    B.chunks = ctx->d_chunks.p;
    B.chunk_cap = ctx->d_chunks.cap;
    B.sets = ctx->d_sets.p;
    B.set_cap = ctx->d_sets.cap;
    B.arena = ctx->d_arena.p + ctx->arena_shift;
    B.arena_cap = ctx->d_arena.cap - ctx->arena_shift;
    B.proc_counts = d_proc;
    B.cap_pad_windows = ctx->cap_pad_windows;
    B.recmap = nullptr;
    B.dsum = nullptr;
    static const bool dsum_on = ngz_knob("NGZ_DSUM", 1) != 0;
    if (dsum_on && N) {
        if (ctx->d_dsum.ensure(N)) return fail(ctx, NGZ_E_NOMEM, "device alloc (datagram summaries)");
        B.dsum = ctx->d_dsum.p;
    }
    B.recoff = nullptr;
    B.recoff_div = 0;
    B.split = 0;
    if (any_vlen && recmap_env != 0) {
        if (lists) {
            if (ctx->d_recoff.ensure(in->bytes_size / min_vlen_rec + 8ull * N + 16))
                return fail(ctx, NGZ_E_NOMEM, "device alloc (record offsets)");
            B.recoff = ctx->d_recoff.p;
            B.recoff_div = min_vlen_rec;
        } else {
            if (ctx->d_recmap.ensure(in->bytes_size / 32 + 8)) return fail(ctx, NGZ_E_NOMEM, "device alloc (record map)");
            B.recmap = ctx->d_recmap.p;
        }
    }
    B.summary = d_sum;
    // split framing: phase B has its own count matrix, scan and rows and writes the record-offset
    // lists; phase A defers the variable-length sets
    BatchDev B2 = B;
    if (split) {
        B2.split = 2;
        B2.counts = ctx->d_counts2.p;
        B2.scan = ctx->d_scan2.p;
        B2.slot_row = ctx->d_slot_row2.p;
        B2.n_rows = A2;
        B2.dsum = nullptr;
        B.split = 1;
        B.recoff = nullptr;
    }

    HIPCHK(hipEventRecord(ctx->ev[0], st));
    // k_frame zeroes the count matrix itself; the summary and increments of
    // this parity were zeroed by the previous batch's k_export
    if (!N) HIPCHK(hipMemsetAsync(ctx->d_counts.p, 0, n_items * 4, st));
    if (B.recmap) HIPCHK(hipMemsetAsync(B.recmap, 0, (in->bytes_size / 32 + 8) * 4, st));
    if (!ctx->clean[par]) {
        HIPCHK(hipMemsetAsync(d_sum, 0, sizeof(BatchSummary), st));
        HIPCHK(hipMemsetAsync(d_proc, 0, NGZ_MAX_SLOTS * 8, st));
    }
    ctx->clean[par] = false;
    BatchSummary *next_sum = ctx->d_summary.p + (par ^ 1);
    unsigned long long *next_proc = ctx->d_proc.p + (size_t)(par ^ 1) * NGZ_MAX_SLOTS;
    auto export_results = [&]() -> int {
        const unsigned long long seq = ++ctx->export_seq;
        if (ngz_launch_export(&B, ctx->dh_summary, ctx->dh_slots, ctx->dh_proc, next_sum, next_proc, ctx->dh_done,
                              seq, st))
            return fail(ctx, NGZ_E_DEVICE, "export launch");
        // spin on the completion word (the export is the stream's last command);
        // a stream synchronisation covers errors and very long batches
        bool done = false;
        if (ctx->spin_wait) {
            const auto t0 = std::chrono::steady_clock::now();
            for (uint32_t k = 0;; ++k) {
                if (__atomic_load_n(ctx->h_done, __ATOMIC_ACQUIRE) == seq) { done = true; break; }
                if ((k & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) break;
                __builtin_ia32_pause();
            }
        }
        if (!done) HIPCHK(hipStreamSynchronize(st));
        ctx->clean[par ^ 1] = true;
        return 0;
    };
    const hipStream_t ss = split ? ctx->split_stream : st;
    if (split) {
        // phase B starts with the batch (the summary zeroed, the plans uploaded)
        HIPCHK(hipEventRecord(ctx->split_ev[0], st));
        HIPCHK(hipStreamWaitEvent(ss, ctx->split_ev[0], 0));
        if (ngz_launch_frame_vlen(&B2, ss)) return fail(ctx, NGZ_E_DEVICE, "k_frame_vlen launch");
        if (ngz_launch_scan(ctx->d_scan_tmp2.p, scan_tmp2, ctx->d_counts2.p, ctx->d_scan2.p, n_items2, ss))
            return fail(ctx, NGZ_E_DEVICE, "scan launch (phase B)");
    }
    if (ngz_launch_frame(&B, hf_flag, hf_first, st)) return fail(ctx, NGZ_E_DEVICE, "k_frame launch");
    if (ngz_launch_scan(ctx->d_scan_tmp.p, scan_tmp, ctx->d_counts.p, ctx->d_scan.p, n_items, st))
        return fail(ctx, NGZ_E_DEVICE, "scan launch");
    if (!split) {
        if (ngz_launch_layout_emit(&B, hf_flag, hf_first, st)) return fail(ctx, NGZ_E_DEVICE, "layout/emit launch");
    } else {
        // phase B lays its templates out after phase A's (and reads phase A's headers in k_emit)
        if (ngz_launch_layout(&B, st)) return fail(ctx, NGZ_E_DEVICE, "layout launch");
        HIPCHK(hipEventRecord(ctx->split_ev[1], st));
        if (ngz_launch_emit(&B, st)) return fail(ctx, NGZ_E_DEVICE, "emit launch");
        HIPCHK(hipStreamWaitEvent(ss, ctx->split_ev[1], 0));
        if (ngz_launch_layout(&B2, ss) || ngz_launch_emit(&B2, ss)) return fail(ctx, NGZ_E_DEVICE, "layout/emit launch (phase B)");
    }
    // Decode launches.  The record counts per slot are known on the device
    // only; reading them back costs a host round trip in the middle of the
    // pipeline.  In steady state (same slots as the previous batch) the
    // decode kernels of the slots that had records last time are launched
    // right away, with grid-strided geometry that needs no counts, and the
    // counts are checked after the final synchronisation: a slot that gained
    // records is decoded then, and processed counts / statuses are redone.
    const uint32_t grid = (uint32_t)ctx->n_cus * ctx->blocks_per_cu;  // 256-thread blocks
    const bool predict = ctx->pred_valid && ctx->pred_versions == ctx->slot_version && !hf;
    if (predict) ctx->batch_info |= NGZ_BATCH_PREDICTED;
    else ctx->batch_info &= ~(uint32_t)NGZ_BATCH_PREDICTED;
    // launch the decode of slot s (rt: its counts when known)
    auto launch_slot = [&](uint32_t s, const SlotRT *rt, bool &generic, hipStream_t ls) -> int {
        const Version &v = ctx->versions[ctx->slot_version[s]];
        if (!v.plan.rpl) return 0;
        if (ctx->specialize && v.rtc_state == 1) {
            // one specialised kernel per active template, over that slot's chunks only
            uint32_t g, block = 256;
            if (v.plan.lds_waves) {
                // one workgroup per window of 256*lds_waves rows (grid-strided)
                const uint32_t rows = NGZ_REG_WINDOW * v.plan.lds_waves;
                g = (uint32_t)ctx->n_cus * ctx->lds_blocks_per_cu;
                if (rt) g = std::min<uint32_t>(g, (rt->total + rows - 1) / rows);
                block = 64 * v.plan.lds_waves;
            } else {
                g = grid;
                if (rt) {
                    const uint32_t units =
                        rt->mode == NGZ_MODE_ROW ? (rt->total + NGZ_REG_WINDOW - 1) / NGZ_REG_WINDOW : rt->nchunks;
                    g = std::min<uint32_t>(grid, (units + 3) / 4);
                }
            }
            if (g && ngz_rtc_launch(v.rtc_fn, split && is_v[s] ? &B2 : &B, s, g, block, split && is_v[s] ? ss : ls))
                return fail(ctx, NGZ_E_DEVICE, "specialised decode launch");
        } else {
            generic = true;
        }
        return 0;
    };
    auto check_summary = [&]() -> int {
        ctx->summary = *ctx->h_summary;
        if (ctx->summary.overflow) {
            if (ctx->summary.overflow & 8) ctx->rows_all = true;  // a slot without a count row had a set
            if (ctx->summary.overflow & 16) ctx->split_skip = 64;  // a record error phase A went past
            if (ctx->summary.overflow & 1) ctx->d_arena.ensure(ctx->summary.arena_used + 4096);
            if (ctx->summary.overflow & 2) ctx->d_chunks.ensure(ctx->summary.n_chunks + 1024);
            if (ctx->summary.overflow & 4) ctx->d_sets.ensure(ctx->summary.n_sets + 1024);
            ctx->pred_valid = false;
            return 1;  // retry
        }
        return 0;
    };
    std::vector<uint8_t> launched(S, 0);
    bool generic = false;
    if (!predict) {
        // the kernels that run depend on the per-slot counts: read them first
        HIPCHK(hipMemcpyAsync(ctx->h_summary, d_sum, sizeof(BatchSummary), hipMemcpyDeviceToHost, st));
        if (S) HIPCHK(hipMemcpyAsync(ctx->h_slots, ctx->d_slots.p, S * sizeof(SlotRT), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        const int r = check_summary();
        if (r) return r;
    }
    HIPCHK(hipEventRecord(ctx->ev[1], st));
    std::vector<std::pair<uint32_t, const SlotRT *>> todo;
    for (uint32_t s = 0; s < S; ++s) {
        if (predict) {
            if (!ctx->pred_active[s]) continue;
            todo.push_back({s, nullptr});
        } else {
            const SlotRT &rt = ctx->h_slots[s];
            if (!rt.total || (rt.mode == NGZ_MODE_CHUNK && !rt.nchunks)) continue;
            todo.push_back({s, &rt});
        }
        launched[s] = 1;
    }
    // Several LDS-staged specialised templates of one workgroup shape: one
    // multi-template launch deals all their windows over the grid (one ramp and
    // one tail for the batch instead of one per template).  Its kernel compiles
    // like a template's (in the background unless NGZ_OPT_RTC_SYNC); until it is
    // ready the templates launch one by one.
    if (ctx->group_launch && ctx->specialize && todo.size() >= 2) {
        std::map<uint32_t, std::vector<uint32_t>> by_lw;
        for (const auto &t : todo) {
            const Version &v = ctx->versions[ctx->slot_version[t.first]];
            if (v.rtc_state == 1 && v.plan.lds_waves && !v.plan.has_vlen) by_lw[v.plan.lds_waves].push_back(t.first);
        }
        for (auto &kv : by_lw) {
            std::vector<uint32_t> &sl = kv.second;
            if (sl.size() < 2) continue;
            if (sl.size() > NGZ_RTC_GROUP_MAX) sl.resize(NGZ_RTC_GROUP_MAX);
            std::vector<int32_t> key;
            std::vector<const DevPlan *> pp;
            for (uint32_t s : sl) {
                key.push_back(ctx->slot_version[s]);
                pp.push_back(&ctx->versions[ctx->slot_version[s]].plan);
            }
            ngz_ctx::GroupKernel &gk = ctx->group_kernels[key];
            if (gk.state == 0) {
                if (ctx->rtc_sync) {
                    gk.fn = ngz_rtc_group(ctx->device, pp.data(), (uint32_t)pp.size());
                    gk.state = gk.fn ? 1 : 2;
                } else {
                    const int r = ngz_rtc_group_async(ctx->device, pp.data(), (uint32_t)pp.size(), &gk.fn, &gk.entry);
                    gk.state = r == 1 ? 1 : r < 0 ? 2 : 3;
                }
            } else if (gk.state == 3) {
                const int r = ngz_rtc_poll(gk.entry, &gk.fn);
                if (r) gk.state = r > 0 ? 1 : 2;
            }
            if (gk.state != 1) continue;
            const uint32_t g = (uint32_t)ctx->n_cus * ctx->lds_blocks_per_cu;
            if (ngz_rtc_launch_group(gk.fn, &B, sl.data(), (uint32_t)sl.size(), g, 64 * kv.first, st))
                return fail(ctx, NGZ_E_DEVICE, "multi-template decode launch");
            std::set<uint32_t> done(sl.begin(), sl.end());
            todo.erase(std::remove_if(todo.begin(), todo.end(), [&](const auto &t) { return done.count(t.first) != 0; }),
                       todo.end());
        }
    }
    // several active templates: their kernels run side by side on the context's
    // auxiliary streams (fork/join with events), so one kernel's tail overlaps
    // the next one's start instead of draining the GPU between templates
    const uint32_t n_aux = todo.size() >= 2 && !split ? std::min<uint32_t>(ctx->n_aux, (uint32_t)todo.size() - 1) : 0;
    if (n_aux) {
        HIPCHK(hipEventRecord(ctx->fork_ev, st));
        for (uint32_t i = 0; i < n_aux; ++i) HIPCHK(hipStreamWaitEvent(ctx->aux[i], ctx->fork_ev, 0));
    }
    for (size_t k = 0; k < todo.size(); ++k) {
        const hipStream_t ls = (n_aux && k > 0) ? ctx->aux[(k - 1) % n_aux] : st;
        if (launch_slot(todo[k].first, todo[k].second, generic, ls)) return -1;
    }
    if (generic && ngz_launch_decode_generic(&B, grid, st)) return fail(ctx, NGZ_E_DEVICE, "decode launch");
    if (split) {  // join phase B before the counts
        HIPCHK(hipEventRecord(ctx->split_ev[2], ss));
        HIPCHK(hipStreamWaitEvent(st, ctx->split_ev[2], 0));
    }
    for (uint32_t i = 0; i < n_aux; ++i) {
        HIPCHK(hipEventRecord(ctx->join_ev[i], ctx->aux[i]));
        HIPCHK(hipStreamWaitEvent(st, ctx->join_ev[i], 0));
    }
    HIPCHK(hipEventRecord(ctx->ev[2], st));
    if (ngz_launch_counts(&B, ctx->d_sets.cap, st)) return fail(ctx, NGZ_E_DEVICE, "counts launch");
    HIPCHK(hipEventRecord(ctx->ev[3], st));
    // summary, slot table and processed_count increments straight into pinned memory, one synchronisation
    int rc = export_results();
    if (rc) return rc;
    if (predict) {
        const int r = check_summary();
        if (r) return r;
        // slots that gained records since the last batch
        bool missed = false, generic2 = false;
        for (uint32_t s = 0; s < S; ++s) {
            const SlotRT &rt = ctx->h_slots[s];
            if (launched[s] || !rt.total || (rt.mode == NGZ_MODE_CHUNK && !rt.nchunks)) continue;
            missed = true;
            const Version &v = ctx->versions[ctx->slot_version[s]];
            const bool spec = ctx->specialize && v.rtc_state == 1;
            if (!spec && generic) continue;  // the generic kernel walked every non-specialised slot
            if (launch_slot(s, &rt, generic2, st)) return -1;
            launched[s] = 1;
        }
        if (missed) {
            if (generic2 && ngz_launch_decode_generic(&B, grid, st)) return fail(ctx, NGZ_E_DEVICE, "decode launch");
            HIPCHK(hipMemsetAsync(d_proc, 0, NGZ_MAX_SLOTS * 8, st));
            if (ngz_launch_counts(&B, ctx->d_sets.cap, st)) return fail(ctx, NGZ_E_DEVICE, "counts launch");
            HIPCHK(hipEventRecord(ctx->ev[3], st));
            rc = export_results();
            if (rc) return rc;
        }
    }
    if (B.trace) trace_report(ctx, S, st);
    ctx->parity ^= 1;
    // slots with records this batch: launched without a round trip next time
    ctx->pred_versions = ctx->slot_version;
    ctx->pred_active.assign(S, 0);
    for (uint32_t s = 0; s < S; ++s) {
        const SlotRT &rt = ctx->h_slots[s];
        ctx->pred_active[s] = rt.total && !(rt.mode == NGZ_MODE_CHUNK && !rt.nchunks);
    }
    ctx->pred_valid = !hf;
    ctx->rows_all = false;
    hipEventElapsedTime(&ctx->t_decode, ctx->ev[1], ctx->ev[2]);
    hipEventElapsedTime(&ctx->t_pipeline, ctx->ev[0], ctx->ev[3]);
    return 0;
}

// NGZ_TRACE: per slot, the windows' start / end clocks (100 MHz) summarised on stderr: the launch
// span, the mean window time in each tenth of it, and the windows finished per tenth
static void trace_report(ngz_ctx *ctx, uint32_t S, hipStream_t st) {
    if (hipStreamSynchronize(st) != hipSuccess) return;
    std::vector<unsigned long long> t(2ull * NGZ_TRACE_WINDOWS * S);
    if (hipMemcpy(t.data(), ctx->d_trace.p, t.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    for (uint32_t s = 0; s < S; ++s) {
        const unsigned long long *w = t.data() + 2ull * NGZ_TRACE_WINDOWS * s;
        unsigned long long lo = ~0ull, hi = 0;
        uint32_t n = 0;
        for (uint32_t i = 0; i < NGZ_TRACE_WINDOWS; ++i)
            if (w[2 * i + 1]) {
                lo = std::min(lo, w[2 * i]);
                hi = std::max(hi, w[2 * i + 1]);
                ++n;
            }
        if (!n || hi <= lo) continue;
        double sum[10] = {}, cnt[10] = {}, fin[10] = {};
        for (uint32_t i = 0; i < NGZ_TRACE_WINDOWS; ++i)
            if (w[2 * i + 1]) {
                const int b0 = (int)std::min<unsigned long long>(9, (w[2 * i] - lo) * 10 / (hi - lo));
                const int b1 = (int)std::min<unsigned long long>(9, (w[2 * i + 1] - lo) * 10 / (hi - lo));
                sum[b0] += (double)(w[2 * i + 1] - w[2 * i]) * 0.01;
                cnt[b0] += 1;
                fin[b1] += 1;
            }
        fprintf(stderr, "[ngz] trace slot %u: %u windows over %.1f us; mean window us by start tenth:", s, n,
                (double)(hi - lo) * 0.01);
        for (int b = 0; b < 10; ++b) fprintf(stderr, " %.1f", cnt[b] ? sum[b] / cnt[b] : 0.0);
        fprintf(stderr, "; finished per tenth:");
        for (int b = 0; b < 10; ++b) fprintf(stderr, " %.0f", fin[b]);
        fprintf(stderr, "\n");
    }
}

// Arena placement.  The decode kernel's speed depends on where in HBM the
// column arena was allocated: on MI355X some allocations run the same decode
// up to 15 % slower than others, stably for the allocation's lifetime and
// independent of offsets inside it (tools/arena_shift.py, tools/cap_pad.py,
// tools/alloc_var3.py).  The first large device batch of a
// context is therefore decoded on up to NGZ_PLACE_TRIALS fresh arenas (each
// kept while the next is allocated, so every trial gets other memory); the
// fastest is kept and the batch's results are the ones decoded on it.
// The probe of one arena (k_place_probe over every slot with records, the first frac16 sixteenths of
// each XCD's windows): device milliseconds.  Overwrites the columns of that arena.
float place_probe(ngz_ctx *ctx, const ngz_batch_in *in, hipStream_t st, uint32_t frac16) {
    const uint32_t S = (uint32_t)ctx->slot_version.size();
    const uint32_t grid = ctx->lds_blocks_per_cu * (uint32_t)ctx->n_cus;
    HIPCHK(hipEventRecord(ctx->ev[0], st));
    for (uint32_t s = 0; s < S; ++s) {
        const SlotRT &rt = ctx->h_slots[s];
        if (!rt.total) continue;
        const Version &v = ctx->versions[ctx->slot_version[s]];
        std::vector<uint32_t> w, off;
        for (uint32_t f = 0; f < v.plan.n_fields && f < 32; ++f) {
            w.push_back(v.plan.f[f].width);
            off.push_back(v.plan.f[f].col_off);
        }
        if (ngz_launch_place_probe(in->bytes, in->bytes_size, ctx->d_arena.p + ctx->arena_shift + rt.block, rt.cap,
                                   rt.total, std::max<uint32_t>(v.plan.rec_len, 16), frac16, w.data(), off.data(),
                                   (uint32_t)w.size(), grid, st))
            return -1.f;
    }
    HIPCHK(hipEventRecord(ctx->ev[1], st));
    HIPCHK(hipEventSynchronize(ctx->ev[1]));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]));
    return ms;
}

int place_arena(ngz_ctx *ctx, const ngz_batch_in *in, hipStream_t st) {
    if (ctx->placed || ctx->place_trials <= 1) return 0;
    if (ctx->t_decode < 0.25f) return 0;  // small batches: launch-bound, placement does not show; try the next
    ctx->placed = true;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) return 0;
    const size_t cap = ctx->d_arena.cap;
    const int trials = (int)std::min<size_t>((size_t)ctx->place_trials, free_b / std::max<size_t>(cap, 1) / 2 + 1);
    // NGZ_OPT_PLACE_PROBE: 0 every trial decodes the batch; 1 every trial runs the probe (a fraction
    // of the decode's memory traffic) and only the kept arena decodes; 2 (diagnostics) both, the
    // decodes decide
    const int mode = ctx->place_probe;
    const uint32_t frac16 = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(16, ngz_knob("NGZ_PLACE_PROBE_FRAC", 2)));
    std::vector<DevBuf<uint8_t>> arenas{ctx->d_arena};
    std::vector<float> ms{ctx->t_decode}, pms;
    auto redo = [&]() {
        int rc;
        for (int tries = 0; (rc = run_pipeline(ctx, in, st, nullptr)) == 1 && tries < 4; ++tries) {}
        return rc;
    };
    if (mode) pms.push_back(place_probe(ctx, in, st, frac16));  // (arena 0's columns are rewritten below)
    for (int k = 1; k < trials; ++k) {
        DevBuf<uint8_t> a;
        if (a.ensure(cap)) break;  // out of room: keep what was tried
        ctx->d_arena = a;
        if (mode) pms.push_back(place_probe(ctx, in, st, frac16));
        int rc = mode == 1 ? 0 : redo();
        arenas.push_back(ctx->d_arena);  // (a retry may have regrown it)
        if (rc) {
            ctx->d_arena = arenas[0];
            for (size_t i = 1; i < arenas.size(); ++i) arenas[i].release();
            return rc < 0 ? rc : fail(ctx, NGZ_E_NOMEM, "batch buffers kept overflowing");
        }
        if (mode != 1) ms.push_back(ctx->t_decode);
    }
    const std::vector<float> &by = mode == 1 ? pms : ms;
    const size_t best = (size_t)(std::min_element(by.begin(), by.end()) - by.begin());
    ctx->place_ms = mode == 1 ? std::vector<float>() : ms;
    ctx->place_probe_ms = pms;
    ctx->place_kept = (uint32_t)best;
    if (ngz_debug()) {
        fprintf(stderr, "[ngz] arena placement (probe mode %d, %u/16):", mode, frac16);
        for (size_t i = 0; i < by.size(); ++i)
            fprintf(stderr, " %.3f/%.3f", i < ms.size() ? ms[i] : 0.f, i < pms.size() ? pms[i] : 0.f);
        fprintf(stderr, " ms -> %zu\n", best);
    }
    ctx->d_arena = arenas[best];
    for (size_t i = 0; i < arenas.size(); ++i)
        if (i != best) arenas[i].release();
    if (mode != 1) ctx->t_decode = ms[best];
    // Every trial decoded the batch into its own arena (its columns and row tables; the headers, sets,
    // chunks and counts outside the arena are the same for every trial), so the kept arena already
    // holds this batch's results -- unless the probe ran over it after its decode (every arena in
    // mode 1; arena 0, decoded before the trials, in mode 2): decode it there once more
    if (mode == 1 || (mode == 2 && best == 0)) {
        int rc;
        for (int tries = 0; (rc = run_pipeline(ctx, in, st, nullptr)) == 1 && tries < 4; ++tries) {}
        if (rc) return rc < 0 ? rc : fail(ctx, NGZ_E_NOMEM, "batch buffers kept overflowing");
    }
    return 0;
}

int finish_batch(ngz_ctx *ctx, const ngz_batch_in *in, ngz_batch_out *out, hipStream_t st) {
    const uint32_t S = (uint32_t)ctx->slot_version.size();
    (void)st;
    // run_pipeline left the slot table and the processed_count increments in pinned memory
    ctx->slot_rt.assign(ctx->h_slots, ctx->h_slots + S);
    std::vector<unsigned long long> proc(ctx->h_proc, ctx->h_proc + S);
    ctx->slot_infos.resize(S);
    for (uint32_t s = 0; s < S; ++s) {
        Version &v = ctx->versions[ctx->slot_version[s]];
        // re-announced in this batch: the count restarted there (k_counts counted only later sets)
        v.processed = (ctx->count_from.count(ctx->slot_version[s]) ? 0 : v.processed) + proc[s];
        v.seen_records += ctx->slot_rt[s].total;
        if (ctx->specialize == 2 && v.rtc_state == 0 && v.seen_records >= NGZ_SPECIALIZE_MIN_RECORDS)
            ctx->plans_dirty = true;  // the next batch compiles its kernel
        ngz_slot_info &si = ctx->slot_infos[s];
        si.version_id = (uint32_t)ctx->slot_version[s];
        si.template_id = v.tid;
        si.proto = v.proto;
        si.n_fields = (uint32_t)v.specs.size();
        si.reserved = 0;
        si.reserved2 = 0;
        si.n_records = ctx->slot_rt[s].total;
        si.capacity = ctx->slot_rt[s].cap;
        si.columns = ctx->d_arena.p + ctx->arena_shift + ctx->slot_rt[s].block;
    }
    out->n_dgrams = in->n;
    out->n_sets = ctx->summary.n_sets;
    out->n_slots = S;
    out->n_records = ctx->summary.n_records_total;
    out->dgrams = ctx->d_hdr.p;
    out->sets = ctx->d_sets.p;
    out->slots = ctx->slot_infos.data();
    out->n_template_dgrams = ctx->n_template_dgrams;
    ctx->last_in = *in;
    return 0;
}

}  // namespace

// ------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------
extern "C" {

int ngz_abi_version(void) { return NGZ_ABI_VERSION; }

int ngz_ctx_create(int device, ngz_ctx **out) {
    if (!out) return NGZ_E_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return NGZ_E_DEVICE;
    if (hipSetDevice(device) != hipSuccess) return NGZ_E_DEVICE;
    ngz_ctx *ctx = new ngz_ctx();
    ctx->device = device;
    ctx->cur[0].assign(65536, -1);
    ctx->cur[1].assign(65536, -1);
    if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return NGZ_E_DEVICE;
    }
    for (auto &e : ctx->ev) hipEventCreate(&e);
    if (const int64_t e = ngz_knob("NGZ_DECODE_STREAMS", 0)) ctx->n_aux = (uint32_t)std::max<int64_t>(0, std::min<int64_t>(NGZ_MAX_AUX, e - 1));
    for (uint32_t i = 0; i < ctx->n_aux; ++i) {
        if (hipStreamCreateWithFlags(&ctx->aux[i], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&ctx->join_ev[i], hipEventDisableTiming) != hipSuccess) {
            ctx->n_aux = i;
            break;
        }
    }
    hipEventCreateWithFlags(&ctx->fork_ev, hipEventDisableTiming);
    hipDeviceGetAttribute(&ctx->n_cus, hipDeviceAttributeMultiprocessorCount, device);
    // fine-grained (coherent) pinned memory: k_export writes it directly
    const unsigned hf = hipHostMallocCoherent | hipHostMallocMapped;
    if (hipHostMalloc((void **)&ctx->h_summary, sizeof(BatchSummary), hf) != hipSuccess ||
        hipHostMalloc((void **)&ctx->h_slots, NGZ_MAX_SLOTS * sizeof(SlotRT), hf) != hipSuccess ||
        hipHostMalloc((void **)&ctx->h_proc, NGZ_MAX_SLOTS * sizeof(unsigned long long), hf) != hipSuccess ||
        hipHostGetDevicePointer((void **)&ctx->dh_summary, ctx->h_summary, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&ctx->dh_slots, ctx->h_slots, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&ctx->dh_proc, ctx->h_proc, 0) != hipSuccess ||
        hipHostMalloc((void **)&ctx->h_done, 64, hf) != hipSuccess ||
        hipHostGetDevicePointer((void **)&ctx->dh_done, ctx->h_done, 0) != hipSuccess) {
        ngz_ctx_destroy(ctx);
        return NGZ_E_NOMEM;
    }
    // defaults; hosts choose through ngz_ctx_set_option (experiment builds also read NGZ_<name>)
    ctx->specialize = (int)ngz_knob("NGZ_SPECIALIZE", ctx->specialize);
    ctx->spin_wait = ngz_knob("NGZ_SPIN", ctx->spin_wait) != 0;
    ctx->d_arena.contiguous = ngz_knob("NGZ_ARENA_CONTIG", ctx->d_arena.contiguous) != 0;
    ctx->place_trials = (int)ngz_knob("NGZ_PLACE_TRIALS", ctx->place_trials);
    ctx->cap_pad_windows = (uint32_t)std::max<int64_t>(0, std::min<int64_t>(200000, ngz_knob("NGZ_CAP_PAD", ctx->cap_pad_windows)));
    *ctx->h_done = 0;
    ctx->blocks_per_cu = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(32, ngz_knob("NGZ_BLOCKS_PER_CU", ctx->blocks_per_cu)));
    ctx->lds_blocks_per_cu = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(512, ngz_knob("NGZ_LDS_BLOCKS_PER_CU", ctx->lds_blocks_per_cu)));
    ctx->group_launch = ngz_knob("NGZ_GROUP", ctx->group_launch) != 0;
    *out = ctx;
    return NGZ_OK;
}

void ngz_ctx_destroy(ngz_ctx *ctx) {
    if (!ctx) return;
    if (ctx->async.th.joinable()) {  // the decode worker finishes a submitted batch, then exits
        {
            std::lock_guard<std::mutex> lk(ctx->async.m);
            ctx->async.stop = true;
        }
        ctx->async.cv.notify_all();
        ctx->async.th.join();
    }
    {
        // Synchronous drop, as the reference codec's (codec.rs:68-82): no kernel compile this context
        // started or waits on is still running once it returns, so a C / Rust host may return from main
        // right after (a compile inside hiprtc/comgr during exit can hang it, ngz_rtc.cpp Workers)
        std::vector<void *> entries;
        for (const ngzh::Version &v : ctx->versions)
            if (v.rtc_entry) entries.push_back(v.rtc_entry);
        for (const auto &kv : ctx->group_kernels)
            if (kv.second.entry) entries.push_back(kv.second.entry);
        ngz_rtc_join(entries.data(), entries.size());
    }
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    if (ctx->d2h_ev) {
        hipEventSynchronize(ctx->d2h_ev);
        hipEventDestroy(ctx->d2h_ev);
    }
    ctx->d_plans.release(); ctx->d_fields.release(); ctx->d_cur_slot.release(); ctx->d_tl_key.release(); ctx->d_tl_dgram.release();
    ctx->d_tl_slot.release(); ctx->d_hf_flag.release(); ctx->d_hf_hdr.release(); ctx->d_hf_first.release(); ctx->d_hf_sets.release();
    ctx->d_hdr.release(); ctx->d_counts.release(); ctx->d_scan.release(); ctx->d_scan_tmp.release();
    ctx->d_slots.release(); ctx->d_chunks.release(); ctx->d_sets.release(); ctx->d_arena.release();
    ctx->d_proc.release(); ctx->d_summary.release(); ctx->d_recmap.release(); ctx->d_recoff.release(); ctx->d_dsum.release(); ctx->d_slot_row.release(); ctx->d_in_bytes.release(); ctx->d_in_off.release();
    ctx->d_in_len.release();
    ctx->d_trace.release();
    ctx->d_counts2.release(); ctx->d_scan2.release(); ctx->d_scan_tmp2.release(); ctx->d_slot_row2.release();
    if (ctx->split_stream) {
        hipStreamSynchronize(ctx->split_stream);
        hipStreamDestroy(ctx->split_stream);
    }
    for (auto &e : ctx->split_ev)
        if (e) hipEventDestroy(e);
    for (auto &e : ctx->ev) hipEventDestroy(e);
    for (uint32_t i = 0; i < ctx->n_aux; ++i) {
        hipStreamSynchronize(ctx->aux[i]);
        hipStreamDestroy(ctx->aux[i]);
        hipEventDestroy(ctx->join_ev[i]);
    }
    if (ctx->fork_ev) hipEventDestroy(ctx->fork_ev);
    if (ctx->h_summary) hipHostFree(ctx->h_summary);
    if (ctx->h_slots) hipHostFree(ctx->h_slots);
    if (ctx->h_proc) hipHostFree(ctx->h_proc);
    if (ctx->h_done) hipHostFree(ctx->h_done);
    for (int i = 0; i < ngz_ctx::COUNTS_RING; ++i) {
        if (ctx->counts_ev[i]) { hipEventSynchronize(ctx->counts_ev[i]); hipEventDestroy(ctx->counts_ev[i]); }
        if (ctx->h_counts_stage[i]) hipHostFree(ctx->h_counts_stage[i]);
    }
    hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char *ngz_last_error(ngz_ctx *ctx) { return ctx ? ctx->last_error.c_str() : "null context"; }

int ngz_ctx_set_option(ngz_ctx *ctx, int opt, int64_t value) {
    if (!ctx) return NGZ_E_INVALID;
    switch (opt) {
    case NGZ_OPT_SPECIALIZE:
        if (value < 0 || value > 2) return fail(ctx, NGZ_E_INVALID, "NGZ_OPT_SPECIALIZE takes 0, 1 or 2");
        if (ctx->specialize != (int)value) ctx->plans_dirty = true;  // device plans carry the spec flag
        ctx->specialize = (int)value;
        return NGZ_OK;
    case NGZ_OPT_ARENA_SHIFT:
        if (value < 0 || value > (1ll << 32) || value % 256) return fail(ctx, NGZ_E_INVALID, "NGZ_OPT_ARENA_SHIFT: 0..4 GiB, 256-byte multiple");
        ctx->arena_shift = (uint64_t)value;
        return NGZ_OK;
    case NGZ_OPT_CAP_PAD:
        if (value < 0 || value > 4096) return fail(ctx, NGZ_E_INVALID, "NGZ_OPT_CAP_PAD takes 0..4096");
        ctx->cap_pad_windows = (uint32_t)value;
        return NGZ_OK;
    case NGZ_OPT_RTC_SYNC:
        if (value < 0 || value > 1) return fail(ctx, NGZ_E_INVALID, "NGZ_OPT_RTC_SYNC takes 0 or 1");
        ctx->rtc_sync = value != 0;
        return NGZ_OK;
    case NGZ_OPT_BLOCKS_PER_CU:
        if (value < 1 || value > 32) return fail(ctx, NGZ_E_INVALID, "NGZ_OPT_BLOCKS_PER_CU takes 1..32");
        ctx->blocks_per_cu = (uint32_t)value;
        return NGZ_OK;
    case NGZ_OPT_SPLIT:
        if (value < 0 || value > 1) return fail(ctx, NGZ_E_INVALID, "NGZ_OPT_SPLIT takes 0 or 1");
        ctx->split_framing = (int)value;
        return NGZ_OK;
    case NGZ_OPT_GROUP:
        if (value < 0 || value > 1) return fail(ctx, NGZ_E_INVALID, "NGZ_OPT_GROUP takes 0 or 1");
        ctx->group_launch = value != 0;
        return NGZ_OK;
    case NGZ_OPT_PLACE_TRIALS:
        if (value < 1 || value > 16) return fail(ctx, NGZ_E_INVALID, "NGZ_OPT_PLACE_TRIALS takes 1..16");
        ctx->place_trials = (int)value;
        return NGZ_OK;
    case NGZ_OPT_PLACE_PROBE:
        if (value < 0 || value > 2) return fail(ctx, NGZ_E_INVALID, "NGZ_OPT_PLACE_PROBE takes 0, 1 or 2");
        ctx->place_probe = (int)value;
        return NGZ_OK;
    }
    return fail(ctx, NGZ_E_INVALID, "unknown option");
}

static int wait_d2h(ngz_ctx *ctx);

int ngz_decode_batch(ngz_ctx *ctx, const ngz_batch_in *in, ngz_batch_out *out, void *hip_stream) {
    if (!ctx || !in || !out) return NGZ_E_INVALID;
    if (ctx->async.pending.load() && std::this_thread::get_id() != ctx->async.th.get_id())
        return NGZ_E_INVALID;  // (no message: the worker may be writing the context's error text)
    if (in->n && (!in->bytes || !in->offsets || !in->lengths)) return fail(ctx, NGZ_E_INVALID, "null batch arrays");
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : ctx->stream;
    if (wait_d2h(ctx)) return NGZ_E_DEVICE;
    ctx->host_errors.clear();
    ctx->tmpl_sets.clear();
    ctx->batch_serial++;
    ctx->json_view.reset();
    ctx->batch_info = 0;
    ctx->pipeline_runs = 0;
    if (!ctx->count_from.empty()) {  // the last batch's restarts are in its counts already
        ctx->count_from.clear();
        ctx->plans_dirty = true;
    }
    memset(out, 0, sizeof *out);
    int rc = ctx->assigned_gen == ctx->tmpl_gen ? 0 : assign_slots(ctx, {});
    if (rc) return rc;
    // templates whose kernel was compiling: switch to it once it is ready
    for (int32_t vid : ctx->slot_version) {
        Version &v = ctx->versions[vid];
        if (v.rtc_state != 3 || !v.rtc_entry) continue;
        const int r = ngz_rtc_poll(v.rtc_entry, &v.rtc_fn);
        if (r != 0) {
            v.rtc_state = r > 0 ? 1 : 2;
            ctx->plans_dirty = true;
        }
    }
    if (ctx->plans_dirty || ctx->uploaded_gen != ctx->tmpl_gen) {
        rc = upload_slots(ctx, ctx->cur, st);
        if (rc) return rc;
        ctx->uploaded_gen = ctx->tmpl_gen;
    }
    // fast path: no template sets expected
    for (int tries = 0; (rc = run_pipeline(ctx, in, st, nullptr)) == 1 && tries < 4; ++tries) {}
    if (rc < 0) return rc;
    if (rc == 1) return fail(ctx, NGZ_E_NOMEM, "batch buffers kept overflowing");
    ctx->n_template_dgrams = ctx->summary.n_host;
    if (ctx->summary.n_host == 0) {
        rc = place_arena(ctx, in, st);
        if (rc) return rc;
        return finish_batch(ctx, in, out, st);
    }

    // slow path: frame template-bearing datagrams on the host, in stream order.
    // The fast pass left the template state untouched: it is the batch-start state.
    const size_t nver0 = ctx->versions.size();
    const std::vector<int32_t> cur0[2] = {ctx->cur[0], ctx->cur[1]};
    const uint32_t N = in->n;
    std::vector<ngz_dgram_hdr> hdr(N);
    std::vector<uint64_t> offs(N);
    std::vector<uint32_t> lens(N);
    HIPCHK(hipMemcpyAsync(hdr.data(), ctx->d_hdr.p, N * sizeof(ngz_dgram_hdr), hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(offs.data(), in->offsets, N * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(lens.data(), in->lengths, N * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    std::vector<uint32_t> host_idx;
    for (uint32_t d = 0; d < N; ++d)
        if (hdr[d].status == NGZ_FR_HOST) host_idx.push_back(d);
    std::vector<std::vector<uint8_t>> dbytes(host_idx.size());
    for (size_t i = 0; i < host_idx.size(); ++i) {
        const uint32_t d = host_idx[i];
        dbytes[i].resize(lens[d] + 8);
        HIPCHK(hipMemcpy(dbytes[i].data(), in->bytes + offs[d], lens[d], hipMemcpyDeviceToHost));
    }
    ctx->n_template_dgrams = (uint32_t)host_idx.size();
    std::vector<uint32_t> limit(host_idx.size(), 0xFFFFFFFFu);
    std::vector<TemplateSetJson> tsets;
    for (int round = 0; round < 16; ++round) {
        tsets.clear();
        // roll the template state back to the batch start
        ctx->uploaded_gen = 0;  // device tables will describe the batch start, not the end state
        ctx->versions.resize(nver0);
        ctx->cur[0] = cur0[0];
        ctx->cur[1] = cur0[1];
        ctx->host_errors.clear();
        ctx->count_from.clear();
        HostFramed hf;
        hf.flag.assign(N, 0);
        hf.first.assign(N + 1, 0);
        std::vector<std::vector<std::pair<uint32_t, int32_t>>> defs(host_idx.size());
        std::vector<std::pair<uint32_t, uint32_t>> tl_entries;  // (version, dgram)
        std::vector<std::pair<uint32_t, std::vector<HostSet>>> per;
        for (size_t i = 0; i < host_idx.size(); ++i) {
            const uint32_t d = host_idx[i];
            HostFrameOut o;
            host_frame(ctx, dbytes[i].data(), lens[d], limit[i], o);
            hf.hdrs.push_back(o.hdr);
            hf.flag[d] = (uint32_t)hf.hdrs.size();
            per.push_back({d, std::move(o.sets)});
            defs[i] = o.defs;
            for (auto &df : o.defs) tl_entries.push_back({(uint32_t)df.second, d});
            for (auto &rs : o.restarts) {  // the last re-announcement of a version in the batch wins
                uint64_t &cf = ctx->count_from[rs.second];
                cf = std::max<uint64_t>(cf, ((uint64_t)d << 16) | rs.first);
            }
            for (auto &ts : o.tsets) tsets.push_back({d, ts.first, std::move(ts.second)});
        }
        std::vector<int32_t> extra;
        for (auto &t : tl_entries) extra.push_back((int32_t)t.first);
        for (int pi = 0; pi < 2; ++pi)
            for (uint32_t id = 0; id < 65536; ++id)
                if (cur0[pi][id] >= 0) extra.push_back(cur0[pi][id]);
        rc = assign_slots(ctx, extra);
        if (rc) return rc;
        // slot ids inside host sets are version ids until now
        for (auto &pr : per)
            for (auto &hs : pr.second) hs.slot = (uint16_t)ctx->version_slot[hs.reserved2];
        uint32_t at = 0, pi = 0;
        for (uint32_t d = 0; d < N; ++d) {
            hf.first[d] = at;
            if (pi < per.size() && per[pi].first == d) {
                for (auto &hs : per[pi].second) hf.sets.push_back(hs);
                at += (uint32_t)per[pi].second.size();
                ++pi;
            }
        }
        hf.first[N] = at;
        // timeline sorted by (proto<<16|id, dgram)
        std::vector<std::tuple<uint32_t, uint32_t, uint16_t>> tl;
        for (auto &t : tl_entries) {
            const Version &v = ctx->versions[t.first];
            tl.emplace_back(((v.proto == 10 ? 0u : 1u) << 16) | v.tid, t.second, (uint16_t)ctx->version_slot[t.first]);
        }
        std::stable_sort(tl.begin(), tl.end(), [](const auto &a, const auto &b) {
            return std::get<0>(a) != std::get<0>(b) ? std::get<0>(a) < std::get<0>(b) : std::get<1>(a) < std::get<1>(b);
        });
        // several definitions of one id inside one datagram: keep the last
        std::vector<std::tuple<uint32_t, uint32_t, uint16_t>> tl2;
        for (auto &e : tl) {
            if (!tl2.empty() && std::get<0>(tl2.back()) == std::get<0>(e) && std::get<1>(tl2.back()) == std::get<1>(e))
                tl2.back() = e;
            else
                tl2.push_back(e);
        }
        for (auto &e : tl2) {
            hf.tl.key.push_back(std::get<0>(e));
            hf.tl.dgram.push_back(std::get<1>(e));
            hf.tl.slot.push_back(std::get<2>(e));
        }
        rc = upload_slots(ctx, cur0, st);
        if (rc) return rc;
        if (ngz_debug()) {
            fprintf(stderr, "[ngz] slow path round %d: host dgrams %zu, slots %zu, timeline %zu\n", round,
                    host_idx.size(), ctx->slot_version.size(), hf.tl.key.size());
            for (size_t i = 0; i < hf.tl.key.size(); ++i)
                fprintf(stderr, "[ngz]   tl key %u dgram %u slot %u\n", hf.tl.key[i], hf.tl.dgram[i], hf.tl.slot[i]);
            for (size_t s2 = 0; s2 < ctx->slot_version.size(); ++s2) {
                const DevPlan &P = ctx->versions[ctx->slot_version[s2]].plan;
                fprintf(stderr, "[ngz]   slot %zu version %d tid %u rec_len %u rpl %u nf %u spec %u\n", s2,
                        ctx->slot_version[s2], P.template_id, P.rec_len, P.rpl, P.n_fields, P.spec);
            }
        }
        for (int tries = 0; (rc = run_pipeline(ctx, in, st, &hf)) == 1 && tries < 4; ++tries) {}
        if (rc < 0) return rc;
        if (rc == 1) return fail(ctx, NGZ_E_NOMEM, "batch buffers kept overflowing");
        // a device-found record error that precedes a template set voids that
        // definition (the reference stops parsing the message there)
        std::vector<ngz_dgram_hdr> h2(N);
        HIPCHK(hipMemcpy(h2.data(), ctx->d_hdr.p, N * sizeof(ngz_dgram_hdr), hipMemcpyDeviceToHost));
        bool redo = false;
        if (ngz_debug())
            for (size_t i = 0; i < host_idx.size(); ++i)
                fprintf(stderr, "[ngz]   host dgram %u flag %u status %u err %016llx limit %u defs %zu\n", host_idx[i],
                        hf.flag[host_idx[i]], h2[host_idx[i]].status, (unsigned long long)h2[host_idx[i]].err_key,
                        limit[i], defs[i].size());
        for (size_t i = 0; i < host_idx.size(); ++i) {
            const uint64_t k = h2[host_idx[i]].err_key;
            if (k == NGZ_NO_ERR) continue;
            const uint32_t stop = (uint32_t)(k >> 48);
            const uint32_t code = (uint32_t)(k >> 40) & 0xFF;
            if (code == E_HOST) continue;
            bool later_def = false;
            for (auto &df : defs[i])
                if (df.first > stop) later_def = true;
            if (later_def && limit[i] != stop) {
                limit[i] = stop;
                redo = true;
            }
        }
        if (!redo) break;
    }
    ctx->tmpl_sets = std::move(tsets);
    return finish_batch(ctx, in, out, st);
}

// The decode worker of ngz_decode_batch_submit: runs one submitted batch at a time through
// ngz_decode_batch on its own thread; exits when the context is destroyed (after a pending batch)
static void async_worker(ngz_ctx *ctx) {
    ngz_ctx::AsyncDecode &A = ctx->async;
    std::unique_lock<std::mutex> lk(A.m);
    for (;;) {
        A.cv.wait(lk, [&] { return A.job || A.stop; });
        if (!A.job) return;
        const ngz_batch_in in = A.in;
        ngz_batch_out *out = A.out;
        void *stream = A.stream;
        lk.unlock();
        int rc;
        try {
            rc = ngz_decode_batch(ctx, &in, out, stream);
        } catch (...) {  // (host allocation failure: no exception may leave the worker thread)
            rc = NGZ_E_NOMEM;
        }
        lk.lock();
        A.rc = rc;
        A.job = false;
        A.result = true;
        A.cv.notify_all();
    }
}

int ngz_decode_batch_submit(ngz_ctx *ctx, const ngz_batch_in *in, ngz_batch_out *out, void *hip_stream) {
    if (!ctx || !in || !out) return NGZ_E_INVALID;
    if (in->n && (!in->bytes || !in->offsets || !in->lengths)) return fail(ctx, NGZ_E_INVALID, "null batch arrays");
    ngz_ctx::AsyncDecode &A = ctx->async;
    std::unique_lock<std::mutex> lk(A.m);
    if (A.job || A.result) return NGZ_E_INVALID;  // pending: ngz_decode_batch_wait first (no message, see above)
    if (!A.th.joinable()) {
        try {
            A.th = std::thread(async_worker, ctx);
        } catch (...) {
            return fail(ctx, NGZ_E_NOMEM, "decode worker thread");
        }
    }
    A.in = *in;
    A.out = out;
    A.stream = hip_stream;
    A.job = true;
    A.pending.store(true);
    A.cv.notify_all();
    return NGZ_OK;
}

int ngz_decode_batch_wait(ngz_ctx *ctx) {
    if (!ctx) return NGZ_E_INVALID;
    ngz_ctx::AsyncDecode &A = ctx->async;
    std::unique_lock<std::mutex> lk(A.m);
    if (!A.job && !A.result) return NGZ_E_INVALID;
    A.cv.wait(lk, [&] { return A.result; });
    A.result = false;
    A.pending.store(false);
    return A.rc;
}

int ngz_decode_batch_host(ngz_ctx *ctx, const uint8_t *bytes, uint64_t bytes_size, const uint64_t *offsets,
                          const uint32_t *lengths, uint32_t n, ngz_batch_out *out) {
    if (!ctx || !out || (n && (!bytes || !offsets || !lengths))) return NGZ_E_INVALID;
    if (ctx->async.pending.load()) return NGZ_E_INVALID;  // a submitted batch is pending
    HIPCHK(hipSetDevice(ctx->device));
    if (wait_d2h(ctx)) return NGZ_E_DEVICE;
    if (ctx->d_in_bytes.ensure(bytes_size + 16) || ctx->d_in_off.ensure(n + 1) || ctx->d_in_len.ensure(n + 1))
        return fail(ctx, NGZ_E_NOMEM, "device alloc (input)");
    HIPCHK(hipMemcpyAsync(ctx->d_in_bytes.p, bytes, bytes_size, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->d_in_off.p, offsets, n * 8ull, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(ctx->d_in_len.p, lengths, n * 4ull, hipMemcpyHostToDevice, ctx->stream));
    ngz_batch_in in{ctx->d_in_bytes.p, bytes_size, ctx->d_in_off.p, ctx->d_in_len.p, n};
    return ngz_decode_batch(ctx, &in, out, nullptr);
}

// The columns of the last batch stay valid until the context's next decode: one that starts while a
// queued copy may still read them waits for it first (host side, so no reallocation can race it)
static int wait_d2h(ngz_ctx *ctx) {
    if (!ctx->d2h_pending) return 0;
    ctx->d2h_pending = false;
    HIPCHK(hipEventSynchronize(ctx->d2h_ev));
    return 0;
}

int64_t ngz_columns_to_host_async(ngz_ctx *ctx, void *dst, uint64_t cap, void *hip_stream, uint32_t flags) {
    if (!ctx || (!dst && cap) || (flags & ~NGZ_D2H_KERNEL)) return NGZ_E_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : ctx->stream;
    uint8_t *to = (uint8_t *)dst;
    if ((flags & NGZ_D2H_KERNEL) && dst) {
        void *dp = nullptr;
        if (hipHostGetDevicePointer(&dp, dst, 0) != hipSuccess || !dp) {
            (void)hipGetLastError();
            return fail(ctx, NGZ_E_INVALID, "NGZ_D2H_KERNEL: dst is not pinned host memory mapped for the device");
        }
        to = (uint8_t *)dp;
    }
    // the whole size first: a copy too large for dst queues nothing
    uint64_t total = 0;
    for (size_t s = 0; s < ctx->slot_infos.size(); ++s) {
        const ngz_slot_info &si = ctx->slot_infos[s];
        if (si.n_records)
            total = ((total + 255) & ~255ull) + (uint64_t)si.capacity * ctx->versions[si.version_id].plan.row_bytes;
    }
    if (total > cap) return fail(ctx, NGZ_E_INVALID, "ngz_columns_to_host: destination too small");
    if (!ctx->d2h_ev) HIPCHK(hipEventCreateWithFlags(&ctx->d2h_ev, hipEventDisableTiming));
    HIPCHK(hipStreamWaitEvent(st, ctx->ev[3], 0));  // the end of the last batch's pipeline
    // one event covers every queued copy: a copy queued earlier on another stream is waited for
    // by this one's stream before the event is recorded again (the next decode waits on it)
    if (ctx->d2h_pending) HIPCHK(hipStreamWaitEvent(st, ctx->d2h_ev, 0));
    uint64_t at = 0;
    for (size_t s = 0; s < ctx->slot_infos.size(); ++s) {
        const ngz_slot_info &si = ctx->slot_infos[s];
        if (!si.n_records) continue;
        const uint64_t bytes = (uint64_t)si.capacity * ctx->versions[si.version_id].plan.row_bytes;
        at = (at + 255) & ~255ull;
        if (flags & NGZ_D2H_KERNEL) {
            if (ngz_launch_to_host(si.columns, to + at, bytes, st)) {
                ctx->d2h_pending = at > 0 || ctx->d2h_pending;
                if (ctx->d2h_pending) (void)hipEventRecord(ctx->d2h_ev, st);
                return fail(ctx, NGZ_E_DEVICE, "k_to_host launch");
            }
        } else {
            HIPCHK(hipMemcpyAsync(to + at, si.columns, bytes, hipMemcpyDeviceToHost, st));
        }
        at += bytes;
    }
    HIPCHK(hipEventRecord(ctx->d2h_ev, st));
    ctx->d2h_pending = true;
    return (int64_t)at;
}

int64_t ngz_columns_to_host(ngz_ctx *ctx, void *dst, uint64_t cap) {
    const int64_t n = ngz_columns_to_host_async(ctx, dst, cap, nullptr, 0);
    if (n < 0) return n;
    // the event covers this copy and every copy queued before it on any stream
    HIPCHK(hipEventSynchronize(ctx->d2h_ev));
    ctx->d2h_pending = false;
    return n;
}

int ngz_slot_fields(ngz_ctx *ctx, uint32_t slot, ngz_field_info *fields, uint32_t cap) {
    if (!ctx || slot >= ctx->slot_version.size()) return NGZ_E_INVALID;
    const Version &v = ctx->versions[ctx->slot_version[slot]];
    const uint32_t n = (uint32_t)v.specs.size();
    for (uint32_t i = 0; i < n && i < cap; ++i) {
        ngz_field_info &f = fields[i];
        const Spec &s = v.specs[i];
        memset(&f, 0, sizeof f);
        f.wire_length = s.length;
        f.is_scope = i < v.n_scope;
        f.pen = s.pen;
        f.ie_id = s.id;
        f.wire_offset = v.fields[i].off;
        f.width = v.fields[i].width;
        f.kind = v.fields[i].kind;
        f.col_off = v.fields[i].col_off;
    }
    return (int)n;
}

int ngz_last_batch_info(ngz_ctx *ctx) { return ctx ? (int)ctx->batch_info : NGZ_E_INVALID; }

int ngz_message_records(ngz_ctx *ctx, const uint8_t *bytes, const uint64_t *offsets, const uint32_t *lengths,
                        uint32_t n, uint32_t *records) {
    if (!ctx || (n && (!bytes || !offsets || !lengths || !records))) return NGZ_E_INVALID;
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t *p = bytes + offsets[i];
        const uint32_t dl = lengths[i];
        uint32_t r = 0, pos = 0, end = 0, pi = 0;
        const uint32_t ver = dl >= 16 ? rd16(p) : 0, len = dl >= 16 ? rd16(p + 2) : 0;
        if (ver == 10 && len >= 16 && dl >= len) {  // ipfix.rs:54-104: the sets up to the header length
            pos = 16; end = len; pi = 0;
        } else if (ver == 9 && dl >= 20) {          // netflow.rs:56-114: the sets up to the datagram end
            pos = 20; end = dl; pi = 1;
        }
        while (pos + 4 <= end) {
            const uint32_t id = rd16(p + pos), sl = rd16(p + pos + 2);
            if (sl < 4 || sl > end - pos) break;
            const int32_t vid = id >= 256 ? ctx->cur[pi][id] : -1;
            if (vid >= 0) {
                const DevPlan &P = ctx->versions[vid].plan;
                uint64_t err = NGZ_NO_ERR;
                if (P.has_vlen && P.rpl)  // the framing's own record walk (ipfix.rs:219-222)
                    r += ngz_vlen_walk(p, pos + 4, pos + sl, P, &err, [](uint32_t, uint32_t) {});
                else if (P.rec_len)
                    r += (sl - 4) / P.rec_len;
            }
            pos += sl;
        }
        records[i] = r;
    }
    return NGZ_OK;
}

int ngz_placement_trials(ngz_ctx *ctx, float *decode_ms, float *probe_ms, uint32_t cap, uint32_t *kept) {
    if (!ctx) return NGZ_E_INVALID;
    const size_t n = std::max(ctx->place_ms.size(), ctx->place_probe_ms.size());
    for (size_t i = 0; i < n && i < cap; ++i) {
        if (decode_ms) decode_ms[i] = i < ctx->place_ms.size() ? ctx->place_ms[i] : 0.f;
        if (probe_ms) probe_ms[i] = i < ctx->place_probe_ms.size() ? ctx->place_probe_ms[i] : 0.f;
    }
    if (kept) *kept = ctx->place_kept;
    return (int)n;
}

#ifdef NGZ_EXPERIMENTS
extern "C" int ngz_launch_walk_probe(const uint8_t *bytes, uint64_t bytes_size, const uint64_t *offsets,
                                     const ngz_set_info *sets, uint32_t nsets, const DevPlan *plans, uint32_t mode,
                                     uint32_t lds_kb, uint32_t grid, uint32_t *out, hipStream_t st);
// Experiment builds: the walk probe (k_walk_probe, ngz_kernels.hip) over the last batch's sets, `reps`
// launches; out[0] records walked per launch, out[1] sets whose count differs; returns device ms per launch
extern "C" float ngz_exp_walk_probe(ngz_ctx *ctx, uint32_t mode, uint32_t lds_kb, uint32_t blocks_per_cu, uint32_t reps,
                                    uint32_t *out2) {
    if (!ctx || !ctx->summary.n_sets || !reps) return -1.f;
    hipStream_t st = ctx->stream;
    uint32_t *d_out = nullptr;
    if (hipMalloc(&d_out, 8) != hipSuccess) return -1.f;
    const uint32_t grid = blocks_per_cu * (uint32_t)ctx->n_cus;
    float ms = -1.f;
    uint32_t h[2] = {0, 0};
    hipMemsetAsync(d_out, 0, 8, st);
    hipEventRecord(ctx->ev[0], st);
    for (uint32_t r = 0; r < reps; ++r)
        if (ngz_launch_walk_probe(ctx->last_in.bytes, ctx->last_in.bytes_size, ctx->last_in.offsets, ctx->d_sets.p,
                                  ctx->summary.n_sets, ctx->d_plans.p, mode, lds_kb, grid, d_out, st))
            break;
    hipEventRecord(ctx->ev[1], st);
    if (hipEventSynchronize(ctx->ev[1]) == hipSuccess && hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]) == hipSuccess &&
        hipMemcpy(h, d_out, 8, hipMemcpyDeviceToHost) == hipSuccess) {
        ms /= (float)reps;
        out2[0] = h[0] / reps;
        out2[1] = h[1] / reps;
    } else {
        ms = -1.f;
    }
    hipFree(d_out);
    return ms;
}
#endif

int ngz_slot_kernel(ngz_ctx *ctx, uint32_t slot) {
    if (!ctx || slot >= ctx->slot_spec.size()) return NGZ_E_INVALID;
    return ctx->slot_spec[slot];
}

int ngz_last_timing(ngz_ctx *ctx, float *decode_ms, float *pipeline_ms) {
    if (!ctx) return NGZ_E_INVALID;
    if (decode_ms) *decode_ms = ctx->t_decode;
    if (pipeline_ms) *pipeline_ms = ctx->t_pipeline;
    return 0;
}

int ngz_template_counts(ngz_ctx *ctx, int proto, uint16_t *ids, uint64_t *counts, uint32_t cap, int reset) {
    if (!ctx || (proto != 9 && proto != 10)) return NGZ_E_INVALID;
    const int pi = proto == 10 ? 0 : 1;
    uint32_t n = 0;
    for (uint32_t id = 0; id < 65536; ++id) {
        const int32_t v = ctx->cur[pi][id];
        if (v < 0) continue;
        if (n < cap) {
            if (ids) ids[n] = (uint16_t)id;
            if (counts) counts[n] = ctx->versions[v].processed;
        }
        if (reset) ctx->versions[v].processed = 0;
        ++n;
    }
    return (int)n;
}

int ngz_template_counts_device(ngz_ctx *ctx, int proto, uint64_t *dev_table, uint32_t cap, int reset,
                               void *hip_stream) {
    if (!ctx || (proto != 9 && proto != 10) || (cap && !dev_table)) return NGZ_E_INVALID;
    HIPCHK(hipSetDevice(ctx->device));
    hipStream_t st = hip_stream ? (hipStream_t)hip_stream : ctx->stream;
    // staging table of this call: the ring slot whose last copy is the oldest (queued
    // COUNTS_RING calls ago, long complete in a per-step exchange: no host wait in practice)
    const int slot = (int)(ctx->counts_next++ % ngz_ctx::COUNTS_RING);
    if (ctx->counts_ev[slot]) HIPCHK(hipEventSynchronize(ctx->counts_ev[slot]));
    else HIPCHK(hipEventCreateWithFlags(&ctx->counts_ev[slot], hipEventDisableTiming));
    if (cap > ctx->h_counts_cap[slot]) {
        if (ctx->h_counts_stage[slot]) hipHostFree(ctx->h_counts_stage[slot]);
        ctx->h_counts_stage[slot] = nullptr;
        ctx->h_counts_cap[slot] = 0;
        HIPCHK(hipHostMalloc((void **)&ctx->h_counts_stage[slot], 16ull * cap, hipHostMallocDefault));
        ctx->h_counts_cap[slot] = cap;
    }
    uint64_t *stage = ctx->h_counts_stage[slot];
    const int n = ngz_template_counts(ctx, proto, nullptr, nullptr, 0, 0);
    std::vector<uint16_t> ids(std::max(n, 1));
    std::vector<uint64_t> cnt(std::max(n, 1));
    // a table too small resets nothing: the counts carry over to the call that has room for them
    ngz_template_counts(ctx, proto, ids.data(), cnt.data(), (uint32_t)n, reset && (uint32_t)n <= cap);
    for (uint32_t i = 0; i < cap; ++i) {
        stage[2 * i] = (int)i < n ? ids[i] : 0;
        stage[2 * i + 1] = (int)i < n ? cnt[i] : 0;
    }
    if (cap) {
        HIPCHK(hipMemcpyAsync(dev_table, stage, 16ull * cap, hipMemcpyHostToDevice, st));
        HIPCHK(hipEventRecord(ctx->counts_ev[slot], st));
    }
    return n;
}

int ngz_templates_json(ngz_ctx *ctx, int proto, char *buf, size_t cap) {
    if (!ctx || (proto != 9 && proto != 10)) return NGZ_E_INVALID;
    const int pi = proto == 10 ? 0 : 1;
    std::string s = "[";
    bool first = true;
    for (uint32_t id = 0; id < 65536; ++id) {
        const int32_t vid = ctx->cur[pi][id];
        if (vid < 0) continue;
        const Version &v = ctx->versions[vid];
        if (!first) s += ",";
        first = false;
        char b[64];
        snprintf(b, sizeof b, "{\"id\":%u,", id);
        s += b;
        s += "\"scope_field_specifiers\":[";
        for (uint32_t i = 0; i < v.n_scope; ++i) s += (i ? "," : "") + spec_json(v.specs[i]);
        s += "],\"field_specifiers\":[";
        for (uint32_t i = v.n_scope; i < v.specs.size(); ++i) s += (i > v.n_scope ? "," : "") + spec_json(v.specs[i]);
        s += "]}";
    }
    s += "]";
    if (buf && cap) {
        const size_t m = std::min(cap - 1, s.size());
        memcpy(buf, s.data(), m);
        buf[m] = 0;
    }
    return (int)s.size();
}

}  // extern "C"

// ------------------------------------------------------------------------
// Error rendering (serde_json text of FlowInfoCodecDecoderError)
// ------------------------------------------------------------------------
namespace {

std::string utf8_error_msg(const uint8_t *s, uint32_t n) {
    // core::str::Utf8Error Display
    uint32_t i = 0;
    while (i < n) {
        const uint32_t c = s[i];
        if (c < 0x80) { ++i; continue; }
        uint32_t need, lo = 0x80, hi = 0xBF;
        if (c >= 0xC2 && c <= 0xDF) need = 1;
        else if (c >= 0xE0 && c <= 0xEF) { need = 2; if (c == 0xE0) lo = 0xA0; if (c == 0xED) hi = 0x9F; }
        else if (c >= 0xF0 && c <= 0xF4) { need = 3; if (c == 0xF0) lo = 0x90; if (c == 0xF4) hi = 0x8F; }
        else {
            char b[96];
            snprintf(b, sizeof b, "invalid utf-8 sequence of 1 bytes from index %u", i);
            return b;
        }
        uint32_t t = 1;
        for (; t <= need; ++t) {
            if (i + t >= n) {
                char b[96];
                snprintf(b, sizeof b, "incomplete utf-8 byte sequence from index %u", i);
                return b;
            }
            const uint32_t bb = s[i + t];
            const uint32_t l2 = t == 1 ? lo : 0x80, h2 = t == 1 ? hi : 0xBF;
            if (bb < l2 || bb > h2) {
                char b[96];
                snprintf(b, sizeof b, "invalid utf-8 sequence of %u bytes from index %u", t, i);
                return b;
            }
        }
        i += need + 1;
    }
    return "";
}

}  // namespace

namespace ngzh {
// The error key of a datagram as the reference reports it.  The framing walk of a variable-length
// set stops in a record at an UnexpectedEof or a template-constant failure, and that key is the
// datagram's; DataRecord::parse had read the record's fields before the failing one, so a value
// error among them is the record's error (ngz_partial_record_err, ngz_internal.h).  Applied here,
// on the host, whenever an error is rendered (JSON text and ngz_dgram_error alike).
uint64_t record_err_key(ngz_ctx *ctx, uint32_t dgram, uint64_t key) {
    const uint32_t code = (uint32_t)(key >> 40) & 0xFF;
    if (key == NGZ_NO_ERR || (code != E_REC_EOF && code != E_REC_FAIL)) return key;
    const uint32_t stop = (uint32_t)(key >> 48), f = (uint32_t)(key >> 24) & 0xFFFF;
    uint64_t off = 0;
    uint32_t len = 0;
    if (hipMemcpy(&off, ctx->last_in.offsets + dgram, 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&len, ctx->last_in.lengths + dgram, 4, hipMemcpyDeviceToHost) != hipSuccess)
        return key;
    std::vector<uint8_t> p(len + 16, 0);
    std::vector<ngz_set_info> sets(ctx->summary.n_sets);
    if (hipMemcpy(p.data(), ctx->last_in.bytes + off, len, hipMemcpyDeviceToHost) != hipSuccess ||
        (!sets.empty() &&
         hipMemcpy(sets.data(), ctx->d_sets.p, sets.size() * sizeof(ngz_set_info), hipMemcpyDeviceToHost) != hipSuccess))
        return key;
    for (const auto &si : sets) {
        const uint32_t e = si.set_pos + rd16(p.data() + si.set_pos + 2);
        if (si.dgram != dgram || si.set_pos >= stop || stop > e) continue;
        const Version &v = ctx->versions[ctx->slot_version[si.slot]];
        if (!v.plan.has_vlen || f >= v.specs.size()) return key;
        uint64_t werr = NGZ_NO_ERR;
        uint32_t rstart = si.set_pos + 4u;
        ngz_vlen_walk_exact(p.data(), si.set_pos + 4u, e, v.plan, &werr, [](uint32_t, uint32_t) {}, 0u, &rstart);
        const uint64_t ve = werr != NGZ_NO_ERR ? ngz_partial_record_err(p.data(), rstart, f, v.plan) : NGZ_NO_ERR;
        return ve != NGZ_NO_ERR ? ve : key;
    }
    return key;
}
}  // namespace ngzh

extern "C" int ngz_dgram_error_json(ngz_ctx *ctx, uint32_t dgram, char *buf, size_t cap) {
    if (!ctx || dgram >= ctx->last_in.n) return NGZ_E_INVALID;
    ngz_dgram_hdr h;
    if (hipMemcpy(&h, ctx->d_hdr.p + dgram, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return NGZ_E_DEVICE;
    if (h.err_key == NGZ_NO_ERR) return NGZ_E_INVALID;
    h.err_key = record_err_key(ctx, dgram, h.err_key);
    const uint32_t stop = (uint32_t)(h.err_key >> 48);
    const uint32_t code = (uint32_t)(h.err_key >> 40) & 0xFF;
    const uint32_t a = (uint32_t)(h.err_key >> 24) & 0xFFFF;
    const uint32_t bval = (uint32_t)h.err_key & 0xFFFFFF;
    std::string s;
    char b[256];
    if (code == E_HOST) {
        s = bval < ctx->host_errors.size() ? ctx->host_errors[bval].json : "null";
    } else {
        uint64_t off = 0;
        uint32_t len = 0;
        hipMemcpy(&off, ctx->last_in.offsets + dgram, 8, hipMemcpyDeviceToHost);
        hipMemcpy(&len, ctx->last_in.lengths + dgram, 4, hipMemcpyDeviceToHost);
        std::vector<uint8_t> p(len + 16, 0);
        hipMemcpy(p.data(), ctx->last_in.bytes + off, len, hipMemcpyDeviceToHost);
        const bool v10 = h.version == 10;
        const char *W = v10 ? "IpfixParsingError" : "NetFlowV9ParingError";
        const char *SW = v10 ? "SetParsingError" : "SetError";
        auto set_wrap = [&](const std::string &j) { return wrap(W, wrap(SW, j)); };
        switch (code) {
        case E_CODEC_UNSUPPORTED_VERSION: snprintf(b, sizeof b, "{\"UnsupportedVersion\":%u}", a); s = b; break;
        case E_IPFIX_INVALID_LENGTH:
            snprintf(b, sizeof b, "{\"InvalidLength\":{\"offset\":2,\"length\":%u}}", bval); s = wrap(W, b); break;
        case E_HDR_EOF: s = wrap(W, eof_json({stop, a, bval})); break;
        case E_SET_EOF_ID: case E_SET_EOF_LEN: s = set_wrap(eof_json({stop, a, bval})); break;
        case E_SET_EOF_BODY: s = set_wrap(eof_json({stop, a, bval})); break;
        case E_SET_INVALID_ID: snprintf(b, sizeof b, "{\"InvalidSetId\":{\"offset\":%u,\"id\":%u}}", stop, a); s = set_wrap(b); break;
        case E_SET_INVALID_LENGTH:
            snprintf(b, sizeof b, "{\"InvalidLength\":{\"offset\":%u,\"length\":%u}}", stop, bval); s = set_wrap(b); break;
        case E_SET_NO_TEMPLATE:
            snprintf(b, sizeof b, "{\"NoTemplateDefinedFor\":{\"offset\":%u,\"id\":%u}}", stop, a); s = set_wrap(b); break;
        case E_SET_PADDING:
            snprintf(b, sizeof b, "{\"InvalidPaddingValue\":{\"offset\":%u,\"value\":%u}}", stop, bval); s = set_wrap(b); break;
        case E_NF_INVALID_COUNT:
            snprintf(b, sizeof b, "{\"InvalidCount\":{\"offset\":2,\"count\":%u}}", bval); s = wrap(W, b); break;
        case E_REC_DTMS: case E_REC_DTFRAC: case E_REC_UTF8: case E_REC_FAIL: case E_REC_EOF: {
            // find the set and version holding the failing field
            uint32_t nsets = ctx->summary.n_sets;
            std::vector<ngz_set_info> sets(nsets);
            hipMemcpy(sets.data(), ctx->d_sets.p, nsets * sizeof(ngz_set_info), hipMemcpyDeviceToHost);
            const Version *v = nullptr;
            uint32_t set_end = 0;
            for (auto &si : sets) {
                const uint32_t e = si.set_pos + rd16(p.data() + si.set_pos + 2);
                if (si.dgram == dgram && si.set_pos < stop && stop <= e) {
                    v = &ctx->versions[ctx->slot_version[si.slot]];
                    set_end = e;
                }
            }
            if (!v || a >= v->specs.size()) { s = "null"; break; }
            const Spec &sp = v->specs[a];
            std::string fe;
            const char *name = sp.name ? sp.name : "";
            if (code == E_REC_DTMS) {
                unsigned long long ms = 0;
                for (int i = 0; i < 8; ++i) ms = (ms << 8) | p[stop + i];
                snprintf(b, sizeof b, "{\"InvalidTimestampMillis\":{\"offset\":%u,\"ie_name\":%s,\"millis\":%llu}}", stop,
                         json_str(name).c_str(), ms);
                fe = b;
            } else if (code == E_REC_DTFRAC) {
                snprintf(b, sizeof b,
                         "{\"InvalidTimestampFraction\":{\"offset\":%u,\"ie_name\":%s,\"seconds\":%u,\"fraction\":%u}}",
                         stop, json_str(name).c_str(), rd32(p.data() + stop), rd32(p.data() + stop + 4));
                fe = b;
            } else if (code == E_REC_EOF) {  // variable-length record ran past its set
                fe = eof_json({stop, bval, set_end - stop});
            } else if (code == E_REC_UTF8) {
                uint32_t n = 0;
                if (sp.length == 0xFFFF) n = bval;  // variable-length string: every byte
                else while (n < sp.length && p[stop + n]) ++n;  // fixed: up to the first NUL
                snprintf(b, sizeof b, "{\"Utf8Error\":{\"offset\":%u,\"ie_name\":%s,\"error\":", stop, json_str(name).c_str());
                fe = std::string(b) + json_str(utf8_error_msg(p.data() + stop, n).c_str()) + "}}";
            } else {
                const uint8_t sub = v->fail_sub[a];
                if (sub == 3) {
                    snprintf(b, sizeof b, "{\"ScopeFieldError\":{\"InvalidLength\":{\"offset\":%u,\"length\":%u}}}", stop, sp.length);
                    s = set_wrap(wrap("DataRecordError", b));
                    break;
                }
                if (sub == 2)
                    snprintf(b, sizeof b, "{\"Parse\":{\"InvalidPaddingLength\":{\"offset\":%u,\"requested\":%u,\"ret_len\":4}}}",
                             stop, sp.length);
                else
                    snprintf(b, sizeof b, "{\"InvalidLength\":{\"offset\":%u,\"ie_name\":%s,\"length\":%u}}", stop,
                             json_str(name).c_str(), sp.length);
                fe = b;
            }
            if (sp.kind == IK_VENDOR || sp.kind == IK_VENDOR_UNKNOWN) fe = wrap((std::string(sp.vendor) + "Error").c_str(), fe);
            s = set_wrap(wrap("DataRecordError", wrap("FieldError", fe)));
            break;
        }
        default: s = "null";
        }
    }
    if (buf && cap) {
        const size_t m = std::min(cap - 1, s.size());
        memcpy(buf, s.data(), m);
        buf[m] = 0;
    }
    return (int)s.size();
}

extern "C" int ngz_template_kernel(const uint8_t *tmpl, size_t len, int compile, char *buf, size_t cap) {
    if (!tmpl || len < 4 || len > 65535) return NGZ_E_INVALID;
    Cur c{tmpl, 0, (uint32_t)len};
    const uint16_t tid = rd16(tmpl);
    const uint32_t count = rd16(tmpl + 2);
    c.pos = 4;
    Version v;
    v.proto = (compile & 2) ? 9 : 10;  // bit 1: a NetFlow v9 template record (netflow.rs:324-353)
    v.tid = tid;
    v.n_scope = 0;
    for (uint32_t i = 0; i < count; ++i) {
        Spec s;
        std::string err;
        if (!parse_field_spec(c, s, err)) return NGZ_E_INVALID;
        v.specs.push_back(s);
    }
    build_plan(v);
    if (!rtc_eligible(v.plan)) return NGZ_E_INVALID;
    std::string out = ngz_rtc_source(v.plan);
    int rc = NGZ_OK;
    if (compile & 1) {
        std::string log;
        if (ngz_rtc_compile_only(v.plan, &log)) {
            out += "\n// hiprtc log:\n" + log;
            rc = NGZ_E_DEVICE;
        }
    }
    if (buf && cap) {
        const size_t n = std::min(cap - 1, out.size());
        memcpy(buf, out.data(), n);
        buf[n] = 0;
    }
    return rc;
}

extern "C" int ngz_group_kernel(const uint8_t *tmpls, size_t len, int compile, char *buf, size_t cap) {
    if (!tmpls || len < 4 || len > 65535) return NGZ_E_INVALID;
    Cur c{tmpls, 0, (uint32_t)len};
    std::vector<Version> vs;
    while (c.pos + 4 <= len) {
        Version v;
        v.proto = 10;
        v.tid = rd16(tmpls + c.pos);
        const uint32_t count = rd16(tmpls + c.pos + 2);
        v.n_scope = 0;
        c.pos += 4;
        for (uint32_t i = 0; i < count; ++i) {
            Spec s;
            std::string err;
            if (!parse_field_spec(c, s, err)) return NGZ_E_INVALID;
            v.specs.push_back(s);
        }
        vs.push_back(std::move(v));
    }
    if (vs.size() < 2 || vs.size() > NGZ_RTC_GROUP_MAX) return NGZ_E_INVALID;
    std::vector<const DevPlan *> pp;
    for (Version &v : vs) {
        build_plan(v);
        if (!rtc_eligible(v.plan) || !v.plan.lds_waves || v.plan.has_vlen || v.plan.lds_waves != vs[0].plan.lds_waves)
            return NGZ_E_INVALID;
    }
    for (Version &v : vs) pp.push_back(&v.plan);
    std::string out = ngz_rtc_group_source(pp.data(), (uint32_t)pp.size());
    int rc = NGZ_OK;
    if (compile) {
        std::string log;
        if (ngz_rtc_compile_source(out, &log)) {
            out += "\n// hiprtc log:\n" + log;
            rc = NGZ_E_DEVICE;
        }
    }
    if (buf && cap) {
        const size_t n = std::min(cap - 1, out.size());
        memcpy(buf, out.data(), n);
        buf[n] = 0;
    }
    return rc;
}

namespace ngzh {

void state_save(ngz_ctx *ctx, TemplateState &s) {
    s.versions = ctx->versions;
    s.cur[0] = ctx->cur[0];
    s.cur[1] = ctx->cur[1];
}

void state_restore(ngz_ctx *ctx, const TemplateState &s) {
    ctx->versions = s.versions;
    ctx->cur[0] = s.cur[0];
    ctx->cur[1] = s.cur[1];
    ctx->tmpl_gen++;  // device plan tables are re-uploaded by the next batch
    ctx->plans_dirty = true;
    ctx->pred_valid = false;
}

}  // namespace ngzh
