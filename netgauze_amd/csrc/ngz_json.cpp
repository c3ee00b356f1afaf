// serde-JSON rendering of decoded datagrams, straight from the device columns:
// the text serde_json::to_string gives for the reference's FlowInfo value of
// each datagram (IPFIX / NetFlow v9 packet, every set, every record, every
// field), so the GPU path can feed the same JSONL consumers (pcap-decoder,
// the flow pcap tests) as the reference's Box<[Field]> records.
//
// Reference (NetGauze v0.13.0, paths relative to the checkout):
//   crates/flow-pkt/src/ipfix.rs:99-108,212-221,419-424  IpfixPacket / Set / DataRecord serde layout
//   crates/flow-pkt/src/netflow.rs (NetFlowV9Packet, ScopeField)       NetFlow v9 serde layout
//   crates/ipfix-code-generator/src/generator.rs:1412-1846 (Field enum, externally tagged;
//     vendor fields nested under the vendor variant, Unknown{pen,id,value})
//   crates/ipfix-code-generator/src/generator_sub_registries.rs:215-247 (sub-registry enums)
//   crates/iana/src/tcp.rs:165-190                        TCPHeaderFlags (8 named bools)
//   chrono 0.4.45 DateTime<Utc> serde (RFC 3339, AutoSi fraction, 'Z'), serde_json 1.0 (ryu
//   float text, string escaping), core::net Ipv4Addr / Ipv6Addr Display.
// tests/test_gpu_jsonl.py checks the lines against the reference's own golden
// JSON files, byte for byte.
#include <charconv>
#include <cmath>
#include <cstring>

#include "ngz_host.h"

using namespace ngzh;

namespace {

struct SubVal {
    uint32_t v;
    const char *name;
};
struct SubGroup {  // nested sub-registry: reason codes of one 64-value group
    const char *name;
    uint32_t first, count;
};
struct SubReg {
    uint32_t pen;
    uint16_t id;
    uint8_t nested;
    uint32_t first, count;
};
#include "subreg_table.inc"

const SubReg *subreg_find(uint32_t pen, uint16_t id) {
    for (const auto &r : kSubRegs)
        if (r.pen == pen && r.id == id) return &r;
    return nullptr;
}

inline void put(std::string &o, const char *s) { o += s; }

inline void put_u64(std::string &o, uint64_t v) {
    char b[24];
    auto r = std::to_chars(b, b + sizeof b, v);
    o.append(b, r.ptr);
}

inline void put_i64(std::string &o, int64_t v) {
    char b[24];
    auto r = std::to_chars(b, b + sizeof b, v);
    o.append(b, r.ptr);
}

// serde_json string escaping (valid UTF-8 in, escapes '"', '\\' and C0 controls)
void put_str(std::string &o, const uint8_t *s, size_t n) {
    static const char hex[] = "0123456789abcdef";
    o += '"';
    for (size_t i = 0; i < n; ++i) {
        const uint8_t c = s[i];
        if (c >= 0x20 && c != '"' && c != '\\') { o += (char)c; continue; }
        o += '\\';
        switch (c) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '\b': o += 'b'; break;
        case '\f': o += 'f'; break;
        case '\n': o += 'n'; break;
        case '\r': o += 'r'; break;
        case '\t': o += 't'; break;
        default: o += "u00"; o += hex[c >> 4]; o += hex[c & 15];
        }
    }
    o += '"';
}

void put_list(std::string &o, const uint8_t *p, size_t n) {
    o += '[';
    for (size_t i = 0; i < n; ++i) {
        if (i) o += ',';
        put_u64(o, p[i]);
    }
    o += ']';
}

void put_ipv4_raw(std::string &o, uint32_t v) {
    put_u64(o, v >> 24); o += '.';
    put_u64(o, (v >> 16) & 255); o += '.';
    put_u64(o, (v >> 8) & 255); o += '.';
    put_u64(o, v & 255);
}

// core::net::Ipv6Addr Display: RFC 5952 (longest run of >= 2 zero groups, the
// first one on ties, compressed to "::"), IPv4-mapped as ::ffff:a.b.c.d
void put_ipv6_raw(std::string &o, const uint8_t *b) {
    uint32_t g[8];
    for (int i = 0; i < 8; ++i) g[i] = ((uint32_t)b[2 * i] << 8) | b[2 * i + 1];
    if (!g[0] && !g[1] && !g[2] && !g[3] && !g[4] && g[5] == 0xFFFF) {
        o += "::ffff:";
        put_ipv4_raw(o, (g[6] << 16) | g[7]);
        return;
    }
    int best_s = 0, best_l = 0, cur_s = 0, cur_l = 0;
    for (int i = 0; i < 8; ++i) {
        if (g[i] == 0) {
            if (cur_l == 0) cur_s = i;
            if (++cur_l > best_l) { best_s = cur_s; best_l = cur_l; }
        } else cur_l = 0;
    }
    char h[8];
    auto grp = [&](int i) {
        auto r = std::to_chars(h, h + sizeof h, g[i], 16);
        o.append(h, r.ptr);
    };
    if (best_l > 1) {
        for (int i = 0; i < best_s; ++i) { if (i) o += ':'; grp(i); }
        o += "::";
        for (int i = best_s + best_l; i < 8; ++i) { if (i > best_s + best_l) o += ':'; grp(i); }
    } else {
        for (int i = 0; i < 8; ++i) { if (i) o += ':'; grp(i); }
    }
}

int64_t floordiv(int64_t a, int64_t b) { return a / b - ((a % b != 0) && ((a < 0) != (b < 0))); }

// chrono DateTime<Utc> serde text (RFC 3339, 'Z', fraction trimmed to 0/3/6/9
// digits; a leap-second nanos >= 1e9 prints as second 60)
void put_datetime(std::string &o, int64_t secs, uint32_t nanos) {
    const int64_t days = floordiv(secs, 86400);
    const int64_t sod = secs - days * 86400;
    int64_t z = days + 719468;
    const int64_t era = floordiv(z, 146097);
    const int64_t doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    int64_t y = yoe + era * 400;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    const int64_t d = doy - (153 * mp + 2) / 5 + 1;
    const int64_t m = mp < 10 ? mp + 3 : mp - 9;
    if (m <= 2) ++y;
    int64_t ss = sod % 60;
    if (nanos >= 1000000000u) { ss += 1; nanos -= 1000000000u; }
    char b[64];
    int n;
    if (y >= 0 && y <= 9999) n = snprintf(b, sizeof b, "\"%04lld", (long long)y);
    else n = snprintf(b, sizeof b, "\"%+05lld", (long long)y);
    n += snprintf(b + n, sizeof b - n, "-%02lld-%02lldT%02lld:%02lld:%02lld", (long long)m, (long long)d,
                  (long long)(sod / 3600), (long long)(sod % 3600 / 60), (long long)ss);
    if (nanos == 0) {}
    else if (nanos % 1000000 == 0) n += snprintf(b + n, sizeof b - n, ".%03u", nanos / 1000000);
    else if (nanos % 1000 == 0) n += snprintf(b + n, sizeof b - n, ".%06u", nanos / 1000);
    else n += snprintf(b + n, sizeof b - n, ".%09u", nanos);
    o.append(b, n);
    o += "Z\"";
}

// serde_json float text: ryu's shortest round-trip digits in ryu's layout
// (format64 / format32 in ryu's pretty module); NaN and infinities are null.
template <class F>
void put_float(std::string &o, F x, int maxkk, int minkk) {
    if (x != x || x - x != x - x) { o += "null"; return; }
    if (x == 0) { o += std::signbit(x) ? "-0.0" : "0.0"; return; }
    char b[64];
    auto r = std::to_chars(b, b + sizeof b, x, std::chars_format::scientific);
    std::string s(b, r.ptr);
    std::string sign;
    if (s[0] == '-') { sign = "-"; s = s.substr(1); }
    const size_t e = s.find('e');
    std::string digits;
    for (size_t i = 0; i < e; ++i)
        if (s[i] != '.') digits += s[i];
    const int E = atoi(s.c_str() + e + 1);
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    const int n = (int)digits.size();
    const int k = E - (n - 1);  // value = digits * 10^k
    const int kk = n + k;
    o += sign;
    if (0 <= k && kk <= maxkk) {
        o += digits; o.append(k, '0'); o += ".0";
    } else if (0 < kk && kk <= maxkk) {
        o += digits.substr(0, kk); o += '.'; o += digits.substr(kk);
    } else if (minkk < kk && kk <= 0) {
        o += "0."; o.append(-kk, '0'); o += digits;
    } else if (n == 1) {
        o += digits; o += 'e'; o += std::to_string(kk - 1);
    } else {
        o += digits[0]; o += '.'; o += digits.substr(1); o += 'e'; o += std::to_string(kk - 1);
    }
}

uint64_t le(const uint8_t *p, uint32_t w) {
    uint64_t v = 0;
    for (uint32_t i = 0; i < w; ++i) v |= (uint64_t)p[i] << (8 * i);
    return v;
}

// sub-registry enum text (generator_sub_registries.rs:215-247): variant name,
// {"Unassigned": v}; forwardingStatus nests a reason code per 64-value group
void put_subreg(std::string &o, const SubReg &r, uint64_t v) {
    if (!r.nested) {
        for (uint32_t i = r.first; i < r.first + r.count; ++i)
            if (kSubVals[i].v == v) { o += '"'; o += kSubVals[i].name; o += '"'; return; }
        o += "{\"Unassigned\":"; put_u64(o, v); o += '}';
        return;
    }
    const uint64_t gi = v / 64;
    if (gi < r.count) {
        const SubGroup &g = kSubGroups[r.first + gi];
        o += "{\""; o += g.name; o += "\":";
        for (uint32_t i = g.first; i < g.first + g.count; ++i)
            if (kSubVals[i].v == v) { o += '"'; o += kSubVals[i].name; o += "\"}"; return; }
        o += "{\"Unassigned\":"; put_u64(o, v); o += "}}";
        return;
    }
    o += "{\"Unassigned\":"; put_u64(o, v); o += '}';
}

const char *kScopeNames[] = {nullptr, "System", "Interface", "LineCard", "Cache", "Template"};

// Field::serialize of one decoded cell (canonical column encoding)
void put_value(std::string &o, const Spec &s, const DevField &fd, const uint8_t *cell, const uint8_t *bytes) {
    switch (fd.kind) {
    case NGZ_K_UINT: {
        const uint64_t v = le(cell, fd.width);
        if (s.kind == IK_VENDOR || s.kind == IK_IANA) {
            if (s.flags & 4) {
                if (const SubReg *r = subreg_find(s.pen, s.id)) { put_subreg(o, *r, v); return; }
            }
            switch (s.dtype) {
            case DT_float64: { double x; memcpy(&x, &v, 8); put_float(o, x, 16, -5); return; }
            case DT_float32: { float x; uint32_t u = (uint32_t)v; memcpy(&x, &u, 4); put_float(o, x, 13, -6); return; }
            case DT_ipv4Address: o += '"'; put_ipv4_raw(o, (uint32_t)v); o += '"'; return;
            case DT_dateTimeSeconds: put_datetime(o, (int64_t)v, 0); return;
            default: break;
            }
        }
        put_u64(o, v);
        return;
    }
    case NGZ_K_SCOPE32: put_u64(o, le(cell, 4)); return;
    case NGZ_K_TCPFLAGS: {  // TCPHeaderFlags (iana/src/tcp.rs:165-190)
        static const char *nm[8] = {"FIN", "SYN", "RST", "PSH", "ACK", "URG", "ECE", "CWR"};
        o += '{';
        for (int i = 0; i < 8; ++i) {
            if (i) o += ',';
            o += '"'; o += nm[i]; o += "\":";
            o += (cell[0] >> i & 1) ? "true" : "false";
        }
        o += '}';
        return;
    }
    case NGZ_K_SINT: {
        const uint64_t u = le(cell, fd.width);
        const int sh = 64 - 8 * fd.width;
        put_i64(o, (int64_t)(u << sh) >> sh);
        return;
    }
    case NGZ_K_BOOL: o += cell[0] ? "true" : "false"; return;
    case NGZ_K_BYTES:
        if ((s.kind == IK_IANA || s.kind == IK_VENDOR) && s.dtype == DT_ipv6Address && fd.width == 16) {
            o += '"'; put_ipv6_raw(o, cell); o += '"';
            return;
        }
        put_list(o, cell, fd.width);
        return;
    case NGZ_K_U256: put_list(o, cell, 32); return;
    case NGZ_K_DTMS: {
        const int64_t ms = (int64_t)le(cell, 8);
        const int64_t secs = floordiv(ms, 1000);
        put_datetime(o, secs, (uint32_t)(ms - secs * 1000) * 1000000u);
        return;
    }
    case NGZ_K_DTFRAC: put_datetime(o, (int64_t)(uint32_t)le(cell, 4), (uint32_t)le(cell + 4, 4)); return;
    case NGZ_K_STR: {  // fixed string: the reader truncates at the first NUL
        uint32_t n = 0;
        while (n < fd.width && cell[n]) ++n;
        put_str(o, cell, n);
        return;
    }
    case NGZ_K_VLEN: {  // {u64 batch offset, u32 length}
        const uint64_t off = le(cell, 8);
        const uint32_t n = (uint32_t)le(cell + 8, 4);
        if (fd.flags & 0x80) put_str(o, bytes + off, n);
        else put_list(o, bytes + off, n);
        return;
    }
    }
    o += "null";
}

// one Field / ScopeField value with its enum tag
void put_field(std::string &o, const Spec &s, const DevField &fd, const uint8_t *cell, const uint8_t *bytes) {
    char b[80];
    switch (s.kind) {
    case IK_IANA:
        o += "{\""; o += s.name; o += "\":";
        put_value(o, s, fd, cell, bytes);
        o += '}';
        return;
    case IK_VENDOR:
        o += "{\""; o += s.vendor; o += "\":{\""; o += s.name; o += "\":";
        put_value(o, s, fd, cell, bytes);
        o += "}}";
        return;
    case IK_VENDOR_UNKNOWN:
        o += "{\""; o += s.vendor;
        snprintf(b, sizeof b, "\":{\"Unknown\":{\"id\":%u,\"value\":", s.id);
        o += b;
        put_value(o, s, fd, cell, bytes);
        o += "}}}";
        return;
    case IK_UNKNOWN:
        snprintf(b, sizeof b, "{\"Unknown\":{\"pen\":%u,\"id\":%u,\"value\":", s.pen, s.id);
        o += b;
        put_value(o, s, fd, cell, bytes);
        o += "}}";
        return;
    case IK_SCOPE: {  // NFv9 ScopeField (netflow.rs:443-475)
        const char *nm = (s.pen == 0 && s.id >= 1 && s.id <= 5) ? kScopeNames[s.id] : nullptr;
        if (!nm) {
            snprintf(b, sizeof b, "{\"Unknown\":{\"pen\":%u,\"id\":%u,\"value\":", s.pen, s.id);
            o += b;
            put_list(o, cell, fd.width);
            o += "}}";
            return;
        }
        o += "{\""; o += nm; o += "\":";
        if (fd.kind == NGZ_K_SCOPE32) put_u64(o, le(cell, 4));
        else put_list(o, cell, fd.width);
        o += '}';
        return;
    }
    }
}

}  // namespace

namespace ngzh {

int json_view_load(ngz_ctx *ctx, const uint8_t *host_bytes, JsonView &v) {
    const uint32_t N = ctx->last_in.n;
    hipStream_t st = ctx->stream;
    v.serial = ctx->batch_serial;
    v.hdr.resize(N);
    v.offs.resize(N);
    v.lens.resize(N);
    const uint32_t ns = ctx->summary.n_sets;
    v.sets.resize(ns);
    if (N) {
        if (hipMemcpyAsync(v.hdr.data(), ctx->d_hdr.p, N * sizeof(ngz_dgram_hdr), hipMemcpyDeviceToHost, st) ||
            hipMemcpyAsync(v.offs.data(), ctx->last_in.offsets, N * 8ull, hipMemcpyDeviceToHost, st) ||
            hipMemcpyAsync(v.lens.data(), ctx->last_in.lengths, N * 4ull, hipMemcpyDeviceToHost, st))
            return NGZ_E_DEVICE;
    }
    if (ns && hipMemcpyAsync(v.sets.data(), ctx->d_sets.p, ns * sizeof(ngz_set_info), hipMemcpyDeviceToHost, st))
        return NGZ_E_DEVICE;
    const size_t S = ctx->slot_infos.size();
    v.cols.assign(S, {});
    for (size_t s = 0; s < S; ++s) {
        const ngz_slot_info &si = ctx->slot_infos[s];
        if (!si.n_records) continue;
        const uint64_t nb = (uint64_t)si.capacity * ctx->versions[si.version_id].plan.row_bytes;
        v.cols[s].resize(nb);
        if (nb && hipMemcpyAsync(v.cols[s].data(), si.columns, nb, hipMemcpyDeviceToHost, st)) return NGZ_E_DEVICE;
    }
    v.own_bytes.clear();
    if (host_bytes) {
        v.bytes = host_bytes;
    } else {
        v.own_bytes.resize(ctx->last_in.bytes_size + 16);
        if (ctx->last_in.bytes_size &&
            hipMemcpyAsync(v.own_bytes.data(), ctx->last_in.bytes, ctx->last_in.bytes_size, hipMemcpyDeviceToHost, st))
            return NGZ_E_DEVICE;
        v.bytes = v.own_bytes.data();
    }
    if (hipStreamSynchronize(st)) return NGZ_E_DEVICE;
    // CSR of data sets and template sets per datagram (both are in stream order)
    v.set_first.assign(N + 1, 0);
    for (const auto &si : v.sets) v.set_first[si.dgram + 1]++;
    v.tset_first.assign(N + 1, 0);
    for (const auto &t : ctx->tmpl_sets) v.tset_first[t.dgram + 1]++;
    for (uint32_t d = 0; d < N; ++d) {
        v.set_first[d + 1] += v.set_first[d];
        v.tset_first[d + 1] += v.tset_first[d];
    }
    return NGZ_OK;
}

int json_render(ngz_ctx *ctx, const JsonView &v, uint32_t d, std::string &o, uint32_t *consumed) {
    const ngz_dgram_hdr &h = v.hdr[d];
    const uint8_t *p = v.bytes + v.offs[d];
    const uint32_t dl = v.lens[d];
    const uint32_t ver = dl >= 2 ? rd16(p) : 0;
    if (h.status == NGZ_DG_NEED_MORE) {
        if (consumed) *consumed = 0;
        return NGZ_DG_NEED_MORE;
    }
    if (h.status == NGZ_DG_UNSUPPORTED) return NGZ_DG_UNSUPPORTED;
    if (h.status == NGZ_DG_ERROR) {
        // codec.rs:155-159 (IPFIX advances max(5, length)), :178-183 and :214-217 (buffer cleared)
        if (consumed) *consumed = ver == 10 ? std::min<uint32_t>(dl, std::max<uint32_t>(5, rd16(p + 2))) : dl;
        char small[512];
        int n = ngz_dgram_error_json(ctx, d, small, sizeof small);
        if (n < 0) return n;
        if ((size_t)n < sizeof small) o.append(small, n);
        else {
            std::string big(n + 1, '\0');
            ngz_dgram_error_json(ctx, d, &big[0], big.size());
            o.append(big.data(), n);
        }
        return NGZ_DG_ERROR;
    }
    const bool v10 = h.version == 10;
    if (v10) {
        o += "{\"IPFIX\":{\"version\":10,\"export_time\":";
        put_datetime(o, h.time, 0);
        o += ",\"sequence_number\":"; put_u64(o, h.sequence);
        o += ",\"observation_domain_id\":"; put_u64(o, h.domain);
    } else {
        o += "{\"NetFlowV9\":{\"version\":9,\"sys_up_time\":"; put_u64(o, h.sys_up_time);
        o += ",\"unix_time\":"; put_datetime(o, h.time, 0);
        o += ",\"sequence_number\":"; put_u64(o, h.sequence);
        o += ",\"source_id\":"; put_u64(o, h.domain);
    }
    o += ",\"sets\":[";
    uint32_t ds = v.set_first[d], de = v.set_first[d + 1];
    uint32_t ts = v.tset_first[d], te = v.tset_first[d + 1];
    uint32_t end = v10 ? 16 : 20;  // NFv9: bytes the parse consumed (netflow.rs:89 stops early)
    bool first = true;
    while (ds < de || ts < te) {
        const bool take_t = ts < te && (ds >= de || ctx->tmpl_sets[ts].set_pos < v.sets[ds].set_pos);
        if (!first) o += ',';
        first = false;
        if (take_t) {
            const TemplateSetJson &t = ctx->tmpl_sets[ts++];
            o += t.json;
            end = std::max(end, t.set_pos + rd16(p + t.set_pos + 2));
            continue;
        }
        const ngz_set_info &si = v.sets[ds++];
        end = std::max<uint32_t>(end, si.set_pos + rd16(p + si.set_pos + 2));
        const Version &ver_t = ctx->versions[ctx->slot_version[si.slot]];
        const uint32_t cap = ctx->slot_rt[si.slot].cap;
        const uint8_t *cols = v.cols[si.slot].data();
        o += "{\"Data\":{\"id\":"; put_u64(o, ver_t.tid);
        o += ",\"records\":[";
        const uint32_t nf = (uint32_t)ver_t.specs.size();
        for (uint32_t r = 0; r < si.n; ++r) {
            const uint64_t row = (uint64_t)si.rec0 + r;
            o += r ? ",{\"scope_fields\":[" : "{\"scope_fields\":[";
            for (uint32_t f = 0; f < nf; ++f) {
                if (f == ver_t.n_scope) o += "],\"fields\":[";
                else if (f) o += ',';
                const DevField &fd = ver_t.plan.f[f];
                put_field(o, ver_t.specs[f], fd, cols + (uint64_t)cap * fd.col_off + row * fd.width, v.bytes);
            }
            if (ver_t.n_scope == nf) o += "],\"fields\":[";
            o += "]}";
        }
        o += "]}}";
    }
    o += "]}}";
    if (consumed) *consumed = v10 ? h.length : end;
    return NGZ_DG_OK;
}

int subreg_kind(uint32_t pen, uint16_t id) {
    const SubReg *r = subreg_find(pen, id);
    return r ? (r->nested ? 2 : 1) : 0;
}

// Rank of the values 0..255 of a nested sub-registry (forwardingStatus) in the derived Ord of its
// enum (generator_sub_registries.rs:96-140): the outer variant (one per 64-value group, declared in
// group order, then Unassigned), then the reason enum's discriminant (a registered reason is its
// value, its Unassigned(x) the last registered value + 1), then the value: rank = outer << 56 |
// discriminant << 32 | value.  rank[256] is the outer Unassigned's (values from 256 OR into it).
bool subreg_nested_ranks(uint32_t pen, uint16_t id, uint64_t rank[257]) {
    const SubReg *r = subreg_find(pen, id);
    if (!r || !r->nested) return false;
    for (uint64_t x = 0; x < 256; ++x) {
        const uint64_t gi = x / 64;
        if (gi >= r->count) {
            rank[x] = ((uint64_t)r->count << 56) | x;
            continue;
        }
        const SubGroup &g = kSubGroups[r->first + gi];
        uint64_t disc = 0;  // an enum with no registered reason: Unassigned is its only variant
        bool known = false;
        for (uint32_t i = g.first; i < g.first + g.count; ++i) {
            if (kSubVals[i].v == x) known = true;
            disc = kSubVals[i].v + 1;  // implicit discriminant after the last declared one
        }
        if (known) disc = x;
        rank[x] = ((uint64_t)gi << 56) | (disc << 32) | x;
    }
    rank[256] = (uint64_t)r->count << 56;
    return true;
}

bool subreg_known(uint32_t pen, uint16_t id, uint64_t v) {
    const SubReg *r = subreg_find(pen, id);
    if (!r || r->nested) return false;
    for (uint32_t i = r->first; i < r->first + r->count; ++i)
        if (kSubVals[i].v == v) return true;
    return false;
}

}  // namespace ngzh

// ---------------------------------------------------------------------------
// AggFlowInfo::into_flowinfo_with_extra_fields (aggregator.rs:203-277)
// ---------------------------------------------------------------------------
namespace {

Spec spec_of(uint32_t pen, uint16_t id) {
    Spec s{};
    s.pen = pen;
    s.id = id;
    if (pen == 0) {
        const IeRow *r = ie_find(0, id);
        if (r) { s.kind = IK_IANA; s.dtype = r->dtype; s.flags = r->flags; s.name = r->name; }
        else { s.kind = IK_UNKNOWN; s.dtype = DT_octetArray; }
    } else if (const char *vn = vendor_name(pen)) {
        const IeRow *r = ie_find(pen, id);
        s.vendor = vn;
        if (r) { s.kind = IK_VENDOR; s.dtype = r->dtype; s.flags = r->flags; s.name = r->name; }
        else { s.kind = IK_VENDOR_UNKNOWN; s.dtype = DT_octetArray; }
    } else {
        s.kind = IK_UNKNOWN;
        s.dtype = DT_octetArray;
    }
    return s;
}

void put_cell(std::string &o, uint32_t pen, uint16_t id, uint8_t kind, uint16_t width, const uint8_t *cell) {
    DevField fd{};
    fd.kind = kind;
    fd.width = width;
    put_field(o, spec_of(pen, id), fd, cell, nullptr);
}

// a byte value of any length (BVAL keys / values): rendered as the decode path renders a
// variable-length field of the IE (string text, or the bytes as a list)
void put_bytes(std::string &o, uint32_t pen, uint16_t id, const std::vector<uint8_t> &b) {
    const Spec s = spec_of(pen, id);
    DevField fd{};
    fd.kind = NGZ_K_VLEN;
    fd.width = 16;
    fd.flags = s.dtype == DT_string ? 0x80 : 0;
    uint8_t cell[16] = {};
    const uint32_t n = (uint32_t)b.size();
    memcpy(cell + 8, &n, 4);
    put_field(o, s, fd, cell, b.data());
}

// the whole byte value of a row's BVAL key / value; false when the row's tail is not in the
// tails of the last flush / emit (a row of an earlier call): the caller fails, NGZ_E_INVALID
bool row_bytes(ngz_agg *a, const uint8_t *R, int is_value, uint32_t i, std::vector<uint8_t> &b) {
    const int64_t n = ngz_agg_row_bytes(a, R, is_value, i, nullptr, 0);
    if (n < 0) return false;
    b.assign((size_t)n, 0);
    return n == 0 || ngz_agg_row_bytes(a, R, is_value, i, b.data(), b.size()) == n;
}

}  // namespace

extern "C" int64_t ngz_agg_flowinfo_json(ngz_agg *a, const void *rows, uint64_t n, uint32_t shard_id, uint32_t seq0,
                                         int64_t export_time_ms, ngz_json_line_fn fn, void *user) {
    if (!a || (n && (!rows || !fn))) return NGZ_E_INVALID;
    const auto &keys = agg_keys(a);
    const auto &vals = agg_vals(a);
    uint32_t rb = 0;
    std::vector<uint32_t> ko(keys.size() + 1), vo(vals.size() + 1);
    std::vector<uint16_t> kw(keys.size() + 1), vw(vals.size() + 1);
    ngz_agg_layout(a, &rb, ko.data(), kw.data(), vo.data(), vw.data());
    std::vector<ngz_agg_key_desc> kd(keys.size());
    std::vector<ngz_agg_value_desc> vd(vals.size());
    for (uint32_t k = 0; k < keys.size(); ++k) ngz_agg_key_info(a, k, &kd[k]);
    for (uint32_t v = 0; v < vals.size(); ++v) ngz_agg_value_info(a, v, &vd[v]);
    const std::vector<int64_t> *dt, *dp, *dd;
    agg_out_dicts(a, &dt, &dp, &dd);
    const std::vector<ngz_peer> &peers = agg_out_peers(a);
    const uint64_t win_ms = agg_window_ms(a);
    const int64_t es = floordiv(export_time_ms, 1000);
    const uint32_t ens = (uint32_t)(export_time_ms - es * 1000) * 1000000u;
    std::string o;
    for (uint64_t g = 0; g < n; ++g) {
        const uint8_t *R = (const uint8_t *)rows + g * rb;
        ngz_agg_row h;
        memcpy(&h, R, sizeof h);
        o.clear();
        const bool v10 = h.flow_type == 10;
        if (v10) {
            o += "{\"IPFIX\":{\"version\":10,\"export_time\":";
            put_datetime(o, es, ens);
            o += ",\"sequence_number\":"; put_u64(o, (uint32_t)(seq0 + g));
            o += ",\"observation_domain_id\":"; put_u64(o, shard_id);
        } else {
            o += "{\"NetFlowV9\":{\"version\":9,\"sys_up_time\":"; put_u64(o, h.max_sys_up_time);
            o += ",\"unix_time\":"; put_datetime(o, es, ens);
            o += ",\"sequence_number\":"; put_u64(o, (uint32_t)(seq0 + g));
            o += ",\"source_id\":"; put_u64(o, shard_id);
        }
        o += ",\"sets\":[{\"Data\":{\"id\":65535,\"records\":[{\"scope_fields\":[],\"fields\":[";
        bool first = true;
        auto sep = [&]() { if (!first) o += ','; first = false; };
        // key fields, then aggregated fields: the present ones (flatten over Option)
        for (uint32_t k = 0; k < keys.size(); ++k) {
            if (!(h.key_present >> k & 1)) continue;
            sep();
            const uint8_t *c = R + ko[k];
            if (kd[k].kkind == 3) {  // a byte value of any length
                std::vector<uint8_t> b;
                if (!row_bytes(a, R, 0, k, b)) return NGZ_E_INVALID;
                put_bytes(o, keys[k].pen, keys[k].ie_id, b);
            } else {
                put_cell(o, keys[k].pen, keys[k].ie_id, kd[k].kind, kd[k].width, c);
            }
        }
        for (uint32_t v = 0; v < vals.size(); ++v) {
            if (!(h.val_present >> v & 1)) continue;
            sep();
            const uint8_t *c = R + vo[v];
            uint8_t cell[32];
            switch (vd[v].vclass) {
            case 2: {  // secs<<32 | nanos -> {u32 secs, u32 nanos}
                uint64_t x;
                memcpy(&x, c, 8);
                const uint32_t secs = (uint32_t)(x >> 32), ns = (uint32_t)x;
                memcpy(cell, &secs, 4);
                memcpy(cell + 4, &ns, 4);
                put_cell(o, vals[v].pen, vals[v].ie_id, NGZ_K_DTFRAC, 8, cell);
                break;
            }
            case 5: put_cell(o, vals[v].pen, vals[v].ie_id, NGZ_K_UINT, 4, c); break;
            case 6: put_cell(o, vals[v].pen, vals[v].ie_id, NGZ_K_UINT, 8, c); break;
            case 7: put_cell(o, vals[v].pen, vals[v].ie_id, NGZ_K_BYTES, 16, c); break;
            case 8:
            case 9: {
                std::vector<uint8_t> b;
                if (!row_bytes(a, R, 1, v, b)) return NGZ_E_INVALID;
                put_bytes(o, vals[v].pen, vals[v].ie_id, b);
                break;
            }
            default: put_cell(o, vals[v].pen, vals[v].ie_id, vd[v].kind, vd[v].width, c); break;
            }
        }
        uint8_t cell[8];
        sep();
        memcpy(cell, &h.record_count, 8);
        put_cell(o, 0, 375, NGZ_K_UINT, 8, cell);  // originalFlowsPresent
        sep();
        memcpy(cell, &h.min_export_time, 4);
        put_cell(o, 0, 264, NGZ_K_UINT, 4, cell);  // minExportSeconds
        sep();
        memcpy(cell, &h.max_export_time, 4);
        put_cell(o, 0, 260, NGZ_K_UINT, 4, cell);  // maxExportSeconds
        sep();
        memcpy(cell, &h.max_collection_ms, 8);
        put_cell(o, 0, 258, NGZ_K_DTMS, 8, cell);  // collectionTimeMilliseconds
        // the actor's extra fields (actor.rs:222-240): NetGauze windowStart / windowEnd of the
        // emitted window ((start, start + window_duration), aggregation.rs:163-168), then the
        // peer IP as originalExporterIPv4Address / originalExporterIPv6Address
        const int64_t ws_ms = (int64_t)h.window_start * 1000;
        const int64_t we_ms = ws_ms + (int64_t)win_ms;
        sep();
        memcpy(cell, &ws_ms, 8);
        put_cell(o, 3746, 1, NGZ_K_DTMS, 8, cell);  // NetGauze windowStart
        sep();
        memcpy(cell, &we_ms, 8);
        put_cell(o, 3746, 2, NGZ_K_DTMS, 8, cell);  // NetGauze windowEnd
        if (h.peer >= peers.size()) return NGZ_E_INVALID;
        const ngz_peer &pe = peers[h.peer];
        sep();
        if (pe.family == 4) {
            const uint32_t ip = ((uint32_t)pe.addr[0] << 24) | ((uint32_t)pe.addr[1] << 16) |
                                ((uint32_t)pe.addr[2] << 8) | pe.addr[3];
            uint8_t c4[4];
            memcpy(c4, &ip, 4);
            put_cell(o, 0, 403, NGZ_K_UINT, 4, c4);  // originalExporterIPv4Address
        } else {
            put_cell(o, 0, 404, NGZ_K_BYTES, 16, pe.addr);  // originalExporterIPv6Address
        }
        auto bits_sorted = [](const std::vector<int64_t> &d, const uint64_t *bits, int words) {
            std::vector<int64_t> out;
            for (size_t i = 0; i < d.size() && (int)(i / 64) < words; ++i)
                if ((bits[i / 64] >> (i % 64) & 1) && d[i] >= 0) out.push_back(d[i]);
            std::sort(out.begin(), out.end());
            return out;
        };
        for (int64_t p : bits_sorted(*dp, &h.port_bits, 1)) {
            sep();
            const uint16_t x = (uint16_t)p;
            memcpy(cell, &x, 2);
            put_cell(o, 3746, 4, NGZ_K_UINT, 2, cell);  // NetGauze originalExporterTransportPort
        }
        for (int64_t dm : bits_sorted(*dd, h.domain_bits, 2)) {
            sep();
            const uint32_t x = (uint32_t)dm;
            memcpy(cell, &x, 4);
            put_cell(o, 0, 405, NGZ_K_UINT, 4, cell);  // originalObservationDomainId
        }
        std::vector<int64_t> tids;
        for (int64_t t : bits_sorted(*dt, &h.template_bits, 1)) tids.push_back(t & 0xFFFF);
        std::sort(tids.begin(), tids.end());
        for (int64_t t : tids) {
            sep();
            const uint16_t x = (uint16_t)t;
            memcpy(cell, &x, 2);
            put_cell(o, 3746, 3, NGZ_K_UINT, 2, cell);  // NetGauze originalTemplateId
        }
        o += "]}]}}]}}";
        if (fn(user, (uint32_t)g, NGZ_DG_OK, o.data(), o.size(), 0)) return (int64_t)g + 1;
    }
    return (int64_t)n;
}

extern "C" int64_t ngz_dgram_json(ngz_ctx *ctx, uint32_t dgram, char *buf, size_t cap) {
    if (!ctx || dgram >= ctx->last_in.n) return NGZ_E_INVALID;
    if (hipSetDevice(ctx->device)) return NGZ_E_DEVICE;
    if (!ctx->json_view || ctx->json_view->serial != ctx->batch_serial) {
        auto v = std::make_shared<JsonView>();
        const int rc = json_view_load(ctx, nullptr, *v);
        if (rc) return rc;
        ctx->json_view = v;
    }
    std::string s;
    const int st = json_render(ctx, *ctx->json_view, dgram, s, nullptr);
    if (st < 0) return st;
    if (st != NGZ_DG_OK && st != NGZ_DG_ERROR) return NGZ_E_INVALID;
    if (buf && cap) {
        const size_t m = std::min(cap - 1, s.size());
        memcpy(buf, s.data(), m);
        buf[m] = 0;
    }
    return (int64_t)s.size();
}

static_assert(DT_octetArray == NGZ_DT_OCTET_ARRAY && DT_string == NGZ_DT_STRING && DT_ipv6Address == NGZ_DT_IPV6_ADDRESS &&
                  DT_dateTimeNanoseconds == NGZ_DT_DATETIME_NANOSECONDS && DT_unsigned256 == NGZ_DT_UNSIGNED256,
              "registry data types are the ABI's NGZ_DT_*");

extern "C" int ngz_record_fields(ngz_ctx *ctx, uint32_t dgram, uint32_t set, uint32_t rec, ngz_field_value *out,
                                 uint32_t cap) {
    if (!ctx || dgram >= ctx->last_in.n || (cap && !out)) return NGZ_E_INVALID;
    if (hipSetDevice(ctx->device)) return NGZ_E_DEVICE;
    if (!ctx->json_view || ctx->json_view->serial != ctx->batch_serial) {
        auto v = std::make_shared<JsonView>();
        const int rc = json_view_load(ctx, nullptr, *v);
        if (rc) return rc;
        ctx->json_view = v;
    }
    JsonView &v = *ctx->json_view;
    if (v.hdr[dgram].status != NGZ_DG_OK) return NGZ_E_INVALID;
    const uint32_t s0 = v.set_first[dgram];
    if (set >= v.set_first[dgram + 1] - s0) return NGZ_E_INVALID;
    const ngz_set_info &si = v.sets[s0 + set];
    if (rec >= si.n) return NGZ_E_INVALID;
    const Version &ver = ctx->versions[ctx->slot_version[si.slot]];
    const uint8_t *p = v.bytes + v.offs[dgram];
    // the record's offset in the datagram: fixed records follow each other from the set payload;
    // variable-length ones are walked once per set (ngz_vlen_walk, the framing's own walk)
    uint32_t pos;
    if (ver.plan.has_vlen) {
        auto it = v.rec_pos.find(s0 + set);
        if (it == v.rec_pos.end()) {
            std::vector<uint32_t> starts;
            uint64_t err = NGZ_NO_ERR;
            ngz_vlen_walk(p, si.set_pos + 4u, si.set_pos + rd16(p + si.set_pos + 2), ver.plan, &err,
                          [&](uint32_t, uint32_t at) { starts.push_back(at); });
            it = v.rec_pos.emplace(s0 + set, std::move(starts)).first;
        }
        if (rec >= it->second.size()) return NGZ_E_INVALID;
        pos = it->second[rec];
    } else {
        pos = si.set_pos + 4u + rec * ver.plan.rec_len;
    }
    const uint32_t nf = (uint32_t)ver.specs.size();
    const uint32_t cap_rows = ctx->slot_rt[si.slot].cap;
    const uint8_t *cols = v.cols[si.slot].data();
    const uint64_t row = (uint64_t)si.rec0 + rec;
    for (uint32_t f = 0; f < nf; ++f) {
        const Spec &sp = ver.specs[f];
        const DevField &fd = ver.plan.f[f];
        const uint8_t *cell = cols + (uint64_t)cap_rows * fd.col_off + row * fd.width;
        ngz_field_value fv{};
        fv.pen = sp.pen;
        fv.ie_id = sp.id;
        fv.kind = fd.kind;
        fv.dtype = sp.dtype;
        fv.flags = (sp.scope ? NGZ_FV_SCOPE : 0u) |
                   (fd.kind == NGZ_K_STR || (fd.kind == NGZ_K_VLEN && (fd.flags & 0x80)) ? NGZ_FV_STRING : 0u) |
                   (sp.kind == IK_VENDOR || sp.kind == IK_VENDOR_UNKNOWN ? NGZ_FV_VENDOR : 0u) |
                   (sp.kind == IK_UNKNOWN || sp.kind == IK_VENDOR_UNKNOWN ? NGZ_FV_UNKNOWN : 0u) |
                   (sp.flags & 4 ? NGZ_FV_SUBREG : 0u) | (sp.flags & 1 ? NGZ_FV_MPLS : 0u) |
                   (sp.flags & 2 ? NGZ_FV_TCPFLAGS : 0u);
        fv.wire_length = sp.length;
        fv.width = fd.width;
        if (fd.kind == NGZ_K_VLEN) {  // {u64 batch offset, u32 length, u32 0}
            uint64_t off;
            uint32_t len;
            memcpy(&off, cell, 8);
            memcpy(&len, cell + 8, 4);
            fv.value = v.bytes + off;
            fv.len = len;
            fv.wire_offset = (uint32_t)(off - v.offs[dgram]);
            pos = fv.wire_offset + len;
        } else {
            fv.value = cell;
            fv.len = fd.width;
            if (fd.kind == NGZ_K_STR) {  // the string ends at its first NUL (generator.rs:1651-1668)
                uint32_t n = 0;
                while (n < fd.width && cell[n]) ++n;
                fv.len = n;
            }
            fv.wire_offset = pos;
            pos += sp.length;
        }
        if (f < cap) out[f] = fv;
    }
    return (int)nf;
}

extern "C" int64_t ngz_batch_json(ngz_ctx *ctx, const uint8_t *host_bytes, ngz_json_line_fn fn, void *user) {
    if (!ctx || !fn) return NGZ_E_INVALID;
    if (hipSetDevice(ctx->device)) return NGZ_E_DEVICE;
    JsonView v;
    int rc = json_view_load(ctx, host_bytes, v);
    if (rc) return rc;
    int64_t lines = 0;
    std::string s;
    for (uint32_t d = 0; d < ctx->last_in.n; ++d) {
        s.clear();
        uint32_t consumed = 0;
        const int st = json_render(ctx, v, d, s, &consumed);
        if (st < 0) return st;
        if (st != NGZ_DG_OK && st != NGZ_DG_ERROR) continue;
        if (fn(user, d, st, s.data(), s.size(), consumed)) break;
        ++lines;
    }
    return lines;
}
