// Host ingest in front of the decoder (include/ngz/flow_ingest.h):
//   * the capture reader (≙ netgauze_pcap_reader::PcapIter,
//     crates/pcap-reader/src/lib.rs:97-377),
//   * a recvmmsg(2) UDP reader (≙ the collector's socket loop,
//     crates/flow-service/src/flow_actor.rs:828-883),
//   * the per-exporter-peer codec map with stream framing (≙ the pcap
//     decoder's FlowProtocolHandler + decode_buffer,
//     crates/pcap-decoder/src/handlers/{flow.rs:37-59, mod.rs:36-80}, and the
//     flow pcap tests' driver, wire/tests/pcap_tests.rs:79-118), and
//   * `pcap-decoder --protocol flow` (crates/pcap-decoder/src/lib.rs:65-127).
//
// Decoding is not done message by message as in the reference: every peer's
// queued bytes are framed speculatively into messages with the codec's rules
// (codec.rs:189-220) and decoded in one GPU batch per peer.  Two outcomes
// decide where the next message of a byte stream starts and are only known
// after decoding: how many bytes a NetFlow v9 parse consumed (the header has
// no length, netflow.rs:89) and, in pcap-decoder mode, whether a message that
// shares its buffer with later bytes failed (the buffer is then cleared,
// handlers/mod.rs:53-57).  The speculation assumes "whole buffer" / "success";
// if a decoded message contradicts it, the peer's template state is rolled
// back to the batch start, the prefix up to that message is replayed, and
// framing resumes from the true position.  Output is therefore identical to
// the reference's one-message-at-a-time loop.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <poll.h>
#include <sys/socket.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "ngz/flow_ingest.h"
#include "ngz_host.h"

using namespace ngzh;

// ---------------------------------------------------------------------------
// Capture reader
// ---------------------------------------------------------------------------
struct ngz_pcap {
    std::vector<uint8_t> data;
    size_t pos = 0;
    bool ng = false;
    bool be = false;                   // file byte order (legacy header / current pcapng section)
    std::vector<uint32_t> link_types;  // legacy: [network]; pcapng: per interface of the section
    uint64_t frame = 0;
    std::vector<uint8_t> payload;      // the current packet's payload (borrowed by ngz_packet)
};

namespace {

uint16_t be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }
uint32_t rd32f(const uint8_t *p, bool be) {
    return be ? ((uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3])
              : ((uint32_t)p[3] << 24 | (uint32_t)p[2] << 16 | (uint32_t)p[1] << 8 | p[0]);
}
uint16_t rd16f(const uint8_t *p, bool be) { return be ? (uint16_t)(p[0] << 8 | p[1]) : (uint16_t)(p[1] << 8 | p[0]); }

constexpr uint16_t ET_IPV4 = 0x0800, ET_IPV6 = 0x86DD;
bool is_vlan(uint16_t et) { return et == 0x8100 || et == 0x88A8 || et == 0x9100; }

// strip_vlan_tags (lib.rs:97-117): at most MAX_VLAN_TAGS = 4 stacked tags
bool strip_vlan_tags(uint16_t &et, const uint8_t *&p, size_t &n) {
    for (int i = 0; i <= 4; ++i) {
        if (!is_vlan(et)) return true;
        if (n < 4) return false;
        et = be16(p + 2);
        p += 4;
        n -= 4;
    }
    return false;
}

// Ipv4Pdu / Ipv6Pdu + Udp / Tcp (lib.rs:279-377, pdu crate bounds)
bool parse_l4(uint8_t proto, const uint8_t *body, size_t n, bool trim_udp, ngz_packet &pk) {
    if (proto == NGZ_PROTO_UDP) {
        if (n < 8) return false;
        pk.key.src_port = be16(body);
        pk.key.dst_port = be16(body + 2);
        size_t len = n - 8;
        if (trim_udp) {  // IPv4 only: "UDP payload length, to avoiding parsing any padding bytes"
            const uint32_t ulen = be16(body + 4);
            if (ulen < 8 || ulen - 8 > n - 8) return false;  // the reference asserts here
            len = ulen - 8;
        }
        pk.proto = NGZ_PROTO_UDP;
        pk.payload = body + 8;
        pk.len = (uint32_t)len;
        return true;
    }
    if (proto == NGZ_PROTO_TCP) {
        if (n < 20) return false;
        const size_t off = (size_t)(body[12] >> 4) * 4;
        if (off < 20 || off > n) return false;
        pk.key.src_port = be16(body);
        pk.key.dst_port = be16(body + 2);
        pk.proto = NGZ_PROTO_TCP;
        pk.payload = body + off;
        pk.len = (uint32_t)(n - off);
        return true;
    }
    return false;  // ICMP, raw, ...
}

bool parse_l3(uint16_t et, const uint8_t *d, size_t n, ngz_packet &pk) {
    memset(&pk.key, 0, sizeof pk.key);
    if (et == ET_IPV4) {
        if (n < 20 || (d[0] >> 4) != 4) return false;
        const size_t ihl = (size_t)(d[0] & 15) * 4;
        if (ihl < 20 || ihl > n) return false;
        const size_t total = be16(d + 2);
        const size_t end = total >= ihl ? std::min(total, n) : n;
        pk.key.family = 4;
        memcpy(pk.key.src, d + 12, 4);
        memcpy(pk.key.dst, d + 16, 4);
        return parse_l4(d[9], d + ihl, end - ihl, true, pk);
    }
    if (et == ET_IPV6) {
        if (n < 40 || (d[0] >> 4) != 6) return false;
        const size_t plen = be16(d + 4);
        pk.key.family = 6;
        memcpy(pk.key.src, d + 8, 16);
        memcpy(pk.key.dst, d + 24, 16);
        return parse_l4(d[6], d + 40, std::min(plen, n - 40), false, pk);
    }
    return false;
}

// data::get_packetdata by link type, then parse_ethernet / parse_l3 (lib.rs:222-277)
bool parse_frame(uint32_t linktype, const uint8_t *d, size_t n, ngz_packet &pk) {
    uint16_t et;
    switch (linktype) {
    case 1: {  // Ethernet; the pdu crate unwraps one 802.1Q tag itself
        if (n < 14) return false;
        et = be16(d + 12);
        d += 14;
        n -= 14;
        if (et == 0x8100) {
            if (n < 4) return false;
            et = be16(d + 2);
            d += 4;
            n -= 4;
        }
        break;
    }
    case 101: case 12: case 14:  // raw IP
        if (n < 1) return false;
        if ((d[0] >> 4) == 4) et = ET_IPV4;
        else if ((d[0] >> 4) == 6) et = ET_IPV6;
        else return false;
        break;
    case 228: et = ET_IPV4; break;
    case 229: et = ET_IPV6; break;
    case 113:  // Linux cooked capture
        if (n < 16) return false;
        et = be16(d + 14);
        d += 16;
        n -= 16;
        break;
    case 276:  // Linux cooked capture v2
        if (n < 20) return false;
        et = be16(d);
        d += 20;
        n -= 20;
        break;
    case 0: {  // BSD loopback: host-order address family
        if (n < 4) return false;
        uint32_t af = rd32f(d, false);
        if (af > 0xFFFF) af = rd32f(d, true);
        if (af == 2) et = ET_IPV4;
        else if (af == 10 || af == 24 || af == 28 || af == 30) et = ET_IPV6;
        else return false;
        d += 4;
        n -= 4;
        break;
    }
    default: return false;
    }
    if (!strip_vlan_tags(et, d, n)) return false;
    return parse_l3(et, d, n, pk);
}

}  // namespace

extern "C" int ngz_pcap_open(const char *path, ngz_pcap **out) {
    if (!path || !out) return NGZ_E_INVALID;
    *out = nullptr;
    FILE *f = fopen(path, "rb");
    if (!f) return NGZ_E_INVALID;
    auto *p = new ngz_pcap();
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) p->data.insert(p->data.end(), buf, buf + k);
    fclose(f);
    const auto &d = p->data;
    if (d.size() < 24 && !(d.size() >= 12 && rd32f(d.data(), false) == 0x0A0D0D0A)) { delete p; return NGZ_E_INVALID; }
    const uint32_t m = rd32f(d.data(), false);
    if (m == 0xA1B2C3D4 || m == 0xA1B23C4D) p->be = false;
    else if (m == 0xD4C3B2A1 || m == 0x4D3CB2A1) p->be = true;
    else if (m == 0x0A0D0D0A) p->ng = true;
    else { delete p; return NGZ_E_INVALID; }
    if (!p->ng) {
        p->link_types.push_back(rd32f(d.data() + 20, p->be));
        p->pos = 24;
    }
    *out = p;
    return NGZ_OK;
}

extern "C" void ngz_pcap_close(ngz_pcap *p) { delete p; }

extern "C" int ngz_pcap_next(ngz_pcap *p, ngz_packet *pk) {
    if (!p || !pk) return NGZ_E_INVALID;
    const auto &d = p->data;
    for (;;) {
        if (p->pos >= d.size()) return 0;
        if (!p->ng) {  // legacy record: ts_sec, ts_frac, caplen, origlen, data
            if (d.size() - p->pos < 16) return NGZ_E_INVALID;
            const uint32_t caplen = rd32f(d.data() + p->pos + 8, p->be);
            if (d.size() - p->pos - 16 < caplen) return NGZ_E_INVALID;
            const uint8_t *fr = d.data() + p->pos + 16;
            p->pos += 16 + (size_t)caplen;
            p->frame++;
            memset(pk, 0, sizeof *pk);
            if (parse_frame(p->link_types[0], fr, caplen, *pk)) { pk->frame = p->frame; return 1; }
            continue;  // frames we don't extract from must not end iteration (lib.rs:158-165)
        }
        // pcapng block: type, total length, body, total length
        if (d.size() - p->pos < 12) return NGZ_E_INVALID;
        const uint8_t *b = d.data() + p->pos;
        const uint32_t type = rd32f(b, false);
        if (type == 0x0A0D0D0A) {  // section header: byte-order magic decides the section's endianness
            const uint32_t bom = rd32f(b + 8, false);
            if (bom == 0x1A2B3C4D) p->be = false;
            else if (bom == 0x4D3C2B1A) p->be = true;
            else return NGZ_E_INVALID;
            p->link_types.clear();
        }
        const uint32_t blen = rd32f(b + 4, p->be);
        if (blen < 12 || blen % 4 || blen > d.size() - p->pos) return NGZ_E_INVALID;
        p->pos += blen;
        const uint32_t t = rd32f(b, p->be);
        if (t == 1) {  // interface description: link type
            if (blen < 20) return NGZ_E_INVALID;
            p->link_types.push_back(rd16f(b + 8, p->be));
        } else if (t == 6) {  // enhanced packet
            if (blen < 32) return NGZ_E_INVALID;
            const uint32_t ifid = rd32f(b + 8, p->be);
            const uint32_t caplen = rd32f(b + 20, p->be);
            if (caplen > blen - 32 || ifid >= p->link_types.size()) return NGZ_E_INVALID;
            p->frame++;
            memset(pk, 0, sizeof *pk);
            if (parse_frame(p->link_types[ifid], b + 28, caplen, *pk)) { pk->frame = p->frame; return 1; }
        } else if (t == 3) {
            return NGZ_E_INVALID;  // simple packet block: todo!() in the reference (lib.rs:195-197)
        }
    }
}

// ---------------------------------------------------------------------------
// UDP socket ingest
// ---------------------------------------------------------------------------
extern "C" int ngz_udp_recv(int fd, uint8_t *buf, uint64_t cap, ngz_peer_key *keys, uint64_t *offsets,
                            uint32_t *lengths, uint32_t max_dgrams, int timeout_ms) {
    if (fd < 0 || !buf || !keys || !offsets || !lengths) return NGZ_E_INVALID;
    constexpr uint64_t SLOT = 65536;  // largest UDP payload, 16-byte aligned slots
    const uint32_t n = (uint32_t)std::min<uint64_t>(max_dgrams, cap / SLOT);
    if (!n) return NGZ_E_INVALID;
    if (timeout_ms != 0) {
        pollfd pf{fd, POLLIN, 0};
        const int r = poll(&pf, 1, timeout_ms < 0 ? -1 : timeout_ms);
        if (r < 0) return NGZ_E_INVALID;
        if (r == 0) return 0;
    }
    std::vector<mmsghdr> msgs(n);
    std::vector<iovec> iov(n);
    std::vector<sockaddr_storage> from(n);
    for (uint32_t i = 0; i < n; ++i) {
        iov[i].iov_base = buf + i * SLOT;
        iov[i].iov_len = SLOT;
        memset(&msgs[i], 0, sizeof msgs[i]);
        msgs[i].msg_hdr.msg_iov = &iov[i];
        msgs[i].msg_hdr.msg_iovlen = 1;
        msgs[i].msg_hdr.msg_name = &from[i];
        msgs[i].msg_hdr.msg_namelen = sizeof from[i];
    }
    const int got = recvmmsg(fd, msgs.data(), n, MSG_DONTWAIT, nullptr);
    if (got < 0) return (errno == EAGAIN || errno == EWOULDBLOCK) ? 0 : NGZ_E_INVALID;
    sockaddr_storage local{};
    socklen_t ll = sizeof local;
    getsockname(fd, (sockaddr *)&local, &ll);
    auto fill = [](const sockaddr_storage &sa, uint8_t *ip, uint16_t &port, uint8_t &fam) {
        if (sa.ss_family == AF_INET) {
            const auto *s4 = (const sockaddr_in *)&sa;
            fam = 4;
            memcpy(ip, &s4->sin_addr, 4);
            port = ntohs(s4->sin_port);
        } else if (sa.ss_family == AF_INET6) {
            const auto *s6 = (const sockaddr_in6 *)&sa;
            fam = 6;
            memcpy(ip, &s6->sin6_addr, 16);
            port = ntohs(s6->sin6_port);
        }
    };
    for (int i = 0; i < got; ++i) {
        ngz_peer_key &k = keys[i];
        memset(&k, 0, sizeof k);
        uint8_t fam_dst = 0;
        fill(from[i], k.src, k.src_port, k.family);
        fill(local, k.dst, k.dst_port, fam_dst);
        offsets[i] = (uint64_t)i * SLOT;
        lengths[i] = msgs[i].msg_len;
    }
    return got;
}

// ---------------------------------------------------------------------------
// Collector: per-peer stream framing and GPU batches
// ---------------------------------------------------------------------------
namespace {

struct KeyHash {
    size_t operator()(const ngz_peer_key &k) const {
        size_t h = 1469598103934665603ull;
        const uint8_t *p = (const uint8_t *)&k;
        for (size_t i = 0; i < sizeof k; ++i) h = (h ^ p[i]) * 1099511628211ull;
        return h;
    }
};
struct KeyEq {
    bool operator()(const ngz_peer_key &a, const ngz_peer_key &b) const { return !memcmp(&a, &b, sizeof a); }
};

struct Item {           // one queued datagram
    uint64_t off;       // in Peer::data
    uint32_t len;
    uint64_t seq;       // push order (output order)
    uint64_t tag;
};

enum MsgKind { MK_IPFIX, MK_IPFIX_SHORT, MK_NFV9, MK_OTHER };

struct Msg {            // one speculatively framed message
    uint64_t start;     // in the peer's stream buffer
    uint32_t len;       // bytes handed to the decoder
    uint32_t item;      // index of the datagram whose arrival completed it
    uint8_t kind;
    bool tail;          // more bytes followed it in the buffer when it was decoded
};

struct Line {
    uint64_t seq;
    uint64_t sub;
    uint64_t tag;
    std::string text;
};

std::string socket_addr(const uint8_t *ip, uint16_t port, uint8_t fam) {
    std::string s;
    if (fam == 6) {
        // core::net::SocketAddrV6 Display: [addr]:port
        char tmp[64];
        s = "[";  // Ipv6Addr Display, the rules of the JSON values (ngz_json.cpp)
        uint32_t g[8];
        for (int i = 0; i < 8; ++i) g[i] = ((uint32_t)ip[2 * i] << 8) | ip[2 * i + 1];
        if (!g[0] && !g[1] && !g[2] && !g[3] && !g[4] && g[5] == 0xFFFF) {
            snprintf(tmp, sizeof tmp, "::ffff:%u.%u.%u.%u", ip[12], ip[13], ip[14], ip[15]);
            s += tmp;
        } else {
            int bs = 0, bl = 0, cs = 0, cl = 0;
            for (int i = 0; i < 8; ++i) {
                if (!g[i]) { if (!cl) cs = i; if (++cl > bl) { bs = cs; bl = cl; } }
                else cl = 0;
            }
            auto grp = [&](int i) { snprintf(tmp, sizeof tmp, "%x", g[i]); s += tmp; };
            if (bl > 1) {
                for (int i = 0; i < bs; ++i) { if (i) s += ':'; grp(i); }
                s += "::";
                for (int i = bs + bl; i < 8; ++i) { if (i > bs + bl) s += ':'; grp(i); }
            } else {
                for (int i = 0; i < 8; ++i) { if (i) s += ':'; grp(i); }
            }
        }
        snprintf(tmp, sizeof tmp, "]:%u", port);
        return s + tmp;
    }
    char tmp[32];
    snprintf(tmp, sizeof tmp, "%u.%u.%u.%u:%u", ip[0], ip[1], ip[2], ip[3], port);
    return tmp;
}

}  // namespace

struct ngz_collector {
    int device = 0;
    int mode = NGZ_COLLECT_PCAP_DECODER;
    std::string err;
    struct Peer {
        ngz_peer_key key{};
        ngz_ctx *ctx = nullptr;
        std::string prefix;          // {"source_address":..,"destination_address":..,"info":
        std::vector<uint8_t> carry;  // unconsumed stream bytes (BytesMut) from earlier flushes
        std::vector<uint8_t> data;   // datagrams queued since the last flush
        std::vector<Item> items;
        uint64_t sub = 0;
    };
    std::vector<Peer *> peers;
    std::unordered_map<ngz_peer_key, size_t, KeyHash, KeyEq> index;
    uint64_t seq = 0;
    ~ngz_collector() {
        for (Peer *p : peers) {
            if (p->ctx) ngz_ctx_destroy(p->ctx);
            delete p;
        }
    }
    int fail(int code, const std::string &m) {
        err = m;
        return code;
    }
    int flush_peer(Peer &p, std::vector<Line> &out);
};

namespace {

struct JsonLine {
    int status;
    uint32_t consumed;
    std::string json;
};

// decode msgs[0..n) of `S` as one batch; with `lines`, render every message
int decode_msgs(ngz_collector *C, ngz_ctx *ctx, const std::vector<uint8_t> &S, const std::vector<Msg> &msgs, size_t n,
                std::vector<JsonLine> *lines) {
    std::vector<uint64_t> offs(n);
    std::vector<uint32_t> lens(n);
    for (size_t j = 0; j < n; ++j) {
        offs[j] = msgs[j].start;
        lens[j] = msgs[j].len;
    }
    ngz_batch_out out;
    int rc = ngz_decode_batch_host(ctx, S.data(), S.size(), offs.data(), lens.data(), (uint32_t)n, &out);
    if (rc) return C->fail(rc, std::string("decode: ") + ngz_last_error(ctx));
    if (!lines) return 0;
    JsonView v;
    rc = json_view_load(ctx, S.data(), v);
    if (rc) return C->fail(rc, "json view");
    lines->resize(n);
    for (size_t j = 0; j < n; ++j) {
        JsonLine &l = (*lines)[j];
        l.json.clear();
        l.consumed = 0;
        l.status = json_render(ctx, v, (uint32_t)j, l.json, &l.consumed);
        if (l.status < 0) return C->fail(l.status, "render");
        if (l.status == NGZ_DG_UNSUPPORTED) return C->fail(NGZ_E_LIMIT, "template not decodable on the device");
        if (l.status == NGZ_DG_NEED_MORE) return C->fail(NGZ_E_INVALID, "internal: framed message incomplete");
    }
    return 0;
}

}  // namespace

int ngz_collector::flush_peer(Peer &p, std::vector<Line> &out) {
    if (p.items.empty()) return 0;
    // the peer's stream: carried bytes, then every queued datagram
    std::vector<uint8_t> S;
    S.reserve(p.carry.size() + p.data.size() + 16);
    S.insert(S.end(), p.carry.begin(), p.carry.end());
    S.insert(S.end(), p.data.begin(), p.data.end());
    const size_t NI = p.items.size();
    std::vector<uint64_t> bnd(NI);  // stream end after datagram i arrived
    for (size_t i = 0; i < NI; ++i) bnd[i] = p.carry.size() + p.items[i].off + p.items[i].len;
    const bool clear_on_error = mode == NGZ_COLLECT_PCAP_DECODER;
    uint64_t c = 0;      // stream cursor (the BytesMut start)
    size_t it = 0;       // datagram whose arrival the decode loop is handling
    std::vector<Msg> msgs;
    std::vector<JsonLine> lines;
    for (;;) {
        // speculative framing (Decoder::decode gates, codec.rs:194-219)
        msgs.clear();
        uint64_t c_spec = c;
        for (size_t i = it; i < NI; ++i) {
            const uint64_t E = bnd[i];
            while (c_spec < E) {
                const uint64_t avail = E - c_spec;
                if (avail < 16) break;
                const uint8_t *h = S.data() + c_spec;
                const uint32_t ver = be16(h), L = be16(h + 2);
                if (avail < L) break;
                Msg m{c_spec, 0, (uint32_t)i, MK_OTHER, false};
                if (ver == 10 && L >= 16) {
                    m.kind = MK_IPFIX;
                    m.len = L;
                    m.tail = c_spec + L < E;
                    c_spec += L;  // success advances `length`; so does an error (codec.rs:158)
                } else if (ver == 10) {  // InvalidLength: advance max(5, length) (codec.rs:158)
                    m.kind = MK_IPFIX_SHORT;
                    m.len = 16;
                    c_spec = clear_on_error ? E : c_spec + std::max<uint32_t>(5, L);
                } else if (ver == 9) {  // consumed = whatever the parse read; guess: everything
                    if (avail > 0xFFFF) return fail(NGZ_E_LIMIT, "NetFlow v9 stream buffer above 65535 bytes");
                    m.kind = MK_NFV9;
                    m.len = (uint32_t)avail;
                    c_spec = E;
                } else {  // UnsupportedVersion: buffer cleared (codec.rs:214-217)
                    m.len = std::max<uint32_t>(16, L);
                    c_spec = E;
                }
                msgs.push_back(m);
            }
        }
        if (msgs.empty()) break;
        TemplateState snap;
        state_save(p.ctx, snap);
        int rc = decode_msgs(this, p.ctx, S, msgs, msgs.size(), &lines);
        if (rc) return rc;
        // verify the guesses in stream order
        size_t bad = msgs.size();
        uint64_t c_true = 0;
        for (size_t j = 0; j < msgs.size(); ++j) {
            const Msg &m = msgs[j];
            const JsonLine &l = lines[j];
            if (m.kind == MK_NFV9 && l.status == NGZ_DG_OK && l.consumed < m.len) {
                bad = j;
                c_true = m.start + l.consumed;
                break;
            }
            if (m.kind == MK_IPFIX && l.status == NGZ_DG_ERROR && m.tail && clear_on_error) {
                bad = j;
                c_true = bnd[m.item];
                break;
            }
        }
        const size_t keep = bad == msgs.size() ? bad : bad + 1;
        for (size_t j = 0; j < keep; ++j) {
            const Msg &m = msgs[j];
            Line ln{p.items[m.item].seq, p.sub++, p.items[m.item].tag, {}};
            if (mode == NGZ_COLLECT_PCAP_DECODER && lines[j].status == NGZ_DG_OK)
                ln.text = p.prefix + lines[j].json + "}";
            else
                ln.text = std::move(lines[j].json);
            out.push_back(std::move(ln));
        }
        if (bad == msgs.size()) {
            c = c_spec;
            break;
        }
        // roll back and replay the confirmed prefix, then frame again from the true cursor
        state_restore(p.ctx, snap);
        rc = decode_msgs(this, p.ctx, S, msgs, keep, nullptr);
        if (rc) return rc;
        c = c_true;
        it = msgs[bad].item;
    }
    // bytes of an incomplete message wait for the next datagram
    const uint64_t end = S.size();
    p.carry.assign(S.begin() + (ptrdiff_t)std::min(c, end), S.end());
    p.data.clear();
    p.items.clear();
    return 0;
}

extern "C" {

int ngz_collector_create(int device, int mode, ngz_collector **out) {
    if (!out || (mode != NGZ_COLLECT_PCAP_DECODER && mode != NGZ_COLLECT_FLOW_INFO)) return NGZ_E_INVALID;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return NGZ_E_DEVICE;
    auto *c = new ngz_collector();
    c->device = device;
    c->mode = mode;
    *out = c;
    return NGZ_OK;
}

void ngz_collector_destroy(ngz_collector *c) { delete c; }

const char *ngz_collector_last_error(ngz_collector *c) { return c ? c->err.c_str() : "null collector"; }

uint32_t ngz_collector_peers(ngz_collector *c) { return c ? (uint32_t)c->peers.size() : 0; }

int ngz_collector_push(ngz_collector *c, const ngz_peer_key *key, const uint8_t *payload, uint32_t len, uint64_t tag) {
    if (!c || !key || (len && !payload) || (key->family != 4 && key->family != 6)) return NGZ_E_INVALID;
    ngz_peer_key k = *key;
    memset(k.reserved, 0, sizeof k.reserved);
    if (k.family == 4) {
        memset(k.src + 4, 0, 12);
        memset(k.dst + 4, 0, 12);
    }
    auto itr = c->index.find(k);
    ngz_collector::Peer *p;
    if (itr == c->index.end()) {
        p = new ngz_collector::Peer();
        p->key = k;
        const int rc = ngz_ctx_create(c->device, &p->ctx);
        if (rc) {
            delete p;
            return c->fail(rc, "ngz_ctx_create");
        }
        // per-template kernels only for templates that carry volume (captures are mostly short)
        if (ngz_knob("NGZ_SPECIALIZE", -1) < 0) ngz_ctx_set_option(p->ctx, NGZ_OPT_SPECIALIZE, 2);
        p->prefix = "{\"source_address\":\"" + socket_addr(k.src, k.src_port, k.family) +
                    "\",\"destination_address\":\"" + socket_addr(k.dst, k.dst_port, k.family) + "\",\"info\":";
        c->index.emplace(k, c->peers.size());
        c->peers.push_back(p);
    } else {
        p = c->peers[itr->second];
    }
    p->items.push_back({p->data.size(), len, c->seq++, tag});
    p->data.insert(p->data.end(), payload, payload + len);
    return NGZ_OK;
}

int64_t ngz_collector_flush(ngz_collector *c, ngz_collect_line_fn fn, void *user) {
    if (!c || !fn) return NGZ_E_INVALID;
    std::vector<Line> lines;
    for (auto *p : c->peers) {
        const int rc = c->flush_peer(*p, lines);
        if (rc) return rc;
    }
    std::sort(lines.begin(), lines.end(),
              [](const Line &a, const Line &b) { return a.seq != b.seq ? a.seq < b.seq : a.sub < b.sub; });
    int64_t n = 0;
    for (const auto &l : lines) {
        if (fn(user, l.tag, l.text.data(), l.text.size())) break;
        ++n;
    }
    return n;
}

int64_t ngz_pcap_to_jsonl(const char *pcap_path, const uint16_t *ports, uint32_t n_ports, const char *out_path,
                          int device, int64_t input_count, int show_frame_number) {
    if (!pcap_path || (n_ports && !ports)) return NGZ_E_INVALID;
    ngz_pcap *pc = nullptr;
    int rc = ngz_pcap_open(pcap_path, &pc);
    if (rc) return rc;
    ngz_collector *col = nullptr;
    rc = ngz_collector_create(device, NGZ_COLLECT_PCAP_DECODER, &col);
    if (rc) { ngz_pcap_close(pc); return rc; }
    ngz_packet pk;
    while ((rc = ngz_pcap_next(pc, &pk)) == 1) {
        if (input_count >= 0 && pk.frame > (uint64_t)input_count) break;  // lib.rs:98-104
        if (pk.proto != NGZ_PROTO_UDP) continue;                           // handlers/flow.rs:46
        if (std::find(ports, ports + n_ports, pk.key.dst_port) == ports + n_ports) continue;
        if ((rc = ngz_collector_push(col, &pk.key, pk.payload, pk.len, pk.frame))) break;
    }
    ngz_pcap_close(pc);
    if (rc < 0) { ngz_collector_destroy(col); return rc; }
    const bool to_stdout = !out_path || !strcmp(out_path, "-");
    FILE *f = to_stdout ? stdout : fopen(out_path, "wb");
    if (!f) { ngz_collector_destroy(col); return NGZ_E_INVALID; }
    struct W {
        FILE *f;
        int frames;
    } w{f, show_frame_number};
    const int64_t n = ngz_collector_flush(col, [](void *u, uint64_t tag, const char *line, size_t len) -> int {
        W *w = (W *)u;
        if (w->frames) fprintf(w->f, "{\"frame_number\":%llu,\"data\":", (unsigned long long)tag);
        fwrite(line, 1, len, w->f);
        fputs(w->frames ? "}\n" : "\n", w->f);
        return 0;
    }, &w);
    if (!to_stdout) fclose(f);
    else fflush(f);
    if (n < 0) fprintf(stderr, "ngz_pcap_to_jsonl: %s\n", ngz_collector_last_error(col));
    ngz_collector_destroy(col);
    return n;
}

}  // extern "C"
