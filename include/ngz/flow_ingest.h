/*
 * netgauze_amd — host ingest in front of the MI355X decoder (C ABI).
 *
 * The reference feeds its FlowInfoCodec from two places, both restated here:
 *
 *   ngz_pcap_*        ≙ netgauze_pcap_reader::PcapIter
 *                       (crates/pcap-reader/src/lib.rs:97-377): legacy pcap and
 *                       pcapng, Ethernet / raw IP / Linux cooked captures,
 *                       802.1Q / QinQ tags, IPv4 / IPv6, UDP / TCP payloads
 *                       (IPv4 UDP trimmed to the UDP length, lib.rs:303-323).
 *   ngz_udp_recv      ≙ the collector's UDP socket read loop
 *                       (crates/flow-service/src/flow_actor.rs:828-883), batched
 *                       with recvmmsg(2) into one contiguous buffer.
 *   ngz_collector_*   ≙ the per-exporter-peer codec map of the pcap decoder and
 *                       the flow pcap tests: one FlowInfoCodec + BytesMut per
 *                       (src ip, src port, dst ip, dst port)
 *                       (crates/pcap-decoder/src/handlers/flow.rs:37-59,
 *                       handlers/mod.rs:36-80; wire/tests/pcap_tests.rs:79-118).
 *                       Datagrams are queued per peer and decoded on the GPU in
 *                       one batch per peer per flush; output lines come back in
 *                       push order.
 *   ngz_pcap_to_jsonl ≙ `pcap-decoder --protocol flow`
 *                       (crates/pcap-decoder/src/lib.rs:65-127, main.rs:62-95).
 *
 * Return codes are the NGZ_E_* of flow_decode.h.  Objects are not thread-safe.
 */
#ifndef NGZ_FLOW_INGEST_H
#define NGZ_FLOW_INGEST_H

#include <stddef.h>
#include <stdint.h>

#include "ngz/flow_decode.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Exporter peer: the reference's flow_key (IpAddr, u16, IpAddr, u16). */
typedef struct {
    uint8_t family;    /* 4 or 6 */
    uint8_t reserved[3];
    uint8_t src[16];   /* IPv4 in src[0..4], network order */
    uint8_t dst[16];
    uint16_t src_port;
    uint16_t dst_port;
} ngz_peer_key;

#define NGZ_PROTO_TCP 6
#define NGZ_PROTO_UDP 17

/* One transport payload out of a capture (borrowed until the next call). */
typedef struct {
    ngz_peer_key key;
    uint8_t proto;          /* NGZ_PROTO_UDP / NGZ_PROTO_TCP */
    uint8_t reserved[7];
    uint64_t frame;         /* PcapIter::frame_counter after this frame (1-based) */
    const uint8_t *payload;
    uint32_t len;
    uint32_t reserved2;
} ngz_packet;

/* --- pcap reader ------------------------------------------------------- */
typedef struct ngz_pcap ngz_pcap;
int ngz_pcap_open(const char *path, ngz_pcap **out);
/* 1 = *pkt filled, 0 = end of capture, <0 = malformed file / unsupported block. */
int ngz_pcap_next(ngz_pcap *p, ngz_packet *pkt);
void ngz_pcap_close(ngz_pcap *p);

/* --- collector (per-peer stream framing + GPU batches) ----------------- */
/* Output lines of ngz_collector_flush: the pcap decoder's
 * {"source_address":..,"destination_address":..,"info":<FlowInfo>} for a
 * decoded message and the bare FlowInfoCodecDecoderError JSON for an error;
 * the peer's buffer is cleared after an error (handlers/mod.rs:36-60). */
#define NGZ_COLLECT_PCAP_DECODER 0
/* The flow pcap tests' lines: bare FlowInfo / error JSON; after an error only
 * the codec's own advance applies (pcap_tests.rs:79-118, codec.rs:155-217). */
#define NGZ_COLLECT_FLOW_INFO 1

typedef struct ngz_collector ngz_collector;
/* tag: the value given to ngz_collector_push for the datagram whose arrival
 * completed the message (the pcap frame number, for instance). */
typedef int (*ngz_collect_line_fn)(void *user, uint64_t tag, const char *line, size_t len);

int ngz_collector_create(int device, int mode, ngz_collector **out);
void ngz_collector_destroy(ngz_collector *c);
const char *ngz_collector_last_error(ngz_collector *c);
/* Queue one UDP payload from `key` (copied). */
int ngz_collector_push(ngz_collector *c, const ngz_peer_key *key, const uint8_t *payload, uint32_t len, uint64_t tag);
/* Decode everything queued (one GPU batch per peer) and emit the lines in
 * push order.  Bytes of an incomplete trailing message stay buffered for the
 * next flush, as in the reference's BytesMut.  Returns lines emitted or <0. */
int64_t ngz_collector_flush(ngz_collector *c, ngz_collect_line_fn fn, void *user);
/* Exporter peers seen so far. */
uint32_t ngz_collector_peers(ngz_collector *c);

/* --- UDP socket ingest ------------------------------------------------- */
/* recvmmsg(2) up to max_dgrams datagrams from a bound UDP socket into
 * buf[0..cap) (each datagram at a 16-byte aligned offset); fills keys[i]
 * (src = sender, dst = local address/port), offsets[i], lengths[i].
 * timeout_ms < 0 blocks until the first datagram; 0 polls.  Returns the
 * number received (0 on timeout) or <0. */
int ngz_udp_recv(int fd, uint8_t *buf, uint64_t cap, ngz_peer_key *keys, uint64_t *offsets, uint32_t *lengths,
                 uint32_t max_dgrams, int timeout_ms);

/* --- pcap-decoder --protocol flow ------------------------------------- */
/* Decode every UDP payload of the capture whose destination port is in
 * ports[0..n_ports) and write one JSON line per decode outcome to out_path
 * (NULL or "-": stdout).  input_count >= 0 stops at the first yielded frame
 * whose frame counter exceeds it (lib.rs:98-104); show_frame_number wraps each
 * line as {"frame_number":N,"data":..}.  Returns lines written or <0. */
int64_t ngz_pcap_to_jsonl(const char *pcap_path, const uint16_t *ports, uint32_t n_ports, const char *out_path,
                          int device, int64_t input_count, int show_frame_number);

#ifdef __cplusplus
}
#endif
#endif
