/* MI355X flow aggregation over decoded IPFIX / NetFlow v9 columns (C ABI).
 *
 * the step after the decode path.  One ngz_agg
 * replaces one collector shard's windowed aggregation (the AggregationActor's
 * window_aggregate over every exporter peer the shard sees, actor.rs:151-181):
 *
 *   FlowAggregator::push / flush     crates/collector/src/flow/aggregation/aggregator.rs:68-95
 *   FlowCacheRecord::reduce          aggregator.rs:159-198   (Add / Min / Max / BoolMapOr; None + Some -> Some)
 *   explode                          aggregator.rs:286-354   (one AggFlowInfo per data record, FieldRef lookup)
 *   FieldRef::map_fields             crates/collector/src/flow/types.rs:82-100 (index = occurrence of the IE
 *                                                             among the record's non-scope fields)
 *   WindowAggregator::process_item   crates/analytics/src/aggregation.rs:124-172 (lateness drop, window start)
 *   get_window_start                 aggregation.rs:79-89    (timestamp floored to the minute)
 *   validate_operation_compatibility aggregation/config.rs:212-250, generator.rs:580-629
 *
 *   AggFlowInfo::into_flowinfo_with_extra_fields  aggregator.rs:203-277 + actor.rs:222-240 (ngz_agg_flowinfo_json)
 *
 * The group table lives in HBM and persists across ngz_agg_push calls; one
 * aggregator serves every exporter peer of a shard.  Records are grouped by
 * (peer IP, window start, flow type, key fields) exactly -- FlowCacheKey is
 * (peer_ip, flow_type, key_fields) and the window aggregator keys its windows by
 * peer IP (aggregator.rs:109-124, aggregation.rs:96-108): keys are compared,
 * never identified by a hash.  Each peer IP has its own event time: a record
 * whose message export time is more than `lateness` behind its peer's event time
 * is late and is counted, not aggregated (aggregation.rs:139-141), and a peer's
 * windows whose start is at or before get_window_start(its event time -
 * lateness) - window_duration are closed (aggregation.rs:154-160), independently
 * of the other peers: ngz_agg_emit hands the groups of closed windows out and
 * frees their room; ngz_agg_flush hands out every group (WindowAggregator::flush).
 *
 * A push is all-or-nothing: when it fails (NGZ_AGG_E_OVERFLOW, NGZ_E_LIMIT, ...)
 * the groups, the set dictionaries and the event times are as they were before
 * it.  Only a device error or an internal inconsistency poisons the aggregator
 * (NGZ_AGG_E_POISONED from then on, until ngz_agg_reset).
 */
#ifndef NGZ_FLOW_AGGREGATE_H
#define NGZ_FLOW_AGGREGATE_H

#include <stddef.h>
#include <stdint.h>

#include "ngz/flow_decode.h"

#ifdef __cplusplus
extern "C" {
#endif

#define NGZ_AGG_ABI_VERSION 4 /* 2: ngz_agg_create takes max_peers, ngz_agg_push a const ngz_peer * (the
                                 exporter's address; 1 took a uint16 port); 3: byte-valued keys and values
                                 of any length (kkind 3, vclass 8 / 9, ngz_agg_row_bytes); 4:
                                 ngz_agg_set_option */

/* NGZ_AGG_ABI_VERSION the library was built with (checked by hosts like ngz_abi_version). */
int ngz_agg_abi_version(void);

/* Transform ops (config.rs Op).  KEY selects a key field; the others an aggregated field. */
#define NGZ_AGG_KEY 0
#define NGZ_AGG_ADD 1
#define NGZ_AGG_MIN 2
#define NGZ_AGG_MAX 3
#define NGZ_AGG_OR 4 /* BoolMapOr */

#define NGZ_AGG_MAX_KEYS 16
#define NGZ_AGG_MAX_VALUES 32
#define NGZ_AGG_MAX_KEY_BYTES 128   /* sum of key row slots (see ngz_agg_key_desc) */
#define NGZ_AGG_SET_BITS 64         /* distinct template ids / peer ports among the live groups; 128 observation
                                       domains (entries no live group uses are reused) */
#define NGZ_AGG_MAX_PEERS 65536     /* distinct exporter peer IPs between two flushes */

#define NGZ_AGG_E_OVERFLOW (-10)    /* more groups than the capacity, a set dictionary full of live entries, or
                                       more peer IPs than max_peers */
#define NGZ_AGG_E_COLLISION (-11)   /* no longer returned: hash collisions are resolved by comparing keys */
#define NGZ_AGG_E_POISONED (-12)    /* an earlier device error / internal inconsistency; ngz_agg_reset clears it */

/* One transform entry: (IE, occurrence index) -> op  (FieldRef + Op, config.rs:152-176). */
typedef struct {
    uint32_t pen;      /* 0 = IANA */
    uint16_t ie_id;
    uint16_t index;    /* FieldRef index */
    uint8_t op;        /* NGZ_AGG_* */
    uint8_t reserved[7];
} ngz_agg_field;

typedef struct ngz_agg ngz_agg;

/* An exporter peer (std::net::SocketAddr, the `peer` of explode, aggregator.rs:286-292):
 * the IP keys the groups and the windows, the port joins the groups' peer_ports set. */
typedef struct {
    uint8_t family;      /* 4 or 6 */
    uint8_t reserved;
    uint16_t port;
    uint8_t addr[16];    /* network order; IPv4 in addr[0..3] */
} ngz_peer;

/* Validates the config like AggregationConfig::validate + validate_operation_compatibility
 * (window > 0, lateness <= window; the op allowed by IE::supports_{arithmetic,comparison,
 * bitwise}_ops, generator.rs:1176-1272 -- data type, sub-registry and dataTypeSemantics
 * identifier/flags): NGZ_E_INVALID where the reference rejects the config.  Every config the
 * reference accepts runs (NGZ_E_LIMIT only beyond the compiled limits: NGZ_AGG_MAX_KEYS /
 * NGZ_AGG_MAX_VALUES, capacity, max_peers).  Key fields keep their order (key_select), aggregated
 * fields theirs (agg_select).  capacity: live groups held at most, up to 2^30 (the HBM table
 * has at least twice as many slots).  max_peers: distinct peer IPs the aggregator takes
 * between flushes (0 = NGZ_AGG_MAX_PEERS); a small bound leaves more bits of the exact
 * 63-bit group tag to the key fields. */
int ngz_agg_create(int device, const ngz_agg_field *fields, uint32_t n_fields, uint64_t window_ms,
                   uint64_t lateness_ms, uint64_t capacity, uint32_t max_peers, ngz_agg **out);
void ngz_agg_destroy(ngz_agg *a);
const char *ngz_agg_last_error(ngz_agg *a);

/* Explode + push every data record of the batch last decoded on ctx (out from
 * ngz_decode_batch), in datagram order: the FlowInfos one peer sent (a context is one
 * peer's FlowInfoCodec).  peer: its address (a new IP beyond max_peers is
 * NGZ_AGG_E_OVERFLOW); collection_time_ms is the batch's collection time
 * (min/max_collection_time).  Records of failed messages are not pushed (they yield no
 * FlowInfo).  *late_records (may be NULL) receives the records dropped as late.
 * hip_stream: the stream the batch was decoded on (NULL = the context's stream is
 * synchronised by ngz_decode_batch already).  Variable-length key / value cells point into the
 * batch's input bytes (NGZ_K_VLEN): the bytes given to ngz_decode_batch must stay valid and
 * unchanged until ngz_agg_push returns (a host that recycles its H2D buffers pushes first). */
int ngz_agg_push(ngz_agg *a, ngz_ctx *ctx, const ngz_batch_out *out, const ngz_peer *peer,
                 int64_t collection_time_ms, uint64_t *late_records, void *hip_stream);

/* One flushed group (host).  Key and value bytes follow at key_off / val_off of the row
 * (ngz_agg_layout).  Set members are bits into the dictionaries of ngz_agg_sets. */
typedef struct {
    uint32_t window_start;      /* seconds, minute-floored (get_window_start) */
    uint8_t flow_type;          /* 10 IPFIX / 9 NetFlow v9 */
    uint8_t reserved0;
    uint16_t peer;              /* the group's peer IP: entry of ngz_agg_peer */
    uint32_t key_present;       /* bit k: key field k is Some */
    uint32_t val_present;       /* bit v: aggregated field v is Some */
    uint64_t record_count;
    uint32_t min_export_time;   /* seconds */
    uint32_t max_export_time;
    uint32_t max_sys_up_time;
    uint32_t take_id;           /* which ngz_agg_flush / ngz_agg_emit call returned the row (1, 2, ...):
                                   ngz_agg_row_bytes reads byte values of the last call's rows only */
    int64_t min_collection_ms;
    int64_t max_collection_ms;
    uint64_t template_bits;     /* DataSetId set */
    uint64_t port_bits;         /* peer_ports set */
    uint64_t domain_bits[2];    /* observation_domain_ids set */
} ngz_agg_row;

/* Row layout of ngz_agg_flush output: row_bytes per group (a multiple of 128: whole
 * cache lines in the device table); the
 * ngz_agg_row header, 8 bytes of device bookkeeping, then key field k at key_off[k]
 * (column width of the IE, rounded to 4; width in key_width[k]: 0 if the
 * field never appeared), value v at val_off[v] (8 bytes; OR of byte fields: width
 * rounded to 4, in val_width[v]).  Integer values are little-endian at the IE's
 * Rust width (adds wrap at that width, as release-mode `+=`). */
int ngz_agg_layout(ngz_agg *a, uint32_t *row_bytes, uint32_t *key_off, uint16_t *key_width, uint32_t *val_off,
                   uint16_t *val_width);

/* Number of groups held. */
int64_t ngz_agg_groups(ngz_agg *a);

/* Copies every group (unordered) into dst (cap bytes, row_bytes each), then empties
 * the table, the set dictionaries, and forgets every peer and its event time
 * (WindowAggregator::flush).  Returns the groups written or <0 (NGZ_E_INVALID: cap too
 * small; nothing is emptied). */
int64_t ngz_agg_flush(ngz_agg *a, void *dst, uint64_t cap);

/* Groups of the windows their peer's event time has closed (aggregation.rs:154-160), and
 * the emission of those groups: copied into dst like ngz_agg_flush, then removed.  The
 * reference emits a closed window from the process_item call that closes it; here the
 * windows closed by a push are emitted after it, with the same contents (an item is
 * never late for a window that is still open, and never lands in a closed one).
 * ngz_agg_emit returns the groups handed out; if rebuilding the table afterwards fails,
 * the aggregator is poisoned (the next call reports it), the groups are still out. */
int64_t ngz_agg_closed(ngz_agg *a);
int64_t ngz_agg_emit(ngz_agg *a, void *dst, uint64_t cap);

/* Empties the aggregator and clears a poisoned state. */
int ngz_agg_reset(ngz_agg *a);

/* Set dictionaries of the rows last returned by ngz_agg_flush / ngz_agg_emit: template
 * ids (proto<<16 | id), peer ports and observation domain ids, entry i <-> bit i (free
 * entries read all-ones).  Each array receives up to cap entries; returns 0. */
int ngz_agg_sets(ngz_agg *a, uint32_t *templates, uint32_t *n_templates, uint16_t *ports, uint32_t *n_ports,
                 uint32_t *domains, uint32_t *n_domains, uint32_t cap);

/* The peer IP of output rows (ngz_agg_row.peer) last returned by ngz_agg_flush /
 * ngz_agg_emit (port: that of the push that first brought the IP).  out may be NULL.
 * Returns the number of peers, or NGZ_E_INVALID for an index beyond them. */
int ngz_agg_peer(ngz_agg *a, uint32_t index, ngz_peer *out);

/* How a key / value is stored in an output row.
 * Key kkind: 0 the decoded column cell (width bytes); 3 a byte value of any length (string,
 * octetArray, list and unknown IEs; fixed or variable-length on the wire): u32 length, u32
 * reserved, then the first 32 bytes (zero padded) -- the whole value through
 * ngz_agg_row_bytes.  A string key is its text: a fixed-length cell up to its first NUL
 * (Field::String, generator.rs:1654-1669), a variable-length one as sent, so the same text
 * declared at different lengths or variable-length is one key.  (kkinds 1 and 2 are no
 * longer produced.)
 * Value vclass: 0 unsigned / 1 signed integer (little-endian at the IE width, the
 * Rust type's wrap-around for Add), 2 dateTime micro/nanoseconds (u64 secs<<32 | nanos),
 * 3 bytes (OR of a fixed-size type: macAddress, ipv6Address, unsigned256, MPLS label),
 * 4 sub-registry / TCP flags value (little-endian at the width), 5 f32, 6 f64, 7 IPv6
 * address (16 bytes, network order), 8 octetArray BoolMapOr, 9 list Min / Max (both in the
 * kkind 3 form: length, reserved, first 32 bytes; ngz_agg_row_bytes for all of them).
 * kind: the decoded column kind (NGZ_K_*) and width the column width, both as first seen
 * (0 before). */
typedef struct {
    uint8_t kkind;
    uint8_t kind;
    uint16_t slot;      /* row bytes */
    uint16_t width;
    uint16_t reserved;
} ngz_agg_key_desc;
typedef struct {
    uint8_t vclass;
    uint8_t kind;
    uint16_t width;
    uint32_t reserved;
} ngz_agg_value_desc;
int ngz_agg_key_info(ngz_agg *a, uint32_t k, ngz_agg_key_desc *out);
int ngz_agg_value_info(ngz_agg *a, uint32_t v, ngz_agg_value_desc *out);

/* The whole byte value of key k (is_value 0, kkind 3) or aggregated field v (is_value 1,
 * vclass 8 / 9) of an output row of the last ngz_agg_flush / ngz_agg_emit call: up to cap
 * bytes into dst (may be NULL); returns the value's length, or NGZ_E_INVALID.  Byte values can be
 * read only until the next flush / emit: the tails come from that call's copy.  A row of an
 * earlier call (its take_id is not the last call's) is NGZ_E_INVALID, and ngz_agg_flowinfo_json
 * then fails with NGZ_E_INVALID instead of printing another row's bytes. */
int64_t ngz_agg_row_bytes(ngz_agg *a, const void *row, int is_value, uint32_t index, uint8_t *dst, uint64_t cap);

/* AggFlowInfo::into_flowinfo_with_extra_fields (aggregator.rs:203-277) of output rows,
 * with the extra fields the aggregation actor always passes (actor.rs:222-240), for the
 * n rows of one ngz_agg_flush / ngz_agg_emit call, read with that call's dictionaries:
 * one FlowInfo per group, as the serde JSON text of the decode path (ngz_batch_json):
 * an IPFIX or NetFlow v9 packet whose one data set (id 65535) holds one record: the
 * present key fields, the present aggregated fields, originalFlowsPresent,
 * minExportSeconds, maxExportSeconds, collectionTimeMilliseconds (the max), NetGauze
 * windowStart and windowEnd (window start + window duration),
 * originalExporterIPv4Address / originalExporterIPv6Address (the group's peer IP), then
 * one NetGauze originalExporterTransportPort per peer port, one
 * originalObservationDomainId per domain and one NetGauze originalTemplateId per template
 * id, each set in ascending order (the reference iterates HashSets: unspecified order).
 * Packet header: export time export_time_ms (the reference uses Utc::now()), sequence
 * numbers seq0, seq0+1, ..., observation domain / source id shard_id, NetFlow v9
 * sys_up_time = the group's max.  fn gets (row index, NGZ_DG_OK, text, length).  Returns
 * rows rendered or <0. */
int64_t ngz_agg_flowinfo_json(ngz_agg *a, const void *rows, uint64_t n, uint32_t shard_id, uint32_t seq0,
                              int64_t export_time_ms, ngz_json_line_fn fn, void *user);

/* Aggregator options (ngz_agg_set_option).  They choose how a push reduces, never what it
 * computes: every choice gives the same groups (tests/test_gpu_agg.py runs them against each
 * other and the oracle).  The library reads no tuning from the environment. */
#define NGZ_AGG_OPT_LOWCARD 1    /* -1 (default): the low-cardinality path from 2^16 records; 0 never;
                                    1 at any size (where the config allows it) */
#define NGZ_AGG_OPT_PARTITION 2  /* -1 (default): the partitioned reduction for many groups with at least 8
                                    records each per push; 0 never; 1 whenever the config allows it */
#define NGZ_AGG_OPT_OWNER 3      /* 1 (default): per-record owner rows where groups get few records per
                                    push; 0 never */
#define NGZ_AGG_OPT_HASH_BITS 4  /* 0 (default): the full 64-bit hash of hashed keys; 1..63: only that many
                                    bits, so distinct keys collide (tests of the exact key compare).  Only
                                    while the aggregator holds no group (NGZ_E_INVALID otherwise). */
int ngz_agg_set_option(ngz_agg *a, int opt, int64_t value);

/* Device time of the last push (HIP events around its kernels), milliseconds. */
int ngz_agg_last_timing(ngz_agg *a, float *push_ms);

/* The reduction path the last push took: "lowcard" (packed keys with at most 8 distinct
 * key tuples: per-set LDS reduction, no per-record atomics), "general", or "none" (no
 * record to reduce). */
const char *ngz_agg_last_path(ngz_agg *a);

#ifdef __cplusplus
}
#endif
#endif
