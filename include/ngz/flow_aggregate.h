/* MI355X flow aggregation over decoded IPFIX / NetFlow v9 columns (C ABI).
 *
 * the step after the decode path.  One ngz_agg
 * replaces the collector's per-peer windowed FlowAggregator:
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
 * The group table lives in HBM and persists across ngz_agg_push calls; one
 * aggregator serves one exporter peer IP (the window key, aggregator.rs:109-117).
 * Records are grouped by (window start, flow type, key fields); a record whose
 * message export time is more than `lateness` behind the peer's event time is
 * late and is counted, not aggregated (aggregation.rs:139-141).  Window
 * contents do not depend on when windows are flushed, so
 * ngz_agg_flush returns every group at once, as WindowAggregator::flush does.
 */
#ifndef NGZ_FLOW_AGGREGATE_H
#define NGZ_FLOW_AGGREGATE_H

#include <stddef.h>
#include <stdint.h>

#include "ngz/flow_decode.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Transform ops (config.rs Op).  KEY selects a key field; the others an aggregated field. */
#define NGZ_AGG_KEY 0
#define NGZ_AGG_ADD 1
#define NGZ_AGG_MIN 2
#define NGZ_AGG_MAX 3
#define NGZ_AGG_OR 4 /* BoolMapOr */

#define NGZ_AGG_MAX_KEYS 16
#define NGZ_AGG_MAX_VALUES 32
#define NGZ_AGG_MAX_KEY_BYTES 128   /* sum of key column widths, each rounded up to 4 */
#define NGZ_AGG_SET_BITS 64         /* distinct template ids / peer ports; 128 observation domains */

#define NGZ_AGG_E_OVERFLOW (-10)    /* group table full (capacity) or a set dictionary is full */
#define NGZ_AGG_E_COLLISION (-11)   /* two distinct keys share a 64-bit key hash (detected, ~1e-8 per 1e6 groups) */

/* One transform entry: (IE, occurrence index) -> op  (FieldRef + Op, config.rs:152-176). */
typedef struct {
    uint32_t pen;      /* 0 = IANA */
    uint16_t ie_id;
    uint16_t index;    /* FieldRef index */
    uint8_t op;        /* NGZ_AGG_* */
    uint8_t reserved[7];
} ngz_agg_field;

typedef struct ngz_agg ngz_agg;

/* Validates the config like AggregationConfig::validate + validate_operation_compatibility
 * (window > 0, lateness <= window, op allowed for the IE's data type).  Key fields keep
 * their order (key_select), aggregated fields theirs (agg_select).  capacity: groups the
 * HBM table holds (rounded up to a power of two; the table is half full at most). */
int ngz_agg_create(int device, const ngz_agg_field *fields, uint32_t n_fields, uint64_t window_ms,
                   uint64_t lateness_ms, uint64_t capacity, ngz_agg **out);
void ngz_agg_destroy(ngz_agg *a);
const char *ngz_agg_last_error(ngz_agg *a);

/* Explode + push every data record of the batch last decoded on ctx (out from
 * ngz_decode_batch), in datagram order.  peer_port joins peer_ports; collection_time_ms
 * is the batch's collection time (min/max_collection_time).  Records of failed
 * messages are not pushed (they yield no FlowInfo).  *late_records (may be NULL)
 * receives the records dropped as late.  hip_stream: the stream the batch was decoded
 * on (NULL = the context's stream is synchronised by ngz_decode_batch already). */
int ngz_agg_push(ngz_agg *a, ngz_ctx *ctx, const ngz_batch_out *out, uint16_t peer_port,
                 int64_t collection_time_ms, uint64_t *late_records, void *hip_stream);

/* One flushed group (host).  Key and value bytes follow at key_off / val_off of the row
 * (ngz_agg_layout).  Set members are bits into the dictionaries of ngz_agg_sets. */
typedef struct {
    uint32_t window_start;      /* seconds, minute-floored (get_window_start) */
    uint8_t flow_type;          /* 10 IPFIX / 9 NetFlow v9 */
    uint8_t reserved0[3];
    uint32_t key_present;       /* bit k: key field k is Some */
    uint32_t val_present;       /* bit v: aggregated field v is Some */
    uint64_t record_count;
    uint32_t min_export_time;   /* seconds */
    uint32_t max_export_time;
    uint32_t max_sys_up_time;
    uint32_t reserved1;
    int64_t min_collection_ms;
    int64_t max_collection_ms;
    uint64_t template_bits;     /* DataSetId set */
    uint64_t port_bits;         /* peer_ports set */
    uint64_t domain_bits[2];    /* observation_domain_ids set */
} ngz_agg_row;

/* Row layout of ngz_agg_flush output: row_bytes per group; key field k at
 * key_off[k] (column width of the IE, rounded to 4; width in key_width[k]: 0 if the
 * field never appeared), value v at val_off[v] (8 bytes; OR of byte fields: width
 * rounded to 4, in val_width[v]).  Integer values are little-endian at the IE's
 * Rust width (adds wrap at that width, as release-mode `+=`). */
int ngz_agg_layout(ngz_agg *a, uint32_t *row_bytes, uint32_t *key_off, uint16_t *key_width, uint32_t *val_off,
                   uint16_t *val_width);

/* Number of groups held. */
int64_t ngz_agg_groups(ngz_agg *a);

/* Copies every group (unordered) into dst (cap bytes, row_bytes each), then empties
 * the table and forgets the peer's event time (WindowAggregator::flush).  Returns the
 * groups written or <0 (NGZ_E_INVALID: cap too small; nothing is emptied). */
int64_t ngz_agg_flush(ngz_agg *a, void *dst, uint64_t cap);

/* Set dictionaries: template ids (proto<<16 | id), peer ports and observation domain
 * ids, in bit order.  Each array receives up to cap entries; returns 0. */
int ngz_agg_sets(ngz_agg *a, uint32_t *templates, uint32_t *n_templates, uint16_t *ports, uint32_t *n_ports,
                 uint32_t *domains, uint32_t *n_domains, uint32_t cap);

/* Device time of the last push (HIP events around its kernels), milliseconds. */
int ngz_agg_last_timing(ngz_agg *a, float *push_ms);

#ifdef __cplusplus
}
#endif
#endif
