/*
 * netgauze_amd — MI355X-native IPFIX (v10) / NetFlow v9 data-record decoder.
 *
 * C ABI (plain pointers and sizes, no HIP or torch types in the signatures).
 * This is the drop-in boundary for the reference's decode path:
 *
 *   ngz_ctx                 ≙ netgauze_flow_pkt::codec::FlowInfoCodec
 *                             (crates/flow-pkt/src/codec.rs:68-73): one per
 *                             exporter peer, owns the NetFlow v9 and IPFIX
 *                             TemplatesMap (ipfix.rs:73, netflow.rs).
 *   ngz_decode_batch        ≙ FlowCollectorActor::decode_pkt applied to each
 *                             datagram of a batch, in order
 *                             (crates/flow-service/src/flow_actor.rs:342-411):
 *                             one FlowInfoCodec::decode (codec.rs:189-220)
 *                             per datagram -> IpfixPacket::parse
 *                             (wire/deserializer/ipfix.rs:54-104) /
 *                             NetFlowV9Packet::parse (netflow.rs:56-114) ->
 *                             Set::parse -> DataRecord::parse ->
 *                             Field::parse (generated, generator.rs:2901-2980).
 *                             Decoded fields land in per-template columnar
 *                             arrays in HBM instead of Box<[Field]> per record.
 *   ngz_template_counts     ≙ DecodingTemplate::processed_count /
 *                             reset_processed_count (ipfix.rs:55-69), read by
 *                             flow_actor.rs:362-381.
 *   ngz_dgram_error_json    ≙ serde_json::to_string(&FlowInfoCodecDecoderError)
 *                             for a datagram whose decode returned Err.
 *
 * Error convention (mirrors the reference): the first error aborts the whole
 * message; template definitions parsed before the error persist.  Return codes
 * are ints (0 = ok, <0 = NGZ_E_*); no exceptions cross the ABI.  A context is
 * not thread-safe; distinct contexts may be used concurrently.
 */
#ifndef NGZ_FLOW_DECODE_H
#define NGZ_FLOW_DECODE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NGZ_ABI_VERSION 6  /* 2: ngz_slot_info.n_fields is 32-bit (no field cap), ngz_dgram_error,
                              ngz_template_counts_device; 3: ngz_abi_version, ngz_ctx_destroy joins the
                              context's background compiles; 4: ngz_columns_to_host_async;
                              5: ngz_record_fields; 6: ngz_decode_batch_submit / _wait */

/* return codes */
#define NGZ_OK 0
#define NGZ_E_INVALID (-1)     /* bad argument */
#define NGZ_E_DEVICE (-2)      /* HIP runtime error */
#define NGZ_E_NOMEM (-3)       /* device allocation failed */
#define NGZ_E_LIMIT (-4)       /* batch exceeds a compiled limit */

/* per-datagram status (ngz_dgram_hdr.status) */
#define NGZ_DG_OK 0            /* Ok(Some(FlowInfo)) */
#define NGZ_DG_NEED_MORE 1     /* Ok(None): shorter than 16 B or than the header length */
#define NGZ_DG_ERROR 2         /* Err(FlowInfoCodecDecoderError), see ngz_dgram_error_json */
#define NGZ_DG_UNSUPPORTED 3   /* a data set of a template whose fixed record is longer than 65535 bytes
                                  (NGZ_MAX_REC_LEN; every other template is decoded on the device) */

/* field decode kinds (ngz_field_info.kind); column encodings in DESIGN.md */
#define NGZ_K_UINT 1      /* big-endian unsigned, reduced size, zero-extended to width */
#define NGZ_K_TCPFLAGS 2  /* tcpControlBits: u16 (len 1|2) truncated to u8 */
#define NGZ_K_SINT 3      /* big-endian signed, sign-extended to width */
#define NGZ_K_BOOL 4      /* u8 0/1 */
#define NGZ_K_BYTES 5     /* raw wire bytes, width = wire length */
#define NGZ_K_U256 6      /* <=32 bytes left-aligned, zero-padded to 32 */
#define NGZ_K_DTMS 7      /* dateTimeMilliseconds -> i64 millis, range-checked */
#define NGZ_K_DTFRAC 8    /* dateTimeMicro/Nanoseconds -> {u32 secs, u32 nanos} */
#define NGZ_K_STR 9       /* fixed string: raw bytes, NUL-truncated prefix UTF-8 checked */
#define NGZ_K_SCOPE32 10  /* NFv9 System/Interface/LineCard scope: reduced u32 (len<=4) */
#define NGZ_K_VLEN 11     /* variable-length field (65535): column = {u64 offset into the batch bytes,
                             u32 value length, u32 0}; strings UTF-8 checked */
#define NGZ_K_FAIL 12     /* always fails with a template-constant error */

typedef struct ngz_ctx ngz_ctx;

/* One batch of datagrams already resident in device memory.  `offsets` and
 * `lengths` are device arrays of n entries; datagram i is
 * bytes[offsets[i] .. offsets[i]+lengths[i]).  bytes_size bounds every read. */
typedef struct {
    const uint8_t *bytes;
    uint64_t bytes_size;
    const uint64_t *offsets;
    const uint32_t *lengths;
    uint32_t n;
} ngz_batch_in;

/* Per-datagram message header + status (device array in ngz_batch_out). */
typedef struct {
    uint8_t status;       /* NGZ_DG_* */
    uint8_t version;      /* 10 = IPFIX, 9 = NetFlow v9, 0 otherwise */
    uint16_t length;      /* IPFIX header length / NFv9 header count */
    uint32_t time;        /* IPFIX export_time / NFv9 unix_time (seconds) */
    uint32_t sequence;    /* sequence_number */
    uint32_t domain;      /* IPFIX observation_domain_id / NFv9 source_id */
    uint32_t sys_up_time; /* NFv9 only */
    uint32_t n_sets;      /* sets parsed (all kinds) */
    uint64_t err_key;     /* first error, internal encoding; ~0 if none */
} ngz_dgram_hdr;

/* One data set, in stream order (device array in ngz_batch_out). */
typedef struct {
    uint32_t dgram;       /* datagram index */
    uint16_t set_pos;     /* byte offset of the set header in the datagram */
    uint16_t slot;        /* batch template slot (ngz_slot_info) */
    uint32_t rec0;        /* first record's row in the slot's columns */
    uint32_t n;           /* records */
} ngz_set_info;

/* Where one template version's records landed. */
typedef struct {
    uint32_t version_id;  /* context-unique template version id */
    uint16_t template_id;
    uint8_t proto;        /* 10 or 9 */
    uint8_t reserved;
    uint32_t n_records;   /* rows filled in this batch */
    uint32_t capacity;    /* rows allocated (column stride is capacity*width) */
    uint8_t *columns;     /* device base; column f at columns + capacity*col_off[f] */
    uint32_t n_fields;    /* scope + non-scope fields (columns); no cap */
    uint32_t reserved2;
} ngz_slot_info;

typedef struct {
    uint16_t wire_offset;  /* offset inside the record (0xFFFF after a vlen field) */
    uint16_t wire_length;  /* declared length (65535 = variable) */
    uint16_t width;        /* column bytes per record */
    uint8_t kind;          /* NGZ_K_* */
    uint8_t is_scope;
    uint32_t col_off;      /* column offset factor (bytes per row before this column) */
    uint32_t pen;          /* IE enterprise number (0 = IANA) */
    uint16_t ie_id;        /* IE id (NFv9 scope ids keep their raw code) */
    uint16_t reserved;
} ngz_field_info;

typedef struct {
    uint32_t n_dgrams;
    uint32_t n_sets;
    uint32_t n_slots;
    uint64_t n_records;          /* all records of all slots (incl. failed messages) */
    const ngz_dgram_hdr *dgrams; /* device, n_dgrams */
    const ngz_set_info *sets;    /* device, n_sets */
    const ngz_slot_info *slots;  /* HOST array, n_slots */
    uint32_t n_template_dgrams;  /* datagrams with (options) template sets */
} ngz_batch_out;

/* NGZ_ABI_VERSION the library was built with: a host checks it against the header it was
 * compiled with before any other call. */
int ngz_abi_version(void);

/* --- context ------------------------------------------------------------ */
int ngz_ctx_create(int device, ngz_ctx **out);
/* Synchronous, as the reference codec's drop (codec.rs:68-82): waits for the
 * context's stream and joins every background template compile the context
 * started or was waiting on, so a host may return from main right after. */
void ngz_ctx_destroy(ngz_ctx *ctx);
const char *ngz_last_error(ngz_ctx *ctx);

/* Context options (ngz_ctx_set_option). */
#define NGZ_OPT_SPECIALIZE 1    /* 1 (default): decode each template with its own kernel, generated and
                                   compiled at run time (hiprtc) and cached by layout; 0: the generic
                                   field-table kernel for every template; 2: generic kernel until a
                                   template has decoded 65536 records, then its own kernel (short
                                   captures skip the 0.1-0.3 s compile per template) */
#define NGZ_OPT_BLOCKS_PER_CU 2 /* decode grid size: 256-thread blocks per CU (default 4) */
#define NGZ_OPT_CAP_PAD 4       /* extra row windows of column capacity per template slot (column spacing) */
#define NGZ_OPT_ARENA_SHIFT 3   /* bytes (multiple of 256) the column blocks start into the context's
                                   device arena: moves the output onto other HBM pages */
#define NGZ_OPT_RTC_SYNC 5      /* 0 (default): a template's kernel compiles on a background thread and the
                                   generic kernel decodes its records until it is ready (a new template on
                                   one peer never stalls a batch); 1: the first batch after a template
                                   definition waits for its compile (deterministic kernel choice) */
#define NGZ_OPT_SPLIT 6         /* 1: split framing in steady state -- the record walk of variable-length
                                   sets on a second stream beside the fixed-length sets' framing and
                                   decode (measured slower on config 4); 0 (default) */
#define NGZ_OPT_GROUP 7         /* 1: one multi-template decode launch per workgroup shape for the
                                   LDS-staged templates of a batch (ngz_group_kernel); 0 (default): one
                                   launch per template */
#define NGZ_OPT_PLACE_TRIALS 8  /* column arenas tried for a context's first large batch, the fastest
                                   kept (1..16, default 6; 1 = no trials, DESIGN.md §2 "Arena placement") */
#define NGZ_OPT_PLACE_PROBE 9   /* how a placement trial is timed: 0 the batch's decode on each arena; 1 a
                                   probe of the decode's memory streams over a fraction of the windows (one
                                   decode in all, on the kept arena); 2 both, the decodes decide (diagnostics) */
/* Options change how a batch runs, never its results.  The library reads no tuning from the
 * environment (only NGZ_DEBUG, stderr traces). */
int ngz_ctx_set_option(ngz_ctx *ctx, int opt, int64_t value);

/* Wait for every background template compile of the process (NGZ_OPT_RTC_SYNC 0) to finish
 * and load.  A compile still inside hiprtc/comgr when the C exit handlers run can outlive
 * the compiler's own static objects, which exit destroys in an order the library cannot
 * control.  ngz_ctx_destroy (and so ngz_collector_destroy / ngz_pcap_to_jsonl) already
 * joins its context's compiles; this is for hosts that exit with contexts still alive (the
 * Python binding registers it with atexit).  Returns the number of compiles waited for. */
int ngz_rtc_drain(void);

/* --- decode ------------------------------------------------------------- */
/* Decode every datagram of `in` in order against the context's template
 * state.  Synchronous: on return the device arrays in *out are complete and
 * stay valid until the next ngz_decode_batch on this context.
 * hip_stream: a hipStream_t (NULL = the context's own stream). */
int ngz_decode_batch(ngz_ctx *ctx, const ngz_batch_in *in, ngz_batch_out *out, void *hip_stream);

/* ngz_decode_batch without blocking the caller: the context's decode worker (one host thread per
 * context, started on first use) runs it, and ngz_decode_batch_wait returns its result once *out
 * is filled.  One host thread can so keep batches of several contexts in flight, each context on
 * its own stream, as a collector with one socket thread does (FlowCollectorActor's loop).  Until
 * the wait returns, the context takes no other call and *in / *out / the input bytes must stay
 * valid.  Returns NGZ_OK when queued, NGZ_E_INVALID if a batch is already pending. */
int ngz_decode_batch_submit(ngz_ctx *ctx, const ngz_batch_in *in, ngz_batch_out *out, void *hip_stream);

/* Wait for the batch ngz_decode_batch_submit queued on ctx: ngz_decode_batch's return code, or
 * NGZ_E_INVALID when nothing is pending. */
int ngz_decode_batch_wait(ngz_ctx *ctx);

/* Same, with the datagrams in host memory (pinned staging, H2D included). */
int ngz_decode_batch_host(ngz_ctx *ctx, const uint8_t *bytes, uint64_t bytes_size,
                          const uint64_t *offsets, const uint32_t *lengths, uint32_t n,
                          ngz_batch_out *out);

/* Which kernel decoded a slot of the last batch: 1 its specialised kernel,
 * 0 the generic kernel, 2 the generic kernel while its own compiles. */
int ngz_slot_kernel(ngz_ctx *ctx, uint32_t slot);

/* How the last batch ran (bits): NGZ_BATCH_PREDICTED decode launched without a host round trip
 * (steady state), NGZ_BATCH_SPLIT split framing (the record walk of variable-length sets on a
 * second stream beside the fixed-length sets' framing and decode), NGZ_BATCH_RERUN a pass was
 * repeated (buffer growth, a template slot without a count row, a record error split framing
 * went past).  Returns the bits, or NGZ_E_INVALID. */
/* Data records each of n host-memory messages carries under the context's current templates
 * (no device work, nothing decoded or learnt): per data set, its payload over the template's
 * record length, or the framing's record walk for a variable-length template; sets of unknown
 * templates count nothing.  For the multi-GPU shard plan (contiguous message
 * ranges balanced by record count, netgauze_amd/dist.py shard_by_records), the reference's
 * analogue being how the supervisor spreads exporter peers over actors (flow_supervisor.rs:288-305).
 * Returns NGZ_OK or NGZ_E_INVALID. */
int ngz_message_records(ngz_ctx *ctx, const uint8_t *bytes, const uint64_t *offsets, const uint32_t *lengths,
                        uint32_t n, uint32_t *records);

/* The arena placement of the context's first large batch (NGZ_OPT_PLACE_TRIALS, DESIGN.md §2
 * "Arena placement"): per trial arena, in trial order, the batch's decode milliseconds into
 * decode_ms[0, cap) and the probe's into probe_ms[0, cap) (either may be NULL; 0 where the trial
 * did not run it, NGZ_OPT_PLACE_PROBE), and in *kept (may be NULL) the trial whose arena the
 * context kept.  Returns the number of trials: 0 before the placement ran (or with one trial). */
int ngz_placement_trials(ngz_ctx *ctx, float *decode_ms, float *probe_ms, uint32_t cap, uint32_t *kept);

#define NGZ_BATCH_PREDICTED 1
#define NGZ_BATCH_SPLIT 2
#define NGZ_BATCH_RERUN 4
int ngz_last_batch_info(ngz_ctx *ctx);

/* Column layout of a batch slot (valid with the last batch). */
int ngz_slot_fields(ngz_ctx *ctx, uint32_t slot, ngz_field_info *fields, uint32_t cap);

/* serde_json text of the datagram's FlowInfoCodecDecoderError (status ERROR).
 * Returns the string length (excluding NUL) or <0. */
int ngz_dgram_error_json(ngz_ctx *ctx, uint32_t dgram, char *buf, size_t cap);

/* Structured FlowInfoCodecDecoderError of a datagram (status ERROR): the
 * innermost reference error variant and its fields, the layer it was raised
 * in, and the IE it concerns.  It carries the same information as the serde
 * text of ngz_dgram_error_json (which it is derived from), so a host binding
 * can rebuild the reference's nested error enums without parsing JSON:
 *   layer CODEC    FlowInfoCodecDecoderError::UnsupportedVersion (codec.rs:214-217)
 *         MESSAGE  IpfixPacketParsingError / NetFlowV9PacketParsingError (ipfix.rs:54-104, netflow.rs:56-114)
 *         SET      SetParsingError / SetError (ipfix.rs:133-251, netflow.rs:143-248)
 *         TEMPLATE (Options)TemplateRecordError, FieldSpecifierError, ScopeFieldSpecifierError
 *                  (ipfix.rs:276-327,384-413, netflow.rs:265-388, deserializer/mod.rs:50-67)
 *         RECORD   DataRecordError -> FieldError / ScopeFieldError (ipfix.rs:335-370, netflow.rs:399-475)
 * Field meaning per kind (offset is always the absolute message offset the
 * reference reports; NGZ_ERR_INVALID_LENGTH's length is the bad length):
 *   UNSUPPORTED_VERSION value=version | UNEXPECTED_EOF length=needed, available |
 *   INVALID_PADDING_LENGTH length=requested, value=ret_len | INVALID_SET_ID value=id |
 *   NO_TEMPLATE value=template id | INVALID_PADDING_VALUE value | INVALID_COUNT value=count |
 *   INVALID_TEMPLATE_ID value=template id | INVALID_SCOPE_FIELDS_COUNT value=scope count, length=total |
 *   UNDEFINED_IANA_IE ie_id | INVALID_TIMESTAMP value=seconds | INVALID_TIMESTAMP_MILLIS value=millis |
 *   INVALID_TIMESTAMP_FRACTION value=seconds, length=fraction | UTF8 offset of the string. */
#define NGZ_ERR_NONE 0
#define NGZ_ERR_UNSUPPORTED_VERSION 1
#define NGZ_ERR_INVALID_LENGTH 2
#define NGZ_ERR_UNEXPECTED_EOF 3
#define NGZ_ERR_INVALID_PADDING_LENGTH 4
#define NGZ_ERR_INVALID_SET_ID 5
#define NGZ_ERR_NO_TEMPLATE 6
#define NGZ_ERR_INVALID_PADDING_VALUE 7
#define NGZ_ERR_INVALID_COUNT 8
#define NGZ_ERR_INVALID_TEMPLATE_ID 9
#define NGZ_ERR_INVALID_SCOPE_FIELDS_COUNT 10
#define NGZ_ERR_UNDEFINED_IANA_IE 11
#define NGZ_ERR_INVALID_TIMESTAMP 12
#define NGZ_ERR_INVALID_TIMESTAMP_MILLIS 13
#define NGZ_ERR_INVALID_TIMESTAMP_FRACTION 14
#define NGZ_ERR_UTF8 15

#define NGZ_ERRL_CODEC 0
#define NGZ_ERRL_MESSAGE 1
#define NGZ_ERRL_SET 2
#define NGZ_ERRL_TEMPLATE 3
#define NGZ_ERRL_RECORD 4

typedef struct {
    uint16_t kind;       /* NGZ_ERR_* */
    uint8_t layer;       /* NGZ_ERRL_* */
    uint8_t vendor;      /* 1: wrapped in the IE vendor's error ({Vendor}Error, generator.rs:2875-2895) */
    uint32_t offset;     /* absolute byte offset in the message */
    uint64_t value;      /* per kind, above */
    uint32_t length;     /* per kind, above */
    uint32_t available;  /* UNEXPECTED_EOF */
    uint32_t ie_pen;     /* IE the error concerns (field / specifier errors), else 0 */
    uint16_t ie_id;
    uint16_t field;      /* RECORD layer: field index in the template (scope first), else 0xFFFF */
} ngz_error;

/* Returns 0 and fills *err for a datagram with status ERROR; NGZ_E_INVALID otherwise. */
int ngz_dgram_error(ngz_ctx *ctx, uint32_t dgram, ngz_error *err);

/* serde_json text of the datagram's decoded FlowInfo (status OK) or of its
 * FlowInfoCodecDecoderError (status ERROR), rendered from the last batch's
 * columns: the reference's `serde_json::to_string(&flow_info)` for the same
 * bytes (FlowInfo / IpfixPacket / NetFlowV9Packet Serialize, ipfix.rs:99-108,
 * 212-221, 419-424; crates/pcap-decoder/src/handlers/mod.rs:64-80).  The whole
 * batch is copied to the host on the first call after a decode.  Returns the
 * length (excluding NUL; buf is truncated to cap) or <0 (NGZ_E_INVALID for
 * NEED_MORE / UNSUPPORTED datagrams). */
int64_t ngz_dgram_json(ngz_ctx *ctx, uint32_t dgram, char *buf, size_t cap);

/* One decoded field of a record: the reference's `Field` value (DataRecord::parse ->
 * Box<[Field]>, ipfix.rs:335-370, 419-424; NFv9 scope fields ScopeField, netflow.rs:443-475)
 * as the IE that names its variant plus the typed value in the canonical column encoding
 * (the NGZ_K_* list above).  A host builds the `Field` from (pen, ie_id, kind, value)
 * without parsing JSON (INTEGRATION.md §2 `ColumnarBatch::record`). */
#define NGZ_FV_SCOPE 1u      /* a scope field (IPFIX options scope / NFv9 ScopeField) */
#define NGZ_FV_STRING 2u     /* NGZ_K_VLEN / NGZ_K_STR: a UTF-8 string (String), else octets (Box<[u8]>) */
#define NGZ_FV_VENDOR 4u     /* the IE is in a vendor package (Field::<Vendor>(..), generator.rs:2915-2924) */
#define NGZ_FV_UNKNOWN 8u    /* IE::Unknown{pen, id} or a vendor package's Unknown{id}: raw bytes */
#define NGZ_FV_SUBREG 16u    /* the value is a sub-registry enum (From<int>, lossless) */
#define NGZ_FV_MPLS 32u      /* an MPLS label IE ([u8; 3]) */
#define NGZ_FV_TCPFLAGS 64u  /* tcpControlBits (TCPHeaderFlags from the low byte) */
/* IPFIX data types (dtype; the registry's, RFC 7012 s3.1 order) */
#define NGZ_DT_OCTET_ARRAY 0
#define NGZ_DT_UNSIGNED8 1
#define NGZ_DT_UNSIGNED16 2
#define NGZ_DT_UNSIGNED32 3
#define NGZ_DT_UNSIGNED64 4
#define NGZ_DT_SIGNED8 5
#define NGZ_DT_SIGNED16 6
#define NGZ_DT_SIGNED32 7
#define NGZ_DT_SIGNED64 8
#define NGZ_DT_FLOAT32 9
#define NGZ_DT_FLOAT64 10
#define NGZ_DT_BOOLEAN 11
#define NGZ_DT_MAC_ADDRESS 12
#define NGZ_DT_STRING 13
#define NGZ_DT_DATETIME_SECONDS 14
#define NGZ_DT_DATETIME_MILLISECONDS 15
#define NGZ_DT_DATETIME_MICROSECONDS 16
#define NGZ_DT_DATETIME_NANOSECONDS 17
#define NGZ_DT_IPV4_ADDRESS 18
#define NGZ_DT_IPV6_ADDRESS 19
#define NGZ_DT_BASIC_LIST 20
#define NGZ_DT_SUB_TEMPLATE_LIST 21
#define NGZ_DT_SUB_TEMPLATE_MULTI_LIST 22
#define NGZ_DT_UNSIGNED256 23
typedef struct {
    uint32_t pen;          /* IE enterprise number (0 = IANA) */
    uint16_t ie_id;        /* IE id (NFv9 scope fields: the raw scope code) */
    uint8_t kind;          /* NGZ_K_*: the decode rule that produced `value` */
    uint8_t dtype;         /* NGZ_DT_*: the IE's data type (octetArray for unknown IEs and NFv9 scopes) */
    uint16_t wire_length;  /* declared length (65535 = variable length) */
    uint16_t width;        /* column width */
    uint32_t len;          /* bytes at `value`: the width, a fixed string's bytes before its first NUL,
                              a variable-length field's value length */
    uint32_t wire_offset;  /* where the value starts in its datagram (after a vlen prefix) */
    uint32_t flags;        /* NGZ_FV_* */
    uint32_t reserved;
    const uint8_t *value;  /* host memory, valid until the context's next decode: the column cell, or
                              for NGZ_K_VLEN the value's bytes in the batch input */
} ngz_field_value;

/* The fields of record `rec` of data set `set` (its index among datagram `dgram`'s data sets) of
 * the last batch, scope fields first, into out[0, cap).  Returns the field count (> cap: only cap
 * written), or NGZ_E_INVALID (datagram not NGZ_DG_OK, set or record out of range).  The first call
 * after a decode copies the batch's columns to the host (as ngz_dgram_json). */
int ngz_record_fields(ngz_ctx *ctx, uint32_t dgram, uint32_t set, uint32_t rec, ngz_field_value *out, uint32_t cap);

/* Line callback of ngz_batch_json: datagram index, NGZ_DG_OK / NGZ_DG_ERROR,
 * the JSON text (not NUL-terminated), and the bytes FlowInfoCodec::decode
 * consumed from the datagram (codec.rs:151-183).  Non-zero return stops. */
typedef int (*ngz_json_line_fn)(void *user, uint32_t dgram, int status, const char *json, size_t len,
                                uint32_t consumed);

/* Render every datagram of the last batch that produced a FlowInfo or an
 * error, in datagram order (one D2H of headers, sets and columns).
 * host_bytes: the batch bytes in host memory (for variable-length values), or
 * NULL to copy them from the device.  Returns the lines emitted or <0. */
int64_t ngz_batch_json(ngz_ctx *ctx, const uint8_t *host_bytes, ngz_json_line_fn fn, void *user);

/* Template introspection: serde_json text of the current template map for one
 * protocol (10 or 9): [{"id":..,"scope_field_specifiers":[..],"field_specifiers":[..]},..]. */
int ngz_templates_json(ngz_ctx *ctx, int proto, char *buf, size_t cap);

/* processed_count of the current templates of one protocol (10 or 9):
 * fills ids[i], counts[i] for up to cap templates; reset != 0 zeroes them
 * afterwards (reset_processed_count).  Returns the number of templates. */
int ngz_template_counts(ngz_ctx *ctx, int proto, uint16_t *ids, uint64_t *counts, uint32_t cap, int reset);

/* The same table written to DEVICE memory, ready for a collective (the
 * per-template count exchange behind templates.usage, flow_actor.rs:362-381):
 * dev_table[2*i] = template id, dev_table[2*i+1] = processed_count, ids
 * ascending, entries [n, cap) zeroed.  One host-to-device copy queued on
 * hip_stream (NULL = the context's stream): an ncclAllGather / ncclAllReduce
 * queued after it on that stream sees the table, with no host synchronisation.
 * reset as ngz_template_counts, but only when all n templates fit (n <= cap).
 * Returns the number of templates n (> cap: only the first cap were written
 * and nothing was reset; re-agree the table size and call again). */
int ngz_template_counts_device(ngz_ctx *ctx, int proto, uint64_t *dev_table, uint32_t cap, int reset,
                               void *hip_stream);

/* Timing of the last ngz_decode_batch: device milliseconds of the record
 * decode kernel and of the whole device pipeline (HIP events). */
int ngz_last_timing(ngz_ctx *ctx, float *decode_ms, float *pipeline_ms);

/* D2H of the last batch's columns into host memory `dst` (pinned for full
 * PCIe rate): the column block of every slot with records, in slot order,
 * each ngz_slot_info.capacity * (sum of column widths) bytes, starting at a
 * multiple of 256 bytes.  Copied on the context's stream; returns the bytes
 * written, or <0 (NGZ_E_INVALID: cap too small). */
int64_t ngz_columns_to_host(ngz_ctx *ctx, void *dst, uint64_t cap);

/* ngz_columns_to_host queued on hip_stream (NULL = the context's stream) without waiting for it:
 * the copy starts once the last batch's decode is done, and the context's next ngz_decode_batch /
 * ngz_decode_batch_host waits for the copy before it reuses the columns.  Returns the bytes queued.
 * flags: NGZ_D2H_KERNEL copies with a kernel whose stores cross PCIe to dst (dst must be pinned host
 * memory mapped for the device: hipHostMalloc, or hipHostRegister with hipHostRegisterMapped;
 * NGZ_E_INVALID otherwise), leaving the copy engines to the next batch's host-to-device copy so the
 * link carries both directions at once; 0 uses a copy engine. */
#define NGZ_D2H_KERNEL 1u
int64_t ngz_columns_to_host_async(ngz_ctx *ctx, void *dst, uint64_t cap, void *hip_stream, uint32_t flags);

/* Introspection (no device needed): the per-template decode kernel for one
 * IPFIX template record (template id u16, field count u16, field specifiers;
 * the body of a template set entry, ipfix.rs:384-413).  Writes the generated
 * HIP source to buf (NUL-terminated, truncated to cap) and, with compile bit 0,
 * compiles it for gfx950 with hiprtc (the build log follows the source on
 * failure).  compile bit 1: the record is a NetFlow v9 template record of the
 * same layout (netflow.rs:324-353), decoded by the NFv9 kernel shape.  Returns 0 on success, NGZ_E_INVALID if the template does not
 * parse or is not device-decodable, NGZ_E_DEVICE if compilation failed. */
int ngz_template_kernel(const uint8_t *tmpl, size_t len, int compile, char *buf, size_t cap);

/* Introspection (no device needed): the multi-template decode kernel of 2-16 IPFIX
 * template records laid back to back (a template set's body, ipfix.rs:384-413) that
 * are all LDS-staged with one workgroup shape -- the one launch ngz_decode_batch uses
 * for such templates of one batch.  As ngz_template_kernel; NGZ_E_INVALID when the
 * records do not form such a group. */
int ngz_group_kernel(const uint8_t *tmpls, size_t len, int compile, char *buf, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
