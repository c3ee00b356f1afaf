"""ctypes binding of the C ABI in include/ngz/flow_decode.h and flow_ingest.h (libngz.so).

The library is built in-tree by __graft_entry__.build() (hipcc, gfx950).  If
it is missing this module raises at import: there is no CPU fallback.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libngz.so")
# NGZ_EXPERIMENTS=1 (tools only): the experiment build, libngz_exp.so (tools/build_experiments.sh),
# whose knobs are read from NGZ_<name> variables for A/B measurements; NGZ_EXPERIMENTS=<name>:
# libngz_exp_<name>.so, a variant built with extra compile-time defines.  Never the product path.
# They are built outside the package (tools/exp/), so a stray variable in a collector's
# environment finds nothing to load unless a developer built one, and loading one says so.
if os.environ.get("NGZ_EXPERIMENTS"):
    import sys as _sys
    _x = os.environ["NGZ_EXPERIMENTS"]
    LIB_PATH = os.path.join(os.path.dirname(HERE), "tools", "exp",
                            "libngz_exp.so" if _x == "1" else "libngz_exp_%s.so" % _x)
    print("netgauze_amd: NGZ_EXPERIMENTS=%s loads the EXPERIMENT build %s (A/B knobs; timing variants "
          "decode wrong on purpose) -- not the product library" % (_x, LIB_PATH), file=_sys.stderr)

NGZ_DG_OK, NGZ_DG_NEED_MORE, NGZ_DG_ERROR, NGZ_DG_UNSUPPORTED = 0, 1, 2, 3
(K_UINT, K_TCPFLAGS, K_SINT, K_BOOL, K_BYTES, K_U256, K_DTMS, K_DTFRAC, K_STR,
 K_SCOPE32, K_VLEN, K_FAIL) = range(1, 13)

# every function the header declares (tests check the exports)
ABI_FUNCTIONS = [
    "ngz_ctx_create", "ngz_ctx_destroy", "ngz_last_error", "ngz_decode_batch",
    "ngz_decode_batch_host", "ngz_slot_fields", "ngz_dgram_error_json",
    "ngz_templates_json", "ngz_template_counts", "ngz_last_timing", "ngz_ctx_set_option",
    "ngz_template_kernel", "ngz_group_kernel", "ngz_columns_to_host", "ngz_columns_to_host_async", "ngz_dgram_json", "ngz_batch_json",
    "ngz_dgram_error", "ngz_template_counts_device", "ngz_slot_kernel", "ngz_rtc_drain", "ngz_abi_version",
    "ngz_last_batch_info", "ngz_record_fields", "ngz_placement_trials",
    "ngz_message_records", "ngz_decode_batch_submit", "ngz_decode_batch_wait",
]
NGZ_ABI_VERSION = 6
# ngz_field_value.flags
FV_SCOPE, FV_STRING, FV_VENDOR, FV_UNKNOWN, FV_SUBREG, FV_MPLS, FV_TCPFLAGS = 1, 2, 4, 8, 16, 32, 64
NGZ_BATCH_PREDICTED, NGZ_BATCH_SPLIT, NGZ_BATCH_RERUN = 1, 2, 4  # ngz_last_batch_info
# ngz_ctx_set_option
(NGZ_OPT_SPECIALIZE, NGZ_OPT_BLOCKS_PER_CU, NGZ_OPT_ARENA_SHIFT, NGZ_OPT_CAP_PAD, NGZ_OPT_RTC_SYNC, NGZ_OPT_SPLIT,
 NGZ_OPT_GROUP, NGZ_OPT_PLACE_TRIALS) = range(1, 9)
NGZ_AGG_ABI_VERSION = 4
# ngz_error.kind / .layer (flow_decode.h)
ERR_KINDS = ["NONE", "UNSUPPORTED_VERSION", "INVALID_LENGTH", "UNEXPECTED_EOF", "INVALID_PADDING_LENGTH",
             "INVALID_SET_ID", "NO_TEMPLATE", "INVALID_PADDING_VALUE", "INVALID_COUNT", "INVALID_TEMPLATE_ID",
             "INVALID_SCOPE_FIELDS_COUNT", "UNDEFINED_IANA_IE", "INVALID_TIMESTAMP", "INVALID_TIMESTAMP_MILLIS",
             "INVALID_TIMESTAMP_FRACTION", "UTF8"]
ERR_LAYERS = ["CODEC", "MESSAGE", "SET", "TEMPLATE", "RECORD"]
# include/ngz/flow_ingest.h
INGEST_FUNCTIONS = [
    "ngz_pcap_open", "ngz_pcap_next", "ngz_pcap_close", "ngz_collector_create", "ngz_collector_destroy",
    "ngz_collector_last_error", "ngz_collector_push", "ngz_collector_flush", "ngz_collector_peers",
    "ngz_udp_recv", "ngz_pcap_to_jsonl",
]
# include/ngz/flow_aggregate.h
AGG_FUNCTIONS = [
    "ngz_agg_create", "ngz_agg_destroy", "ngz_agg_last_error", "ngz_agg_push", "ngz_agg_layout",
    "ngz_agg_groups", "ngz_agg_flush", "ngz_agg_closed", "ngz_agg_emit", "ngz_agg_reset", "ngz_agg_sets",
    "ngz_agg_key_info", "ngz_agg_value_info", "ngz_agg_flowinfo_json", "ngz_agg_last_timing", "ngz_agg_peer", "ngz_agg_last_path",
    "ngz_agg_abi_version", "ngz_agg_row_bytes", "ngz_agg_set_option",
]
NGZ_AGG_KEY, NGZ_AGG_ADD, NGZ_AGG_MIN, NGZ_AGG_MAX, NGZ_AGG_OR = range(5)
NGZ_AGG_E_OVERFLOW, NGZ_AGG_E_COLLISION, NGZ_AGG_E_POISONED = -10, -11, -12
NGZ_AGG_OPT_LOWCARD, NGZ_AGG_OPT_PARTITION, NGZ_AGG_OPT_OWNER, NGZ_AGG_OPT_HASH_BITS = 1, 2, 3, 4
# ngz_agg_key_desc.kkind / ngz_agg_value_desc.vclass
AGG_KK_FIXED, AGG_KK_BYTES = 0, 3
(AGG_VC_UINT, AGG_VC_SINT, AGG_VC_DTFRAC, AGG_VC_BYTES, AGG_VC_RANK, AGG_VC_F32, AGG_VC_F64, AGG_VC_IPV6,
 AGG_VC_VBYTES, AGG_VC_VLIST) = range(10)
NGZ_COLLECT_PCAP_DECODER, NGZ_COLLECT_FLOW_INFO = 0, 1
NGZ_PROTO_TCP, NGZ_PROTO_UDP = 6, 17

# ngz_json_line_fn(user, dgram, status, json, len, consumed)
JSON_LINE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int,
                                ctypes.POINTER(ctypes.c_char), ctypes.c_size_t, ctypes.c_uint32)
# ngz_collect_line_fn(user, tag, line, len)
COLLECT_LINE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_char),
                                   ctypes.c_size_t)


class PeerKey(ctypes.Structure):
    _fields_ = [("family", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 3), ("src", ctypes.c_uint8 * 16),
                ("dst", ctypes.c_uint8 * 16), ("src_port", ctypes.c_uint16), ("dst_port", ctypes.c_uint16)]


class Packet(ctypes.Structure):
    _fields_ = [("key", PeerKey), ("proto", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 7),
                ("frame", ctypes.c_uint64), ("payload", ctypes.POINTER(ctypes.c_uint8)), ("len", ctypes.c_uint32),
                ("reserved2", ctypes.c_uint32)]


class BatchIn(ctypes.Structure):
    _fields_ = [("bytes", ctypes.c_void_p), ("bytes_size", ctypes.c_uint64),
                ("offsets", ctypes.c_void_p), ("lengths", ctypes.c_void_p), ("n", ctypes.c_uint32)]


class SlotInfo(ctypes.Structure):
    _fields_ = [("version_id", ctypes.c_uint32), ("template_id", ctypes.c_uint16),
                ("proto", ctypes.c_uint8), ("reserved", ctypes.c_uint8),
                ("n_records", ctypes.c_uint32), ("capacity", ctypes.c_uint32),
                ("columns", ctypes.c_void_p), ("n_fields", ctypes.c_uint32), ("reserved2", ctypes.c_uint32)]


class BatchOut(ctypes.Structure):
    _fields_ = [("n_dgrams", ctypes.c_uint32), ("n_sets", ctypes.c_uint32), ("n_slots", ctypes.c_uint32),
                ("n_records", ctypes.c_uint64), ("dgrams", ctypes.c_void_p), ("sets", ctypes.c_void_p),
                ("slots", ctypes.POINTER(SlotInfo)), ("n_template_dgrams", ctypes.c_uint32)]


class Error(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_uint16), ("layer", ctypes.c_uint8), ("vendor", ctypes.c_uint8),
                ("offset", ctypes.c_uint32), ("value", ctypes.c_uint64), ("length", ctypes.c_uint32),
                ("available", ctypes.c_uint32), ("ie_pen", ctypes.c_uint32), ("ie_id", ctypes.c_uint16),
                ("field", ctypes.c_uint16)]


assert ctypes.sizeof(Error) == 32


class FieldInfo(ctypes.Structure):
    _fields_ = [("wire_offset", ctypes.c_uint16), ("wire_length", ctypes.c_uint16), ("width", ctypes.c_uint16),
                ("kind", ctypes.c_uint8), ("is_scope", ctypes.c_uint8), ("col_off", ctypes.c_uint32),
                ("pen", ctypes.c_uint32), ("ie_id", ctypes.c_uint16), ("reserved", ctypes.c_uint16)]


class FieldValue(ctypes.Structure):
    """ngz_field_value: one decoded field of a record (ngz_record_fields)."""
    _fields_ = [("pen", ctypes.c_uint32), ("ie_id", ctypes.c_uint16), ("kind", ctypes.c_uint8),
                ("dtype", ctypes.c_uint8), ("wire_length", ctypes.c_uint16), ("width", ctypes.c_uint16),
                ("len", ctypes.c_uint32), ("wire_offset", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32), ("value", ctypes.c_void_p)]


assert ctypes.sizeof(FieldValue) == 40


class AggField(ctypes.Structure):
    _fields_ = [("pen", ctypes.c_uint32), ("ie_id", ctypes.c_uint16), ("index", ctypes.c_uint16),
                ("op", ctypes.c_uint8), ("reserved", ctypes.c_uint8 * 7)]


class AggKeyDesc(ctypes.Structure):
    _fields_ = [("kkind", ctypes.c_uint8), ("kind", ctypes.c_uint8), ("slot", ctypes.c_uint16),
                ("width", ctypes.c_uint16), ("reserved", ctypes.c_uint16)]


class AggValueDesc(ctypes.Structure):
    _fields_ = [("vclass", ctypes.c_uint8), ("kind", ctypes.c_uint8), ("width", ctypes.c_uint16),
                ("reserved", ctypes.c_uint32)]


assert ctypes.sizeof(AggKeyDesc) == 8 and ctypes.sizeof(AggValueDesc) == 8


class Peer(ctypes.Structure):
    """ngz_peer: an exporter's SocketAddr."""
    _fields_ = [("family", ctypes.c_uint8), ("reserved", ctypes.c_uint8), ("port", ctypes.c_uint16),
                ("addr", ctypes.c_uint8 * 16)]

    @classmethod
    def of(cls, ip, port):
        import ipaddress
        a = ipaddress.ip_address(ip)
        p = cls()
        p.family = a.version
        p.port = port
        b = a.packed
        for i, x in enumerate(b):
            p.addr[i] = x
        return p

    def ip(self):
        import ipaddress
        b = bytes(self.addr)
        return str(ipaddress.ip_address(b[:4] if self.family == 4 else b))


assert ctypes.sizeof(Peer) == 20

AGG_ROW_DTYPE = np.dtype([("window_start", "<u4"), ("flow_type", "u1"), ("reserved0", "u1"), ("peer", "<u2"),
                          ("key_present", "<u4"), ("val_present", "<u4"), ("record_count", "<u8"),
                          ("min_export_time", "<u4"), ("max_export_time", "<u4"), ("max_sys_up_time", "<u4"),
                          ("take_id", "<u4"), ("min_collection_ms", "<i8"), ("max_collection_ms", "<i8"),
                          ("template_bits", "<u8"), ("port_bits", "<u8"), ("domain_bits", "<u8", 2)])
assert AGG_ROW_DTYPE.itemsize == 88


DGRAM_HDR_DTYPE = np.dtype([("status", "u1"), ("version", "u1"), ("length", "<u2"), ("time", "<u4"),
                            ("sequence", "<u4"), ("domain", "<u4"), ("sys_up_time", "<u4"),
                            ("n_sets", "<u4"), ("err_key", "<u8")])
SET_INFO_DTYPE = np.dtype([("dgram", "<u4"), ("set_pos", "<u2"), ("slot", "<u2"), ("rec0", "<u4"), ("n", "<u4")])
assert DGRAM_HDR_DTYPE.itemsize == 32 and SET_INFO_DTYPE.itemsize == 16


_DRAIN_REGISTERED = False


def load():
    if not os.path.exists(LIB_PATH):
        raise RuntimeError("netgauze_amd: %s is missing — run __graft_entry__.build() (hipcc, gfx950); "
                           "there is no CPU fallback" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    P, U32, U64, I = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    # the structs and signatures below are those of NGZ_ABI_VERSION / NGZ_AGG_ABI_VERSION: a library
    # built from other headers is refused before any call that could misread an argument
    lib.ngz_abi_version.argtypes, lib.ngz_abi_version.restype = [], I
    lib.ngz_agg_abi_version.argtypes, lib.ngz_agg_abi_version.restype = [], I
    got = (lib.ngz_abi_version(), lib.ngz_agg_abi_version())
    if got != (NGZ_ABI_VERSION, NGZ_AGG_ABI_VERSION):
        raise RuntimeError("netgauze_amd: %s has ABI versions %s, this binding needs %s -- rebuild it"
                           % (LIB_PATH, got, (NGZ_ABI_VERSION, NGZ_AGG_ABI_VERSION)))
    lib.ngz_ctx_create.argtypes = [I, ctypes.POINTER(P)]
    lib.ngz_ctx_create.restype = I
    lib.ngz_ctx_destroy.argtypes = [P]
    lib.ngz_ctx_destroy.restype = None
    lib.ngz_last_error.argtypes = [P]
    lib.ngz_last_error.restype = ctypes.c_char_p
    lib.ngz_decode_batch.argtypes = [P, ctypes.POINTER(BatchIn), ctypes.POINTER(BatchOut), P]
    lib.ngz_decode_batch.restype = I
    lib.ngz_decode_batch_submit.argtypes = [P, ctypes.POINTER(BatchIn), ctypes.POINTER(BatchOut), P]
    lib.ngz_decode_batch_submit.restype = I
    lib.ngz_decode_batch_wait.argtypes = [P]
    lib.ngz_decode_batch_wait.restype = I
    lib.ngz_decode_batch_host.argtypes = [P, P, U64, P, P, U32, ctypes.POINTER(BatchOut)]
    lib.ngz_decode_batch_host.restype = I
    lib.ngz_slot_fields.argtypes = [P, U32, ctypes.POINTER(FieldInfo), U32]
    lib.ngz_slot_fields.restype = I
    lib.ngz_dgram_error_json.argtypes = [P, U32, ctypes.c_char_p, ctypes.c_size_t]
    lib.ngz_dgram_error_json.restype = I
    lib.ngz_templates_json.argtypes = [P, I, ctypes.c_char_p, ctypes.c_size_t]
    lib.ngz_templates_json.restype = I
    lib.ngz_template_counts.argtypes = [P, I, ctypes.POINTER(ctypes.c_uint16), ctypes.POINTER(ctypes.c_uint64), U32, I]
    lib.ngz_template_counts.restype = I
    lib.ngz_last_timing.argtypes = [P, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
    lib.ngz_last_timing.restype = I
    lib.ngz_columns_to_host.argtypes = [P, P, U64]
    lib.ngz_columns_to_host.restype = ctypes.c_int64
    lib.ngz_columns_to_host_async.argtypes = [P, P, U64, P, ctypes.c_uint32]
    lib.ngz_columns_to_host_async.restype = ctypes.c_int64
    lib.ngz_template_kernel.argtypes = [P, ctypes.c_size_t, I, ctypes.c_char_p, ctypes.c_size_t]
    lib.ngz_template_kernel.restype = I
    lib.ngz_group_kernel.argtypes = [P, ctypes.c_size_t, I, ctypes.c_char_p, ctypes.c_size_t]
    lib.ngz_group_kernel.restype = I
    lib.ngz_ctx_set_option.argtypes = [P, I, ctypes.c_int64]
    lib.ngz_ctx_set_option.restype = I
    lib.ngz_dgram_json.argtypes = [P, U32, ctypes.c_char_p, ctypes.c_size_t]
    lib.ngz_record_fields.argtypes = [P, U32, U32, U32, ctypes.POINTER(FieldValue), U32]
    lib.ngz_record_fields.restype = I
    lib.ngz_placement_trials.argtypes = [P, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float), U32,
                                         ctypes.POINTER(ctypes.c_uint32)]
    lib.ngz_placement_trials.restype = I
    lib.ngz_message_records.argtypes = [P, P, P, P, U32, P]
    lib.ngz_message_records.restype = I
    lib.ngz_dgram_json.restype = ctypes.c_int64
    lib.ngz_batch_json.argtypes = [P, P, JSON_LINE_FN, P]
    lib.ngz_batch_json.restype = ctypes.c_int64
    lib.ngz_slot_kernel.argtypes = [P, U32]
    lib.ngz_slot_kernel.restype = I
    lib.ngz_last_batch_info.argtypes = [P]
    lib.ngz_last_batch_info.restype = I
    lib.ngz_dgram_error.argtypes = [P, U32, ctypes.POINTER(Error)]
    lib.ngz_dgram_error.restype = I
    lib.ngz_template_counts_device.argtypes = [P, I, P, U32, I, P]
    lib.ngz_template_counts_device.restype = I
    lib.ngz_rtc_drain.argtypes = []
    lib.ngz_rtc_drain.restype = I
    global _DRAIN_REGISTERED
    if not _DRAIN_REGISTERED:
        # background template compiles finish before the interpreter tears down and the C
        # exit handlers run (flow_decode.h ngz_rtc_drain; the r2/r3 exit hang of a dist rank)
        import atexit
        atexit.register(lib.ngz_rtc_drain)
        _DRAIN_REGISTERED = True
    # aggregation (flow_aggregate.h)
    lib.ngz_agg_create.argtypes = [I, ctypes.POINTER(AggField), U32, U64, U64, U64, U32, ctypes.POINTER(P)]
    lib.ngz_agg_create.restype = I
    lib.ngz_agg_destroy.argtypes = [P]
    lib.ngz_agg_destroy.restype = None
    lib.ngz_agg_last_error.argtypes = [P]
    lib.ngz_agg_last_error.restype = ctypes.c_char_p
    lib.ngz_agg_push.argtypes = [P, P, ctypes.POINTER(BatchOut), ctypes.POINTER(Peer), ctypes.c_int64,
                                 ctypes.POINTER(ctypes.c_uint64), P]
    lib.ngz_agg_push.restype = I
    lib.ngz_agg_layout.argtypes = [P, ctypes.POINTER(U32), ctypes.POINTER(U32), ctypes.POINTER(ctypes.c_uint16),
                                   ctypes.POINTER(U32), ctypes.POINTER(ctypes.c_uint16)]
    lib.ngz_agg_layout.restype = I
    lib.ngz_agg_groups.argtypes = [P]
    lib.ngz_agg_groups.restype = ctypes.c_int64
    lib.ngz_agg_flush.argtypes = [P, P, U64]
    lib.ngz_agg_flush.restype = ctypes.c_int64
    lib.ngz_agg_sets.argtypes = [P, ctypes.POINTER(U32), ctypes.POINTER(U32), ctypes.POINTER(ctypes.c_uint16),
                                 ctypes.POINTER(U32), ctypes.POINTER(U32), ctypes.POINTER(U32), U32]
    lib.ngz_agg_sets.restype = I
    lib.ngz_agg_last_timing.argtypes = [P, ctypes.POINTER(ctypes.c_float)]
    lib.ngz_agg_last_timing.restype = I
    lib.ngz_agg_closed.argtypes = [P]
    lib.ngz_agg_closed.restype = ctypes.c_int64
    lib.ngz_agg_emit.argtypes = [P, P, U64]
    lib.ngz_agg_emit.restype = ctypes.c_int64
    lib.ngz_agg_reset.argtypes = [P]
    lib.ngz_agg_reset.restype = I
    lib.ngz_agg_key_info.argtypes = [P, U32, ctypes.POINTER(AggKeyDesc)]
    lib.ngz_agg_key_info.restype = I
    lib.ngz_agg_value_info.argtypes = [P, U32, ctypes.POINTER(AggValueDesc)]
    lib.ngz_agg_value_info.restype = I
    lib.ngz_agg_row_bytes.argtypes = [P, P, I, U32, P, U64]
    lib.ngz_agg_row_bytes.restype = ctypes.c_int64
    lib.ngz_agg_flowinfo_json.argtypes = [P, P, U64, U32, U32, ctypes.c_int64, JSON_LINE_FN, P]
    lib.ngz_agg_flowinfo_json.restype = ctypes.c_int64
    lib.ngz_agg_peer.argtypes = [P, U32, ctypes.POINTER(Peer)]
    lib.ngz_agg_peer.restype = I
    lib.ngz_agg_last_path.argtypes = [P]
    lib.ngz_agg_last_path.restype = ctypes.c_char_p
    lib.ngz_agg_set_option.argtypes = [P, I, ctypes.c_int64]
    lib.ngz_agg_set_option.restype = I
    # ingest (flow_ingest.h)
    lib.ngz_pcap_open.argtypes = [ctypes.c_char_p, ctypes.POINTER(P)]
    lib.ngz_pcap_open.restype = I
    lib.ngz_pcap_next.argtypes = [P, ctypes.POINTER(Packet)]
    lib.ngz_pcap_next.restype = I
    lib.ngz_pcap_close.argtypes = [P]
    lib.ngz_pcap_close.restype = None
    lib.ngz_collector_create.argtypes = [I, I, ctypes.POINTER(P)]
    lib.ngz_collector_create.restype = I
    lib.ngz_collector_destroy.argtypes = [P]
    lib.ngz_collector_destroy.restype = None
    lib.ngz_collector_last_error.argtypes = [P]
    lib.ngz_collector_last_error.restype = ctypes.c_char_p
    lib.ngz_collector_push.argtypes = [P, ctypes.POINTER(PeerKey), P, U32, U64]
    lib.ngz_collector_push.restype = I
    lib.ngz_collector_flush.argtypes = [P, COLLECT_LINE_FN, P]
    lib.ngz_collector_flush.restype = ctypes.c_int64
    lib.ngz_collector_peers.argtypes = [P]
    lib.ngz_collector_peers.restype = U32
    lib.ngz_udp_recv.argtypes = [I, P, U64, ctypes.POINTER(PeerKey), P, P, U32, I]
    lib.ngz_udp_recv.restype = I
    lib.ngz_pcap_to_jsonl.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint16), U32, ctypes.c_char_p, I,
                                      ctypes.c_int64, I]
    lib.ngz_pcap_to_jsonl.restype = ctypes.c_int64
    return lib


_HIP = None


def hip():
    """libamdhip64 for device->host copies of result arrays."""
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
        _HIP.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _HIP.hipMemcpy.restype = ctypes.c_int
    return _HIP


def d2h(dev_ptr, nbytes):
    out = np.empty(nbytes, dtype=np.uint8)
    if nbytes:
        rc = hip().hipMemcpy(out.ctypes.data, dev_ptr, nbytes, 2)  # hipMemcpyDeviceToHost
        if rc != 0:
            raise RuntimeError("hipMemcpy D2H failed: %d" % rc)
    return out
