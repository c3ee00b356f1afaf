"""Host-side mirror of the collector's windowed flow aggregation, over the C ABI
in include/ngz/flow_aggregate.h (libngz.so; the group table lives in HBM).

`FlowAggregator(transform, window, lateness)` takes the reference's
AggregationConfig.transform shape (crates/collector/src/flow/aggregation/config.rs:
152-176, 252-335): an ordered mapping IE -> Op, or IE -> {index: Op}, where IE is
(pen, ie_id).  One aggregator serves a collector shard: every exporter peer.
`push(batch, peer_port, collection_ms, peer_ip)` explodes and reduces every data
record of a batch one peer sent (aggregator.rs:78-90, 159-198, 286-354), grouped
by (peer IP, window, flow type, key); `emit()` returns the groups of the windows
each peer's event time has closed (analytics/src/aggregation.rs:154-160) and
`flush()` every group
(WindowAggregator::flush, :175-185), as dicts with canonical values: ints for
integer-like fields, bytes for byte-like ones, str for strings, floats, and
(secs, nanos) for date-times -- each field rendered from its IE's data type in
the registry (netgauze_amd/data/ie_registry.json) and the device's storage
class (ngz_agg_key_info / ngz_agg_value_info).  `flowinfo_json(rows)` renders
output rows as the reference's aggregated FlowInfo
(AggFlowInfo::into_flowinfo_with_extra_fields, aggregator.rs:203-277).
"""
import ctypes
import sys
import json
import os
import struct

import numpy as np

from . import _lib
from ._lib import AGG_ROW_DTYPE

OPS = {"Key": _lib.NGZ_AGG_KEY, "Add": _lib.NGZ_AGG_ADD, "Min": _lib.NGZ_AGG_MIN, "Max": _lib.NGZ_AGG_MAX,
       "BoolMapOr": _lib.NGZ_AGG_OR}

_LIB = None
_DTYPES = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = _lib.load()
    return _LIB


def ie_dtype(pen, ie_id):
    """IE data type from the registry the library is built from (None: IE::Unknown)."""
    global _DTYPES
    if _DTYPES is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "ie_registry.json")
        with open(path) as f:
            reg = json.load(f)
        _DTYPES = {(r["pen"], r["id"]): r["type"] for r in reg["ies"]}
    return _DTYPES.get((pen, ie_id))


class AggError(RuntimeError):
    pass


def unify(transform):
    """AggregationConfig.transform -> [(pen, ie_id, index, op)] (TryInto<UnifiedConfig>,
    config.rs:252-335).  Ops may be names ("Add") or NGZ_AGG_* ints."""
    out = []
    for ie, t in transform.items():
        pen, ie_id = ie
        items = t.items() if isinstance(t, dict) else [(0, t)]
        for index, op in items:
            out.append((pen, ie_id, int(index), OPS.get(op, op)))
    return out


def _datetime_ms(ms):
    secs = ms // 1000
    return (secs, (ms - secs * 1000) * 1_000_000)


class FlowAggregator:
    DEFAULT_PEER = "192.0.2.1"  # TEST-NET-1: the exporter of pushes that name none

    def __init__(self, transform, window_s=60, lateness_s=10, capacity=1 << 20, device=0, kinds=None, max_peers=0,
                 options=None):
        """max_peers: distinct exporter IPs the aggregator takes between flushes (0: the library's
        NGZ_AGG_MAX_PEERS, 65536).  Entries are kept until flush / reset, as each peer's event time
        is; a push from a new IP beyond it fails (AggError, NGZ_AGG_E_OVERFLOW).  A smaller bound
        leaves more bits of the exact 63-bit group tag to the key fields (flow_aggregate.h).
        options: {NGZ_AGG_OPT_*: value} for ngz_agg_set_option (how pushes reduce, never what)."""
        self.fields = unify(transform) if isinstance(transform, dict) else list(transform)
        self.key_fields = [f for f in self.fields if f[3] == _lib.NGZ_AGG_KEY]
        self.val_fields = [f for f in self.fields if f[3] != _lib.NGZ_AGG_KEY]
        arr = (_lib.AggField * max(len(self.fields), 1))(*[_lib.AggField(p, i, x, o) for p, i, x, o in self.fields])
        h = ctypes.c_void_p()
        rc = lib().ngz_agg_create(device, arr, len(self.fields), int(window_s * 1000), int(lateness_s * 1000),
                                  capacity, max_peers, ctypes.byref(h))
        if rc != 0:
            raise AggError("ngz_agg_create failed (%d)" % rc)
        self._h = h
        # optional override of the rendering per (pen, ie_id): "sint" | "uint" | "bytes" | "str"
        self.kinds = kinds or {}
        for opt, value in (options or {}).items():
            self.set_option(opt, value)

    def set_option(self, opt, value):
        """ngz_agg_set_option: NGZ_AGG_OPT_LOWCARD / _PARTITION (-1 auto, 0 never, 1 always),
        _OWNER (0 / 1), _HASH_BITS (0 full hash; 1..63, only while no group is held)."""
        self._check(lib().ngz_agg_set_option(self._h, opt, int(value)))

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().ngz_agg_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        if sys.is_finalizing():  # the HIP runtime may be torn down already: leave it to the process exit
            return
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc < 0:
            raise AggError("%s (%d)" % (lib().ngz_agg_last_error(self._h).decode(), rc))
        return rc

    def push(self, batch, peer_port=4739, collection_ms=0, peer_ip=DEFAULT_PEER):
        """Aggregate every data record of a DecodedBatch the peer (peer_ip, peer_port)
        sent; returns the late records.  The batch must be the latest one its codec
        decoded (its device arrays are reused by the next decode)."""
        if batch.generation != batch._codec.generation:
            raise AggError("stale DecodedBatch: its codec has decoded another batch since")
        late = ctypes.c_uint64()
        peer = _lib.Peer.of(peer_ip, peer_port)
        self._check(lib().ngz_agg_push(self._h, batch._codec._ctx, ctypes.byref(batch.out), ctypes.byref(peer),
                                       collection_ms, ctypes.byref(late), None))
        return late.value

    def peers(self):
        """Peer IPs of the rows last returned by flush / emit (row field `peer`)."""
        out = []
        p = _lib.Peer()
        n = lib().ngz_agg_peer(self._h, 0, ctypes.byref(p))
        for i in range(max(n, 0)):
            lib().ngz_agg_peer(self._h, i, ctypes.byref(p))
            out.append(p.ip())
        return out

    def last_path(self):
        """"lowcard" or "general": the reduction path of the last push."""
        return lib().ngz_agg_last_path(self._h).decode()

    def push_ms(self):
        t = ctypes.c_float()
        lib().ngz_agg_last_timing(self._h, ctypes.byref(t))
        return t.value

    def n_groups(self):
        return self._check(lib().ngz_agg_groups(self._h))

    def n_closed(self):
        return self._check(lib().ngz_agg_closed(self._h))

    def reset(self):
        self._check(lib().ngz_agg_reset(self._h))

    def layout(self):
        nk, nv = len(self.key_fields), len(self.val_fields)
        rb = ctypes.c_uint32()
        ko, kw = (ctypes.c_uint32 * max(nk, 1))(), (ctypes.c_uint16 * max(nk, 1))()
        vo, vw = (ctypes.c_uint32 * max(nv, 1))(), (ctypes.c_uint16 * max(nv, 1))()
        self._check(lib().ngz_agg_layout(self._h, ctypes.byref(rb), ko, kw, vo, vw))
        return rb.value, list(ko)[:nk], list(kw)[:nk], list(vo)[:nv], list(vw)[:nv]

    def descs(self):
        kd, vd = [], []
        for k in range(len(self.key_fields)):
            d = _lib.AggKeyDesc()
            self._check(lib().ngz_agg_key_info(self._h, k, ctypes.byref(d)))
            kd.append(d)
        for v in range(len(self.val_fields)):
            d = _lib.AggValueDesc()
            self._check(lib().ngz_agg_value_info(self._h, v, ctypes.byref(d)))
            vd.append(d)
        return kd, vd

    def sets(self):
        cap = 128
        t, p, d = (ctypes.c_uint32 * cap)(), (ctypes.c_uint16 * cap)(), (ctypes.c_uint32 * cap)()
        nt, np_, nd = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        self._check(lib().ngz_agg_sets(self._h, t, ctypes.byref(nt), p, ctypes.byref(np_), d, ctypes.byref(nd), cap))
        return list(t)[:nt.value], list(p)[:np_.value], list(d)[:nd.value]

    def _take(self, fn, n):
        rb = self.layout()[0]
        buf = np.zeros(max(n, 1) * rb, dtype=np.uint8)
        got = self._check(fn(self._h, buf.ctypes.data, buf.nbytes))
        raw = buf[:got * rb].reshape(got, rb)
        return raw[:, :88].copy().view(AGG_ROW_DTYPE).reshape(got), raw

    def flush_raw(self):
        """Every group as (rows: AGG_ROW_DTYPE view, raw bytes [n, row_bytes]); empties the table."""
        return self._take(lib().ngz_agg_flush, self.n_groups())

    def emit_raw(self):
        """The groups of closed windows as (rows, raw bytes); removes them."""
        return self._take(lib().ngz_agg_emit, self.n_closed())

    def flush(self):
        return self.render(*self.flush_raw())

    def emit(self):
        return self.render(*self.emit_raw())

    def flowinfo_json(self, raw, shard_id=0, seq0=0, export_time_ms=0):
        """AggFlowInfo -> FlowInfo serde JSON of rows just returned by flush_raw / emit_raw."""
        out = []

        def cb(_user, _i, _status, text, n, _consumed):
            out.append(ctypes.string_at(text, n).decode())
            return 0

        fn = _lib.JSON_LINE_FN(cb)
        raw = np.ascontiguousarray(raw)
        self._check(lib().ngz_agg_flowinfo_json(self._h, raw.ctypes.data if len(raw) else None, len(raw), shard_id,
                                                seq0, export_time_ms, fn, None))
        return out

    def render(self, hdr, raw):
        rb, ko, kw, vo, vw = self.layout()
        kd, vd = self.descs()
        tpl, ports, doms = self.sets()
        peers = self.peers() if len(hdr) else []

        def bits(x, dictionary):
            return {dictionary[i] for i in range(len(dictionary)) if (int(x) >> i) & 1}

        out = []
        for g in range(len(hdr)):
            h, r = hdr[g], raw[g]
            key = []
            for k, (pen, ie, _i, _op) in enumerate(self.key_fields):
                if not (int(h["key_present"]) >> k) & 1:
                    key.append(None)
                    continue
                if kd[k].kkind == _lib.AGG_KK_BYTES:
                    key.append(self._render_bytes(pen, ie, self._row_bytes(r, 0, k)))
                    continue
                key.append(self._render_key(pen, ie, kd[k], bytes(r[ko[k]:ko[k] + kd[k].slot])))
            vals = []
            for v, (pen, ie, _i, op) in enumerate(self.val_fields):
                if not (int(h["val_present"]) >> v) & 1:
                    vals.append(None)
                    continue
                if vd[v].vclass in (_lib.AGG_VC_VBYTES, _lib.AGG_VC_VLIST):
                    vals.append(self._row_bytes(r, 1, v))
                    continue
                vals.append(self._render_value(pen, ie, vd[v], bytes(r[vo[v]:vo[v] + 32])))
            dom_bits = int(h["domain_bits"][0]) | (int(h["domain_bits"][1]) << 64)
            out.append(dict(peer=peers[int(h["peer"])], window_start=int(h["window_start"]),
                            flow_type=int(h["flow_type"]), key=tuple(key),
                            vals=tuple(vals), record_count=int(h["record_count"]),
                            min_export=int(h["min_export_time"]), max_export=int(h["max_export_time"]),
                            max_sysup=int(h["max_sys_up_time"]), min_coll=int(h["min_collection_ms"]),
                            max_coll=int(h["max_collection_ms"]),
                            templates={(t >> 16, t & 0xFFFF) for t in bits(h["template_bits"], tpl)},
                            ports=bits(h["port_bits"], ports), domains=bits(dom_bits, doms)))
        return out

    def _row_bytes(self, row, is_value, index):
        """The whole byte value of a BVAL key / value of an output row (ngz_agg_row_bytes)."""
        row = np.ascontiguousarray(row)
        n = self._check(lib().ngz_agg_row_bytes(self._h, row.ctypes.data, is_value, index, None, 0))
        buf = (ctypes.c_uint8 * max(n, 1))()
        lib().ngz_agg_row_bytes(self._h, row.ctypes.data, is_value, index, buf, n)
        return bytes(buf[:n])

    def _render_bytes(self, pen, ie, b):
        kind = self.kinds.get((pen, ie))
        if kind == "str" or (kind is None and ie_dtype(pen, ie) == "string"):
            return b.decode("utf-8")
        return b

    def _render_key(self, pen, ie, d, b):
        kind = self.kinds.get((pen, ie))
        if kind == "str":
            return b.split(b"\0", 1)[0].decode("utf-8")
        return self._render_cell(pen, ie, d.kind, d.width, b, kind)

    def _render_value(self, pen, ie, d, b):
        kind = self.kinds.get((pen, ie))
        vc = d.vclass
        if vc == _lib.AGG_VC_F32:
            return struct.unpack("<f", b[:4])[0]
        if vc == _lib.AGG_VC_F64:
            return struct.unpack("<d", b[:8])[0]
        if vc == _lib.AGG_VC_IPV6:
            return b[:16]
        if vc == _lib.AGG_VC_BYTES:
            return b[:d.width]
        if vc == _lib.AGG_VC_DTFRAC:
            x = int.from_bytes(b[:8], "little")
            return (x >> 32, x & 0xFFFFFFFF)
        return self._render_cell(pen, ie, d.kind, 8, b[:8], kind, value=True)

    def _render_cell(self, pen, ie, ckind, width, b, kind, value=False):
        """A column cell / integer accumulator as the oracle's canonical value."""
        dt = ie_dtype(pen, ie)
        if kind == "bytes" or (kind is None and (dt is None or dt in ("octetArray", "macAddress", "ipv6Address",
                                                                      "unsigned256"))):
            return b[:width]
        signed = kind == "sint" or (kind is None and (dt or "").startswith("signed")) or ckind == 7  # NGZ_K_DTMS
        x = int.from_bytes(b[:width], "little", signed=signed)
        if dt == "dateTimeMilliseconds":
            return _datetime_ms(x)
        if dt in ("dateTimeMicroseconds", "dateTimeNanoseconds"):
            return (x & 0xFFFFFFFF, x >> 32) if not value else (x >> 32, x & 0xFFFFFFFF)
        if dt == "dateTimeSeconds":
            return (x, 0)
        if dt in ("float32", "float64") and not value:
            return struct.unpack("<f" if width == 4 else "<d", b[:width])[0]
        return x
