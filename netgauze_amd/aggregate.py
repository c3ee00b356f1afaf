"""Host-side mirror of the collector's windowed flow aggregation, over the C ABI
in include/ngz/flow_aggregate.h (libngz.so; the group table lives in HBM).

`FlowAggregator(transform, window, lateness)` takes the reference's
AggregationConfig.transform shape (crates/collector/src/flow/aggregation/config.rs:
152-176, 252-335): an ordered mapping IE -> Op, or IE -> {index: Op}, where IE is
(pen, ie_id).  `push(batch, peer_port, collection_ms)` explodes and reduces every
data record of a decoded batch (aggregator.rs:78-90, 159-198, 286-354);
`flush()` returns every group (WindowAggregator::flush, analytics/src/aggregation.rs:
175-185) as dicts with canonical values: ints for integer-like fields, bytes for
byte-like ones, str for fixed strings.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import AGG_ROW_DTYPE

OPS = {"Key": _lib.NGZ_AGG_KEY, "Add": _lib.NGZ_AGG_ADD, "Min": _lib.NGZ_AGG_MIN, "Max": _lib.NGZ_AGG_MAX,
       "BoolMapOr": _lib.NGZ_AGG_OR}

_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = _lib.load()
    return _LIB


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


class FlowAggregator:
    def __init__(self, transform, window_s=60, lateness_s=10, capacity=1 << 20, device=0, kinds=None):
        self.fields = unify(transform) if isinstance(transform, dict) else list(transform)
        self.key_fields = [f for f in self.fields if f[3] == _lib.NGZ_AGG_KEY]
        self.val_fields = [f for f in self.fields if f[3] != _lib.NGZ_AGG_KEY]
        arr = (_lib.AggField * max(len(self.fields), 1))(*[_lib.AggField(p, i, x, o) for p, i, x, o in self.fields])
        h = ctypes.c_void_p()
        rc = lib().ngz_agg_create(device, arr, len(self.fields), int(window_s * 1000), int(lateness_s * 1000),
                                  capacity, ctypes.byref(h))
        if rc != 0:
            raise AggError("ngz_agg_create failed (%d)" % rc)
        self._h = h
        # kinds[(pen, ie_id)] = "sint" | "str" | "bytes" | "uint" (how flush renders values)
        self.kinds = kinds or {}

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().ngz_agg_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc < 0:
            raise AggError("%s (%d)" % (lib().ngz_agg_last_error(self._h).decode(), rc))
        return rc

    def push(self, batch, peer_port=4739, collection_ms=0):
        """Aggregate every data record of a DecodedBatch; returns the late records."""
        late = ctypes.c_uint64()
        self._check(lib().ngz_agg_push(self._h, batch._codec._ctx, ctypes.byref(batch.out), peer_port,
                                       collection_ms, ctypes.byref(late), None))
        return late.value

    def push_ms(self):
        t = ctypes.c_float()
        lib().ngz_agg_last_timing(self._h, ctypes.byref(t))
        return t.value

    def n_groups(self):
        return self._check(lib().ngz_agg_groups(self._h))

    def layout(self):
        nk, nv = len(self.key_fields), len(self.val_fields)
        rb = ctypes.c_uint32()
        ko, kw = (ctypes.c_uint32 * max(nk, 1))(), (ctypes.c_uint16 * max(nk, 1))()
        vo, vw = (ctypes.c_uint32 * max(nv, 1))(), (ctypes.c_uint16 * max(nv, 1))()
        self._check(lib().ngz_agg_layout(self._h, ctypes.byref(rb), ko, kw, vo, vw))
        return rb.value, list(ko)[:nk], list(kw)[:nk], list(vo)[:nv], list(vw)[:nv]

    def sets(self):
        cap = 128
        t, p, d = (ctypes.c_uint32 * cap)(), (ctypes.c_uint16 * cap)(), (ctypes.c_uint32 * cap)()
        nt, np_, nd = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        self._check(lib().ngz_agg_sets(self._h, t, ctypes.byref(nt), p, ctypes.byref(np_), d, ctypes.byref(nd), cap))
        return list(t)[:nt.value], list(p)[:np_.value], list(d)[:nd.value]

    def flush_raw(self):
        """Every group as (rows: AGG_ROW_DTYPE view, raw bytes [n, row_bytes]); empties the table."""
        rb = self.layout()[0]
        n = self.n_groups()
        buf = np.zeros(max(n, 1) * rb, dtype=np.uint8)
        got = self._check(lib().ngz_agg_flush(self._h, buf.ctypes.data, buf.nbytes))
        raw = buf[:got * rb].reshape(got, rb)
        return raw[:, :88].copy().view(AGG_ROW_DTYPE).reshape(got), raw

    def flush(self):
        rb, ko, kw, vo, vw = self.layout()
        tpl, ports, doms = self.sets()
        hdr, raw = self.flush_raw()

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
                b = bytes(r[ko[k]:ko[k] + kw[k]])
                key.append(self._render(pen, ie, b))
            vals = []
            for v, (pen, ie, _i, op) in enumerate(self.val_fields):
                if not (int(h["val_present"]) >> v) & 1:
                    vals.append(None)
                    continue
                kind = self.kinds.get((pen, ie), "uint")
                if kind == "bytes":
                    vals.append(bytes(r[vo[v]:vo[v] + vw[v]]))
                else:
                    x = int.from_bytes(bytes(r[vo[v]:vo[v] + 8]), "little", signed=(kind == "sint"))
                    vals.append((x >> 32, x & 0xFFFFFFFF) if kind == "dtfrac" else x)
            dom_bits = int(h["domain_bits"][0]) | (int(h["domain_bits"][1]) << 64)
            out.append(dict(window_start=int(h["window_start"]), flow_type=int(h["flow_type"]), key=tuple(key),
                            vals=tuple(vals), record_count=int(h["record_count"]),
                            min_export=int(h["min_export_time"]), max_export=int(h["max_export_time"]),
                            max_sysup=int(h["max_sys_up_time"]), min_coll=int(h["min_collection_ms"]),
                            max_coll=int(h["max_collection_ms"]),
                            templates={(t >> 16, t & 0xFFFF) for t in bits(h["template_bits"], tpl)},
                            ports=bits(h["port_bits"], ports), domains=bits(dom_bits, doms)))
        return out

    def _render(self, pen, ie, b):
        kind = self.kinds.get((pen, ie), "uint")
        if kind == "bytes":
            return b
        if kind == "str":
            return b.split(b"\0", 1)[0].decode("utf-8")
        return int.from_bytes(b, "little", signed=(kind == "sint"))
