"""CPU restatement of the collector's windowed flow aggregation (TEST INFRASTRUCTURE ONLY).

This module is the checker for the device aggregation (include/ngz/flow_aggregate.h,
netgauze_amd/csrc/ngz_agg.hip).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may use it; the product path never imports it.

It restates, over the packets of ngz_oracle.FlowInfoCodec:
  - explode                      crates/collector/src/flow/aggregation/aggregator.rs:286-354
  - FieldRef::map_fields         crates/collector/src/flow/types.rs:82-100
  - FlowAggregator::push         aggregator.rs:78-90
  - FlowCacheRecord::reduce      aggregator.rs:159-198
  - Field add/min/max/or         ipfix-code-generator/src/generator.rs:896-1080 (`*lhs += *rhs`,
                                 release-mode wrapping at the Rust width; `min`/`max`; `|=`,
                                 byte-wise zip for arrays)
  - WindowAggregator::process_item crates/analytics/src/aggregation.rs:124-172 (lateness drop,
                                 window start = get_window_start :79-89, minute floor, and the
                                 windows the cutoff closes, :154-160)
  - Ord of the Field types for Min / Max: ordered_float's OrderedFloat (NaN greatest and equal
    to itself, -0 == +0), Ipv6Addr by octets, DateTime chronological, derived Ord of
    TCPHeaderFlags (FIN most significant, iana/src/tcp.rs:41-70) and of sub-registry enums
    (by discriminant: registered value, then Unassigned(x) after every registered variant);
    Ord::min keeps the left argument on equality, Ord::max takes the right one
  - AggFlowInfo::into_flowinfo_with_extra_fields (aggregator.rs:203-277) with the actor's extra
    fields windowStart, windowEnd, originalExporterIPv4Address / IPv6Address (actor.rs:206-240),
    sets in ascending order
One FlowAggregatorOracle is one shard: FlowCacheKey carries the peer IP (aggregator.rs:119-124)
and the window aggregator keeps its windows and event time per peer IP (aggregation.rs:96-108,
TimeSeriesData<IpAddr>::get_key, aggregator.rs:109-117).
Pinned by the reference's own unit tests (aggregator/tests.rs :72-1377 and the window tests of
analytics/src/aggregation.rs :579-789), restated as vectors in tests/kats_agg.py.

Values are canonical Python values: ints for integer / ipv4 / tcpControlBits / bool / date-time
seconds, bytes for byte-like fields, str for strings.
"""
import ipaddress
import struct

import ngz_oracle as O

OP_KEY, OP_ADD, OP_MIN, OP_MAX, OP_OR = 0, 1, 2, 3, 4

RUST_WIDTH = {"unsigned8": 1, "unsigned16": 2, "unsigned32": 4, "unsigned64": 8, "signed8": 1, "signed16": 2,
              "signed32": 4, "signed64": 8}


def canon(field):
    """Field value -> canonical value (see module doc)."""
    v = field.value
    if field.ie.kind == "iana" and field.ie.id == 6:  # tcpControlBits -> TCPHeaderFlags::from(u16) keeps the
        return v & 0xFF                                # low 8 bits (iana/src/tcp.rs:165-168)
    if isinstance(v, tuple) and v and v[0] in ("v4", "v6"):
        return v[1] if v[0] == "v4" else v[1].to_bytes(16, "big")
    if isinstance(v, tuple) and v and v[0] == "f32":
        return struct.unpack("<f", struct.pack("<I", v[1]))[0]
    if isinstance(v, tuple) and v and v[0] == "f64":
        return struct.unpack("<d", struct.pack("<Q", v[1]))[0]
    if isinstance(v, bool):
        return int(v)
    if isinstance(v, O.DateTime):
        return (v.secs, v.nanos)
    return v


def _wrap(ie, x):
    w = RUST_WIDTH.get(ie.dtype)
    if w is None:
        return x
    x &= (1 << (8 * w)) - 1
    if ie.dtype.startswith("signed") and x >> (8 * w - 1):
        x -= 1 << (8 * w)
    return x


def _f32(x):
    return struct.unpack("<f", struct.pack("<f", x))[0]


def _ofloat_cmp(a, b):
    """ordered_float::OrderedFloat Ord: NaN == NaN, NaN > every number, -0 == +0."""
    na, nb = a != a, b != b
    if na or nb:
        return 0 if na == nb else (1 if na else -1)
    return -1 if a < b else (1 if a > b else 0)


def _rank(ie, v):
    """Position of a value in the Rust Ord of its Field type (derived Ord)."""
    if ie.kind == "iana" and ie.id == 6:  # TCPHeaderFlags {FIN, SYN, ...}: FIN most significant
        return int("{:08b}".format(v & 0xFF)[::-1], 2)
    if ie.subreg is not None and ie.subreg["kind"] == "vnd":
        known = {val for val, _ in ie.subreg["entries"]}
        return v if v in known else (1 << 32) | v  # Unassigned(x) after every registered variant
    if ie.subreg is not None and ie.subreg["kind"] == "nested":
        # forwardingStatus (generator_sub_registries.rs:96-140): one outer variant per 64-value
        # group in declaration order, then Unassigned(x); inside a group the reason enum's
        # discriminant (a registered reason is its value, its Unassigned(x) the last declared
        # value + 1 -- Rust's implicit discriminant), then the value
        groups = ie.subreg["entries"]
        gi = v // 64
        if gi >= len(groups):
            return (len(groups), 0, v)
        reasons = [rv for rv, _ in groups[gi][2]]
        return (gi, v if v in reasons else (reasons[-1] + 1 if reasons else 0), v)
    return v


def reduce_value(ie, op, lhs, rhs):
    """Field::{add,min,max,bitwise_or}_assign_field on canonical values (generator.rs:896-1080).
    Ord::min keeps lhs on equality, Ord::max takes rhs (core::cmp::min_by / max_by)."""
    flt = ie.dtype in ("float32", "float64")
    if op == OP_ADD:
        if flt:
            return _f32(lhs + rhs) if ie.dtype == "float32" else lhs + rhs
        return _wrap(ie, lhs + rhs)
    if op in (OP_MIN, OP_MAX):
        if flt:
            c = _ofloat_cmp(lhs, rhs)
        else:
            a, b = _rank(ie, lhs), _rank(ie, rhs)
            c = -1 if a < b else (1 if a > b else 0)
        if op == OP_MIN:
            return rhs if c > 0 else lhs
        return lhs if c > 0 else rhs
    if isinstance(lhs, (bytes, bytearray)):  # lhs.iter_mut().zip(rhs): lhs keeps its length
        out = bytearray(lhs)
        for i, b in enumerate(rhs[:len(out)]):
            out[i] |= b
        return bytes(out)
    return lhs | rhs


# IE::supports_{arithmetic,comparison,bitwise}_ops (ipfix-code-generator/src/generator.rs:1176-1272)
_NUMERIC = {"signed8", "signed16", "signed32", "signed64", "unsigned8", "unsigned16", "unsigned32", "unsigned64",
            "float32", "float64"}
_CMP_TYPES = _NUMERIC | {"dateTimeSeconds", "dateTimeMilliseconds", "dateTimeMicroseconds", "dateTimeNanoseconds",
                         "ipv4Address", "ipv6Address", "basicList", "subTemplateList", "subTemplateMultiList"}
_BIT_TYPES = (_NUMERIC - {"float32", "float64"}) | {"octetArray", "boolean", "macAddress", "ipv4Address",
                                                    "ipv6Address", "unsigned256"}
_SEMANTICS = None


def _semantics(ie):
    global _SEMANTICS
    if _SEMANTICS is None:
        import json
        with open(O._REG_PATH) as f:
            _SEMANTICS = {(r["pen"], r["id"]): r.get("semantics") for r in json.load(f)["ies"]}
    return _SEMANTICS.get((ie.pen, ie.id)) if ie.kind in ("iana", "vendor") else None


def supports(ie, op):
    """generator.rs:1176-1272.  Arithmetic: a numeric type (unsigned256 excluded) without a
    sub-registry and without identifier / flags dataTypeSemantics; comparison and bitwise by data
    type alone."""
    if op == OP_ADD:
        if _semantics(ie) in ("identifier", "flags") or ie.subreg is not None:
            return False
        return ie.dtype in _NUMERIC
    if op in (OP_MIN, OP_MAX):
        return ie.dtype in _CMP_TYPES
    if op == OP_OR:
        return ie.dtype in _BIT_TYPES
    raise ValueError(op)


class FieldOperationError(Exception):
    """FieldOperationError::Inapplicable{Add,Min,Max,Bitwise}(IE, IE) (generator.rs:801-807; the
    vendor enums' own variants map into it, :2476-2492)."""
    VARIANT = {OP_ADD: "InapplicableAdd", OP_MIN: "InapplicableMin", OP_MAX: "InapplicableMax",
               OP_OR: "InapplicableBitwise"}

    def __init__(self, op, lhs_ie, rhs_ie):
        super().__init__(self.VARIANT[op], lhs_ie, rhs_ie)
        self.variant, self.lhs, self.rhs = self.VARIANT[op], lhs_ie, rhs_ie


def field_op(op, lhs_ie, lhs, rhs_ie, rhs):
    """Field::{add,min,max,bitwise_or}_field (generator.rs:812-880, vendor Field :2514-2580): the
    generated match has an arm for (IE x, IE x) of every IE whose type supports the op; any other
    pair -- two different IEs, or an IE without the op -- falls to Inapplicable*(lhs.ie(), rhs.ie())."""
    if lhs_ie != rhs_ie or not supports(lhs_ie, op):
        raise FieldOperationError(op, lhs_ie, rhs_ie)
    return reduce_value(lhs_ie, op, lhs, rhs)


def map_fields(fields):
    """FieldRef::map_fields (types.rs:82-100): (IE key, occurrence index) -> Field."""
    seen, out = {}, {}
    for f in fields:
        k = (f.ie.pen, f.ie.id)
        i = seen.get(k, 0)
        seen[k] = i + 1
        out[(k, i)] = f
    return out


DEFAULT_PEER = "192.0.2.1"  # the exporter of pushes that name none (netgauze_amd.aggregate)


class FlowAggregatorOracle:
    """One shard's WindowAggregator<IpAddr, UnifiedConfig, FlowAggregator> (aggregation.rs:96-186):
    windows and event time per peer IP.

    fields: [(pen, ie_id, index, op)] in transform order; keys and aggregated fields keep
    their relative order (config.rs:252-335)."""

    def __init__(self, fields, window_s=60, lateness_s=10):
        self.keys = [(pen, ie, idx) for pen, ie, idx, op in fields if op == OP_KEY]
        self.vals = [((pen, ie, idx), op) for pen, ie, idx, op in fields if op != OP_KEY]
        self.window_s, self.lateness_s = window_s, lateness_s
        self.current_time = {}   # peer IP -> event time
        self.groups = {}   # (peer IP, window_start, flow_type, key tuple) -> record dict
        self.late = 0
        self.closed = []   # groups of the windows the cutoff closed, not yet taken by emit()
        self._cutoff = {}

    def explode(self, pkt, peer_port, collection_ms):
        """aggregator.rs:286-354: one item per data record (non-scope fields)."""
        if isinstance(pkt, O.IpfixPacket):
            flow_type, ts, sysup, domain = 10, pkt.export_time.secs, 0, pkt.observation_domain_id
        else:
            flow_type, ts, sysup, domain = 9, pkt.unix_time.secs, pkt.sys_up_time, pkt.source_id
        for sid, rec in pkt.data_records():
            fields = rec[1] if isinstance(rec, tuple) else rec.fields
            m = map_fields(fields)
            key = tuple(canon(m[((p, i), x)]) if ((p, i), x) in m else None for p, i, x in self.keys)
            vals = [(m[((p, i), x)].ie, canon(m[((p, i), x)])) if ((p, i), x) in m else None
                    for (p, i, x), _op in self.vals]
            yield flow_type, ts, key, dict(ports={peer_port}, domains={domain}, templates={(flow_type, sid)},
                                           min_export=ts, max_export=ts, min_coll=collection_ms,
                                           max_coll=collection_ms, max_sysup=sysup, vals=vals, count=1)

    def push_packet(self, pkt, peer_port, collection_ms, peer_ip=DEFAULT_PEER):
        for flow_type, ts, key, rec in self.explode(pkt, peer_port, collection_ms):
            self.process_item(peer_ip, flow_type, ts, key, rec)

    def process_item(self, peer_ip, flow_type, ts, key, rec):
        """WindowAggregator::process_item (aggregation.rs:124-172), times in seconds (lateness
        in s): the item's key is its peer IP (aggregator.rs:109-117)."""
        ct = self.current_time.setdefault(peer_ip, ts)
        if ts < ct - self.lateness_s:
            self.late += 1
            return False
        self.current_time[peer_ip] = ct = max(ct, ts)
        g = (peer_ip, ts - ts % 60, flow_type, key)
        cur = self.groups.get(g)
        if cur is None:
            self.groups[g] = rec
        else:
            self.reduce(cur, rec)
        self._close_windows(peer_ip)
        return True

    def _close_windows(self, peer_ip):
        """aggregation.rs:154-160: the peer's windows starting at or before
        get_window_start(current_time - lateness) - window_duration leave its active set."""
        t = self.current_time[peer_ip] - self.lateness_s
        cutoff = t - t % 60 - self.window_s
        last = self._cutoff.get(peer_ip)
        if last is not None and cutoff <= last:
            return
        self._cutoff[peer_ip] = cutoff
        for g in [g for g in self.groups if g[0] == peer_ip and g[1] <= cutoff]:
            self.closed.append(self._out(g, self.groups.pop(g)))

    def reduce(self, lhs, rhs):
        """FlowCacheRecord::reduce (aggregator.rs:159-198)."""
        lhs["ports"] |= rhs["ports"]
        lhs["domains"] |= rhs["domains"]
        lhs["templates"] |= rhs["templates"]
        lhs["min_export"] = min(lhs["min_export"], rhs["min_export"])
        lhs["max_export"] = max(lhs["max_export"], rhs["max_export"])
        lhs["min_coll"] = min(lhs["min_coll"], rhs["min_coll"])
        lhs["max_coll"] = max(lhs["max_coll"], rhs["max_coll"])
        lhs["max_sysup"] = max(lhs["max_sysup"], rhs["max_sysup"])
        lhs["count"] += rhs["count"]
        for i, (_ref, op) in enumerate(self.vals):
            a, b = lhs["vals"][i], rhs["vals"][i]
            if a is not None and b is not None:
                lhs["vals"][i] = (a[0], reduce_value(a[0], op, a[1], b[1]))
            elif a is None and b is not None:
                lhs["vals"][i] = b

    @staticmethod
    def _out(g, r):
        peer, win, ft, key = g
        return dict(peer=peer, window_start=win, flow_type=ft, key=key,
                    vals=tuple(None if v is None else v[1] for v in r["vals"]),
                    record_count=r["count"], min_export=r["min_export"], max_export=r["max_export"],
                    max_sysup=r["max_sysup"], min_coll=r["min_coll"], max_coll=r["max_coll"],
                    templates=set(r["templates"]), ports=set(r["ports"]), domains=set(r["domains"]))

    def emit(self):
        """The groups of every window closed so far (and not emitted yet)."""
        out, self.closed = self.closed, []
        return out

    def flush(self):
        """WindowAggregator::flush: every active group, then forget the event time."""
        out = [self._out(g, r) for g, r in self.groups.items()]
        self.groups = {}
        self.current_time = {}
        self._cutoff = {}
        return out

    def flowinfo_json(self, group, shard_id=0, seq=0, export_time_ms=0):
        """AggFlowInfo::into_flowinfo_with_extra_fields (aggregator.rs:203-277) of one output
        group with the actor's extra fields (actor.rs:222-240): windowStart = the window start,
        windowEnd = start + window duration, the peer IP as originalExporterIPv4Address /
        IPv6Address; serde JSON text; the peer port / domain / template sets in ascending order."""
        return O.dumps(self.flowinfo(group, shard_id, seq, export_time_ms))

    def flowinfo(self, group, shard_id=0, seq=0, export_time_ms=0):
        """The FlowInfo of flowinfo_json as serde's JSON value (dicts and lists)."""
        reg = O.REGISTRY
        fields = []
        for (p, i, _x), v in zip(self.keys, group["key"]):
            if v is not None:
                ie = reg.lookup(p, i)
                fields.append(O.Field(ie, to_field_value(ie, v)))
        for ((p, i, _x), _op), v in zip(self.vals, group["vals"]):
            if v is not None:
                ie = reg.lookup(p, i)
                fields.append(O.Field(ie, to_field_value(ie, v)))
        ms = group["max_coll"]
        fields += [O.Field(reg.lookup(0, 375), group["record_count"]),
                   O.Field(reg.lookup(0, 264), O.DateTime(group["min_export"], 0)),
                   O.Field(reg.lookup(0, 260), O.DateTime(group["max_export"], 0)),
                   O.Field(reg.lookup(0, 258), O.DateTime(ms // 1000, (ms % 1000) * 1_000_000))]
        ws, we = group["window_start"], group["window_start"] * 1000 + int(round(self.window_s * 1000))
        fields += [O.Field(reg.lookup(3746, 1), O.DateTime(ws, 0)),
                   O.Field(reg.lookup(3746, 2), O.DateTime(we // 1000, (we % 1000) * 1_000_000))]
        ip = ipaddress.ip_address(group["peer"])
        fields.append(O.Field(reg.lookup(0, 403), ("v4", int(ip))) if ip.version == 4
                      else O.Field(reg.lookup(0, 404), ("v6", int(ip))))
        fields += [O.Field(reg.lookup(3746, 4), p) for p in sorted(group["ports"])]
        fields += [O.Field(reg.lookup(0, 405), d) for d in sorted(group["domains"])]
        fields += [O.Field(reg.lookup(3746, 3), t) for t in sorted(t for _ft, t in group["templates"])]
        es = export_time_ms // 1000
        et = O.DateTime(es, (export_time_ms - es * 1000) * 1_000_000).to_json()
        sets = [{"Data": {"id": 65535, "records": [{"scope_fields": [],
                                                     "fields": [O.field_json(f) for f in fields]}]}}]
        if group["flow_type"] == 10:
            pkt = {"IPFIX": {"version": 10, "export_time": et, "sequence_number": seq,
                             "observation_domain_id": shard_id, "sets": sets}}
        else:
            pkt = {"NetFlowV9": {"version": 9, "sys_up_time": group["max_sysup"], "unix_time": et,
                                 "sequence_number": seq, "source_id": shard_id, "sets": sets}}
        return pkt


def to_field_value(ie, v):
    """Canonical value -> the oracle's Field value convention (ngz_oracle.Field)."""
    dt = ie.dtype
    if ie.kind in ("unknown", "vendor_unknown"):
        return v
    if dt == "ipv4Address":
        return ("v4", v)
    if dt == "ipv6Address":
        return ("v6", int.from_bytes(v, "big"))
    if dt == "float32":
        return ("f32", struct.unpack("<I", struct.pack("<f", v))[0])
    if dt == "float64":
        return ("f64", struct.unpack("<Q", struct.pack("<d", v))[0])
    if dt == "boolean":
        return bool(v)
    if dt.startswith("dateTime"):
        return O.DateTime(*v)
    return v


def aggregate_datagrams(fields, datagrams, peer_port=4739, collection_ms=0, window_s=60, lateness_s=10,
                        peer_ip=DEFAULT_PEER, agg=None, codec=None):
    """Decode `datagrams` in order with one codec (FlowInfoCodec::decode per datagram) and
    aggregate every decoded packet as sent by (peer_ip, peer_port); failed datagrams yield
    nothing.  agg / codec: continue an aggregator (a shard) / a peer's codec."""
    codec = codec if codec is not None else O.FlowInfoCodec()
    agg = agg if agg is not None else FlowAggregatorOracle(fields, window_s, lateness_s)
    for d in datagrams:
        buf = bytearray(d)
        try:
            pkt = codec.decode(buf)
        except O.ParseFail:
            continue
        if pkt is not None:
            agg.push_packet(pkt, peer_port, collection_ms, peer_ip)
    return agg
