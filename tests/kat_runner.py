"""Runs the packet-level KATs of tests/kats_packets.py through the CPU oracle
(packet level, as the reference test does) and builds the codec-level
datagram streams the device tests feed through the C ABI."""
import json
import struct

import kats_packets as K
import ngz_oracle as O

_BY_NAME = {}
for (_pen, _id), _ie in O.REGISTRY.by_key.items():
    _BY_NAME[(_ie.vendor if _pen else None, _ie.name)] = _ie
_VENDOR_PEN = {name: pen for pen, name in O.REGISTRY.vendors.items()}
_SCOPE_IDS = {v: k for k, v in O.SCOPE_NAMES.items()}


def ie_of(el):
    """element_id JSON -> oracle IE (IE::try_from semantics)."""
    if isinstance(el, str):
        return _BY_NAME[(None, el)]
    (k, v), = el.items()
    if k == "Unknown":
        return O.REGISTRY.lookup(v["pen"], v["id"])
    if isinstance(v, dict):
        return O.REGISTRY.lookup(_VENDOR_PEN[k], v["Unknown"]["id"])
    return _BY_NAME[(k, v)]


def spec_of(s):
    return O.FieldSpec(ie_of(s["element_id"]), s["length"])


def _spec_wire(s, scope_v9=False):
    el, ln = s["element_id"], s["length"]
    if scope_v9:
        return struct.pack(">HH", _SCOPE_IDS[el], ln)
    ie = ie_of(el)
    if ie.pen == 0:
        return struct.pack(">HH", ie.id, ln)
    return struct.pack(">HHI", ie.id | 0x8000, ln, ie.pen)


def template_datagram(proto, tid, scope, fields):
    """A message whose only set defines template `tid` as the DecodingTemplate
    a test inserts into its map (TemplateRecord / OptionsTemplateRecord wire
    forms, ipfix.rs:276-327,384-413; netflow.rs:265-353)."""
    if proto == 10:
        if scope:
            body = struct.pack(">HHH", tid, len(scope) + len(fields), len(scope))
            set_id = 3
        else:
            body = struct.pack(">HH", tid, len(fields))
            set_id = 2
        body += b"".join(_spec_wire(s) for s in list(scope) + list(fields))
        st = struct.pack(">HH", set_id, 4 + len(body)) + body
        return struct.pack(">HHIII", 10, 16 + len(st), 0, 0, 0) + st
    if scope:
        sw = b"".join(_spec_wire(s, True) for s in scope)
        fw = b"".join(_spec_wire(s) for s in fields)
        body = struct.pack(">HHH", tid, len(sw), len(fw)) + sw + fw
        set_id = 1
    else:
        body = struct.pack(">HH", tid, len(fields)) + b"".join(_spec_wire(s) for s in fields)
        set_id = 0
    st = struct.pack(">HH", set_id, 4 + len(body)) + body
    return struct.pack(">HHIIII", 9, 1, 0, 0, 0, 0) + st


def nf9_wrap(set_wire):
    """A lone v9 set inside a one-set v9 message (count 1, zero header)."""
    return struct.pack(">HHIIII", 9, 1, 0, 0, 0, 0) + set_wire


NF9_WRAP_HDR = {"version": 9, "sys_up_time": 0, "unix_time": "1970-01-01T00:00:00Z", "sequence_number": 0,
                "source_id": 0}


IPFIX_WRAP_HDR = {"version": 10, "export_time": "1970-01-01T00:00:00Z", "sequence_number": 0,
                  "observation_domain_id": 0}
IPFIX_WRAPPED = ("ipfixset", "tplrec", "fspec", "datarec")
# where the lone item starts inside its wrapping message
_WRAP_AT = {"ipfixset": 16, "tplrec": 20, "fspec": 24, "datarec": 20}


def ipfix_wrap(kind, b, tid=None):
    """A lone IPFIX set / template record / field specifier / data record of
    template `tid` inside a one-set IPFIX message (zero header fields)."""
    if kind == "ipfixset":
        st = b
    else:
        body = {"tplrec": b, "fspec": struct.pack(">HH", 256, 1) + b, "datarec": b}[kind]
        st = struct.pack(">HH", tid if kind == "datarec" else 2, 4 + len(body)) + body
    return struct.pack(">HHIII", 10, 16 + len(st), 0, 0, 0) + st


def _shift_offsets(v, by):
    if isinstance(v, dict):
        return {k: (x + by if k == "offset" else _shift_offsets(x, by)) for k, x in v.items()}
    return v


def ipfix_wrapped_expect(kind, ek, ev, tid=None):
    """The packet value (ek "ok") or IpfixPacketParsingError (ek "err") the
    wrapping message must give for an item-level expectation: the item nested
    as the reference's types nest it (Set / TemplateRecord / FieldSpecifier /
    DataRecord, ipfix.rs:99-108,212-221,419-424), errors wrapped as
    IpfixPacketParsingError::SetParsingError(SetParsingError::
    TemplateRecordError(..)) (ipfix.rs:51,124) with offsets made absolute."""
    if ek == "ok":
        st = {"ipfixset": ev, "tplrec": {"Template": [ev]},
              "fspec": {"Template": [{"id": 256, "field_specifiers": [ev]}]},
              "datarec": {"Data": {"id": tid, "records": [ev]}}}[kind]
        return dict(IPFIX_WRAP_HDR, sets=[st])
    if ek == "err" and kind == "tplrec":
        return {"SetParsingError": {"TemplateRecordError": _shift_offsets(ev, _WRAP_AT[kind])}}
    return None


def step_wire(w):
    return K.wire(w) if isinstance(w, str) else bytes(w)


def preload(tmap, pre):
    for tid, (scope, fields) in pre.items():
        tmap[tid] = O.DecodingTemplate([spec_of(s) for s in scope], [spec_of(s) for s in fields])


def jsonify(obj):
    return json.loads(O.dumps(obj))


def oracle_step(kind, wire, tmap):
    """Packet-level parse as the reference test does it.  Returns
    ("ok", json, consumed) or ("err", error_json, None)."""
    cur = O.Reader(bytes(wire))
    try:
        if kind == "ipfix":
            pkt = O.parse_ipfix_packet(cur, tmap)
            return "ok", jsonify(pkt.to_json())["IPFIX"], cur.offset()
        if kind == "nf9":
            pkt = O.parse_netflow_packet(cur, tmap)
            return "ok", jsonify(pkt.to_json())["NetFlowV9"], cur.offset()
        if kind == "nf9set":
            s = O._nf_set(cur, tmap)
            return "ok", jsonify(O._set_json(s, True)), cur.offset()
        if kind == "ipfixset":
            return "ok", jsonify(O._set_json(O._ipfix_set(cur, tmap), False)), cur.offset()
        if kind == "tplrec":
            return "ok", jsonify(O._ipfix_template_record(cur, tmap)), cur.offset()
        if kind == "fspec":
            return "ok", jsonify(O.parse_field_specifier(cur).to_json()), cur.offset()
        if kind == "datarec":
            (t,) = tmap.values()
            scope, fields = O._ipfix_data_record(cur, t)
            return "ok", jsonify({"scope_fields": [O.field_json(x) for x in scope],
                                  "fields": [O.field_json(x) for x in fields]}), cur.offset()
        raise AssertionError(kind)
    except O.ParseFail as e:
        return "err", jsonify(e.err), None


def codec_datagrams(case_map):
    """Datagram stream of one map at codec level: synthesized template
    messages for preloaded templates, then every step's wire (nf9set wrapped
    into a message).  Returns (preamble datagrams, [(step, datagram)])."""
    pre = []
    for tid, (scope, fields) in case_map.get("preload", {}).items():
        proto = 9 if case_map["steps"][0][0].startswith("nf9") else 10
        pre.append(template_datagram(proto, tid, scope, fields))
    steps = []
    for i, (kind, w, exp) in enumerate(case_map["steps"]):
        b = step_wire(w)
        if kind == "nf9set":
            b = nf9_wrap(b)
        elif kind in IPFIX_WRAPPED:
            b = ipfix_wrap(kind, b, next(iter(case_map.get("preload", {})), None))
        steps.append((i, b))
    return pre, steps
