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
        s = O._nf_set(cur, tmap)
        return "ok", jsonify(O._set_json(s, True)), cur.offset()
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
        steps.append((i, nf9_wrap(b) if kind == "nf9set" else b))
    return pre, steps
