"""Parity checker: product (HIP path through the C ABI) vs the CPU oracle.

Datagram mode = FlowCollectorActor::decode_pkt semantics: one template state
per peer, one FlowInfoCodec::decode per datagram (flow_actor.rs:342-411).
Every datagram must agree on: status (Ok(None) / Ok(Some) / Err), the
serde-JSON error text, the message header, and every decoded field of every
record (bit-exact against the canonical column encoding).
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))

import ngz_oracle as O  # noqa: E402

from netgauze_amd import _lib as L  # noqa: E402


def oracle_datagrams(dgrams, codec=None):
    codec = codec or O.FlowInfoCodec()
    out = []
    for dg in dgrams:
        buf = bytearray(dg)
        try:
            m = codec.decode(buf)
            out.append(("none", None) if m is None else ("ok", m))
        except O.ParseFail as e:
            out.append(("err", e.err))
    return out, codec


def canon(val, fi):
    """Oracle value -> the column bytes the product must hold."""
    k, w = fi.kind, fi.width
    if isinstance(val, O.Field):
        val = val.value
    if isinstance(val, O.ScopeFieldValue):
        val = val.value
    if k in (L.K_UINT, L.K_SCOPE32):
        if isinstance(val, tuple):
            val = val[1]
        if isinstance(val, O.DateTime):
            val = val.secs
        return int(val).to_bytes(w, "little")
    if k == L.K_TCPFLAGS:
        return bytes([val & 0xFF])
    if k == L.K_SINT:
        return (val % (1 << (8 * w))).to_bytes(w, "little")
    if k == L.K_BOOL:
        return bytes([1 if val else 0])
    if k == L.K_BYTES:
        if isinstance(val, tuple):
            return val[1].to_bytes(16, "big")
        return bytes(val)
    if k == L.K_U256:
        return bytes(val)
    if k == L.K_DTMS:
        ms = val.secs * 1000 + val.nanos // 1_000_000
        return (ms % (1 << 64)).to_bytes(8, "little")
    if k == L.K_DTFRAC:
        return val.secs.to_bytes(4, "little") + val.nanos.to_bytes(4, "little")
    raise AssertionError("kind %d" % k)


# innermost serde variant -> ngz_error.kind (flow_decode.h)
_ERR_KIND = {"UnsupportedVersion": "UNSUPPORTED_VERSION", "InvalidLength": "INVALID_LENGTH",
             "UnexpectedEof": "UNEXPECTED_EOF", "InvalidPaddingLength": "INVALID_PADDING_LENGTH",
             "InvalidSetId": "INVALID_SET_ID", "NoTemplateDefinedFor": "NO_TEMPLATE",
             "InvalidPaddingValue": "INVALID_PADDING_VALUE", "InvalidCount": "INVALID_COUNT",
             "InvalidTemplateId": "INVALID_TEMPLATE_ID", "InvalidScopeFieldsCount": "INVALID_SCOPE_FIELDS_COUNT",
             "UndefinedIANAIE": "UNDEFINED_IANA_IE", "InvalidTimestamp": "INVALID_TIMESTAMP",
             "InvalidTimestampMillis": "INVALID_TIMESTAMP_MILLIS",
             "InvalidTimestampFraction": "INVALID_TIMESTAMP_FRACTION", "Utf8Error": "UTF8"}


def check_error_struct(batch, d, err):
    """ngz_dgram_error of datagram d against the oracle's serde error value."""
    st = batch.error_struct(d)
    assert st is not None, d
    tags, v = [], err
    while isinstance(v, dict) and len(v) == 1:
        (k, v), = v.items()
        tags.append(k)
    kind = tags[-1]
    assert st["kind"] == _ERR_KIND[kind], (d, st, err)
    layer = ("RECORD" if "DataRecordError" in tags else
             "TEMPLATE" if {"TemplateRecordError", "OptionsTemplateRecordError", "FieldSpecifierError",
                            "ScopeFieldSpecifierError", "IEError"} & set(tags) else
             "SET" if {"SetParsingError", "SetError"} & set(tags) else
             "MESSAGE" if {"IpfixParsingError", "NetFlowV9ParingError"} & set(tags) else "CODEC")
    assert st["layer"] == layer, (d, st, err)
    vendors = {n + "Error" for n in O.REGISTRY.vendors.values()}
    assert st["vendor"] == (1 if vendors & set(tags) else 0), (d, st, err)
    if isinstance(v, dict):
        assert st["offset"] == v.get("offset", 0), (d, st, err)
        expect = {"UnexpectedEof": {"length": v.get("needed"), "available": v.get("available")},
                  "InvalidPaddingLength": {"length": v.get("requested"), "value": v.get("ret_len")},
                  "InvalidSetId": {"value": v.get("id")}, "NoTemplateDefinedFor": {"value": v.get("id")},
                  "InvalidPaddingValue": {"value": v.get("value")}, "InvalidCount": {"value": v.get("count")},
                  "InvalidTemplateId": {"value": v.get("template_id")},
                  "InvalidScopeFieldsCount": {"value": v.get("scope_fields_count"),
                                              "length": v.get("total_fields_count")},
                  "InvalidTimestamp": {"value": v.get("seconds")},
                  "InvalidTimestampMillis": {"value": v.get("millis")},
                  "InvalidTimestampFraction": {"value": v.get("seconds"), "length": v.get("fraction")},
                  "InvalidLength": {"length": v.get("length")},
                  "UnsupportedVersion": {"value": v.get("version")}}.get(kind, {})
        for k, x in expect.items():
            assert st[k] == x, (d, k, st, err)
    elif kind == "UnsupportedVersion":
        assert st["value"] == v
    elif kind == "UndefinedIANAIE":
        assert (st["ie_pen"], st["ie_id"]) == (0, v)
    elif kind == "InvalidLength":  # FieldSpecifierError::InvalidLength(length, IE)
        assert st["length"] == v[0]
    if layer == "RECORD" and isinstance(v, dict) and "ie_name" in v:
        assert st["field"] != 0xFFFF, (d, st)
        ie = O.REGISTRY.by_key.get((st["ie_pen"], st["ie_id"]))
        assert ie is not None and ie.name == v["ie_name"], (d, st, err)
    return st


def check_batch(batch, oracle, check_records=True, max_fail=5, failures=None):
    """Compare; returns stats dict; raises AssertionError with context.  With a `failures`
    list, a datagram that disagrees is appended as (datagram, message) and the comparison
    goes on with the next one (the fuzz corpus wants every divergence of a batch)."""
    hdr = batch.dgram_headers()
    sets = batch.sets()
    by_dg = {}
    for i in range(len(sets)):
        by_dg.setdefault(int(sets[i]["dgram"]), []).append(sets[i])
    cols = {}

    def col(slot, f):
        key = (slot, f)
        if key not in cols:
            cols[key] = batch.slots[slot].column_bytes(f)
        return cols[key]

    stats = {"ok": 0, "none": 0, "err": 0, "unsupported": 0, "records": 0, "fields": 0}
    assert len(oracle) == batch.n_dgrams
    for d, (kind, val) in enumerate(oracle):
        if failures is None:
            _check_dgram(batch, d, kind, val, hdr, by_dg, col, stats, check_records)
            continue
        try:
            _check_dgram(batch, d, kind, val, hdr, by_dg, col, stats, check_records)
        except AssertionError as e:
            failures.append((d, str(e)[:1500]))
    return stats


def _check_dgram(batch, d, kind, val, hdr, by_dg, col, stats, check_records):
    st = int(hdr[d]["status"])
    if st == L.NGZ_DG_UNSUPPORTED:
        stats["unsupported"] += 1
        return
    if kind == "none":
        assert st == L.NGZ_DG_NEED_MORE, "dgram %d: expected Ok(None), status %d" % (d, st)
        stats["none"] += 1
        return
    if kind == "err":
        assert st == L.NGZ_DG_ERROR, "dgram %d: expected error %s, status %d" % (d, O.dumps(val), st)
        got = batch.error_json(d)
        assert got == O.dumps(val), "dgram %d error:\n got %s\n exp %s" % (d, got, O.dumps(val))
        check_error_struct(batch, d, val)
        stats["err"] += 1
        return
    assert st == L.NGZ_DG_OK, "dgram %d: expected Ok(Some), status %d err %s" % (d, st, batch.error_json(d))
    stats["ok"] += 1
    h = hdr[d]
    if isinstance(val, O.IpfixPacket):
        assert (h["version"], h["time"], h["sequence"], h["domain"]) == (
            10, val.export_time.secs, val.sequence_number, val.observation_domain_id), d
    else:
        assert (h["version"], h["sys_up_time"], h["time"], h["sequence"], h["domain"]) == (
            9, val.sys_up_time, val.unix_time.secs, val.sequence_number, val.source_id), d
    data_sets = [s for s in val.sets if s[0] == "Data"]
    got_sets = by_dg.get(d, [])
    assert len(data_sets) == len(got_sets), "dgram %d: %d data sets vs %d" % (d, len(data_sets), len(got_sets))
    for (_, sid, recs), gs in zip(data_sets, got_sets):
        slot = batch.slots[int(gs["slot"])]
        assert slot.template_id == sid and int(gs["n"]) == len(recs), (d, sid, int(gs["n"]), len(recs))
        if not check_records:
            continue
        rec0 = int(gs["rec0"])
        for r, (scope, fields) in enumerate(recs):
            allf = list(scope) + list(fields)
            assert len(allf) == len(slot.fields)
            for f, fv in enumerate(allf):
                fi = slot.fields[f]
                got = bytes(col(int(gs["slot"]), f)[rec0 + r])
                if fi.kind == L.K_VLEN:
                    # {u64 batch offset, u32 length, u32 0} -> the value's bytes in the input batch
                    off = int.from_bytes(got[:8], "little")
                    ln = int.from_bytes(got[8:12], "little")
                    assert got[12:] == bytes(4), (d, r, f, got.hex())
                    v = fv.value
                    exp = v.encode("utf-8") if isinstance(v, str) else bytes(v)
                    assert batch.input_bytes(off, ln) == exp, (d, r, f, off, ln, exp[:32])
                elif fi.kind == L.K_STR:
                    raw = got.split(b"\0", 1)[0]
                    exp = fv.value.encode("utf-8")
                    assert raw == exp, (d, r, f, raw, exp)
                else:
                    exp = canon(fv, fi)
                    assert got == exp, "dgram %d rec %d field %d kind %d: got %s exp %s" % (
                        d, r, f, fi.kind, got.hex(), exp.hex())
                stats["fields"] += 1
            stats["records"] += 1
