"""CPU ORACLE — test infrastructure only, never part of the product path.

Pure-Python restatement of the NetGauze (v0.13.0) IPFIX / NetFlow v9 decoder,
used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as
the *checker* for the HIP path.  Nothing in netgauze_amd/ imports this file.

Parity pinning: this restatement is checked byte-for-byte against the
reference's own golden pcap -> JSON outputs (assets/pcaps/**/-flow.json and
crates/pcap-decoder/tests/data/502-...-flow.jsonl, copied as data into
tests/golden/) and against the byte-array known-answer tests transcribed from
crates/flow-pkt/src/wire/tests/*.rs (tests/test_oracle_kat.py).  The Rust
reference itself cannot be built here (no cargo/rustc, crates.io
dependencies not vendored; see DESIGN.md "Oracle").

Each function cites the reference file:line it restates.  Paths are relative
to the reference checkout (crates/...).
"""
import json
import math
import os
import struct

_HERE = os.path.dirname(os.path.abspath(__file__))
_REG_PATH = os.path.join(os.path.dirname(_HERE), "netgauze_amd", "data", "ie_registry.json")

IPFIX_VERSION = 10            # crates/flow-pkt/src/ipfix.rs:23
NETFLOW_V9_VERSION = 9        # crates/flow-pkt/src/netflow.rs
IPFIX_HEADER_LENGTH = 16      # wire/deserializer/ipfix.rs:28
DATA_SET_MIN_ID = 256         # crates/flow-pkt/src/lib.rs:174


class ParseFail(Exception):
    """Carries a serde-shaped (externally tagged) error value."""

    def __init__(self, err):
        Exception.__init__(self, err)
        self.err = err


def _wrap(tag, fn, *args):
    try:
        return fn(*args)
    except ParseFail as e:
        raise ParseFail({tag: e.err})


# ---------------------------------------------------------------------------
# L1 byte reader — crates/parse-utils/src/reader.rs:33-296, error.rs:21-40
# ---------------------------------------------------------------------------
def eof(offset, needed, available):
    return ParseFail({"Parse": {"UnexpectedEof": {"offset": offset, "needed": needed, "available": available}}})


def bad_pad(offset, requested, ret_len):
    return ParseFail({"Parse": {"InvalidPaddingLength": {"offset": offset, "requested": requested, "ret_len": ret_len}}})


class Reader:
    """SliceReader: zero-copy cursor, offset absolute from the original buffer
    (reader.rs:33-37, take_slice keeps the absolute offset :157-161)."""
    __slots__ = ("buf", "pos", "end", "base")

    def __init__(self, buf, pos=0, end=None, base=None):
        self.buf = buf
        self.pos = pos
        self.end = len(buf) if end is None else end
        self.base = pos if base is None else base  # offset origin

    def offset(self):
        return self.pos - self.base

    def remaining(self):
        return self.end - self.pos

    def is_empty(self):
        return self.pos >= self.end

    def read_bytes(self, n):  # reader.rs:143-152
        if n > self.end - self.pos:
            raise eof(self.offset(), n, self.end - self.pos)
        b = self.buf[self.pos:self.pos + n]
        self.pos += n
        return b

    def take_slice(self, n):  # reader.rs:157-161
        if n > self.end - self.pos:
            raise eof(self.offset(), n, self.end - self.pos)
        r = Reader(self.buf, self.pos, self.pos + n, self.base)
        self.pos += n
        return r

    def read_uint(self, n):
        return int.from_bytes(self.read_bytes(n), "big")

    def peek_uint(self, n):
        if n > self.end - self.pos:
            raise eof(self.offset(), n, self.end - self.pos)
        return int.from_bytes(self.buf[self.pos:self.pos + n], "big")

    def read_u8(self):  # reader.rs:72-81 (eof reports needed 1, available 0)
        if self.pos >= self.end:
            raise eof(self.offset(), 1, 0)
        v = self.buf[self.pos]
        self.pos += 1
        return v

    def peek_u8(self):  # reader.rs:164-169
        if self.pos >= self.end:
            raise eof(self.offset(), 1, 0)
        return self.buf[self.pos]

    def read_unsigned_be(self, n, cap):
        """read_unsigned32_be / read_unsigned64_be (reader.rs:214-264):
        reduced-size right-aligned big endian; len > cap rejected."""
        if n > cap:
            raise bad_pad(self.offset(), n, cap)
        if n == 0:
            return 0
        return self.read_uint(n)

    def read_signed_be(self, n, cap):  # reader.rs:272-295
        v = self.read_unsigned_be(n, cap)
        if n == 0:
            return 0
        bits = 8 * n
        if v >> (bits - 1):
            v -= 1 << bits
        return v

    def read_padded(self, n, cap):  # reader.rs:192-200
        if n > cap:
            raise bad_pad(self.offset(), n, cap)
        b = self.read_bytes(n)
        return bytes(b) + bytes(cap - n)


# ---------------------------------------------------------------------------
# L0 IE registry — generated from the reference XML by tools/gen_ie_registry.py
# (restating ipfix-code-generator/src/xml_parsers/ipfix.rs:141-291)
# ---------------------------------------------------------------------------
# length_range per data type — crates/flow-pkt/src/ie.rs:114-149 (half-open)
LENGTH_RANGE = {
    "octetArray": None, "unsigned8": (1, 2), "unsigned16": (1, 3), "unsigned32": (1, 5),
    "unsigned64": (1, 9), "signed8": (1, 2), "signed16": (1, 3), "signed32": (1, 5),
    "signed64": (1, 9), "float32": (4, 5), "float64": (8, 9), "boolean": (1, 2),
    "macAddress": (6, 7), "string": None, "dateTimeSeconds": (4, 5),
    "dateTimeMilliseconds": (8, 9), "dateTimeMicroseconds": (8, 9),
    "dateTimeNanoseconds": (8, 9), "ipv4Address": (4, 5), "ipv6Address": (16, 17),
    "basicList": None, "subTemplateList": None, "subTemplateMultiList": None,
    "unsigned256": (1, 33),
}


class IE:
    """IE / vendor IE / IE::Unknown.  kind in {iana, vendor, vendor_unknown, unknown}.
    TryFrom<(u32,u16)> semantics: generator.rs:390-430 and :270-293."""
    __slots__ = ("kind", "pen", "id", "name", "dtype", "subreg", "vendor")

    def __init__(self, kind, pen, id, name=None, dtype="octetArray", subreg=None, vendor=None):
        self.kind, self.pen, self.id, self.name = kind, pen, id, name
        self.dtype, self.subreg, self.vendor = dtype, subreg, vendor

    def length_range(self):
        return LENGTH_RANGE[self.dtype]

    def to_json(self):
        if self.kind == "iana":
            return self.name
        if self.kind == "vendor":
            return {self.vendor: self.name}
        if self.kind == "vendor_unknown":
            return {self.vendor: {"Unknown": {"id": self.id}}}
        return {"Unknown": {"pen": self.pen, "id": self.id}}

    def __eq__(self, other):
        return isinstance(other, IE) and (self.kind, self.pen, self.id) == (other.kind, other.pen, other.id)

    def __hash__(self):
        return hash((self.kind, self.pen, self.id))

    def __repr__(self):
        return "IE(%s,%d,%d,%s)" % (self.kind, self.pen, self.id, self.name)


class Registry:
    def __init__(self, path=_REG_PATH):
        with open(path) as f:
            d = json.load(f)
        self.by_key = {}
        self.vendors = {v["pen"]: v["name"] for v in d["vendors"]}
        for ie in d["ies"]:
            pen = ie["pen"]
            kind = "iana" if pen == 0 else "vendor"
            self.by_key[(pen, ie["id"])] = IE(kind, pen, ie["id"], ie["name"], ie["type"],
                                               ie["subreg"], self.vendors.get(pen))

    def lookup(self, pen, code):
        """IE::try_from((pen, code)) — generator.rs:410-428."""
        if pen == 0:
            ie = self.by_key.get((0, code))
            if ie is None:
                raise ParseFail({"IEError": {"UndefinedIANAIE": code}})
            return ie
        if pen in self.vendors:
            code &= 0x7FFF  # vendor try_from removes the enterprise bit (generator.rs:285-286)
            ie = self.by_key.get((pen, code))
            if ie is None:
                return IE("vendor_unknown", pen, code, None, "octetArray", None, self.vendors[pen])
            return ie
        return IE("unknown", pen, code)


REGISTRY = Registry()


# ---------------------------------------------------------------------------
# chrono 0.4.45 restatement (Cargo.lock): validity of timestamp_opt /
# timestamp_millis_opt and the RFC 3339 serde form (AutoSi, 'Z').
# ---------------------------------------------------------------------------
_MIN_YEAR, _MAX_YEAR = -262143, 262142  # chrono NaiveDate::MIN / MAX (0.4.45)


def _civil_from_days(z):
    z += 719468
    era = (z if z >= 0 else z - 146096) // 146097
    doe = z - era * 146097
    yoe = (doe - doe // 1460 + doe // 36524 - doe // 146096) // 365
    y = yoe + era * 400
    doy = doe - (365 * yoe + yoe // 4 - yoe // 100)
    mp = (5 * doy + 2) // 153
    d = doy - (153 * mp + 2) // 5 + 1
    m = mp + 3 if mp < 10 else mp - 9
    return (y + 1 if m <= 2 else y), m, d


class DateTime:
    __slots__ = ("secs", "nanos")

    def __init__(self, secs, nanos):
        self.secs, self.nanos = secs, nanos

    def __eq__(self, other):
        return isinstance(other, DateTime) and (self.secs, self.nanos) == (other.secs, other.nanos)

    def __repr__(self):
        return "DateTime(%d,%d)" % (self.secs, self.nanos)

    def to_json(self):
        days, sod = divmod(self.secs, 86400)
        y, mo, d = _civil_from_days(days)
        hh, rem = divmod(sod, 3600)
        mm, ss = divmod(rem, 60)
        nanos = self.nanos
        if nanos >= 1_000_000_000:  # leap second displayed as :60
            ss += 1
            nanos -= 1_000_000_000
        ys = "%04d" % y if 0 <= y <= 9999 else "%+05d" % y
        s = "%s-%02d-%02dT%02d:%02d:%02d" % (ys, mo, d, hh, mm, ss)
        if nanos == 0:
            pass
        elif nanos % 1_000_000 == 0:
            s += ".%03d" % (nanos // 1_000_000)
        elif nanos % 1_000 == 0:
            s += ".%06d" % (nanos // 1_000)
        else:
            s += ".%09d" % nanos
        return s + "Z"


def timestamp_opt(secs, nanos):
    """Utc.timestamp_opt(secs, nsecs): None on out-of-range date or invalid
    nanos; nanos in [1e9, 2e9) accepted only at second 59 (leap second)."""
    days, sod = divmod(secs, 86400)
    if nanos >= 2_000_000_000 or (nanos >= 1_000_000_000 and sod % 60 != 59):
        return None
    y, _, _ = _civil_from_days(days)
    if y < _MIN_YEAR or y > _MAX_YEAR:
        return None
    return DateTime(secs, nanos)


def timestamp_millis_opt(millis):
    secs, ms = divmod(millis, 1000)
    return timestamp_opt(secs, ms * 1_000_000)


# ---------------------------------------------------------------------------
# Field values and the generated Field::parse — generator.rs:1412-1846,2841-2980
# ---------------------------------------------------------------------------
class Field:
    """A decoded Field: (IE, python value).  Value conventions:
    ints for unsigned/signed/tcp/subregistry IEs, bytes for octet-like and
    mac/mpls/u256, str for strings, DateTime, ('v4', int) / ('v6', int) for
    addresses, ('f64', bits) for floats, bool."""
    __slots__ = ("ie", "value")

    def __init__(self, ie, value):
        self.ie, self.value = ie, value

    def __eq__(self, other):
        return isinstance(other, Field) and self.ie == other.ie and self.value == other.value

    def __repr__(self):
        return "Field(%r=%r)" % (self.ie, self.value)


def _invalid_length(cur, ie, length):
    # generator.rs:1423-1437: offset captured before reading
    return ParseFail({"InvalidLength": {"offset": cur.offset(), "ie_name": ie.name, "length": length}})


def _vlen(cur, length):
    """u16::MAX marks a variable-length field: 1-byte length, 0xFF escape to a
    3-byte length (generator.rs:1775-1793, RFC 7011 s7)."""
    if length == 0xFFFF:
        short = cur.read_u8()
        if short == 0xFF:
            return cur.read_unsigned_be(3, 4)
        return short
    return length


def _decode_typed(cur, ie, length):
    dt = ie.dtype
    name = ie.name
    if dt == "octetArray":
        if name == "mplsTopLabelStackSection" or name.startswith("mplsLabelStackSection"):
            if length != 3:  # generator.rs:1795-1807
                raise _invalid_length(cur, ie, length)
            return bytes(cur.read_bytes(3))
        return bytes(cur.read_bytes(_vlen(cur, length)))
    if dt in ("basicList", "subTemplateList", "subTemplateMultiList"):
        return bytes(cur.read_bytes(_vlen(cur, length)))
    if dt in ("unsigned8",):  # :1439-1451
        if length != 1:
            raise _invalid_length(cur, ie, length)
        return cur.read_u8()
    if dt == "unsigned16":  # :1453-1466
        if length == 1:
            return cur.read_u8()
        if length == 2:
            return cur.read_uint(2)
        raise _invalid_length(cur, ie, length)
    if dt == "unsigned32":  # :1468-1481
        if length > 4:
            raise _invalid_length(cur, ie, length)
        return cur.read_unsigned_be(length, 4)
    if dt == "unsigned64":  # :1483-1496
        if length > 8:
            raise _invalid_length(cur, ie, length)
        return cur.read_unsigned_be(length, 8)
    if dt == "unsigned256":  # :1498-1518
        if length > 32:
            raise _invalid_length(cur, ie, length)
        return cur.read_padded(length, 32)
    if dt == "signed8":
        if length != 1:
            raise _invalid_length(cur, ie, length)
        v = cur.read_u8()
        return v - 256 if v >= 128 else v
    if dt == "signed32":  # :1549-1562 (len<=8 check, read_signed32_be caps at 4)
        if length > 8:
            raise _invalid_length(cur, ie, length)
        return cur.read_signed_be(length, 4)
    if dt == "signed64":
        if length > 8:
            raise _invalid_length(cur, ie, length)
        return cur.read_signed_be(length, 8)
    if dt == "float32":
        if length != 4:
            raise _invalid_length(cur, ie, length)
        return ("f32", cur.read_uint(4))
    if dt == "float64":  # :1593-1605
        if length != 8:
            raise _invalid_length(cur, ie, length)
        return ("f64", cur.read_uint(8))
    if dt == "boolean":  # :1607-1619
        if length != 1:
            raise _invalid_length(cur, ie, length)
        return cur.read_u8() != 0
    if dt == "macAddress":  # :1621-1633
        if length != 6:
            raise _invalid_length(cur, ie, length)
        return bytes(cur.read_bytes(6))
    if dt == "string":  # :1635-1672
        if length == 0xFFFF:
            short = cur.read_u8()
            ln = cur.read_unsigned_be(3, 4) if short == 0xFF else short
            off = cur.offset()
            raw = bytes(cur.read_bytes(ln))
        else:
            off = cur.offset()
            raw = bytes(cur.read_bytes(length))
            nul = raw.find(b"\0")
            if nul >= 0:
                raw = raw[:nul]
        try:
            return raw.decode("utf-8")
        except UnicodeDecodeError as e:
            raise ParseFail({"Utf8Error": {"offset": off, "ie_name": name, "error": _rust_utf8_msg(raw, e)}})
    if dt == "ipv4Address":  # :1674-1686
        if length != 4:
            raise _invalid_length(cur, ie, length)
        return ("v4", cur.read_uint(4))
    if dt == "ipv6Address":  # :1688-1700
        if length != 16:
            raise _invalid_length(cur, ie, length)
        return ("v6", cur.read_uint(16))
    if dt == "dateTimeSeconds":  # :1702-1723
        if length != 4:
            raise _invalid_length(cur, ie, length)
        off = cur.offset()
        secs = cur.read_uint(4)
        v = timestamp_opt(secs, 0)
        if v is None:
            raise ParseFail({"InvalidTimestamp": {"offset": off, "ie_name": name, "seconds": secs}})
        return v
    if dt == "dateTimeMilliseconds":  # :1725-1746
        if length != 8:
            raise _invalid_length(cur, ie, length)
        off = cur.offset()
        millis = cur.read_uint(8)
        signed = millis - (1 << 64) if millis >= (1 << 63) else millis  # u64 as i64
        v = timestamp_millis_opt(signed)
        if v is None:
            raise ParseFail({"InvalidTimestampMillis": {"offset": off, "ie_name": name, "millis": millis}})
        return v
    if dt in ("dateTimeMicroseconds", "dateTimeNanoseconds"):  # :1748-1773
        if length != 8:
            raise _invalid_length(cur, ie, length)
        off = cur.offset()
        secs = cur.read_uint(4)
        frac = cur.read_uint(4)
        nanos = fraction_to_nanos(frac)
        v = timestamp_opt(secs, nanos)
        if v is None:
            raise ParseFail({"InvalidTimestampFraction": {"offset": off, "ie_name": name, "seconds": secs, "fraction": frac}})
        return v
    raise NotImplementedError(dt)


def fraction_to_nanos(frac):
    """(1_000_000_000f64 * (fraction as f64 / u32::MAX as f64)) as u32
    (generator.rs:1764).  IEEE double, divide then multiply, truncate."""
    return int(1000000000.0 * (float(frac) / 4294967295.0))


def _rust_utf8_msg(raw, e):
    """core::str::Utf8Error Display."""
    valid_up_to = e.start
    # error_len: None if incomplete sequence at end
    rest = raw[valid_up_to:]
    lead = rest[0]
    need = 1 if lead < 0x80 else 2 if 0xC2 <= lead <= 0xDF else 3 if 0xE0 <= lead <= 0xEF else 4 if 0xF0 <= lead <= 0xF4 else 0
    if need == 0:
        return "invalid utf-8 sequence of 1 bytes from index %d" % valid_up_to
    # count how many bytes form a valid prefix of the sequence
    i = 1
    while i < need and i < len(rest):
        b = rest[i]
        lo, hi = 0x80, 0xBF
        if i == 1:
            if lead == 0xE0:
                lo = 0xA0
            elif lead == 0xED:
                hi = 0x9F
            elif lead == 0xF0:
                lo = 0x90
            elif lead == 0xF4:
                hi = 0x8F
        if not (lo <= b <= hi):
            return "invalid utf-8 sequence of %d bytes from index %d" % (i, valid_up_to)
        i += 1
    if i < need:
        return "incomplete utf-8 byte sequence from index %d" % valid_up_to
    return "invalid utf-8 sequence of %d bytes from index %d" % (i, valid_up_to)


def parse_field(cur, ie, length):
    """Field::parse — main dispatch generator.rs:2959-2978; vendor package
    dispatch :2875-2895 (vendor Unknown is vlen-aware, IE::Unknown is not)."""
    if ie.kind == "unknown":
        return Field(ie, bytes(cur.read_bytes(length)))
    if ie.kind == "vendor_unknown":
        try:
            return Field(ie, bytes(cur.read_bytes(_vlen(cur, length))))
        except ParseFail as e:
            raise ParseFail({ie.vendor + "Error": e.err})
    if ie.kind == "vendor":
        try:
            return Field(ie, _decode_typed(cur, ie, length))
        except ParseFail as e:
            raise ParseFail({ie.vendor + "Error": e.err})
    return Field(ie, _decode_typed(cur, ie, length))


# ---------------------------------------------------------------------------
# Templates — lib.rs:147-154 (FieldSpecifier::new), deserializer/mod.rs:50-67
# ---------------------------------------------------------------------------
class FieldSpec:
    __slots__ = ("ie", "length")

    def __init__(self, ie, length):
        self.ie, self.length = ie, length

    def to_json(self):
        return {"element_id": self.ie.to_json(), "length": self.length}

    def __eq__(self, o):
        return isinstance(o, FieldSpec) and (self.ie, self.length) == (o.ie, o.length)

    def __repr__(self):
        return "FieldSpec(%r,%d)" % (self.ie, self.length)


def parse_field_specifier(cur):
    """FieldSpecifier::parse (deserializer/mod.rs:53-66)."""
    code = cur.read_uint(2)
    enterprise = code & 0x8000 != 0
    length = cur.read_uint(2)
    if enterprise:
        pen = cur.read_uint(4)
        code &= 0x7FFF
    else:
        pen = 0
    ie = REGISTRY.lookup(pen, code)
    rng = ie.length_range()
    if rng is not None and not (rng[0] <= length < rng[1]):
        raise ParseFail({"FieldSpecifierError": {"InvalidLength": [length, ie.to_json()]}})
    return FieldSpec(ie, length)


class DecodingTemplate:
    """ipfix.rs:32-70 / netflow.rs:37 — scope specs, field specs, processed_count."""
    __slots__ = ("scope", "fields", "processed_count")

    def __init__(self, scope, fields):
        self.scope, self.fields, self.processed_count = list(scope), list(fields), 0


# ---------------------------------------------------------------------------
# IPFIX — wire/deserializer/ipfix.rs
# ---------------------------------------------------------------------------
def _check_padding(buf):  # ipfix.rs:240-251 / netflow.rs:237-248
    while not buf.is_empty():
        off = buf.offset()
        v = buf.peek_u8()
        if v != 0:
            raise ParseFail({"InvalidPaddingValue": {"offset": off, "value": v}})
        buf.read_u8()


def _ipfix_template_record(cur, tmap):  # ipfix.rs:384-413
    off = cur.offset()
    tid = cur.peek_uint(2)
    if tid < 256:
        raise ParseFail({"InvalidTemplateId": {"offset": off, "template_id": tid}})
    cur.read_uint(2)
    count = cur.read_uint(2)
    fields = [_wrap("FieldSpecifierError", parse_field_specifier, cur) for _ in range(count)]
    tmap[tid] = DecodingTemplate([], fields)
    return {"id": tid, "field_specifiers": [f.to_json() for f in fields]}


def _ipfix_options_template_record(cur, tmap):  # ipfix.rs:276-327
    off = cur.offset()
    tid = cur.peek_uint(2)
    if tid < 256:
        raise ParseFail({"InvalidTemplateId": {"offset": off, "template_id": tid}})
    cur.read_uint(2)
    total = cur.read_uint(2)
    soff = cur.offset()
    scount = cur.peek_uint(2)
    if scount > total:
        raise ParseFail({"InvalidScopeFieldsCount": {"offset": soff, "scope_fields_count": scount, "total_fields_count": total}})
    cur.read_uint(2)
    scope = [_wrap("FieldError", parse_field_specifier, cur) for _ in range(scount)]
    fields = [_wrap("FieldError", parse_field_specifier, cur) for _ in range(total - scount)]
    tmap[tid] = DecodingTemplate(scope, fields)
    return {"id": tid, "scope_field_specifiers": [f.to_json() for f in scope],
            "field_specifiers": [f.to_json() for f in fields]}


def _ipfix_data_record(cur, t):  # ipfix.rs:335-370
    scope = [parse_field(cur, s.ie, s.length) for s in t.scope]
    fields = [parse_field(cur, s.ie, s.length) for s in t.fields]
    return (scope, fields)


def min_record_length(t):
    """ipfix.rs:193-214: sum of lengths, vlen (65535) counted as 1."""
    return sum(1 if s.length == 0xFFFF else s.length for s in t.scope) + \
        sum(1 if s.length == 0xFFFF else s.length for s in t.fields)


def _ipfix_set(cur, tmap):  # ipfix.rs:133-238
    id_off = cur.offset()
    sid = cur.peek_uint(2)
    if sid != 2 and sid != 3 and sid < DATA_SET_MIN_ID:
        raise ParseFail({"InvalidSetId": {"offset": id_off, "id": sid}})
    cur.read_uint(2)
    length = cur.peek_uint(2)
    if length < 4:
        raise ParseFail({"InvalidLength": {"offset": cur.offset(), "length": length}})
    cur.read_uint(2)
    buf = cur.take_slice(length - 4)
    if sid == 2:
        recs = []
        while not buf.is_empty():
            recs.append(_wrap("TemplateRecordError", _ipfix_template_record, buf, tmap))
        return ("Template", sid, recs)
    if sid == 3:
        recs = []
        while buf.remaining() > 3:
            recs.append(_wrap("OptionsTemplateRecordError", _ipfix_options_template_record, buf, tmap))
        _check_padding(buf)
        return ("OptionsTemplate", sid, recs)
    t = tmap.get(sid)
    if t is None:
        raise ParseFail({"NoTemplateDefinedFor": {"offset": id_off, "id": sid}})
    mlen = min_record_length(t)
    records = []
    while buf.remaining() >= mlen and mlen > 0:
        records.append(_wrap("DataRecordError", _wrap, "FieldError", _ipfix_data_record, buf, t))
    t.processed_count = (t.processed_count + 1) & 0xFFFFFFFFFFFFFFFF  # once per SET (:223)
    while not buf.is_empty() and buf.peek_u8() == 0:
        buf.read_u8()
    return ("Data", sid, records)


def parse_ipfix_packet(cur, tmap):  # ipfix.rs:54-104
    version = cur.peek_uint(2)
    if version != IPFIX_VERSION:
        raise ParseFail({"UnsupportedVersion": {"offset": cur.offset(), "version": version}})
    cur.read_uint(2)
    length = cur.peek_uint(2)
    if length < IPFIX_HEADER_LENGTH:
        raise ParseFail({"InvalidLength": {"offset": cur.offset(), "length": length}})
    cur.read_uint(2)
    buf = cur.take_slice(length - 4)
    export_time = buf.peek_uint(4)
    et = timestamp_opt(export_time, 0)
    if et is None:
        raise ParseFail({"InvalidExportTime": {"offset": buf.offset(), "export_time": export_time}})
    buf.read_uint(4)
    seq = buf.read_uint(4)
    obs = buf.read_uint(4)
    sets = []
    while not buf.is_empty():
        sets.append(_wrap("SetParsingError", _ipfix_set, buf, tmap))
    return IpfixPacket(et, seq, obs, sets)


class IpfixPacket:
    def __init__(self, export_time, seq, obs, sets):
        self.export_time, self.sequence_number, self.observation_domain_id, self.sets = export_time, seq, obs, sets

    def to_json(self):
        return {"IPFIX": {"version": 10, "export_time": self.export_time.to_json(),
                          "sequence_number": self.sequence_number,
                          "observation_domain_id": self.observation_domain_id,
                          "sets": [_set_json(s, False) for s in self.sets]}}

    def data_records(self):
        for kind, sid, recs in self.sets:
            if kind == "Data":
                for r in recs:
                    yield sid, r


# ---------------------------------------------------------------------------
# NetFlow v9 — wire/deserializer/netflow.rs
# ---------------------------------------------------------------------------
SCOPE_NAMES = {1: "System", 2: "Interface", 3: "LineCard", 4: "Cache", 5: "Template"}


class ScopeIE:
    """ScopeIE::from((pen, code)) — crates/flow-pkt/src/netflow.rs:404-416.
    Note: the enterprise bit is NOT masked off the code."""
    __slots__ = ("pen", "id")

    def __init__(self, pen, code):
        self.pen, self.id = pen, code

    def name(self):
        return SCOPE_NAMES.get(self.id) if self.pen == 0 else None

    def length_range(self):  # netflow.rs:424-437 data types
        n = self.name()
        if n in ("Interface", "LineCard"):
            return (1, 5)
        return None

    def to_json(self):
        n = self.name()
        return n if n is not None else {"Unknown": {"pen": self.pen, "id": self.id}}

    def __eq__(self, o):
        return isinstance(o, ScopeIE) and (self.pen, self.id) == (o.pen, o.id)

    def __hash__(self):
        return hash((self.pen, self.id))


class ScopeSpec:
    __slots__ = ("ie", "length")

    def __init__(self, ie, length):
        self.ie, self.length = ie, length

    def to_json(self):
        return {"element_id": self.ie.to_json(), "length": self.length}


def parse_scope_field_specifier(cur):  # netflow.rs:368-388
    off = cur.offset()
    code = cur.read_uint(2)
    enterprise = code & 0x8000 != 0
    length = cur.read_uint(2)
    pen = cur.read_uint(4) if enterprise else 0
    ie = ScopeIE(pen, code)
    rng = ie.length_range()
    if rng is not None and not (rng[0] <= length < rng[1]):
        raise ParseFail({"InvalidLength": {"offset": off, "ie": ie.to_json(), "length": length}})
    return ScopeSpec(ie, length)


class ScopeFieldValue:
    __slots__ = ("ie", "value")

    def __init__(self, ie, value):
        self.ie, self.value = ie, value

    def to_json(self):
        n = self.ie.name()
        if n is None:
            return {"Unknown": {"pen": self.ie.pen, "id": self.ie.id, "value": list(self.value)}}
        if n in ("Cache", "Template"):
            return {n: list(self.value)}
        return {n: self.value}

    def __eq__(self, o):
        return isinstance(o, ScopeFieldValue) and self.ie == o.ie and self.value == o.value


def parse_scope_field(cur, ie, length):  # netflow.rs:443-475
    n = ie.name()
    if n in ("System", "Interface", "LineCard"):
        if length > 4:
            raise ParseFail({"InvalidLength": {"offset": cur.offset(), "length": length}})
        return ScopeFieldValue(ie, cur.read_unsigned_be(length, 8) & 0xFFFFFFFF)
    return ScopeFieldValue(ie, bytes(cur.read_bytes(length)))


def _nf_template_record(cur, tmap):  # netflow.rs:324-353
    off = cur.offset()
    tid = cur.peek_uint(2)
    if tid < 256:
        raise ParseFail({"InvalidTemplateId": {"offset": off, "template_id": tid}})
    cur.read_uint(2)
    count = cur.read_uint(2)
    fields = [_wrap("FieldSpecifierError", parse_field_specifier, cur) for _ in range(count)]
    tmap[tid] = DecodingTemplate([], fields)
    return {"id": tid, "field_specifiers": [f.to_json() for f in fields]}


def _nf_options_template_record(cur, tmap):  # netflow.rs:265-310
    off = cur.offset()
    tid = cur.peek_uint(2)
    if tid < 256:
        raise ParseFail({"InvalidTemplateId": {"offset": off, "template_id": tid}})
    cur.read_uint(2)
    scope_len = cur.read_uint(2)
    opt_len = cur.read_uint(2)
    sbuf = cur.take_slice(scope_len)
    obuf = cur.take_slice(opt_len)
    scope = []
    while not sbuf.is_empty():
        scope.append(_wrap("ScopeFieldSpecifierError", parse_scope_field_specifier, sbuf))
    fields = []
    while not obuf.is_empty():
        fields.append(_wrap("FieldSpecifierError", parse_field_specifier, obuf))
    tmap[tid] = DecodingTemplate(scope, fields)
    return {"id": tid, "scope_field_specifiers": [s.to_json() for s in scope],
            "field_specifiers": [f.to_json() for f in fields]}


def _nf_data_record(cur, t):  # netflow.rs:399-432
    scope = [_wrap("ScopeFieldError", parse_scope_field, cur, s.ie, s.length) for s in t.scope]
    fields = [_wrap("FieldError", parse_field, cur, s.ie, s.length) for s in t.fields]
    return (scope, fields)


def _nf_set(cur, tmap):  # netflow.rs:143-235
    id_off = cur.offset()
    sid = cur.peek_uint(2)
    if sid != 0 and sid != 1 and sid < DATA_SET_MIN_ID:
        raise ParseFail({"InvalidSetId": {"offset": id_off, "id": sid}})
    cur.read_uint(2)
    length = cur.peek_uint(2)
    if length < 4:
        raise ParseFail({"InvalidLength": {"offset": cur.offset(), "length": length}})
    cur.read_uint(2)
    buf = cur.take_slice(length - 4)
    if sid == 0:
        recs = []
        while not buf.is_empty():
            recs.append(_wrap("TemplateRecordError", _nf_template_record, buf, tmap))
        return ("Template", sid, recs)
    if sid == 1:
        recs = []
        while buf.remaining() > 3:
            recs.append(_wrap("OptionsTemplateRecordError", _nf_options_template_record, buf, tmap))
        _check_padding(buf)
        return ("OptionsTemplate", sid, recs)
    t = tmap.get(sid)
    if t is None:
        raise ParseFail({"NoTemplateDefinedFor": {"offset": id_off, "id": sid}})
    rlen = sum(s.length for s in t.scope) + sum(s.length for s in t.fields)  # 65535 literal
    records = []
    if rlen != 0:
        while buf.remaining() >= rlen:
            records.append(_wrap("DataRecordError", _nf_data_record, buf, t))
            t.processed_count = (t.processed_count + 1) & 0xFFFFFFFFFFFFFFFF  # per RECORD (:218)
    _check_padding(buf)
    return ("Data", sid, records)


def parse_netflow_packet(cur, tmap):  # netflow.rs:56-114
    version = cur.peek_uint(2)
    if version != NETFLOW_V9_VERSION:
        raise ParseFail({"UnsupportedVersion": {"offset": cur.offset(), "version": version}})
    cur.read_uint(2)
    count_off = cur.offset()
    count = cur.read_uint(2)
    sys_up = cur.read_uint(4)
    unix = cur.peek_uint(4)
    ut = timestamp_opt(unix, 0)
    if ut is None:
        raise ParseFail({"InvalidUnixTime": {"offset": cur.offset(), "unix_time": unix}})
    cur.read_uint(4)
    seq = cur.read_uint(4)
    src = cur.read_uint(4)
    sets = []
    i = count
    while i > 0 and cur.remaining() > 3:
        s = _wrap("SetError", _nf_set, cur, tmap)
        if s[0] == "Data":
            if len(s[2]) > i:
                raise ParseFail({"InvalidCount": {"offset": count_off, "count": count}})
            i -= len(s[2])
        else:
            i -= 1
        sets.append(s)
    return NetFlowV9Packet(sys_up, ut, seq, src, sets)


class NetFlowV9Packet:
    def __init__(self, sys_up, unix_time, seq, source_id, sets):
        self.sys_up_time, self.unix_time, self.sequence_number = sys_up, unix_time, seq
        self.source_id, self.sets = source_id, sets

    def to_json(self):
        return {"NetFlowV9": {"version": 9, "sys_up_time": self.sys_up_time,
                              "unix_time": self.unix_time.to_json(),
                              "sequence_number": self.sequence_number, "source_id": self.source_id,
                              "sets": [_set_json(s, True) for s in self.sets]}}

    def data_records(self):
        for kind, sid, recs in self.sets:
            if kind == "Data":
                for r in recs:
                    yield sid, r


# ---------------------------------------------------------------------------
# FlowInfoCodec — crates/flow-pkt/src/codec.rs:68-220
# ---------------------------------------------------------------------------
class FlowInfoCodec:
    """One codec per exporter peer: owns the v9 and v10 template maps."""

    def __init__(self):
        self.netflow_templates = {}
        self.ipfix_templates = {}

    def decode(self, buf):
        """Decoder::decode over a bytearray `buf` (consumed in place).
        Returns None (need more data), a packet, or raises ParseFail with the
        FlowInfoCodecDecoderError value."""
        if len(buf) < IPFIX_HEADER_LENGTH:
            return None
        version = (buf[0] << 8) | buf[1]
        length = (buf[2] << 8) | buf[3]
        if len(buf) < length:
            return None
        if version == IPFIX_VERSION:
            cur = Reader(bytes(buf))
            try:
                msg = parse_ipfix_packet(cur, self.ipfix_templates)
            except ParseFail as e:
                del buf[:max(5, length)]
                raise ParseFail({"IpfixParsingError": e.err})
            del buf[:cur.offset()]
            return msg
        if version == NETFLOW_V9_VERSION:
            cur = Reader(bytes(buf))
            try:
                msg = parse_netflow_packet(cur, self.netflow_templates)
            except ParseFail as e:
                del buf[:]
                raise ParseFail({"NetFlowV9ParingError": e.err})
            del buf[:cur.offset()]
            return msg
        del buf[:]
        raise ParseFail({"UnsupportedVersion": version})


# ---------------------------------------------------------------------------
# serde JSON layer (pinning only): externally tagged enums, serde_json text
# ---------------------------------------------------------------------------
def _ipv4_str(v):
    return "%d.%d.%d.%d" % ((v >> 24) & 255, (v >> 16) & 255, (v >> 8) & 255, v & 255)


def ipv6_str(v):
    """core::net::Ipv6Addr Display (RFC 5952; ::ffff:a.b.c.d for v4-mapped)."""
    segs = [(v >> (112 - 16 * i)) & 0xFFFF for i in range(8)]
    if segs[:5] == [0, 0, 0, 0, 0] and segs[5] == 0xFFFF:
        return "::ffff:" + _ipv4_str(v & 0xFFFFFFFF)
    best_s, best_l, cur_s, cur_l = 0, 0, 0, 0
    for i, s in enumerate(segs):
        if s == 0:
            if cur_l == 0:
                cur_s = i
            cur_l += 1
            if cur_l > best_l:
                best_s, best_l = cur_s, cur_l
        else:
            cur_l = 0
    if best_l > 1:
        return ":".join("%x" % s for s in segs[:best_s]) + "::" + ":".join("%x" % s for s in segs[best_s + best_l:])
    return ":".join("%x" % s for s in segs)


def ryu_format(x, shortest_repr):
    """serde_json float text (ryu crate format64/format32 layout) from the
    shortest round-trip digits."""
    from decimal import Decimal
    if x == 0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    sign = "-" if x < 0 else ""
    t = Decimal(shortest_repr(abs(x))).as_tuple()
    digits = "".join(str(d) for d in t.digits).lstrip("0")
    k = t.exponent
    stripped = digits.rstrip("0")
    k += len(digits) - len(stripped)
    digits = stripped
    n = len(digits)
    kk = n + k
    if 0 <= k and kk <= 16:
        out = digits + "0" * k + ".0"
    elif 0 < kk <= 16:
        out = digits[:kk] + "." + digits[kk:]
    elif -5 < kk <= 0:
        out = "0." + "0" * (-kk) + digits
    elif n == 1:
        out = digits + "e" + str(kk - 1)
    else:
        out = digits[0] + "." + digits[1:] + "e" + str(kk - 1)
    return sign + out


def _f32_shortest(x):
    for p in range(1, 18):
        s = "%.*g" % (p, x)
        if struct.unpack(">f", struct.pack(">f", float(s)))[0] == x:
            return s
    return repr(x)


def _f64_json(bits):
    x = struct.unpack(">d", bits.to_bytes(8, "big"))[0]
    if math.isnan(x) or math.isinf(x):
        return None
    return _RawNum(ryu_format(x, repr))


def _f32_json(bits):
    x = struct.unpack(">f", bits.to_bytes(4, "big"))[0]
    if math.isnan(x) or math.isinf(x):
        return None
    return _RawNum(ryu_format(x, _f32_shortest))


class _RawNum(str):
    pass


def _subreg_json(sub, v):
    if sub["kind"] == "vnd":
        for val, name in sub["entries"]:
            if val == v:
                return name
        return {"Unassigned": v}
    for idx, (_, name, reasons) in enumerate(sub["entries"]):
        if 64 * idx <= v <= 64 * idx + 63:
            for rv, rn in reasons:
                if rv == v:
                    return {name: rn}
            return {name: {"Unassigned": v}}
    return {"Unassigned": v}


TCP_FLAGS = ["FIN", "SYN", "RST", "PSH", "ACK", "URG", "ECE", "CWR"]


def field_value_json(ie, value):
    dt = ie.dtype
    if ie.kind in ("unknown", "vendor_unknown"):
        return list(value)
    if ie.subreg is not None:
        return _subreg_json(ie.subreg, value)
    if ie.name == "tcpControlBits" and ie.kind == "iana":
        b = value & 0xFF
        return {n: bool(b >> i & 1) for i, n in enumerate(TCP_FLAGS)}
    if isinstance(value, DateTime):
        return value.to_json()
    if isinstance(value, tuple):
        tag, x = value
        if tag == "v4":
            return _ipv4_str(x)
        if tag == "v6":
            return ipv6_str(x)
        if tag == "f64":
            return _f64_json(x)
        if tag == "f32":
            return _f32_json(x)
    if isinstance(value, (bytes, bytearray)):
        return list(value)
    return value


def field_json(f):
    ie = f.ie
    v = field_value_json(ie, f.value)
    if ie.kind == "iana":
        return {ie.name: v}
    if ie.kind == "vendor":
        return {ie.vendor: {ie.name: v}}
    if ie.kind == "vendor_unknown":
        return {ie.vendor: {"Unknown": {"id": ie.id, "value": v}}}
    return {"Unknown": {"pen": ie.pen, "id": ie.id, "value": v}}


def _set_json(s, netflow):
    kind, sid, recs = s
    if kind in ("Template", "OptionsTemplate"):
        return {kind: recs}
    out = []
    for scope, fields in recs:
        if netflow:
            sj = [x.to_json() for x in scope]
        else:
            sj = [field_json(x) for x in scope]
        out.append({"scope_fields": sj, "fields": [field_json(x) for x in fields]})
    return {"Data": {"id": sid, "records": out}}


def dumps(obj):
    """serde_json::to_string compatible text for the value shapes above."""
    if isinstance(obj, _RawNum):
        return str(obj)
    if obj is None:
        return "null"
    if obj is True:
        return "true"
    if obj is False:
        return "false"
    if isinstance(obj, int):
        return str(obj)
    if isinstance(obj, str):
        return json.dumps(obj, ensure_ascii=False)
    if isinstance(obj, list):
        return "[" + ",".join(dumps(x) for x in obj) + "]"
    if isinstance(obj, dict):
        return "{" + ",".join(json.dumps(k, ensure_ascii=False) + ":" + dumps(v) for k, v in obj.items()) + "}"
    raise TypeError(type(obj))


def socket_addr_str(ip, port):
    if isinstance(ip, tuple) and ip[0] == "v6":
        return "[%s]:%d" % (ipv6_str(ip[1]), port)
    return "%s:%d" % (_ipv4_str(ip[1]), port)
