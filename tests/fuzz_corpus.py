"""Seeded, structure-aware mutation corpus for differential fuzzing (TEST INFRASTRUCTURE).

The reference fuzzes exactly the decode path this repo rebuilds:
  fuzz/fuzz_targets/fuzz_ipfix_pkt.rs:23-36      IpfixPacket::parse over arbitrary bytes
  fuzz/fuzz_targets/fuzz_netflow_v9_pkt.rs        NetFlowV9Packet::parse over arbitrary bytes
  fuzz/fuzz_targets/fuzz_flow_codec.rs:22-30      FlowInfoCodec::decode over an arbitrary stream
Those targets only assert "no panic".  Here the same idea is differential: every generated
datagram goes through the device path (C ABI) and through the CPU oracle, and the two must
agree on status, error text, structured error, headers and every decoded field
(tests/test_gpu_fuzz.py).  libFuzzer's coverage feedback is replaced by a deterministic,
seeded mutator that knows the wire format, so the mutations land on the checks the reference
makes (ipfix.rs:54-238,276-413, netflow.rs:56-475, generator.rs:1775-1793 vlen prefixes,
codec.rs:189-220 gates):

  header     version / length / NFv9 count bits and boundary values
  set        set ids (0-3, < 256, unknown templates) and set lengths (< 4, past the message
             end, off by 1-3 = unaligned records)
  template   field counts, field lengths 0 / 65535 / outside length_range, enterprise bits,
             IE ids, template ids < 256, scope counts
  vlen       length prefixes 0, 254, 255 + 3-byte lengths, lengths past the set end, values
             resized for real (set and message lengths fixed up)
  padding    zero and non-zero bytes after the records
  truncation at every header boundary, with and without the message length fixed up
  splice     two datagrams cut and joined, or concatenated
  bits       random bit flips and "interesting" bytes anywhere

Seeds: every reference golden capture (tests/golden/*.dgrams, per exporter peer) plus
synthetic T20, config-3 templates, NFv9 313 and the variable-length / enterprise template
900 (netgauze_amd/synth.py).  Nothing here is imported by the product.
"""
import random
import struct

import golden_io

IPFIX, NFV9 = 10, 9


def _u16(b, o):
    return (b[o] << 8) | b[o + 1]


def _put16(b, o, v):
    b[o] = (v >> 8) & 0xFF
    b[o + 1] = v & 0xFF


def version(dg):
    return _u16(dg, 0) if len(dg) >= 2 else -1


def sets_of(dg):
    """[(pos, id, length)] of the well-formed prefix of the set chain."""
    if len(dg) < 16:
        return []
    ver = _u16(dg, 0)
    if ver == IPFIX:
        pos, end = 16, min(len(dg), _u16(dg, 2))
    elif ver == NFV9:
        pos, end = 20, len(dg)
    else:
        return []
    out = []
    while pos + 4 <= end:
        sid, sl = _u16(dg, pos), _u16(dg, pos + 2)
        if sl < 4 or pos + sl > end:
            break
        out.append((pos, sid, sl))
        pos += sl
    return out


def is_template_set(ver, sid):
    return sid in ((2, 3) if ver == IPFIX else (0, 1))


def has_template_sets(dg):
    ver = version(dg)
    return any(is_template_set(ver, sid) for _, sid, _ in sets_of(dg))


def _specs(dg, pos, end, n):
    """n field specifiers from pos: [(spec_pos, ie, length, pen)], pos after; None past end."""
    out = []
    for _ in range(n):
        if pos + 4 > end:
            return None, pos
        code, ln = _u16(dg, pos), _u16(dg, pos + 2)
        pen = None
        step = 4
        if code & 0x8000:
            if pos + 8 > end:
                return None, pos
            pen = int.from_bytes(dg[pos + 4:pos + 8], "big")
            step = 8
        out.append((pos, code, ln, pen))
        pos += step
    return out, pos


def template_records(dg, ver, pos, sid, sl):
    """(Options) template records of one template set as far as they parse:
    [dict(pos, tid, count_pos, specs, scope)] (deserializer/mod.rs:50-67, ipfix.rs:276-413,
    netflow.rs:265-353 record layouts)."""
    recs = []
    p, end = pos + 4, pos + sl
    options = sid in (3, 1)
    while end - p >= (4 if not options else 6):
        tid = _u16(dg, p)
        if not options:
            n = _u16(dg, p + 2)
            specs, q = _specs(dg, p + 4, end, n)
            if specs is None:
                break
            recs.append(dict(pos=p, tid=tid, count_pos=p + 2, specs=specs, scope=0))
        elif ver == IPFIX:
            total, scount = _u16(dg, p + 2), _u16(dg, p + 4)
            if scount > total:
                break
            specs, q = _specs(dg, p + 6, end, total)
            if specs is None:
                break
            recs.append(dict(pos=p, tid=tid, count_pos=p + 2, specs=specs, scope=scount))
        else:
            slen, olen = _u16(dg, p + 2), _u16(dg, p + 4)
            q = p + 6 + slen + olen
            if q > end:
                break
            specs, _ = _specs(dg, p + 6, p + 6 + slen, slen // 4)
            ospecs, _ = _specs(dg, p + 6 + slen, q, olen // 4)
            if specs is None or ospecs is None:
                break
            recs.append(dict(pos=p, tid=tid, count_pos=p + 2, specs=specs + ospecs, scope=len(specs)))
        p = q
    return recs


def learn_templates(dgrams, layouts=None):
    """{(version, template id): [field lengths, scope first]} from the template sets."""
    layouts = {} if layouts is None else layouts
    for dg in dgrams:
        ver = version(dg)
        for pos, sid, sl in sets_of(dg):
            if is_template_set(ver, sid):
                for r in template_records(dg, ver, pos, sid, sl):
                    layouts[(ver, r["tid"])] = [s[2] for s in r["specs"]]
    return layouts


def record_walk(dg, ver, start, end, lengths):
    """Records of a data set as the reference walks them (ipfix.rs:193-222, netflow.rs:201-218):
    (record starts, vlen prefix positions, fixed fields [(pos, length)])."""
    if ver == IPFIX:
        minlen = sum(1 if ln == 0xFFFF else ln for ln in lengths)
    else:
        minlen = sum(lengths)
    recs, prefixes, fields = [], [], []
    pos = start
    while minlen > 0 and end - pos >= minlen:
        r0, ok = pos, True
        for ln in lengths:
            if ln == 0xFFFF and ver == IPFIX:
                if pos >= end:
                    ok = False
                    break
                prefixes.append(pos)
                n, h = dg[pos], 1
                if n == 255:
                    if pos + 4 > end:
                        ok = False
                        break
                    n, h = int.from_bytes(dg[pos + 1:pos + 4], "big"), 4
                pos += h + n
            else:
                fields.append((pos, ln))
                pos += ln
            if pos > end:
                ok = False
                break
        if not ok:
            break
        recs.append(r0)
    return recs, prefixes, fields


class Anatomy:
    """Where the interesting bytes of one datagram are, given the peer's templates."""

    def __init__(self, dg, layouts):
        self.ver = version(dg)
        self.sets = sets_of(dg)
        self.tmpl = []      # template records (with their set)
        self.data = []      # (set pos, set len, records, prefixes, fields)
        for pos, sid, sl in self.sets:
            if is_template_set(self.ver, sid):
                for r in template_records(dg, self.ver, pos, sid, sl):
                    self.tmpl.append((pos, sid, sl, r))
            else:
                lengths = layouts.get((self.ver, sid))
                if lengths is not None:
                    recs, pre, fields = record_walk(dg, self.ver, pos + 4, pos + sl, lengths)
                    self.data.append((pos, sl, recs, pre, fields))
        self.boundaries = sorted(set(
            list(range(0, min(len(dg), 24))) +
            [p + k for p, _, _ in self.sets for k in (0, 1, 2, 3, 4, 5)] +
            [r + k for _, _, recs, _, _ in self.data for r in recs[:8] for k in (0, 1)] +
            [q + k for _, _, _, pre, _ in self.data for q in pre[:16] for k in (0, 1, 2, 3, 4)] +
            [len(dg) - k for k in (1, 2, 3)]))


# ---------------------------------------------------------------------------
# mutation operators: f(rng, dg bytearray, anatomy, ctx) -> bytearray or None (not applicable)
# ---------------------------------------------------------------------------
INTERESTING16 = [0, 1, 2, 3, 4, 5, 7, 8, 9, 15, 16, 17, 19, 20, 21, 255, 256, 257, 0x7FFF, 0x8000, 0xFFFE, 0xFFFF]


def fix_message_length(dg):
    """IPFIX: header length := datagram length (capped); NFv9 has no length."""
    if version(dg) == IPFIX and len(dg) >= 4:
        _put16(dg, 2, min(len(dg), 0xFFFF))
    return dg


def resize(dg, at, delete, insert, set_pos=None):
    """Replace dg[at:at+delete] by insert; fix the enclosing set's length and the message length."""
    out = dg[:at] + bytearray(insert) + dg[at + delete:]
    delta = len(insert) - delete
    if set_pos is not None and set_pos + 4 <= len(out):
        _put16(out, set_pos + 2, (_u16(out, set_pos + 2) + delta) & 0xFFFF)
    return fix_message_length(out)


def m_hdr_bits(rng, dg, a, ctx):
    for _ in range(rng.randint(1, 2)):
        i = rng.randrange(min(4, len(dg)) or 1)
        if i < len(dg):
            dg[i] ^= 1 << rng.randrange(8)
    return dg


def m_hdr_field(rng, dg, a, ctx):
    if len(dg) < 4:
        return None
    if rng.random() < 0.3:
        _put16(dg, 0, rng.choice([9, 10, 0, 1, 5, 8, 11, 0x0A00, 0xFFFF]))
    else:
        v = _u16(dg, 2)
        _put16(dg, 2, rng.choice([0, 1, 15, 16, 17, 19, 20, 21, v - 1, v + 1, v + 4, len(dg), len(dg) + 1,
                                  len(dg) - 1, 0xFFFF, rng.randrange(0x10000)]) & 0xFFFF)
    return dg


def m_set_len(rng, dg, a, ctx):
    if not a.sets:
        return None
    pos, sid, sl = rng.choice(a.sets)
    rest = len(dg) - pos
    _put16(dg, pos + 2, rng.choice([0, 1, 2, 3, 4, 5, sl - 1, sl - 2, sl - 3, sl + 1, sl + 2, sl + 3, sl + 4,
                                    rest, rest + 1, rest - 1, 0xFFFF, rng.randrange(0x10000)]) & 0xFFFF)
    return dg


def m_set_id(rng, dg, a, ctx):
    if not a.sets:
        return None
    pos, sid, sl = rng.choice(a.sets)
    known = [tid for (v, tid) in ctx["layouts"] if v == a.ver] or [256]
    _put16(dg, pos, rng.choice([0, 1, 2, 3, 4, 255, 256, 257, rng.choice(known), rng.choice(known),
                                rng.randrange(0x10000), 0xFFFF]))
    return dg


def m_trunc(rng, dg, a, ctx):
    cut = rng.choice(a.boundaries) if a.boundaries else rng.randrange(len(dg) + 1)
    out = dg[:max(0, min(cut, len(dg)))]
    if rng.random() < 0.6:
        fix_message_length(out)
    return out


def m_trunc_set(rng, dg, a, ctx):
    """Shorten the last set's body (set and message lengths fixed): record-level EOFs."""
    if not a.sets:
        return None
    pos, sid, sl = a.sets[-1]
    if sl <= 4:
        return None
    keep = rng.randrange(0, sl - 4)
    return resize(dg, pos + 4 + keep, pos + sl - (pos + 4 + keep), b"", set_pos=pos)


def m_vlen(rng, dg, a, ctx):
    pres = [(sp, sl, q) for sp, sl, _, pre, _ in a.data for q in pre]
    if not pres:
        return None
    sp, sl, q = rng.choice(pres)
    end = sp + sl
    n, h = dg[q], 1
    if n == 255 and q + 4 <= end:
        n, h = int.from_bytes(dg[q + 1:q + 4], "big"), 4
    k = rng.random()
    if k < 0.45:  # rewrite the prefix only (the rest of the record shifts)
        choice = rng.choice(["0", "254", "255", "esc", "past"])
        if choice == "0":
            pre = b"\x00"
        elif choice == "254":
            pre = b"\xfe"
        elif choice == "255":
            pre = b"\xff"
        elif choice == "esc":
            pre = b"\xff" + rng.choice([0, 1, 3, 254, 255, 256, 0xFFFF, 0xFFFFFF, end - q]).to_bytes(3, "big")[-3:]
        else:
            left = end - q
            pre = bytes([min(254, left)]) if left < 255 else b"\xff" + (left + rng.randrange(0, 4)).to_bytes(3, "big")
        return dg[:q] + bytearray(pre) + dg[q + h:]
    if k < 0.55:  # escape at the very end of the set
        return resize(dg, end, 0, b"\xff" + bytes(rng.randrange(3)), set_pos=sp)
    # resize the value for real: a valid record of another value length
    new = rng.choice([0, 1, 2, 253, 254, 255, 256, 300, 600, rng.randrange(0, 40)])
    fill = rng.choice([b"a", b"\x00", b"\xc3\xa9", b"\xff", b"\xe2\x82"])
    val = (fill * (new // len(fill) + 1))[:new]
    escape = new >= 255 or rng.random() < 0.15
    pre = (b"\xff" + new.to_bytes(3, "big")) if escape else bytes([new])
    return resize(dg, q, h + n, pre + val, set_pos=sp)


def m_pad(rng, dg, a, ctx):
    if not a.sets:
        return None
    pos, sid, sl = rng.choice(a.sets)
    k = rng.choice([1, 2, 3, 4, 5, 7, 8])
    pad = bytearray(k)
    if rng.random() < 0.5:
        pad[rng.randrange(k)] = rng.choice([1, 0x80, 0xFF, rng.randrange(1, 256)])
    return resize(dg, pos + sl, 0, pad, set_pos=pos)


def m_splice(rng, dg, a, ctx):
    other = rng.choice(ctx["pool"])
    oa = Anatomy(other, ctx["layouts"])
    cut = rng.choice(a.boundaries) if a.boundaries and rng.random() < 0.7 else rng.randrange(len(dg) + 1)
    ocut = rng.choice(oa.boundaries) if oa.boundaries and rng.random() < 0.7 else rng.randrange(len(other) + 1)
    out = dg[:cut] + other[ocut:]
    if rng.random() < 0.5:
        fix_message_length(out)
    return out


def m_concat(rng, dg, a, ctx):
    out = dg + rng.choice(ctx["pool"])
    if rng.random() < 0.3:
        fix_message_length(out)
    return out


def m_dup_drop_set(rng, dg, a, ctx):
    if not a.sets:
        return None
    pos, sid, sl = rng.choice(a.sets)
    if rng.random() < 0.5:
        out = dg[:pos + sl] + dg[pos:pos + sl] + dg[pos + sl:]
    else:
        out = dg[:pos] + dg[pos + sl:]
    fix_message_length(out)
    if a.ver == NFV9 and rng.random() < 0.5:
        _put16(out, 2, rng.randrange(0, 64))
    return out


def m_nf_count(rng, dg, a, ctx):
    if a.ver != NFV9 or len(dg) < 4:
        return None
    nrec = sum(len(r) for _, _, r, _, _ in a.data) + sum(1 for _, s, _ in a.sets if s in (0, 1))
    _put16(dg, 2, rng.choice([0, 1, 2, nrec - 1, nrec, nrec + 1, 0xFFFF, rng.randrange(64)]) & 0xFFFF)
    return dg


def m_tmpl_len(rng, dg, a, ctx):
    specs = [s for _, _, _, r in a.tmpl for s in r["specs"]]
    if not specs:
        return None
    sp = rng.choice(specs)
    _put16(dg, sp[0] + 2, rng.choice([0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 16, 17, 31, 32, 33, 0xFFFE, 0xFFFF,
                                      sp[2] + 1, sp[2] - 1]) & 0xFFFF)
    return dg


def m_tmpl_count(rng, dg, a, ctx):
    if not a.tmpl:
        return None
    pos, sid, sl, r = rng.choice(a.tmpl)
    cp = r["count_pos"]
    if sid in (3,) and rng.random() < 0.5:  # IPFIX options: the scope count
        cp += 2
    n = _u16(dg, cp)
    _put16(dg, cp, rng.choice([0, 1, n - 1, n + 1, n + 2, 0xFFFF, rng.randrange(64)]) & 0xFFFF)
    return dg


def m_tmpl_ebit(rng, dg, a, ctx):
    specs = [(pos, s) for pos, _, _, r in a.tmpl for s in r["specs"]]
    if not specs:
        return None
    set_pos, sp = rng.choice(specs)
    if rng.random() < 0.4:  # flip the bit only: the specifier chain shifts by the PEN
        dg[sp[0]] ^= 0x80
        return dg
    if sp[3] is None:  # IANA -> enterprise: insert a PEN
        pen = rng.choice([0, 2011, 6876, 29305, 213, 9, 0xFFFFFFFF, rng.randrange(1 << 32)])
        out = resize(dg, sp[0] + 4, 0, pen.to_bytes(4, "big"), set_pos=set_pos)
        out[sp[0]] |= 0x80
        return out
    out = resize(dg, sp[0] + 4, 4, b"", set_pos=set_pos)  # enterprise -> IANA
    out[sp[0]] &= 0x7F
    return out


def m_tmpl_ie(rng, dg, a, ctx):
    specs = [s for _, _, _, r in a.tmpl for s in r["specs"]]
    if not specs:
        return None
    sp = rng.choice(specs)
    ie = rng.choice([0, 1, 2, 4, 6, 8, 22, 27, 82, 89, 96, 152, 154, 156, 160, 210, 291, 292, 313, 341, 433,
                     500, 999, 0x7FFF, rng.randrange(0x8000)])
    _put16(dg, sp[0], ie | (dg[sp[0]] << 8 & 0x8000))
    return dg


def m_tmpl_id(rng, dg, a, ctx):
    if not a.tmpl:
        return None
    pos, sid, sl, r = rng.choice(a.tmpl)
    known = [tid for (v, tid) in ctx["layouts"] if v == a.ver] or [256]
    _put16(dg, r["pos"], rng.choice([0, 2, 255, 256, 0xFFFF, rng.choice(known), rng.randrange(0x10000)]))
    return dg


def m_value(rng, dg, a, ctx):
    fields = [f for _, _, _, _, fl in a.data for f in fl if f[1] <= 64]
    if not fields:
        return None
    pos, ln = rng.choice(fields)
    k = rng.random()
    if k < 0.3:
        v = bytes([0xFF]) * ln
    elif k < 0.5:
        v = bytes(ln)
    elif k < 0.7:
        v = bytes([0x80]) + bytes([0xFF] * (ln - 1)) if ln else b""
    else:
        bad = rng.choice([b"\xc3\x28", b"\xe2\x82", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\xc0\xaf", b"\x80"])
        v = (bytes([0x61] * rng.randrange(ln + 1)) + bad + bytes(ln))[:ln]
    dg[pos:pos + ln] = v
    return dg


def m_bits(rng, dg, a, ctx):
    if not dg:
        return None
    for _ in range(rng.randint(1, 8)):
        dg[rng.randrange(len(dg))] ^= 1 << rng.randrange(8)
    return dg


def m_bytes(rng, dg, a, ctx):
    if not dg:
        return None
    for _ in range(rng.randint(1, 4)):
        dg[rng.randrange(len(dg))] = rng.choice([0x00, 0xFF, 0x7F, 0x80, 0x01, 0xFE])
    return dg


OPERATORS = {
    "hdr_bits": (m_hdr_bits, 3), "hdr_field": (m_hdr_field, 4), "set_len": (m_set_len, 8), "set_id": (m_set_id, 5),
    "trunc": (m_trunc, 8), "trunc_set": (m_trunc_set, 6), "vlen": (m_vlen, 10), "pad": (m_pad, 5),
    "splice": (m_splice, 4), "concat": (m_concat, 2), "dup_drop_set": (m_dup_drop_set, 3), "nf_count": (m_nf_count, 5),
    "tmpl_len": (m_tmpl_len, 4), "tmpl_count": (m_tmpl_count, 2), "tmpl_ebit": (m_tmpl_ebit, 2),
    "tmpl_ie": (m_tmpl_ie, 2), "tmpl_id": (m_tmpl_id, 1), "value": (m_value, 8), "bits": (m_bits, 8),
    "bytes": (m_bytes, 4),
}
_TMPL_OPS = {"tmpl_len", "tmpl_count", "tmpl_ebit", "tmpl_ie", "tmpl_id"}


def mutate(rng, dg, ctx, max_ops=3):
    """1..max_ops operators applied in turn (each re-reads the anatomy); returns (bytes, [names])."""
    cur = bytearray(dg)
    names = []
    tmpl_dg = has_template_sets(cur)
    ops = [k for k in OPERATORS if tmpl_dg or k not in _TMPL_OPS]
    weights = [OPERATORS[k][1] * (4 if tmpl_dg and k in _TMPL_OPS else 1) for k in ops]
    for _ in range(rng.randint(1, max_ops)):
        a = Anatomy(cur, ctx["layouts"])
        has_pre = any(pre for _, _, _, pre, _ in a.data)
        w = [x * (8 if has_pre and k == "vlen" else 1) for k, x in zip(ops, weights)]
        for _try in range(6):
            name = rng.choices(ops, w)[0]
            out = OPERATORS[name][0](rng, bytearray(cur), a, ctx)
            if out is not None:
                cur = out[:0xFFFF + 64]
                names.append(name)
                break
        if rng.random() < 0.5:
            break
    return bytes(cur), names


# ---------------------------------------------------------------------------
# seeds
# ---------------------------------------------------------------------------
def _synthetic_ipfix():
    from netgauze_amd import synth
    out = []
    # T20, 1-12 records per message
    rec = synth.t20_records(400, seed=synth.SEED_CFG2).numpy()
    msgs, i = [], 0
    while i < len(rec):
        k = 1 + (i * 7) % 12
        body = rec[i:i + k].tobytes()
        msgs.append(struct.pack(">HHIIIHH", 10, 20 + len(body), 1_700_000_000 + i, i, 1, synth.T20_ID, 4 + len(body))
                    + body)
        i += k
    out.append(("synthetic_t20", [synth.template_message()], msgs))
    # config-3 templates, two data sets of different templates per message
    tpls = synth.CFG3_TEMPLATES
    recs = {tid: synth.template_records(f, 24, synth.SEED_CFG3 + j).numpy() for j, (tid, f) in enumerate(tpls)}
    msgs = []
    for m in range(60):
        sets = b""
        for tid in (tpls[m % len(tpls)][0], tpls[(m * 3 + 1) % len(tpls)][0]):
            k = 1 + m % 4
            r = recs[tid][(m % 6) * 4:(m % 6) * 4 + k].tobytes()
            sets += struct.pack(">HH", tid, 4 + len(r)) + r
        msgs.append(struct.pack(">HHIII", 10, 16 + len(sets), 1_700_000_100 + m, m, 2) + sets)
    out.append(("synthetic_cfg3", [synth.templates_message(tpls)], msgs))
    # variable-length / enterprise template 900, small messages
    flat, lens = synth.vlen_records(300, synth.V900, synth.SEED_CFG4 + 1)
    msgs = synth._pack_ipfix(flat, lens, synth.V900_ID, max_msg=500)
    # an options template with scope fields and its records (ipfix.rs:276-327)
    opt = struct.pack(">HHH", 400, 3, 1) + struct.pack(">HHHHHH", 149, 4, 34, 4, 36, 2) + b"\0\0"
    oset = struct.pack(">HH", 3, 4 + len(opt)) + opt
    tm_opt = struct.pack(">HHIII", 10, 16 + len(oset), 1_700_000_000, 0, 1) + oset
    orecs = b"".join(struct.pack(">IIH", 7 + k, 1000 * k, k) for k in range(5))
    msgs += [struct.pack(">HHIIIHH", 10, 20 + len(orecs), 1_700_000_000, 9, 1, 400, 4 + len(orecs)) + orecs]
    out.append(("synthetic_v900", [synth._ipfix_template_v900(), tm_opt], msgs))
    out.append(_zoo())
    return out


# one field of every decode rule (generator.rs:1439-1807): date-times of all four kinds, fixed
# string, bool, float64, mac, signed32, u256 (full and reduced), MPLS label, sub-registries,
# tcpControlBits (2 and 1 bytes), reduced unsigned, vendor / unknown-PEN fields and lists
ZOO = [(8, 4), (27, 16), (150, 4), (152, 8), (154, 8), (156, 8), (82, 16), (276, 1), (320, 8), (56, 6), (434, 4),
       (515, 32), (520, 5), (70, 3), (89, 1), (61, 1), (6, 2), (6, 1), (1, 3), (10, 2), (7, 1), (434, 2),
       (1000, 4, 2011), (5, 2, 213), (880, 1, 6876), (291, 0xFFFF), (83, 0xFFFF), (12, 4)]


def _zoo():
    body = struct.pack(">HH", 700, len(ZOO))
    for f in ZOO:
        body += struct.pack(">HH", f[0], f[1]) if len(f) == 2 else struct.pack(">HHI", f[0] | 0x8000, f[1], f[2])
    tset = struct.pack(">HH", 2, 4 + len(body)) + body
    tm = struct.pack(">HHIII", 10, 16 + len(tset), 1_700_000_000, 0, 3) + tset
    rng = random.Random(0x5A4F4F)
    msgs = []
    for m in range(80):
        recs = b""
        for _ in range(1 + m % 5):
            for f in ZOO:
                ie, ln = f[0], f[1]
                if ln == 0xFFFF:
                    n = rng.choice([0, 1, 5, 30, 254, 255, 300])
                    v = bytes(rng.randrange(97, 123) for _ in range(n))
                    recs += (bytes([n]) if n < 255 else b"\xff" + n.to_bytes(3, "big")) + v
                elif ie in (150,):
                    recs += struct.pack(">I", 1_700_000_000 + rng.randrange(1 << 20))
                elif ie == 152:
                    recs += struct.pack(">Q", 1_700_000_000_000 + rng.randrange(1 << 36))
                elif ie in (154, 156):
                    recs += struct.pack(">II", 1_700_000_000 + rng.randrange(1 << 20), rng.getrandbits(32))
                elif ie in (82,):
                    s = bytes(rng.randrange(97, 123) for _ in range(rng.randrange(ln + 1)))
                    recs += (s + bytes(ln))[:ln]
                else:
                    recs += bytes(rng.getrandbits(8) for _ in range(ln))
        dset = struct.pack(">HH", 700, 4 + len(recs)) + recs
        msgs.append(struct.pack(">HHIII", 10, 16 + len(dset), 1_700_000_000 + m, m, 3) + dset)
    return ("synthetic_zoo", [tm], msgs)


def _synthetic_nfv9():
    from netgauze_amd import synth
    out = []
    _, rl = synth.field_offsets(synth.NF313)
    nf = synth.template_records(synth.NF313, 120, synth.SEED_CFG4).numpy()
    msgs = []
    i = 0
    while i < len(nf):
        k = 1 + i % 5
        msgs += synth._pack_nfv9(nf[i:i + k], rl, synth.NF313_ID, per_msg=k, unix0=1_700_000_000 + i)
        i += k
    # options template: scope System (4) + Interface (2), option samplingInterval (4) (netflow.rs:265-310)
    oset = struct.pack(">HH", 1, 4 + 6 + 8 + 4 + 2) + struct.pack(">HHH", 270, 8, 4) + \
        struct.pack(">HHHH", 1, 4, 2, 2) + struct.pack(">HH", 34, 4) + b"\0\0"
    tset = struct.pack(">HH", 0, 4 + 4 + 16) + struct.pack(">HH", 260, 4) + struct.pack(">HHHHHHHH", 8, 4, 1, 4, 7, 2,
                                                                                          6, 1)
    tm = struct.pack(">HHIIII", 9, 2, 1000, 1_700_000_000, 0, 5) + tset + oset
    rec = struct.pack(">IIHB", 0x0A000001, 1500, 80, 0x12)
    orec = struct.pack(">IHI", 77, 3, 1000)
    small = []
    for m in range(40):
        k = 1 + m % 4
        body = rec * k
        pad = (-(4 + len(body))) % 4
        s1 = struct.pack(">HH", 260, 4 + len(body) + pad) + body + b"\0" * pad
        s2 = struct.pack(">HH", 270, 4 + 10 * 2) + orec * 2
        small.append(struct.pack(">HHIIII", 9, k + (2 if m % 2 else 0), 1000 + m, 1_700_000_000 + m, m, 5) +
                     s1 + (s2 if m % 2 else b""))
    out.append(("synthetic_nf313", [synth.nfv9_template_message()], msgs))
    out.append(("synthetic_nf_small", [tm], small))
    return out


def seed_streams(proto):
    """[(name, clean template datagrams, every datagram of the stream)] for one protocol:
    each golden capture's exporter peers (tests/golden/*.dgrams) and the synthetic streams."""
    out = []
    for name, kind, _ in golden_io.cases():
        if kind != "pcap_tests":
            continue
        peers = {}
        for src, sp, dst, dp, payload in golden_io.datagrams(name):
            peers.setdefault((src, sp, dst, dp), []).append(payload)
        for k, dgs in sorted(peers.items(), key=lambda kv: str(kv[0])):
            if version(dgs[0]) != proto:
                continue
            tm, seen = [], set()
            for d in dgs:
                if has_template_sets(d):
                    body = bytes(d[16:]) if proto == IPFIX else bytes(d[20:])
                    if body not in seen:
                        seen.add(body)
                        tm.append(d)
            out.append(("%s/%d" % (name, k[1]), tm, dgs))
    syn = _synthetic_ipfix() if proto == IPFIX else _synthetic_nfv9()
    for name, tm, msgs in syn:
        out.append((name, tm, tm + msgs))
    return out


def corpus(proto, n_cases, seed=0x46555A5A, batch_cases=500):
    """Deterministic batches for one protocol: [(stream name, [datagram], [case flags])].
    Every batch starts with its stream's clean template datagrams (flag None); each case is
    one mutated datagram (flag: the operator names), and a case that carried template sets is
    followed by the clean templates again so later cases still meet the real layouts."""
    rng = random.Random(seed * 31 + proto)
    streams = seed_streams(proto)
    pool = [bytes(d) for _, _, dgs in streams for d in dgs]
    batches = []
    done = 0
    s = 0
    while done < n_cases:
        name, tm, dgs = streams[s % len(streams)]
        s += 1
        ctx = {"layouts": learn_templates(tm), "pool": pool}
        dgrams = list(tm)
        flags = [None] * len(tm)
        k = min(batch_cases, n_cases - done)
        for _ in range(k):
            base = rng.choice(dgs)
            dg, names = mutate(rng, base, ctx)
            dgrams.append(dg)
            flags.append(names)
            if has_template_sets(base) or has_template_sets(dg):
                dgrams += tm
                flags += [None] * len(tm)
        batches.append((name, dgrams, flags))
        done += k
    return batches


def streams_corpus(n_streams, seed=0x5354524D):
    """Stream-mode cases (fuzz_flow_codec.rs:22-30): per case, a byte stream of clean templates
    and mutated messages of both protocols, cut into datagrams of random sizes for one or two
    exporter peers: [[(peer index, payload)]]."""
    rng = random.Random(seed)
    per = {p: corpus(p, n_streams * 6, seed=seed + p, batch_cases=6) for p in (IPFIX, NFV9)}
    out = []
    for i in range(n_streams):
        dg = []
        for p in (IPFIX, NFV9):
            _, d, _ = per[p][i % len(per[p])]
            dg += [(p, x) for x in d]
        if rng.random() < 0.5:
            rng.shuffle(dg)
        chunks = []
        for p, x in dg:
            peer = 0 if rng.random() < 0.7 else 1
            j = 0
            while j < len(x):
                n = len(x) - j if rng.random() < 0.6 else rng.randint(1, max(1, len(x) - j))
                chunks.append((peer, x[j:j + n]))
                j += n
        out.append(chunks)
    return out
