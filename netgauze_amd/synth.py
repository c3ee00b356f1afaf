"""Synthetic IPFIX / NetFlow v9 exporter streams (benchmark and test input).

Deterministic: record bytes come from a counter-based splitmix64 stream, so
the same (template, seed, n) gives identical bytes on CPU (tests, oracle) and
on the GPU (bench, generated in HBM without an H2D copy).  Layout per
SURVEY.md §8(d): one template message, then data messages of up to
`rec_per_msg` records in one data set (1023 x 64-byte T20 records = a
65,492-byte message), export time 1,700,000,000 + message index, sequence
number = records sent before the message, observation domain 1.
"""
import struct

import torch

SEED_CFG2 = 0x4E475A4500000002
SEED_CFG3 = 0x4E475A4500000003

# T20: 20 fixed-width IANA fields, 64 bytes (modelled on
# wire/tests/ipfix.rs:212-236)
T20 = [
    (8, 4), (12, 4), (15, 4), (10, 4), (14, 4), (2, 8), (1, 8), (22, 4), (21, 4),
    (7, 2), (11, 2), (6, 2), (4, 1), (5, 1), (9, 1), (13, 1), (16, 4), (17, 4), (61, 1), (60, 1),
]
T20_ID = 256


def _i64(c):
    return c - (1 << 64) if c >= (1 << 63) else c


_G = _i64(0x9E3779B97F4A7C15)
_M1 = _i64(0xBF58476D1CE4E5B9)
_M2 = _i64(0x94D049BB133111EB)


def _lsr(x, k):
    return (x >> k) & ((1 << (64 - k)) - 1)


def splitmix64(idx, seed):
    """splitmix64 of (seed + idx) for an int64 tensor of counters."""
    z = idx + _i64(seed & 0xFFFFFFFFFFFFFFFF) + _G
    z = (z ^ _lsr(z, 30)) * _M1
    z = (z ^ _lsr(z, 27)) * _M2
    return z ^ _lsr(z, 31)


def field_offsets(fields):
    offs, o = [], 0
    for _, ln in fields:
        offs.append(o)
        o += ln
    return offs, o


def t20_records(n, seed=SEED_CFG2, device="cpu", first=0):
    """(n, 64) uint8 tensor of T20 records (wire order, big endian fields)."""
    words = splitmix64(torch.arange(first * 8, (first + n) * 8, dtype=torch.int64, device=device), seed)
    rec = words.view(torch.uint8).view(n, 64).clone()
    offs, _ = field_offsets(T20)
    o = dict(zip([f for f, _ in T20], offs))
    proto_tab = torch.tensor([6, 17, 1], dtype=torch.uint8, device=device)
    rec[:, o[4]] = proto_tab[(rec[:, o[4]].to(torch.int64) % 3)]
    rec[:, o[9]] = (rec[:, o[9]].to(torch.int64) % 33).to(torch.uint8)
    rec[:, o[13]] = (rec[:, o[13]].to(torch.int64) % 33).to(torch.uint8)
    rec[:, o[61]] = rec[:, o[61]] & 1
    rec[:, o[60]] = 4
    return rec


def template_message(tid=T20_ID, fields=T20, export_time=1_700_000_000, seq=0, domain=1):
    body = struct.pack(">HH", tid, len(fields)) + b"".join(struct.pack(">HH", i, ln) for i, ln in fields)
    sset = struct.pack(">HH", 2, 4 + len(body)) + body
    return struct.pack(">HHIII", 10, 16 + len(sset), export_time, seq, domain) + sset


def ipfix_data_stream(records, rec_len, tid=T20_ID, rec_per_msg=1023, export_time0=1_700_000_000, seq0=0,
                      domain=1):
    """Pack an (n, rec_len) uint8 tensor into IPFIX data messages, one data
    set per message.  Returns (bytes uint8 tensor, offsets int64, lengths int32)
    on the records' device."""
    dev = records.device
    n = records.shape[0]
    n_msgs = (n + rec_per_msg - 1) // rec_per_msg
    full = n // rec_per_msg
    msg_len_full = 20 + rec_per_msg * rec_len
    tail = n - full * rec_per_msg
    total = full * msg_len_full + (20 + tail * rec_len if tail else 0)
    buf = torch.zeros(total + 16, dtype=torch.uint8, device=dev)
    m = torch.arange(n_msgs, dtype=torch.int64, device=dev)
    k = torch.full((n_msgs,), rec_per_msg, dtype=torch.int64, device=dev)
    if tail:
        k[-1] = tail
    lens = 20 + k * rec_len
    offs = torch.zeros(n_msgs, dtype=torch.int64, device=dev)
    if n_msgs > 1:
        offs[1:] = torch.cumsum(lens[:-1], 0)
    # headers: version, length, export time, sequence, domain, set id, set length
    hdr = torch.zeros(n_msgs, 20, dtype=torch.uint8, device=dev)

    def put_be(col, width, vals):
        for b in range(width):
            hdr[:, col + b] = _lsr(vals, 8 * (width - 1 - b)).bitwise_and(0xFF).to(torch.uint8)

    put_be(0, 2, torch.full_like(m, 10))
    put_be(2, 2, lens)
    put_be(4, 4, (export_time0 + m) & 0xFFFFFFFF)
    put_be(8, 4, (seq0 + m * rec_per_msg) & 0xFFFFFFFF)
    put_be(12, 4, torch.full_like(m, domain))
    put_be(16, 2, torch.full_like(m, tid))
    put_be(18, 2, 4 + k * rec_len)
    idx = offs.unsqueeze(1) + torch.arange(20, device=dev).unsqueeze(0)
    buf[idx.reshape(-1)] = hdr.reshape(-1)
    if full:
        body = buf[: full * msg_len_full].view(full, msg_len_full)
        body[:, 20:] = records[: full * rec_per_msg].reshape(full, rec_per_msg * rec_len)
    if tail:
        start = full * msg_len_full + 20
        buf[start:start + tail * rec_len] = records[full * rec_per_msg:].reshape(-1)
    return buf, offs, lens.to(torch.int32)


def host_batch(datagrams, device="cpu"):
    """List of bytes -> (bytes uint8, offsets int64, lengths int32) tensors."""
    lens = [len(d) for d in datagrams]
    offs = [0] * len(datagrams)
    for i in range(1, len(datagrams)):
        offs[i] = offs[i - 1] + lens[i - 1]
    blob = b"".join(datagrams) + b"\0" * 16
    return (torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(device),
            torch.tensor(offs, dtype=torch.int64, device=device),
            torch.tensor(lens, dtype=torch.int32, device=device))


# --- config 3: mixed templates ------------------------------
# Field lists are the reference's own: 347/348/342/313 as announced in
# crates/pcap-decoder/tests/data/502-IPFIXv10-BGP-IPv6-CISCO-SRv6-lcomms.pcap,
# 307 from wire/tests/ipfix.rs:212-236, 1024 from benches/serde_benchmark.rs:36-39.
_F347 = [(2, 8), (1, 8), (8, 4), (12, 4), (10, 4), (14, 4), (21, 4), (22, 4), (7, 2), (11, 2), (16, 4), (17, 4),
         (18, 4), (9, 1), (13, 1), (4, 1), (6, 2), (5, 1), (61, 1), (89, 4), (302, 4), (234, 4), (235, 4), (52, 1),
         (53, 1), (198, 8), (56, 6), (80, 6), (256, 2), (243, 2), (245, 2), (244, 1)]
_F342 = [(2, 8), (1, 8), (27, 16), (28, 16), (10, 4), (14, 4), (22, 4), (21, 4), (31, 4), (64, 4), (7, 2), (11, 2),
         (16, 4), (17, 4), (63, 16), (30, 1), (29, 1), (4, 1), (6, 2), (5, 1), (61, 1), (89, 4), (302, 4), (234, 4),
         (235, 4), (52, 1), (53, 1), (198, 8)]
_F348 = _F342 + [(56, 6), (80, 6), (256, 2), (243, 2), (245, 2), (244, 1)]
_F313 = [(70, 3), (71, 3), (72, 3), (73, 3), (74, 3), (75, 3), (10, 4), (14, 4), (1, 8), (2, 8), (21, 4), (22, 4),
         (47, 4), (140, 16), (27, 16), (28, 16), (31, 4), (91, 1), (64, 4), (8, 4), (12, 4), (7, 2), (11, 2), (46, 1),
         (89, 4), (61, 1), (5, 1), (4, 1), (6, 2), (302, 4), (234, 4), (235, 4), (198, 8)]
_F307 = [(8, 4), (12, 4), (5, 1), (4, 1), (7, 2), (11, 2), (32, 2), (10, 4), (16, 4), (17, 4), (18, 4), (14, 4),
         (1, 4), (2, 4), (22, 4), (21, 4), (15, 4), (9, 1), (13, 1), (6, 1), (60, 1), (152, 8), (153, 8)]
_F1024 = [(8, 4), (12, 4), (22, 4), (21, 4), (1, 4), (2, 4), (10, 4), (14, 4), (7, 2), (11, 2), (4, 1), (6, 1),
          (60, 1), (5, 1)]
# 313 with NFv9-style reduced-size counters (reduced-size encoding, RFC 7011 §6.2)
_F313R = [(f, {1: 4, 2: 4, 198: 4, 89: 1, 234: 2, 235: 2}.get(f, ln)) for f, ln in _F313]

CFG3_TEMPLATES = [(256, T20), (347, _F347), (348, _F348), (342, _F342), (313, _F313), (307, _F307), (1024, _F1024),
                  (2313, _F313R)]

# Config 5: the 8 config-3 templates plus 8 width permutations (the same IEs
# in reverse order: other field offsets, another per-template kernel each)
SEED_CFG5 = 0x4E475A4500000005
CFG5_TEMPLATES = CFG3_TEMPLATES + [(tid + 4000, list(reversed(f))) for tid, f in CFG3_TEMPLATES]

_DT_MS = {152, 153, 154, 155, 156, 157, 158, 159}  # dateTime{Milli,Micro,Nano}seconds IEs used here (152/153 ms)


def template_records(fields, n, seed, device="cpu", first=0):
    """(n, rec_len) uint8 tensor of records for an arbitrary fixed-width IANA
    template: splitmix64 bytes, with dateTimeMilliseconds fields (152/153)
    moved into chrono's valid range (2023-11-14 + up to ~11.6 days)."""
    offs, rl = field_offsets(fields)
    nw = (rl + 7) // 8
    words = splitmix64(torch.arange(first * nw, (first + n) * nw, dtype=torch.int64, device=device), seed)
    rec = words.view(torch.uint8).view(n, nw * 8)[:, :rl].clone()
    for (ie, ln), o in zip(fields, offs):
        if ie in (152, 153) and ln == 8:
            ms = 1_700_000_000_000 + (torch.arange(first, first + n, dtype=torch.int64, device=device) * 7919) % 1_000_000_000
            for b in range(8):
                rec[:, o + b] = _lsr(ms, 8 * (7 - b)).bitwise_and(0xFF).to(torch.uint8)
    return rec


def templates_message(templates, export_time=1_700_000_000, seq=0, domain=1):
    """One IPFIX message announcing several templates in one template set."""
    body = b""
    for tid, fields in templates:
        body += struct.pack(">HH", tid, len(fields)) + b"".join(struct.pack(">HH", i, ln) for i, ln in fields)
    sset = struct.pack(">HH", 2, 4 + len(body)) + body
    return struct.pack(">HHIII", 10, 16 + len(sset), export_time, seq, domain) + sset


def mixed_stream(n, templates=CFG3_TEMPLATES, seed=SEED_CFG3, device="cpu"):
    """Config 3: n records split evenly over the templates, each template's
    records packed as many per message as fit in 65,535 bytes, messages
    interleaved round-robin across templates.  Returns (bytes, offsets,
    lengths, {template id: records tensor})."""
    parts, recs = [], {}
    T = len(templates)
    for t, (tid, fields) in enumerate(templates):
        nt = n // T + (1 if t < n % T else 0)
        _, rl = field_offsets(fields)
        r = template_records(fields, nt, seed + t, device)
        recs[tid] = r
        per = (65535 - 20) // rl
        parts.append(ipfix_data_stream(r, rl, tid=tid, rec_per_msg=per))
    bufs, offs, lens, keys = [], [], [], []
    base = 0
    for t, (b, o, ln) in enumerate(parts):
        bufs.append(b[:-16])
        offs.append(o + base)
        lens.append(ln)
        keys.append(torch.arange(o.numel(), dtype=torch.int64, device=o.device) * T + t)
        base += b.numel() - 16
    buf = torch.cat(bufs + [torch.zeros(16, dtype=torch.uint8, device=bufs[0].device)])
    order = torch.argsort(torch.cat(keys))
    return buf, torch.cat(offs)[order], torch.cat(lens)[order], recs


def stream_index(n, templates=None):
    """Message index of the stream t20 (templates None: ipfix_data_stream of t20_records, 1023 per
    message) or mixed_stream(n, templates) builds, without its bytes: per message, numpy arrays
    (template index, first record within the template's records, records).  A multi-GPU host
    shards this one index by records (dist.shard_by_records) and builds only its range
    (stream_range), so the ranks together decode exactly the one stream."""
    import numpy as np
    if templates is None:
        m = (n + 1022) // 1023
        first = np.arange(m, dtype=np.int64) * 1023
        return np.zeros(m, dtype=np.int64), first, np.minimum(1023, n - first)
    T = len(templates)
    tix, firsts, counts, keys = [], [], [], []
    for t, (tid, fields) in enumerate(templates):
        nt = n // T + (1 if t < n % T else 0)
        _, rl = field_offsets(fields)
        per = (65535 - 20) // rl
        m = (nt + per - 1) // per
        f = np.arange(m, dtype=np.int64) * per
        tix.append(np.full(m, t, dtype=np.int64))
        firsts.append(f)
        counts.append(np.minimum(per, nt - f))
        keys.append(np.arange(m, dtype=np.int64) * T + t)  # mixed_stream's round-robin order
    order = np.argsort(np.concatenate(keys), kind="stable")
    return np.concatenate(tix)[order], np.concatenate(firsts)[order], np.concatenate(counts)[order]


def stream_range(n, m0, m1, templates=None, seed=None, device="cpu"):
    """Messages [m0, m1) of the stream_index(n, templates) stream, byte for byte as the whole
    stream has them (records from the counter-based generator at their global position; export
    time and sequence number of their message): (bytes, offsets, lengths, records)."""
    import numpy as np
    tix, first, count = stream_index(n, templates)
    if templates is None:
        seed = SEED_CFG2 if seed is None else seed
        r0 = int(first[m0]) if m1 > m0 else 0
        r1 = int(first[m1 - 1] + count[m1 - 1]) if m1 > m0 else 0
        rec = t20_records(r1 - r0, seed=seed, device=device, first=r0)
        buf, offs, lens = ipfix_data_stream(rec, 64, export_time0=1_700_000_000 + m0, seq0=r0)
        return buf, offs, lens, r1 - r0
    seed = SEED_CFG3 if seed is None else seed
    parts, keys = [], []
    for t, (tid, fields) in enumerate(templates):
        sel = (np.nonzero(tix[m0:m1] == t)[0] + m0).tolist()
        if not sel:
            continue
        _, rl = field_offsets(fields)
        per = (65535 - 20) // rl
        r0, r1 = int(first[sel[0]]), int(first[sel[-1]] + count[sel[-1]])
        r = template_records(fields, r1 - r0, seed + t, device, first=r0)
        b, o, ln = ipfix_data_stream(r, rl, tid=tid, rec_per_msg=per, export_time0=1_700_000_000 + r0 // per, seq0=r0)
        parts.append((b, o, ln))
        keys.append(torch.tensor(sel, dtype=torch.int64, device=b.device))
    bufs, offs, lens = [], [], []
    base = 0
    for b, o, ln in parts:
        bufs.append(b[:-16])
        offs.append(o + base)
        lens.append(ln)
        base += b.numel() - 16
    buf = torch.cat(bufs + [torch.zeros(16, dtype=torch.uint8, device=bufs[0].device)])
    order = torch.argsort(torch.cat(keys))
    return buf, torch.cat(offs)[order], torch.cat(lens)[order], int(count[m0:m1].sum())


# --- config 4: NetFlow v9 + IPFIX variable-length / enterprise IEs ------------
# NFv9 template 313 exactly as announced in the reference capture
# assets/pcaps/101-NFv9-CISCO-cust_primitives (130-byte records, reduced sizes).
NF313 = [(70, 3), (71, 3), (72, 3), (73, 3), (74, 3), (75, 3), (10, 4), (14, 4), (1, 4), (2, 4), (21, 4), (22, 4),
         (47, 4), (140, 16), (27, 16), (28, 16), (31, 3), (91, 1), (64, 4), (8, 4), (12, 4), (7, 2), (11, 2), (46, 1),
         (89, 1), (61, 1), (5, 1), (4, 1), (6, 1), (48, 2), (234, 4), (235, 4)]
# IPFIX template with variable-length strings / octets and enterprise IEs:
# VMware (PEN 6876) tenantProtocol, vmUuid (string, vlen), vifUuid (octets, vlen);
# Huawei (PEN 2011) unregistered id 1000 (vendor Unknown, vlen-aware).
V900 = [(8, 4), (12, 4), (82, 0xFFFF), (7, 2), (11, 2), (4, 1), (1, 8), (2, 8), (96, 0xFFFF),
        (880, 1, 6876), (951, 0xFFFF, 6876), (960, 0xFFFF, 6876), (1000, 0xFFFF, 2011), (152, 8)]
V900_ID = 900
NF313_ID = 313
SEED_CFG4 = 0x4E475A4500000004


def _u64s(n, seed, salt):
    return splitmix64(torch.arange(n, dtype=torch.int64) * 16 + salt, seed).numpy().view("uint64")


def vlen_records(n, fields=V900, seed=SEED_CFG4, max_len=40, spans=False):
    """n IPFIX records of a template with variable-length fields (numpy, host).
    Variable-length values are printable ASCII of 0..max_len bytes (valid
    UTF-8), written with the 1-byte length prefix, every 97th record's first
    variable field with the 255 + 3-byte escape.  dateTimeMilliseconds stays in
    chrono's range.  Returns (flat uint8 bytes, record lengths int64), and with
    spans=True also every field's value span per record: [(start in flat
    int64[n], length int64[n])] in template order (the generator's ground
    truth for full-size checks)."""
    import numpy as np
    lens = []
    parts = []
    for k, f in enumerate(fields):
        ln = f[1]
        if ln == 0xFFFF:
            L = (_u64s(n, seed, k) % (max_len + 1)).astype(np.int64)
            esc = np.zeros(n, dtype=bool)
            if k == next(i for i, g in enumerate(fields) if g[1] == 0xFFFF):
                esc = (np.arange(n) % 97) == 0
            lens.append(L + np.where(esc, 4, 1))
            parts.append(("v", L, esc, k))
        else:
            lens.append(np.full(n, ln, dtype=np.int64))
            parts.append(("f", ln, f[0], k))
    rec_len = np.sum(lens, axis=0)
    starts = np.zeros(n + 1, dtype=np.int64)
    starts[1:] = np.cumsum(rec_len)
    out = np.zeros(int(starts[-1]), dtype=np.uint8)
    cur = starts[:-1].copy()
    span = []
    for kind, a, b, k in parts:
        if kind == "f":
            ln, ie = a, b
            span.append((cur.copy(), np.full(n, ln, dtype=np.int64)))
            if ie in (152, 153) and ln == 8:
                v = 1_700_000_000_000 + (np.arange(n, dtype=np.int64) * 7919) % 1_000_000_000
            else:
                v = _u64s(n, seed, 100 + k)
            vb = v.astype(">u8").view(np.uint8).reshape(n, 8)[:, 8 - ln:] if ln <= 8 else None
            for j in range(ln):
                out[cur + j] = vb[:, j] if vb is not None else (_u64s(n, seed, 200 + 16 * k + j) & 0xFF)
            cur += ln
        else:
            L, esc = a, b
            out[cur] = np.where(esc, 255, L).astype(np.uint8)
            e = np.nonzero(esc)[0]
            out[cur[e] + 1] = 0
            out[cur[e] + 2] = (L[e] >> 8).astype(np.uint8)
            out[cur[e] + 3] = (L[e] & 0xFF).astype(np.uint8)
            cur += np.where(esc, 4, 1)
            span.append((cur.copy(), L.copy()))
            # printable bytes 'a'..'z' for every value byte
            total = int(L.sum())
            if total:
                rep = np.repeat(cur, L)
                within = np.arange(total) - np.repeat(np.cumsum(L) - L, L)
                out[rep + within] = (97 + (rep + within) % 26).astype(np.uint8)
            cur += L
    return (out, rec_len, span) if spans else (out, rec_len)


def _pack_ipfix(flat, rec_len, tid, max_msg=65000, export_time0=1_700_000_000, domain=1, firsts=None):
    import numpy as np
    starts = np.zeros(len(rec_len) + 1, dtype=np.int64)
    starts[1:] = np.cumsum(rec_len)
    msgs = []
    i = 0
    n = len(rec_len)
    while i < n:
        j = int(np.searchsorted(starts, starts[i] + max_msg - 20, side="right")) - 1
        j = max(j, i + 1)
        body = flat[starts[i]:starts[j]].tobytes()
        if firsts is not None:
            firsts.append(i)
        msgs.append(struct.pack(">HHIIIHH", 10, 20 + len(body), export_time0 + len(msgs), i, domain, tid,
                                4 + len(body)) + body)
        i = j
    return msgs


def nfv9_template_message(tid=NF313_ID, fields=NF313, unix=1_700_000_000, seq=0, src=1):
    body = struct.pack(">HH", tid, len(fields)) + b"".join(struct.pack(">HH", i, ln) for i, ln in fields)
    fs = struct.pack(">HH", 0, 4 + len(body)) + body
    return struct.pack(">HHIIII", 9, 1, 1000, unix, seq, src) + fs


def _pack_nfv9(recs, rec_len, tid, per_msg=10, unix0=1_700_000_000, src=1):
    """NetFlow v9 export packets of per_msg records in one data flowset,
    zero-padded to 4 bytes (netflow.rs:225,237-248)."""
    msgs = []
    n = recs.shape[0]
    for m, i in enumerate(range(0, n, per_msg)):
        k = min(per_msg, n - i)
        body = recs[i:i + k].tobytes()
        pad = (-(4 + len(body))) % 4
        fs = struct.pack(">HH", tid, 4 + len(body) + pad) + body + b"\0" * pad
        msgs.append(struct.pack(">HHIIII", 9, k, 1000 + m, unix0 + m, i, src) + fs)
    return msgs


def cfg4_datagrams(n, seed=SEED_CFG4, ipfix_msg_bytes=1400, layout=False):
    """Config 4: n records, half NetFlow v9 (template 313, 130 B, 10 records
    per packet as Cisco exporters send), half IPFIX with variable-length and
    enterprise IEs (template 900) in MTU-sized messages (~1400 B, ~15
    records), packets interleaved.  The two template packets come first.
    Returns a list of datagrams (bytes); layout=True also returns the IPFIX
    records' generator layout: dict(flat, rec_len, spans (vlen_records),
    v_first: first record of each template-900 message, v_pos: index of each
    such message in the returned list)."""
    import numpy as np
    n_nf = n // 2
    n_v = n - n_nf
    _, rl = field_offsets(NF313)
    nf = template_records(NF313, n_nf, seed, "cpu").numpy()
    nf_msgs = _pack_nfv9(nf, rl, NF313_ID)
    flat, lens, spans = vlen_records(n_v, V900, seed + 1, spans=True)
    v_first = []
    v_msgs = _pack_ipfix(flat, lens, V900_ID, max_msg=ipfix_msg_bytes, firsts=v_first)
    out = [nfv9_template_message(), _ipfix_template_v900()]
    # interleave proportionally: packet i of a stream of m packets at position i/m
    keys = [(i / len(nf_msgs), 0, i) for i in range(len(nf_msgs))] + [(i / len(v_msgs), 1, i) for i in range(len(v_msgs))]
    keys.sort()
    out += [nf_msgs[i] if s == 0 else v_msgs[i] for _, s, i in keys]
    if not layout:
        return out
    v_pos = [0] * len(v_msgs)
    for p, (_, s, i) in enumerate(keys):
        if s == 1:
            v_pos[i] = 2 + p
    return out, dict(flat=flat, rec_len=lens, spans=spans, v_first=v_first, v_pos=v_pos)


def _ipfix_template_v900():
    body = struct.pack(">HH", V900_ID, len(V900))
    for f in V900:
        if len(f) == 2:
            body += struct.pack(">HH", f[0], f[1])
        else:
            body += struct.pack(">HHI", f[0] | 0x8000, f[1], f[2])
    sset = struct.pack(">HH", 2, 4 + len(body)) + body
    return struct.pack(">HHIII", 10, 16 + len(sset), 1_700_000_000, 0, 1) + sset
