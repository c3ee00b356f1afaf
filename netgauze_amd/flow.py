"""Host-side mirror of the reference decode interface, over the C ABI.

`FlowInfoCodec` plays the role of netgauze_flow_pkt::codec::FlowInfoCodec
(crates/flow-pkt/src/codec.rs:68-220): one instance per exporter peer, owning
the NetFlow v9 and IPFIX template maps.  `decode_batch` applies
`Decoder::decode` to every datagram of a batch, in order, the way
FlowCollectorActor::decode_pkt does (crates/flow-service/src/flow_actor.rs:
342-411), with the records decoded by the HIP kernels into per-template
columns in HBM.  `template_counts(reset=True)` is reset_processed_count
(crates/flow-pkt/src/ipfix.rs:65-69).
"""
import ctypes
import sys
import json

import numpy as np

from . import _lib
from ._lib import DGRAM_HDR_DTYPE, SET_INFO_DTYPE, d2h

_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        _LIB = _lib.load()
    return _LIB


class NgzError(RuntimeError):
    pass


class Slot:
    """Columns of one template version in the last batch."""

    def __init__(self, codec, index, info):
        self.index = index
        self.version_id = info.version_id
        self.template_id = info.template_id
        self.proto = info.proto
        self.n_records = info.n_records
        self.capacity = info.capacity
        self.columns_ptr = info.columns
        n = lib().ngz_slot_fields(codec._ctx, index, None, 0)
        arr = (_lib.FieldInfo * max(n, 1))()
        lib().ngz_slot_fields(codec._ctx, index, arr, n)
        self.fields = [arr[i] for i in range(n)]

    def column_ptr(self, f):
        return self.columns_ptr + self.capacity * self.fields[f].col_off

    def block_bytes(self):
        """Bytes of this slot's column block (every column, capacity rows)."""
        return self.capacity * sum(fi.width for fi in self.fields)

    def copy_block_to_host(self, host_ptr):
        """D2H of the whole column block (columns are contiguous in it)."""
        n = self.block_bytes()
        if n:
            rc = _lib.hip().hipMemcpy(host_ptr, self.columns_ptr, n, 2)
            if rc != 0:
                raise RuntimeError("hipMemcpy D2H failed: %d" % rc)
        return n

    def column_bytes(self, f, rows=None):
        """Host copy of column f: uint8 array of shape (rows, width)."""
        w = self.fields[f].width
        rows = self.n_records if rows is None else rows
        return d2h(self.column_ptr(f), rows * w).reshape(rows, w)


class DecodedBatch:
    def __init__(self, codec, out, source=None):
        self._codec = codec
        codec.generation += 1
        self.generation = codec.generation  # device arrays valid while it is the codec's latest
        self._source = source  # the batch bytes: host numpy array or device tensor
        self.out = out
        self.n_dgrams = out.n_dgrams
        self.n_sets = out.n_sets
        self.n_records = out.n_records
        self.n_template_dgrams = out.n_template_dgrams
        self._slots = None

    @property
    def slots(self):
        """Per template version: where its records landed (built on first use)."""
        if self._slots is None:
            self._slots = [Slot(self._codec, i, self.out.slots[i]) for i in range(self.out.n_slots)]
        return self._slots

    def input_bytes(self, offset, n):
        """Bytes [offset, offset+n) of this batch's input: variable-length
        columns hold {u64 offset into the batch bytes, u32 length} and are
        valid while the input is (the next batch on the context at most)."""
        src = self._source
        if src is None:
            raise ValueError("batch input not retained")
        if isinstance(src, np.ndarray):
            return bytes(src[offset:offset + n])
        return bytes(d2h(src.data_ptr() + offset, n))

    def dgram_headers(self):
        return d2h(self.out.dgrams, self.n_dgrams * 32).view(DGRAM_HDR_DTYPE)

    def sets(self):
        return d2h(self.out.sets, self.n_sets * 16).view(SET_INFO_DTYPE)

    def error_json(self, d):
        n = lib().ngz_dgram_error_json(self._codec._ctx, d, None, 0)
        if n < 0:
            return None
        buf = ctypes.create_string_buffer(n + 1)
        lib().ngz_dgram_error_json(self._codec._ctx, d, buf, n + 1)
        return buf.value.decode("utf-8")

    def error(self, d):
        s = self.error_json(d)
        return None if s is None else json.loads(s)

    def slot_kernel(self, slot):
        """1: the slot was decoded by its specialised kernel, 0: generic, 2: generic while compiling."""
        return lib().ngz_slot_kernel(self._codec._ctx, slot)

    def error_struct(self, d):
        """ngz_dgram_error: the structured FlowInfoCodecDecoderError of datagram
        d as a dict (kind / layer names from flow_decode.h), or None."""
        e = _lib.Error()
        if lib().ngz_dgram_error(self._codec._ctx, d, ctypes.byref(e)) != 0:
            return None
        out = {k: getattr(e, k) for k, _ in _lib.Error._fields_}
        out["kind"] = _lib.ERR_KINDS[e.kind]
        out["layer"] = _lib.ERR_LAYERS[e.layer]
        return out

    def json(self, d):
        """serde_json text of datagram d's FlowInfo (or of its error), rendered
        from the decoded columns (ngz_dgram_json); None for Ok(None)."""
        n = lib().ngz_dgram_json(self._codec._ctx, d, None, 0)
        if n < 0:
            return None
        buf = ctypes.create_string_buffer(n + 1)
        lib().ngz_dgram_json(self._codec._ctx, d, buf, n + 1)
        return buf.raw[:n].decode("utf-8")

    def record_fields(self, d, s, r):
        """ngz_record_fields: the fields of record r of datagram d's data set s (scope first) as
        [(pen, ie_id, kind, dtype, flags, wire_length, wire_offset, value bytes)] -- the reference's
        Box<[Field]> of DataRecord::parse (ipfix.rs:335-370), one typed value per IE."""
        n = lib().ngz_record_fields(self._codec._ctx, d, s, r, None, 0)
        if n < 0:
            raise NgzError("ngz_record_fields(%d, %d, %d) = %d" % (d, s, r, n))
        arr = (_lib.FieldValue * max(n, 1))()
        lib().ngz_record_fields(self._codec._ctx, d, s, r, arr, n)
        return [(f.pen, f.ie_id, f.kind, f.dtype, f.flags, f.wire_length, f.wire_offset,
                 ctypes.string_at(f.value, f.len) if f.len else b"") for f in arr[:n]]

    def json_lines(self):
        """[(dgram, status, json, consumed)] for every datagram with a FlowInfo
        or an error (ngz_batch_json: one host copy of the whole batch)."""
        from netgauze_amd import _lib
        out = []

        def cb(_user, d, status, text, n, consumed):
            out.append((int(d), int(status), ctypes.string_at(text, n).decode("utf-8"), int(consumed)))
            return 0

        fn = _lib.JSON_LINE_FN(cb)
        host = self._source if isinstance(self._source, np.ndarray) else None
        n = lib().ngz_batch_json(self._codec._ctx, host.ctypes.data if host is not None else None, fn, None)
        if n < 0:
            raise NgzError("ngz_batch_json failed: %d" % n)
        return out


OPT_SPECIALIZE = 1
OPT_BLOCKS_PER_CU = 2
OPT_RTC_SYNC = 5
OPT_SPLIT = 6         # split framing (flow_decode.h NGZ_OPT_SPLIT)
OPT_GROUP = 7         # multi-template decode launches
OPT_PLACE_TRIALS = 8  # column arenas tried for the first large batch
OPT_PLACE_PROBE = 9   # placement trials timed by a probe (1) / decode and probe (2)
D2H_KERNEL = 1  # NGZ_D2H_KERNEL


class FlowInfoCodec:
    def __init__(self, device=0, specialize=None, rtc_sync=None, options=None):
        """specialize: None (library default: per-template kernels, compiled in
        the background), True (per-template kernels, each template's first batch
        waits for its compile: deterministic kernel choice), False (generic
        kernel only).  rtc_sync overrides the waiting.  options: {OPT_*: value}
        for ngz_ctx_set_option (how batches run, never their results)."""
        self.generation = 0  # batches decoded so far (DecodedBatch.generation)
        ctx = ctypes.c_void_p()
        rc = lib().ngz_ctx_create(device, ctypes.byref(ctx))
        if rc != 0:
            raise NgzError("ngz_ctx_create(%d) failed: %d (no HIP device?)" % (device, rc))
        self._ctx = ctx
        if specialize is not None:
            self.set_option(OPT_SPECIALIZE, 1 if specialize else 0)
        if rtc_sync is None:
            rtc_sync = bool(specialize)
        self.set_option(OPT_RTC_SYNC, 1 if rtc_sync else 0)
        for opt, value in (options or {}).items():
            self.set_option(opt, value)

    def set_option(self, opt, value):
        self._check(lib().ngz_ctx_set_option(self._ctx, opt, int(value)))

    def close(self):
        if self._ctx:
            lib().ngz_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        if sys.is_finalizing():  # the HIP runtime may be torn down already: leave it to the process exit
            return
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise NgzError("netgauze_amd: %d: %s" % (rc, lib().ngz_last_error(self._ctx).decode()))

    def decode_batch(self, data, offsets, lengths, n=None, stream=None):
        """data/offsets/lengths: device tensors (uint8 / int64 / int32), already in HBM."""
        n = int(offsets.numel()) if n is None else n
        bi = _lib.BatchIn(data.data_ptr(), data.numel(), offsets.data_ptr(), lengths.data_ptr(), n)
        out = _lib.BatchOut()
        self._check(lib().ngz_decode_batch(self._ctx, ctypes.byref(bi), ctypes.byref(out),
                                           ctypes.c_void_p(stream) if stream else None))
        return DecodedBatch(self, out, data)

    def decode_batch_submit(self, data, offsets, lengths, n=None, stream=None):
        """ngz_decode_batch_submit: queue decode_batch on the context's decode worker and return at
        once; decode_batch_wait() gives the DecodedBatch.  One host thread can so keep several
        contexts' batches in flight.  The tensors must stay alive until the wait returns."""
        if getattr(self, "_pending", None) is not None:
            raise RuntimeError("netgauze_amd: a submitted batch is pending (decode_batch_wait first)")
        n = int(offsets.numel()) if n is None else n
        bi = _lib.BatchIn(data.data_ptr(), data.numel(), offsets.data_ptr(), lengths.data_ptr(), n)
        out = _lib.BatchOut()
        self._check(lib().ngz_decode_batch_submit(self._ctx, ctypes.byref(bi), ctypes.byref(out),
                                                  ctypes.c_void_p(stream) if stream else None))
        self._pending = (bi, out, data, offsets, lengths)
        return self

    def decode_batch_wait(self):
        """ngz_decode_batch_wait: the DecodedBatch of the submitted batch."""
        p, self._pending = getattr(self, "_pending", None), None
        if p is None:
            raise RuntimeError("netgauze_amd: no submitted batch")
        self._check(lib().ngz_decode_batch_wait(self._ctx))
        return DecodedBatch(self, p[1], p[2])

    def decode_datagrams(self, datagrams):
        """Host-memory datagrams (list of bytes): H2D through the library."""
        lens = np.array([len(d) for d in datagrams], dtype=np.uint32)
        offs = np.zeros(len(datagrams), dtype=np.uint64)
        if len(datagrams):
            offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        blob = np.frombuffer(b"".join(datagrams) + b"\0" * 16, dtype=np.uint8)
        out = _lib.BatchOut()
        self._check(lib().ngz_decode_batch_host(self._ctx, blob.ctypes.data, int(lens.sum()), offs.ctypes.data,
                                                lens.ctypes.data, len(datagrams), ctypes.byref(out)))
        return DecodedBatch(self, out, blob)

    def decode_host_buffers(self, data_ptr, data_size, offsets_ptr, lengths_ptr, n):
        """Host-resident batch given as raw pointers (pinned memory gives full
        PCIe rate): H2D through the library, then the device decode."""
        out = _lib.BatchOut()
        self._check(lib().ngz_decode_batch_host(self._ctx, data_ptr, data_size, offsets_ptr, lengths_ptr, n,
                                                ctypes.byref(out)))
        return DecodedBatch(self, out)

    def columns_to_host(self, host_ptr, cap):
        """D2H of the last batch's column blocks (slot order, 256-byte aligned)
        on the context's stream; returns the bytes written."""
        n = lib().ngz_columns_to_host(self._ctx, host_ptr, cap)
        if n < 0:
            self._check(int(n))
        return int(n)

    def columns_to_host_async(self, host_ptr, cap, stream=None, kernel=False):
        """ngz_columns_to_host_async: the same copy queued on `stream` (None: the context's) without
        waiting; kernel=True stores through the CUs (host_ptr pinned and mapped: hipHostMalloc /
        torch pin_memory) so the copy engines stay free for host-to-device copies.  The context's
        next decode waits for it.  Returns the bytes queued."""
        n = lib().ngz_columns_to_host_async(self._ctx, host_ptr, cap, ctypes.c_void_p(stream) if stream else None,
                                            D2H_KERNEL if kernel else 0)
        if n < 0:
            self._check(int(n))
        return int(n)

    def templates(self, proto):
        n = lib().ngz_templates_json(self._ctx, proto, None, 0)
        buf = ctypes.create_string_buffer(n + 1)
        lib().ngz_templates_json(self._ctx, proto, buf, n + 1)
        return json.loads(buf.value.decode())

    def template_counts(self, proto, reset=False):
        n = lib().ngz_template_counts(self._ctx, proto, None, None, 0, 0)
        ids = (ctypes.c_uint16 * max(n, 1))()
        cnt = (ctypes.c_uint64 * max(n, 1))()
        lib().ngz_template_counts(self._ctx, proto, ids, cnt, n, 1 if reset else 0)
        return {ids[i]: cnt[i] for i in range(n)}

    def template_counts_device(self, proto, dev_ptr, cap, reset=False, stream=None):
        """ngz_template_counts_device: (id, processed_count) u64 pairs written to
        device memory at dev_ptr (cap entries) on `stream`; returns the
        template count (> cap: table too small)."""
        n = lib().ngz_template_counts_device(self._ctx, proto, ctypes.c_void_p(dev_ptr), cap, 1 if reset else 0,
                                             ctypes.c_void_p(stream) if stream else None)
        if n < 0:
            self._check(n)
        return n

    def last_batch_info(self):
        """ngz_last_batch_info bits: 1 predicted launches, 2 split framing, 4 a pass repeated."""
        return lib().ngz_last_batch_info(self._ctx)

    def message_records(self, data, offsets, lengths):
        """ngz_message_records: data records per message (host numpy arrays / bytes) under this
        codec's current templates, for the record-balanced shard plan (dist.shard_by_records)."""
        buf = np.frombuffer(bytes(data), dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else \
            np.ascontiguousarray(data, dtype=np.uint8)
        offs = np.ascontiguousarray(offsets, dtype=np.uint64)
        lens = np.ascontiguousarray(lengths, dtype=np.uint32)
        out = np.zeros(len(offs), dtype=np.uint32)
        self._check(lib().ngz_message_records(self._ctx, buf.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                              len(offs), out.ctypes.data))
        return out.astype(np.int64)

    def placement_trials(self, probes=False):
        """ngz_placement_trials: ([decode ms of each arena trial], index of the kept arena), ([], 0)
        before the context's first large batch placed its arena; probes=True adds the probe ms
        (NGZ_OPT_PLACE_PROBE) as a third item."""
        n = lib().ngz_placement_trials(self._ctx, None, None, 0, None)
        ms = (ctypes.c_float * max(n, 1))()
        pm = (ctypes.c_float * max(n, 1))()
        kept = ctypes.c_uint32()
        lib().ngz_placement_trials(self._ctx, ms, pm, n, ctypes.byref(kept))
        out = ([float(x) for x in ms[:n] if x], int(kept.value))
        return out + ([float(x) for x in pm[:n]],) if probes else out

    def last_timing(self):
        a, b = ctypes.c_float(), ctypes.c_float()
        lib().ngz_last_timing(self._ctx, ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value
