"""GPU: ngz_decode_batch_submit / ngz_decode_batch_wait -- several contexts' batches in flight from one
host thread, as the reference collector's single receive task keeps decoding while packets arrive
(flow-service/src/flow_actor.rs:850-869).  Every result must equal the blocking ngz_decode_batch's:
datagram headers, set table, every column byte and the processed counts, for T20 and config 4
(NFv9 + IPFIX variable-length) over three rounds; plus the pending-batch rules of the C ABI."""
import ctypes

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

NGZ_E_INVALID = -1  # include/ngz/flow_decode.h


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from netgauze_amd.flow import FlowInfoCodec  # noqa: F401  (loads libngz.so, fails loudly if missing)
    return torch.device("cuda:0")


def snapshot(batch, codec):
    cols = {}
    for s in batch.slots:
        cols[(s.proto, s.template_id)] = [s.column_bytes(f).tobytes() for f in range(len(s.fields))]
    return (batch.dgram_headers().tobytes(), batch.sets().tobytes(), cols,
            codec.template_counts(9), codec.template_counts(10))


def workloads(dev):
    from netgauze_amd import synth
    n = 500_000
    t20 = synth.stream_range(n, 0, len(synth.stream_index(n)[2]), None, device=dev)[:3]
    dg = synth.cfg4_datagrams(200_000)
    return [("t20", [synth.template_message()], t20), ("cfg4", dg[:2], synth.host_batch(dg[2:], device=dev))]


def test_submit_wait_from_one_thread_equals_blocking(dev):
    from netgauze_amd.flow import FlowInfoCodec
    for name, learn, b in workloads(dev):
        ref = FlowInfoCodec(0, rtc_sync=True)
        ref.decode_datagrams(learn)
        codecs = [FlowInfoCodec(0, rtc_sync=True) for _ in range(3)]
        streams = [torch.cuda.Stream(dev) for _ in codecs]
        for c in codecs:
            c.decode_datagrams(learn)
        torch.cuda.synchronize()
        for rnd in range(3):
            want = snapshot(ref.decode_batch(*b), ref)
            for c, s in zip(codecs, streams):
                c.decode_batch_submit(*b, stream=s.cuda_stream)
            for k, c in enumerate(codecs):
                got = snapshot(c.decode_batch_wait(), c)
                assert got[:3] == want[:3], (name, rnd, k)
                assert got[3:] == want[3:], (name, rnd, k, got[3:], want[3:])
        for c in codecs + [ref]:
            c.close()


def test_pending_batch_rules(dev):
    from netgauze_amd import _lib as L
    from netgauze_amd.flow import FlowInfoCodec, lib
    _, learn, b = workloads(dev)[0]
    c = FlowInfoCodec(0, rtc_sync=True)
    c.decode_datagrams(learn)
    data, offs, lens = b
    bi = L.BatchIn(data.data_ptr(), data.numel(), offs.data_ptr(), lens.data_ptr(), int(offs.numel()))
    out, out2 = L.BatchOut(), L.BatchOut()
    assert lib().ngz_decode_batch_wait(c._ctx) == NGZ_E_INVALID  # nothing submitted
    assert lib().ngz_decode_batch_submit(c._ctx, ctypes.byref(bi), ctypes.byref(out), None) == 0
    # while it is pending the context takes no other batch
    assert lib().ngz_decode_batch_submit(c._ctx, ctypes.byref(bi), ctypes.byref(out2), None) == NGZ_E_INVALID
    assert lib().ngz_decode_batch(c._ctx, ctypes.byref(bi), ctypes.byref(out2), None) == NGZ_E_INVALID
    assert lib().ngz_decode_batch_wait(c._ctx) == 0
    assert out.n_records == 500_000 and out.n_dgrams == int(offs.numel())
    assert lib().ngz_decode_batch_wait(c._ctx) == NGZ_E_INVALID  # collected already
    # the blocking call works again, and destroying a context with a batch in flight waits for it
    assert lib().ngz_decode_batch(c._ctx, ctypes.byref(bi), ctypes.byref(out2), None) == 0
    assert lib().ngz_decode_batch_submit(c._ctx, ctypes.byref(bi), ctypes.byref(out), None) == 0
    c.close()
