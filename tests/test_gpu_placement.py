"""GPU: arena placement trials leave the first large batch's results in the kept arena.  Every trial
decodes the batch into its own column arena (the headers, sets and counts outside it are the same for
every trial), so the kept arena is used as it is -- except where a placement probe ran over it after
its decode (NGZ_OPT_PLACE_PROBE 1, and arena 0 under 2), which decodes it once more.  T20 (1.5*10^7
records, a decode above the 0.25 ms trial threshold) and config 4 (6*10^6 records; row tables in the
arena) against a context without trials: sampled column bytes, datagram headers, sets, processed counts."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from netgauze_amd.flow import FlowInfoCodec  # noqa: F401  (loads libngz.so, fails loudly if missing)
    return torch.device("cuda:0")


def digest(batch, codec):
    from netgauze_amd._lib import d2h
    cols = []
    for s in batch.slots:
        if not s.n_records:
            continue
        for f, fi in enumerate(s.fields):
            n = s.n_records * fi.width
            for at in sorted({0, (n // 2) & ~15, max(0, n - 4096)}):
                cols.append(d2h(s.column_ptr(f) + at, min(4096, n - at)).tobytes())
    return (batch.dgram_headers().tobytes(), batch.sets().tobytes(), cols,
            codec.template_counts(9), codec.template_counts(10))


@pytest.fixture(scope="module")
def batches(dev):
    from netgauze_amd import synth
    n = 15_000_000
    t20 = synth.stream_range(n, 0, len(synth.stream_index(n)[2]), None, device=dev)[:3]
    dg = synth.cfg4_datagrams(6_000_000)
    return {"t20": ([synth.template_message()], t20), "cfg4": (dg[:2], synth.host_batch(dg[2:], device=dev))}


@pytest.mark.parametrize("probe", [0, 1, 2])
@pytest.mark.parametrize("work", ["t20", "cfg4"])
def test_trials_keep_the_batch_results(dev, batches, work, probe):
    from netgauze_amd.flow import FlowInfoCodec, OPT_PLACE_PROBE, OPT_PLACE_TRIALS
    learn, b = batches[work]
    ref = FlowInfoCodec(0, rtc_sync=True, options={OPT_PLACE_TRIALS: 1})
    ref.decode_datagrams(learn)
    want = digest(ref.decode_batch(*b), ref)
    ref.close()
    c = FlowInfoCodec(0, rtc_sync=True, options={OPT_PLACE_TRIALS: 4, OPT_PLACE_PROBE: probe})
    c.decode_datagrams(learn)
    got = digest(c.decode_batch(*b), c)
    ms, kept, pms = c.placement_trials(probes=True)
    assert len(ms) + len([x for x in pms if x]) >= 2, (ms, kept, pms)  # the trials ran
    assert got[:2] == want[:2]
    assert all(np.array_equal(np.frombuffer(x, np.uint8), np.frombuffer(y, np.uint8)) for x, y in zip(got[2], want[2]))
    assert len(got[2]) == len(want[2])
    assert got[3:] == want[3:]
    # the next batch on the kept arena decodes the same
    again = digest(c.decode_batch(*b), c)
    assert again[:3] == want[:3]
    c.close()
