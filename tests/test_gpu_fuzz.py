"""GPU differential fuzz: the device path against the CPU oracle on a seeded mutation corpus.

The reference fuzzes this path for panics (fuzz/fuzz_targets/fuzz_ipfix_pkt.rs:23-36,
fuzz_netflow_v9_pkt.rs, fuzz_flow_codec.rs:22-30).  Here every mutated datagram
(tests/fuzz_corpus.py: header / set / template / vlen-prefix / padding / truncation / splice /
bit mutations of every reference golden capture and of synthetic T20, config-3, NFv9 313,
variable-length 900 and all-decode-rules streams) goes through both device kernel paths and
must equal the oracle: status, serde error text, structured ngz_dgram_error, message header,
every decoded field, the template map and the processed counts; the JSON rendered from the
columns must equal the oracle's serde text.  Stream mode (the codec target) cuts mutated
streams of both protocols into random datagrams for two peers and runs them through the
collector in both reference driver modes.

Each batch runs under a wall-clock guard (a hang fails the test; pytest-timeout ends a hard
one).  Divergences are written to gpurun_out/fuzz/ (hex datagrams + messages) before the test
fails, so one GPU run shows all of them.  Cases fixed after a divergence are kept as
regression vectors in tests/golden/fuzz_regressions.json.
"""
import json
import os
import time

import pytest

import fuzz_corpus as F
import drivers
import ngz_oracle as O
import parity

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_CASES = int(os.environ.get("NGZ_FUZZ_CASES", "20000"))      # per protocol
N_STREAMS = int(os.environ.get("NGZ_FUZZ_STREAMS", "400"))
BATCH_WALL_S = 30.0


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from netgauze_amd.flow import FlowInfoCodec  # noqa: F401  (loads libngz.so, fails loudly if missing)
    return torch.device("cuda:0")


_CORPUS = {}


def oracle_corpus(proto):
    """[(name, dgrams, flags, oracle per datagram, oracle codec after the batch)], cached."""
    if proto not in _CORPUS:
        out = []
        for name, dgrams, flags in F.corpus(proto, N_CASES):
            oracle, oc = parity.oracle_datagrams(dgrams)
            out.append((name, dgrams, flags, oracle, oc))
        _CORPUS[proto] = out
    return _CORPUS[proto]


def _report(tag, items):
    d = os.path.join(os.environ.get("GRAFT_REPO_ROOT", ROOT), "gpurun_out", "fuzz")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, tag + ".json"), "w") as f:
        json.dump(items, f, indent=1)


def _tjson(t):
    return {"scope_field_specifiers": [s.to_json() for s in t.scope],
            "field_specifiers": [f.to_json() for f in t.fields]}


def oracle_json(oracle):
    return [None if k == "none" else O.dumps(v if k == "err" else v.to_json()) for k, v in oracle]


def run_batch(codec_args, proto, name, dgrams, flags, oracle, oc, check_json, failures):
    from netgauze_amd.flow import FlowInfoCodec
    codec = FlowInfoCodec(0, **codec_args)
    try:
        t0 = time.time()
        batch = codec.decode_datagrams(dgrams)
        wall = time.time() - t0
        fails = []
        if wall > BATCH_WALL_S:
            fails.append((-1, "batch took %.1f s" % wall))
        stats = parity.check_batch(batch, oracle, failures=fails)
        tm = oc.ipfix_templates if proto == 10 else oc.netflow_templates
        got_t = codec.templates(proto)
        exp_t = [{"id": k, **_tjson(v)} for k, v in sorted(tm.items())]
        if got_t != exp_t:
            fails.append((-1, "template map differs:\n got %s\n exp %s" % (str(got_t)[:600], str(exp_t)[:600])))
        got_c = codec.template_counts(proto)
        exp_c = {k: v.processed_count for k, v in tm.items()}
        if got_c != exp_c:
            fails.append((-1, "processed counts differ: got %s exp %s" % (got_c, exp_c)))
        if check_json:
            exp = oracle_json(oracle)
            got = {d: js for d, st, js, _ in batch.json_lines()}
            for d, e in enumerate(exp):
                if got.get(d) != e:
                    fails.append((d, "json:\n got %s\n exp %s" % (str(got.get(d))[:600], str(e)[:600])))
        pending = any(batch.slot_kernel(s) == 2 for s in range(batch.out.n_slots))
        if fails:
            failures.append({"stream": name, "proto": proto, "codec": {k: str(v) for k, v in codec_args.items()},
                             "dgrams": [bytes(x).hex() for x in dgrams],
                             "flags": flags, "fails": [(d, m) for d, m in fails[:20]], "n_fails": len(fails)})
        return stats, pending
    finally:
        codec.close()


@pytest.mark.parametrize("proto", [10, 9], ids=["ipfix", "nfv9"])
@pytest.mark.parametrize("path", ["specialized", "generic"])
def test_fuzz_datagrams(dev, proto, path):
    """>= 20 000 mutated datagrams per protocol through one kernel path against the oracle
    (datagram mode: one FlowInfoCodec::decode per datagram, flow_actor.rs:342-411)."""
    from netgauze_amd import _lib as L
    from netgauze_amd.flow import FlowInfoCodec
    corpus = oracle_corpus(proto)
    if path == "specialized":
        # the clean templates' kernels first (compiled and loaded); mutated layouts then decode
        # with the generic kernel while their own compile (bounded pool) runs, and the batches
        # that had such a slot run again once every compile is done
        warm = {}
        for name, dgrams, flags, *_ in corpus:
            warm.setdefault(name, [d for d, f in zip(dgrams, flags) if f is None])
        for tm in warm.values():
            FlowInfoCodec(0, specialize=True, rtc_sync=True).decode_datagrams(tm)
        args = dict(specialize=True, rtc_sync=False)
    else:
        args = dict(specialize=False)
    failures, again = [], []
    tot = {"ok": 0, "err": 0, "none": 0, "records": 0, "fields": 0, "unsupported": 0}
    cases = 0
    for i, (name, dgrams, flags, oracle, oc) in enumerate(corpus):
        stats, pending = run_batch(args, proto, name, dgrams, flags, oracle, oc, path == "specialized", failures)
        for k in tot:
            tot[k] += stats.get(k, 0)
        cases += sum(1 for f in flags if f is not None)
        if pending:
            again.append(i)
        if i % 10 == 9:
            print("  fuzz %d %s: %d/%d batches, %d failing" % (proto, path, i + 1, len(corpus), len(failures)),
                  flush=True)
    if path == "specialized":
        L.load().ngz_rtc_drain()
        for i in again:
            run_batch(args, proto, *corpus[i], False, failures)
    print("fuzz %s %s: %d cases, %s, %d batches re-run specialised" % (proto, path, cases, tot, len(again)))
    if failures:
        _report("dgram_%d_%s" % (proto, path), failures)
    assert not failures, "%d batches diverge; first: %s" % (
        len(failures), json.dumps(failures[0]["fails"][:3])[:3000])
    assert cases >= N_CASES and tot["unsupported"] == 0
    assert tot["ok"] > N_CASES // 5 and tot["err"] > N_CASES // 5 and tot["records"] > 0


def test_fuzz_streams(dev):
    """Stream mode (fuzz_flow_codec.rs:22-30): mutated IPFIX and NFv9 messages of both
    protocols in one byte stream per peer, cut into datagrams of random sizes, two peers
    interleaved, through the GPU collector in both driver modes against oracle/drivers.py."""
    from netgauze_amd import ingest as I
    cases = F.streams_corpus(N_STREAMS)
    failures = []
    lines = 0
    per_col = 25
    for mode, drv in ((I.PCAP_DECODER, drivers.run_pcap_decoder_driver),
                      (I.FLOW_INFO, drivers.run_pcap_tests_driver)):
        for c0 in range(0, len(cases), per_col):
            group = cases[c0:c0 + per_col]
            dg = []
            for k, chunks in enumerate(group):
                for peer, payload in chunks:
                    src = ("v4", 0x0A000000 + 2 * (c0 + k) + peer)
                    dg.append((src, 4000 + peer, ("v4", 0x0A0000FE), 9991, payload))
            exp = drv(dg)
            col = I.Collector(0, mode)
            t0 = time.time()
            for i, (src, sp, dst, dp, pl) in enumerate(dg):
                col.push(src, sp, dst, dp, pl, tag=i)
            got = [line for _, line in col.flush()]
            wall = time.time() - t0
            col.close()
            lines += len(exp)
            print("  fuzz streams mode %d: cases %d-%d, %d lines" % (int(mode), c0, c0 + len(group), len(exp)),
                  flush=True)
            if got != exp or wall > BATCH_WALL_S:
                diff = next((i for i, (g, e) in enumerate(zip(got, exp)) if g != e), min(len(got), len(exp)))
                failures.append({"mode": int(mode), "cases": [c0, c0 + len(group)], "wall": wall,
                                 "n_got": len(got), "n_exp": len(exp), "first_diff": diff,
                                 "got": got[diff][:800] if diff < len(got) else None,
                                 "exp": exp[diff][:800] if diff < len(exp) else None,
                                 "dgrams": [(s[1], sp, pl.hex()) for s, sp, _, _, pl in dg]})
    print("fuzz streams: %d cases, %d lines per mode pair" % (len(cases), lines))
    if failures:
        _report("streams", failures)
    assert not failures, json.dumps({k: v for k, v in failures[0].items() if k != "dgrams"})[:3000]


def test_fuzz_regressions(dev):
    """Divergences the corpus found, kept after their fix (both kernel paths)."""
    path = os.path.join(ROOT, "tests", "golden", "fuzz_regressions.json")
    with open(path) as f:
        vecs = json.load(f)
    failures = []
    for v in vecs:
        dgrams = [bytes.fromhex(x) for x in v["dgrams"]]
        oracle, oc = parity.oracle_datagrams(dgrams)
        for args in (dict(specialize=True, rtc_sync=True), dict(specialize=False)):
            run_batch(args, v["proto"], v["name"], dgrams, [None] * len(dgrams), oracle, oc, True, failures)
    assert not failures, json.dumps(failures[0]["fails"][:3])[:3000]
