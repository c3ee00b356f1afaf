"""CPU: the fuzz corpus (tests/fuzz_corpus.py) is deterministic, reaches every check the
reference makes on this path, and the oracle survives it (only the reference's own error
values come out: fuzz/fuzz_targets/fuzz_ipfix_pkt.rs:23-36, fuzz_netflow_v9_pkt.rs and
fuzz_flow_codec.rs:22-30 assert exactly that of the Rust parser)."""
import collections
import hashlib

import pytest

import drivers
import fuzz_corpus as F
import parity


def _digest(batches):
    h = hashlib.sha256()
    for name, dgrams, flags in batches:
        h.update(name.encode())
        for d in dgrams:
            h.update(len(d).to_bytes(4, "little") + d)
    return h.hexdigest()


def _innermost(err):
    tags = []
    while isinstance(err, dict) and len(err) == 1:
        (k, err), = err.items()
        tags.append(k)
    return tags[-1]


def test_corpus_is_deterministic():
    assert _digest(F.corpus(10, 1500)) == _digest(F.corpus(10, 1500))
    assert _digest(F.corpus(9, 1500)) == _digest(F.corpus(9, 1500))


@pytest.mark.parametrize("proto,kinds", [
    (10, {"UnsupportedVersion", "InvalidLength", "UnexpectedEof", "InvalidSetId", "NoTemplateDefinedFor",
          "InvalidTemplateId", "UndefinedIANAIE", "InvalidScopeFieldsCount", "InvalidPaddingValue",
          "InvalidTimestampMillis", "Utf8Error"}),
    (9, {"UnsupportedVersion", "InvalidLength", "UnexpectedEof", "InvalidSetId", "NoTemplateDefinedFor",
         "InvalidTemplateId", "UndefinedIANAIE", "InvalidPaddingValue", "InvalidCount"}),
])
def test_oracle_survives_corpus(proto, kinds):
    """6 000 cases per protocol: every outcome is Ok(None), a packet or a reference error value
    (anything else raised here is an oracle bug); the corpus reaches the listed error kinds
    and every mutation operator that applies to the protocol."""
    seen, outcomes, ops = set(), collections.Counter(), collections.Counter()
    for name, dgrams, flags in F.corpus(proto, 6000):
        out, _ = parity.oracle_datagrams(dgrams)
        for (k, v), f in zip(out, flags):
            if f is None:
                continue
            outcomes[k] += 1
            ops.update(f)
            if k == "err":
                seen.add(_innermost(v))
    assert kinds <= seen, kinds - seen
    assert outcomes["ok"] > 600 and outcomes["err"] > 600 and outcomes["none"] > 100
    expect_ops = set(F.OPERATORS) - ({"nf_count"} if proto == 10 else {"vlen"})
    assert expect_ops <= set(ops), expect_ops - set(ops)


def test_stream_corpus_drivers_survive():
    """Stream mode: both reference drivers run every stream case to the end."""
    cases = F.streams_corpus(60)
    for chunks in cases:
        dg = [(("v4", 0x0A000000 + p), 4000 + p, ("v4", 0x0A0000FE), 9991, x) for p, x in chunks]
        a = drivers.run_pcap_decoder_driver(dg)
        b = drivers.run_pcap_tests_driver(dg)
        assert len(a) > 0 and len(b) > 0
