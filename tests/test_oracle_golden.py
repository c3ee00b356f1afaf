"""Pin the CPU oracle to the reference's own golden outputs (CPU only).

For every flow pcap the reference's pcap_tests.rs walks, and for the
pcap-decoder integration golden, the oracle must reproduce the reference's
JSON lines byte for byte (tests/golden/, built by tests/golden/make_golden.py).
"""
import pytest

import drivers
import golden_io

CASES = golden_io.cases()


@pytest.mark.parametrize("name,kind,n", CASES, ids=[c[0] for c in CASES])
def test_oracle_matches_reference_golden(name, kind, n):
    dgrams = golden_io.datagrams(name)
    assert len(dgrams) == n
    expected = golden_io.expected_lines(name)
    run = drivers.run_pcap_tests_driver if kind == "pcap_tests" else drivers.run_pcap_decoder_driver
    got = run(dgrams)
    assert len(got) == len(expected)
    for i, (g, e) in enumerate(zip(got, expected)):
        assert g == e, "line %d differs" % i
