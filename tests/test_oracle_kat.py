"""Pin the CPU oracle's field rules to the reference's own unit-test vectors
(tests/kats.py, transcribed from crates/flow-pkt/src/wire/tests/*.rs)."""
import pytest

import kats
import ngz_oracle as O


@pytest.mark.parametrize("name,ie_id,length,wire,expected", kats.KATS, ids=[k[0] for k in kats.KATS])
def test_oracle_field_kat(name, ie_id, length, wire, expected):
    ie = O.REGISTRY.lookup(0, ie_id)
    cur = O.Reader(bytearray(wire))
    if isinstance(expected, dict):
        with pytest.raises(O.ParseFail) as e:
            O.parse_field(cur, ie, length)
        assert e.value.err == expected
        return
    f = O.parse_field(cur, ie, length)
    assert cur.is_empty(), "parsed completely"
    assert f.value == expected
