"""Field-level known-answer vectors transcribed from the reference's own unit
tests (crates/flow-pkt/src/wire/tests/mod.rs and ipfix.rs).  Each entry is
(name, ie_id, length, wire bytes, expected oracle value or expected error).
Expected values are restated in the oracle's value model:
  unsigned -> int; float64 -> ("f64", raw bits); dateTime -> DateTime(secs, nanos);
  strings -> str; octet arrays / u256 -> bytes.
"""
import calendar
import struct

import kats_packets as K
import ngz_oracle as O


def _utc(y, mo, d, h, mi, s):
    return calendar.timegm((y, mo, d, h, mi, s, 0, 0, 0))


SMALL = "abcdefghijklmnopqrstuvwxyz"
LARGE = SMALL * 10  # 260 characters
SMALL_DATA = bytes(range(26))
LARGE_DATA = bytes((i % 256) for i in range(260))

KATS = [
    # mod.rs:77-99 test_u8_value: protocolIdentifier 123 (PTP)
    ("u8_value", 4, 1, bytes([123]), 123),
    ("u8_invalid_length", 4, 2, bytes([123]),
     {"InvalidLength": {"offset": 0, "ie_name": "protocolIdentifier", "length": 2}}),
    # mod.rs:102-129 test_f64_value: samplingProbability 123.4
    ("f64_value", 311, 8, bytes([64, 94, 217, 153, 153, 153, 153, 154]),
     ("f64", struct.unpack(">Q", struct.pack(">d", 123.4))[0])),
    ("f64_invalid_length", 311, 4, bytes([64, 94, 217, 153, 153, 153, 153, 154]),
     {"InvalidLength": {"offset": 0, "ie_name": "samplingProbability", "length": 4}}),
    # mod.rs:223-239 test_milli_value: 2016-11-29T20:05:31.519Z
    ("milli_value", 152, 8, bytes([0, 0, 1, 88, 177, 177, 56, 255]),
     O.DateTime(_utc(2016, 11, 29, 20, 5, 31), 519_000_000)),
    # mod.rs:242-295 test_time_fraction_value: full (leap second at :59), half (rounded), zero
    ("fraction_full_leap", 154, 8, bytes([0x58, 0x3d, 0xdf, 0xa7, 0xff, 0xff, 0xff, 0xff]),
     O.DateTime(_utc(2016, 11, 29, 20, 5, 59), 1_000_000_000)),
    ("fraction_half", 154, 8, bytes([0x58, 0x3d, 0xdf, 0x8b, 0x7f, 0xff, 0xff, 0xff]),
     O.DateTime(_utc(2016, 11, 29, 20, 5, 31), 499_999_999)),
    ("fraction_zero", 154, 8, bytes([0x58, 0x3d, 0xdf, 0x8b, 0, 0, 0, 0]),
     O.DateTime(_utc(2016, 11, 29, 20, 5, 31), 0)),
] + [
    # mod.rs:423-509 test_u64_reduced_size_encoding: packetDeltaCount, 1..8 bytes
    ("u64_reduced_%d" % n, 2, n, bytes([0xff, 0xee, 0xdd, 0xcc, 0xbb, 0xaa, 0x99, 0x88][:n]),
     int.from_bytes(bytes([0xff, 0xee, 0xdd, 0xcc, 0xbb, 0xaa, 0x99, 0x88][:n]), "big"))
    for n in range(1, 9)
] + [
    # mod.rs:512-552 test_u256_value: full, reduced (left-aligned, zero padded), too long
    ("u256_full", 515, 32, bytes([0x11] * 32), bytes([0x11] * 32)),
    ("u256_reduced", 515, 8, bytes([0x11] * 8), bytes([0x11] * 8) + bytes(24)),
    ("u256_invalid_length", 515, 33, bytes([0x11] * 32),
     {"InvalidLength": {"offset": 0, "ie_name": "ipv6ExtensionHeadersFull", "length": 33}}),
    # ipfix.rs:1704-1788 test_string_variable_length: applicationName, u8 / 3-byte length, fixed
    ("string_vlen_small", 96, 0xFFFF, bytes([26]) + SMALL.encode(), SMALL),
    ("string_fixed_small", 96, 26, SMALL.encode(), SMALL),
    ("string_vlen_large", 96, 0xFFFF, bytes([0xff, 0x00, 0x01, 0x04]) + LARGE.encode(), LARGE),
    ("string_fixed_large", 96, 260, LARGE.encode(), LARGE),
    # ipfix.rs:1791-1875 test_octet_array_variable_length: paddingOctets
    ("octets_vlen_small", 210, 0xFFFF, bytes([26]) + SMALL_DATA, SMALL_DATA),
    ("octets_fixed_small", 210, 26, SMALL_DATA, SMALL_DATA),
    ("octets_vlen_large", 210, 0xFFFF, bytes([0xff, 0x00, 0x01, 0x04]) + LARGE_DATA, LARGE_DATA),
    ("octets_fixed_large", 210, 260, LARGE_DATA, LARGE_DATA),
] + [
    # parse-utils/src/reader.rs:400-412, 481-493 (uint*_be_right_aligns_shortened_values): 0x0000ABCD in
    # 2, 3 and 4 octets through the IEs whose decoders call read_unsigned64_be / read_unsigned32_be
    # (packetDeltaCount unsigned64, ingressInterface unsigned32; generator.rs:1468-1496)
    ("reader_u64_shortened_%d" % len(w), 2, len(w), w, 0xABCD)
    for w in (bytes([0xAB, 0xCD]), bytes([0, 0xAB, 0xCD]), bytes([0, 0, 0xAB, 0xCD]))
] + [
    ("reader_u32_shortened_%d" % len(w), 10, len(w), w, 0xABCD)
    for w in (bytes([0xAB, 0xCD]), bytes([0, 0xAB, 0xCD]), bytes([0, 0, 0xAB, 0xCD]))
] + [
    # reader.rs:414-420, 495-501 (full width equals the fixed read)
    ("reader_u64_full_width", 2, 8, bytes([0x01, 0x23, 0x45, 0x67, 0x89, 0xAB, 0xCD, 0xEF]), 0x0123456789ABCDEF),
    ("reader_u32_full_width", 10, 4, bytes([0x01, 0x23, 0x45, 0x67]), 0x01234567),
    # reader.rs:529-551 through the one IANA signed32 IE, mibObjectValueInteger (read_signed32_be,
    # generator.rs:1549-1562): -2 shortened to one octet sign-extends, 0x7F stays positive, full width
    ("reader_i32_sign_extends_shortened", 434, 1, bytes([0xFE]), -2),
    ("reader_i32_keeps_positive", 434, 1, bytes([0x7F]), 127),
    ("reader_i32_full_width", 434, 4, bytes([0xFF, 0xFF, 0xFF, 0xFE]), -2),
    # reader.rs:360-369 (read_padded left-aligns, zero-pads the tail) through an unsigned256 IE
    ("reader_padded_short", 515, 2, bytes([0xAA, 0xBB]), bytes([0xAA, 0xBB]) + bytes(30)),
] + [
    # mod.rs:131-157 test_mac_address_value, :187-214 test_pkg_record_value and :316-344
    # test_record_value (the same vector in three tests): sourceMacAddress 12:c6:21:12:69:32; length 2 is
    # InvalidLength at the field start
    (t + suffix, 56, ln, K.wire("mod.rs:%s:value_wire" % t), exp)
    for t in ("test_mac_address_value", "test_pkg_record_value", "test_record_value")
    for suffix, ln, exp in (
        ("", 6, bytes([0x12, 0xc6, 0x21, 0x12, 0x69, 0x32])),
        ("_invalid_length", 2, {"InvalidLength": {"offset": 0, "ie_name": "sourceMacAddress", "length": 2}}))
] + [
    # mod.rs:159-185 test_ipv4_address_value: sourceIPv4Address 70.1.115.1; length 2 is InvalidLength
    ("ipv4_address_value", 8, 4, K.wire("mod.rs:test_ipv4_address_value:good_wire"), ("v4", 0x46017301)),
    ("ipv4_address_invalid_length", 8, 2, K.wire("mod.rs:test_ipv4_address_value:good_wire"),
     {"InvalidLength": {"offset": 0, "ie_name": "sourceIPv4Address", "length": 2}}),
    # mod.rs:297-314 test_string_value: interfaceName declared 16 bytes, "lo" + 14 NULs -> "lo"
    # (a fixed-length string is cut at its first NUL, generator.rs:1635-1672)
    ("string_fixed_nul_truncated", 82, 16, K.wire("mod.rs:test_string_value:good_wire"), "lo"),
]
