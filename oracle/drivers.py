"""CPU ORACLE drivers — test infrastructure only.

Restatements of the reference's two pcap -> JSON test drivers on top of
ngz_oracle:
  * crates/flow-pkt/src/wire/tests/pcap_tests.rs:79-118 (per 5-tuple codec and
    buffer; decode until incomplete; errors serialized, buffer NOT cleared)
  * crates/pcap-decoder/src/handlers/{flow.rs:37-59, mod.rs:36-60,64-80}
    (same, but the buffer is cleared on error, and each success line is
    {"source_address", "destination_address", "info"}).
"""
import ngz_oracle as O


def run_pcap_tests_driver(dgrams):
    peers = {}
    lines = []
    for src, sp, dst, dp, payload in dgrams:
        key = (src, sp, dst, dp)
        if key not in peers:
            peers[key] = (O.FlowInfoCodec(), bytearray())
        codec, buf = peers[key]
        buf += payload
        while len(buf):
            try:
                msg = codec.decode(buf)
            except O.ParseFail as e:
                lines.append(O.dumps(e.err))
                continue
            if msg is None:
                break
            lines.append(O.dumps(msg.to_json()))
    return lines


def run_pcap_decoder_driver(dgrams):
    peers = {}
    lines = []
    for src, sp, dst, dp, payload in dgrams:
        key = (src, sp, dst, dp)
        if key not in peers:
            peers[key] = (O.FlowInfoCodec(), bytearray())
        codec, buf = peers[key]
        buf += payload
        while len(buf):
            try:
                msg = codec.decode(buf)
            except O.ParseFail as e:
                del buf[:]
                lines.append(O.dumps(e.err))
                continue
            if msg is None:
                break
            lines.append(O.dumps({"source_address": O.socket_addr_str(src, sp),
                                  "destination_address": O.socket_addr_str(dst, dp),
                                  "info": msg.to_json()}))
    return lines
