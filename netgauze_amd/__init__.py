"""netgauze_amd — MI355X-native IPFIX / NetFlow v9 data-record decoder.

A drop-in for the data-record decode path of NetGauze's netgauze-flow-pkt
(crates/flow-pkt/src/wire/deserializer/), re-built for gfx950: the C ABI in
include/ngz/flow_decode.h (libngz.so, hand-written HIP kernels) with a Python
mirror of FlowInfoCodec in netgauze_amd.flow.
"""
from ._lib import LIB_PATH  # noqa: F401

__all__ = ["FlowInfoCodec", "LIB_PATH"]


def __getattr__(name):
    if name == "FlowInfoCodec":
        from .flow import FlowInfoCodec
        return FlowInfoCodec
    raise AttributeError(name)
