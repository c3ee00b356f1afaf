"""Identity of the product build: SHA-256 digests over the sources libngz.so is
built from.  Profiles committed under profiles/ carry them
(tools/summarize_profile.py), and bench.py reports a committed PMC traffic
figure only when the profile was taken of the same decode sources (the GPU box
gets the tree without .git, so a git sha cannot be checked there; the source
hash can).

source_hash() covers every library source.  decode_source_hash() covers the
sources the decode step is built from (the kernels and host pipeline of
ngz_decode_batch, the run-time kernel generator and its device headers, the IE
table and the decode ABI): a change to aggregation, JSON or capture code does
not change a decode kernel's HBM traffic, and does not void its profile.
agg_source_hash() covers the aggregation kernels' sources the same way."""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_PATTERNS = ("netgauze_amd/csrc/*.hip", "netgauze_amd/csrc/*.cpp", "netgauze_amd/csrc/*.h",
             "netgauze_amd/csrc/ie_table.inc", "netgauze_amd/csrc/subreg_table.inc", "include/ngz/*.h")
_DECODE = ("netgauze_amd/csrc/ngz_kernels.hip", "netgauze_amd/csrc/ngz_host.cpp", "netgauze_amd/csrc/ngz_host.h",
           "netgauze_amd/csrc/ngz_rtc.cpp", "netgauze_amd/csrc/ngz_dev.h", "netgauze_amd/csrc/ngz_internal.h",
           "netgauze_amd/csrc/ie_table.inc", "include/ngz/flow_decode.h")


def _digest(patterns):
    h = hashlib.sha256()
    files = sorted({f for p in patterns for f in glob.glob(os.path.join(ROOT, p))})
    for f in files:
        h.update(os.path.relpath(f, ROOT).encode())
        with open(f, "rb") as fh:
            h.update(hashlib.sha256(fh.read()).digest())
    return h.hexdigest()[:16]


_AGG = ("netgauze_amd/csrc/ngz_agg.hip", "netgauze_amd/csrc/ngz_host.h", "netgauze_amd/csrc/ngz_internal.h",
        "include/ngz/flow_aggregate.h", "include/ngz/flow_decode.h", "netgauze_amd/csrc/ie_table.inc")


def source_hash():
    return _digest(_PATTERNS)


def decode_source_hash():
    return _digest(_DECODE)


def agg_source_hash():
    """The aggregation kernels' sources (ngz_agg.hip and the headers it includes)."""
    return _digest(_AGG)
