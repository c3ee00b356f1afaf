"""Identity of the product build: a SHA-256 over the sources libngz.so is built
from.  Profiles committed under profiles/ carry it (tools/summarize_profile.py),
and bench.py reports a committed PMC traffic figure only when the profile was
taken of this exact source tree (the GPU box gets the tree without .git, so a
git sha cannot be checked there; the source hash can)."""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_PATTERNS = ("netgauze_amd/csrc/*.hip", "netgauze_amd/csrc/*.cpp", "netgauze_amd/csrc/*.h",
             "netgauze_amd/csrc/ie_table.inc", "netgauze_amd/csrc/subreg_table.inc", "include/ngz/*.h")


def source_hash():
    h = hashlib.sha256()
    files = sorted({f for p in _PATTERNS for f in glob.glob(os.path.join(ROOT, p))})
    for f in files:
        h.update(os.path.relpath(f, ROOT).encode())
        with open(f, "rb") as fh:
            h.update(hashlib.sha256(fh.read()).digest())
    return h.hexdigest()[:16]
