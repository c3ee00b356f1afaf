"""Write the generated per-template decode kernel of a synthetic template to a
.hip file (for offline hipcc resource-usage / ISA inspection):
python tools/rtc_dump.py t20|v900|nf313 /tmp/rtc/t20.hip"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from netgauze_amd import _lib, synth  # noqa: E402


def template_record(name):
    if name == "t20":
        return synth.template_message()[20:]
    if name == "v900":
        return synth._ipfix_template_v900()[20:]
    if name == "nf313":
        return synth.nfv9_template_message()[24:]
    raise SystemExit("unknown template " + name)


def main():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    rec = template_record(sys.argv[1])
    buf = ctypes.create_string_buffer(1 << 20)
    rc = lib.ngz_template_kernel(rec, len(rec), 2 if sys.argv[1].startswith("nf") else 0, buf, len(buf))
    assert rc == 0, rc
    open(sys.argv[2], "w").write("#include <hip/hip_runtime.h>\n" + buf.value.decode())


if __name__ == "__main__":
    main()
