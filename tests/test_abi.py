"""CPU checks of the C-ABI library: it is built, it loads, and it exports
every function include/ngz/flow_decode.h declares (no compute calls here)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", "ngz", h) for h in ("flow_decode.h", "flow_ingest.h",
                                                                        "flow_aggregate.h")]


def declared_functions(headers=HEADERS):
    names = set()
    for h in headers:
        text = open(h).read()
        names |= set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(ngz_[a-z_0-9]+)\s*\(", text, re.M))
    return sorted(names)


def test_header_declares_abi():
    from netgauze_amd import _lib
    assert declared_functions(HEADERS[:1]) == sorted(_lib.ABI_FUNCTIONS)
    assert declared_functions(HEADERS[1:2]) == sorted(_lib.INGEST_FUNCTIONS)
    assert declared_functions(HEADERS[2:]) == sorted(_lib.AGG_FUNCTIONS)


def test_abi_versions_match_headers():
    """The library reports the NGZ_ABI_VERSION / NGZ_AGG_ABI_VERSION of the headers it was built
    from, and the binding refuses any other (a host built against an older flow_aggregate.h would
    pass a port where ngz_agg_push takes a const ngz_peer *)."""
    from netgauze_amd import _lib
    lib = _lib.load()
    hdr = {m.group(1): int(m.group(2)) for h in HEADERS for m in
           re.finditer(r"#define (NGZ_(?:AGG_)?ABI_VERSION) (\d+)", open(h).read())}
    assert hdr == {"NGZ_ABI_VERSION": _lib.NGZ_ABI_VERSION, "NGZ_AGG_ABI_VERSION": _lib.NGZ_AGG_ABI_VERSION}
    assert (lib.ngz_abi_version(), lib.ngz_agg_abi_version()) == (_lib.NGZ_ABI_VERSION, _lib.NGZ_AGG_ABI_VERSION)


def test_agg_config_validation_without_device():
    """AggregationConfig::validate / validate_operation_compatibility are checked before any
    device call (config.rs:107-119, 212-250) with IE::supports_{arithmetic,comparison,bitwise}_ops
    (generator.rs:1176-1272): the reference's accept / reject table, row by row.  Accepted
    configs go on to the device (no GPU here: NGZ_E_DEVICE / NGZ_E_NOMEM); rejected ones
    return NGZ_E_INVALID.  Every accepted config runs on the device: Min / Max over lists
    (Box<[u8]> order) and over forwardingStatus's nested reason codes, octet-array ORs and
    string / octet / list keys of any length included (no NGZ_E_LIMIT row is left)."""
    from netgauze_amd import _lib
    lib = _lib.load()
    A = _lib.AggField

    def create(fields, window=60000, lateness=10000):
        arr = (A * max(len(fields), 1))(*[A(p, i, x, o) for p, i, x, o in fields])
        h = ctypes.c_void_p()
        return lib.ngz_agg_create(0, arr, len(fields), window, lateness, 1024, 0, ctypes.byref(h))
    ok = [(0, 8, 0, _lib.NGZ_AGG_KEY), (0, 1, 0, _lib.NGZ_AGG_ADD)]
    assert create(ok, window=0) == -1
    assert create(ok, window=1000, lateness=2000) == -1
    assert create([(0, 1, 0, 9)]) == -1                       # unknown op
    ADD, MIN, MAX, OR = _lib.NGZ_AGG_ADD, _lib.NGZ_AGG_MIN, _lib.NGZ_AGG_MAX, _lib.NGZ_AGG_OR
    ACCEPT, REJECT, LIMIT = "accept", "reject", "limit"
    table = [
        # (IE, op, reference verdict): arithmetic = numeric type, no sub-registry, not identifier / flags
        ((0, 1), ADD, ACCEPT),      # octetDeltaCount unsigned64 deltaCounter
        ((0, 434), ADD, ACCEPT),    # mibObjectValueInteger signed32
        ((0, 311), ADD, ACCEPT),    # samplingProbability float64
        ((0, 10), ADD, REJECT),     # ingressInterface: identifier semantics
        ((0, 6), ADD, REJECT),      # tcpControlBits: flags semantics
        ((0, 4), ADD, REJECT),      # protocolIdentifier: sub-registry
        ((0, 8), ADD, REJECT),      # sourceIPv4Address
        ((0, 56), ADD, REJECT),     # sourceMacAddress
        ((0, 515), ADD, REJECT),    # unsigned256
        ((0, 150), ADD, REJECT),    # dateTimeSeconds
        # comparison: by data type only
        ((0, 311), MIN, ACCEPT),    # float64
        ((0, 27), MAX, ACCEPT),     # ipv6Address
        ((0, 8), MIN, ACCEPT),      # ipv4Address
        ((0, 150), MAX, ACCEPT),    # dateTimeSeconds
        ((0, 152), MIN, ACCEPT),    # dateTimeMilliseconds
        ((0, 154), MAX, ACCEPT),    # dateTimeMicroseconds
        ((0, 156), MIN, ACCEPT),    # dateTimeNanoseconds
        ((0, 4), MAX, ACCEPT),      # protocolIdentifier: sub-registry enum order
        ((0, 6), MIN, ACCEPT),      # tcpControlBits: TCPHeaderFlags order
        ((0, 10), MAX, ACCEPT),     # identifier semantics do not matter for comparison
        ((0, 56), MIN, REJECT),     # macAddress
        ((0, 276), MAX, REJECT),    # boolean
        ((0, 82), MIN, REJECT),     # string
        ((0, 70), MAX, REJECT),     # octetArray
        ((0, 515), MIN, REJECT),    # unsigned256
        ((0, 291), MIN, ACCEPT),    # basicList: Box<[u8]> lexicographic order
        ((0, 292), MAX, ACCEPT),    # subTemplateList
        ((0, 293), MIN, ACCEPT),    # subTemplateMultiList
        ((0, 89), MAX, ACCEPT),     # forwardingStatus: nested reason-code sub-registry order
        # bitwise
        ((0, 6), OR, ACCEPT),       # tcpControlBits
        ((0, 4), OR, ACCEPT),       # protocolIdentifier: BitOrAssign of the raw values
        ((0, 56), OR, ACCEPT),      # macAddress
        ((0, 27), OR, ACCEPT),      # ipv6Address
        ((0, 276), OR, ACCEPT),     # boolean
        ((0, 515), OR, ACCEPT),     # unsigned256
        ((0, 70), OR, ACCEPT),      # mplsTopLabelStackSection: [u8; 3]
        ((0, 210), OR, ACCEPT),     # paddingOctets: octetArray of any length
        ((0, 311), OR, REJECT),     # float64
        ((0, 82), OR, REJECT),      # string
        ((0, 150), OR, REJECT),     # dateTimeSeconds
        ((0, 292), OR, REJECT),     # subTemplateList
    ]
    # key fields of every kind are accepted: strings, octet arrays, lists, unknown IEs
    for key in [(0, 82), (0, 236), (0, 210), (0, 291), (2011, 1000), (213, 5)]:
        assert create([key + (0, _lib.NGZ_AGG_KEY), (0, 1, 0, ADD)]) in (-2, -3, 0), key
    assert LIMIT not in {v for _, _, v in table}
    for (pen, ie), op, verdict in table:
        rc = create([(pen, ie, 0, op)])
        if verdict == ACCEPT:
            assert rc in (-2, -3) or rc == 0, ((pen, ie), op, rc)
        elif verdict == REJECT:
            assert rc == -1, ((pen, ie), op, rc)
        else:
            assert rc == -4, ((pen, ie), op, rc)


def test_agg_config_follows_reference_supports_kats():
    """The IE::supports_{arithmetic,bitwise,comparison}_ops asserts of lib.rs:267-358
    (tests/kats_agg.py SUPPORTS_KATS) through ngz_agg_create's validation: an op the reference
    supports is accepted (the call goes on to the device: no GPU here), one it does not is
    NGZ_E_INVALID."""
    import json
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import kats_agg as K
    from netgauze_amd import _lib
    lib = _lib.load()
    reg = json.load(open(os.path.join(ROOT, "netgauze_amd", "data", "ie_registry.json")))
    ids = {r["name"]: r["id"] for r in reg["ies"] if r["pen"] == 0}
    for name, (arith, bit, cmp_) in K.SUPPORTS_KATS.items():
        for op, want in ((_lib.NGZ_AGG_ADD, arith), (_lib.NGZ_AGG_OR, bit), (_lib.NGZ_AGG_MIN, cmp_),
                         (_lib.NGZ_AGG_MAX, cmp_)):
            if want is None:
                continue
            arr = (_lib.AggField * 1)(_lib.AggField(0, ids[name], 0, op))
            h = ctypes.c_void_p()
            rc = lib.ngz_agg_create(0, arr, 1, 60000, 10000, 1024, 0, ctypes.byref(h))
            assert (rc != -1) == want, (name, op, rc)

def test_library_exports_every_declared_symbol():
    from netgauze_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.fail("libngz.so not built: run __graft_entry__.build()")
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_functions():
        assert hasattr(lib, name), name
    _lib.load()


def test_ctx_create_without_device_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    from netgauze_amd import _lib
    lib = _lib.load()
    ctx = ctypes.c_void_p()
    assert lib.ngz_ctx_create(0, ctypes.byref(ctx)) != 0
    assert not ctx.value


def test_column_copies_reject_bad_arguments_without_device():
    """ngz_columns_to_host / _async: a null context, a null destination with room, or an unknown
    flag is NGZ_E_INVALID before any device call."""
    from netgauze_amd import _lib
    lib = _lib.load()
    buf = ctypes.create_string_buffer(64)
    assert lib.ngz_columns_to_host(None, buf, 64) == -1
    assert lib.ngz_columns_to_host_async(None, buf, 64, None, 0) == -1
    assert lib.ngz_columns_to_host_async(None, None, 64, None, 1) == -1
    assert lib.ngz_columns_to_host_async(None, buf, 64, None, 2) == -1


def test_product_does_not_import_oracle():
    """The product path never routes through the CPU oracle."""
    pkg = os.path.join(ROOT, "netgauze_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                text = open(os.path.join(dirpath, f), errors="ignore").read()
                assert "ngz_oracle" not in text and "oracle/" not in text, f


@pytest.mark.parametrize("tid", [t for t, _ in __import__("netgauze_amd.synth", fromlist=["x"]).CFG5_TEMPLATES])
def test_template_kernels_compile_for_gfx950(tid):
    """The per-template decode kernel of every config-5 template (config 3 and
    its width permutations) is generated
    and compiled for gfx950 by hiprtc (no device needed): LDS-staged where the
    rows fit the workgroup budget, direct column stores otherwise."""
    import struct
    from netgauze_amd import _lib, synth
    fields = dict(synth.CFG5_TEMPLATES)[tid]
    rec = struct.pack(">HH", tid, len(fields)) + b"".join(struct.pack(">HH", i, ln) for i, ln in fields)
    lib = ctypes.CDLL(_lib.LIB_PATH)
    buf = ctypes.create_string_buffer(1 << 20)
    rc = lib.ngz_template_kernel(rec, len(rec), 1, buf, len(buf))
    src = buf.value.decode()
    assert rc == 0, src[-2000:]
    assert "ngz_tpl" in src
    assert ("run_lds" in src) == ("NGZ_LDS_WAVES" in src)


@pytest.mark.parametrize("workload", ["cfg3", "cfg5"])
def test_group_kernels_compile_for_gfx950(workload):
    """The multi-template decode kernel (one launch for the LDS-staged templates of a batch that
    share a workgroup shape, ngz_rtc.cpp generate_group) of every such group of config 3 / 5 is
    generated and compiled for gfx950 by hiprtc; each template keeps its own constant-offset
    body."""
    import re
    import struct
    from netgauze_amd import _lib, synth
    tpls = synth.CFG3_TEMPLATES if workload == "cfg3" else synth.CFG5_TEMPLATES
    lib = ctypes.CDLL(_lib.LIB_PATH)
    buf = ctypes.create_string_buffer(4 << 20)
    groups = {}
    for tid, fields in tpls:
        rec = struct.pack(">HH", tid, len(fields)) + b"".join(struct.pack(">HH", i, ln) for i, ln in fields)
        assert lib.ngz_template_kernel(rec, len(rec), 0, buf, len(buf)) == 0
        lw = int(re.search(r"NGZ_LDS_WAVES (\d+)", buf.value.decode()).group(1))
        groups.setdefault(lw, []).append(rec)
    assert sum(len(g) for g in groups.values()) == len(tpls)
    for lw, recs in groups.items():
        body = b"".join(recs)
        rc = lib.ngz_group_kernel(body, len(body), 1, buf, len(buf))
        src = buf.value.decode()
        assert rc == 0, src[-2000:]
        assert "ngz_tplm" in src and src.count("::run(B, S.s[") == len(recs)
        assert "__launch_bounds__(%d)" % (64 * lw) in src
    one = struct.pack(">HH", 256, len(synth.T20)) + b"".join(struct.pack(">HH", i, ln) for i, ln in synth.T20)
    assert lib.ngz_group_kernel(one, len(one), 0, buf, len(buf)) == -1  # a group has at least two templates
