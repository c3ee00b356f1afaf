"""The committed IE registry (netgauze_amd/data/ie_registry.json, shared by the
product and the oracle) checked against the reference's registry XML with an
independent reading: a registry error would otherwise be common-mode and
invisible to oracle-vs-device tests.  For every vendor file
(crates/flow-pkt/registry/*.xml, build.rs:137-255) the set of (id, name, data
type, dataTypeSemantics) of the records the code generator keeps
(xml_parsers/ipfix.rs:141-291: a name that is not "Unassigned" / "Reserved" /
the NetFlow v9 placeholder, a data type, a u16 element id, a status, a
description, a u32 revision and a date; samplerId and forwardingStatus forced to
unsigned32) must equal the committed table's.  Skipped where the reference
checkout is absent."""
import json
import os
import re
import xml.etree.ElementTree as ET

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REG = "/root/reference/crates/flow-pkt/registry"
NS = "{http://www.iana.org/assignments}"
FILES = {0: "iana_ipfix_information_elements.xml", 637: "nokia.xml", 2011: "huawei.xml", 3746: "netgauze.xml",
         6876: "vmware.xml"}


def text(rec, tag):
    for c in rec:
        if c.tag == NS + tag:
            return None if c.text is None else c.text.strip()
    return None


def has(rec, tag):
    return any(c.tag == NS + tag for c in rec)


def records(path):
    root = ET.parse(path).getroot()
    reg = next(n for n in root.iter() if n.attrib.get("id") == "ipfix-information-elements")
    out = set()
    for rec in reg:
        if rec.tag != NS + "record":
            continue
        name, dt, eid, rev = text(rec, "name"), text(rec, "dataType"), text(rec, "elementId"), text(rec, "revision")
        if name is None or name in ("Unassigned", "Reserved", "Assigned for NetFlow v9 compatibility"):
            continue
        if dt is None or eid is None or not re.fullmatch(r"\+?\d+", eid) or int(eid) > 0xFFFF:
            continue
        if text(rec, "status") is None or not has(rec, "description") or text(rec, "date") is None:
            continue
        if rev is None or not re.fullmatch(r"\+?\d+", rev) or int(rev) > 0xFFFFFFFF:
            continue
        if name == "samplerId" or name.lower() == "forwardingstatus":
            dt = "unsigned32"
        out.add((int(eid), name, dt, text(rec, "dataTypeSemantics")))
    return out


@pytest.mark.skipif(not os.path.isdir(REG), reason="reference registry XML not present")
def test_registry_matches_reference_xml():
    with open(os.path.join(ROOT, "netgauze_amd", "data", "ie_registry.json")) as f:
        reg = json.load(f)
    for pen, fname in FILES.items():
        committed = {(r["id"], r["name"], r["type"], r.get("semantics")) for r in reg["ies"] if r["pen"] == pen}
        assert committed == records(os.path.join(REG, fname)), fname
    assert {v["pen"]: v["count"] for v in reg["vendors"]} == {
        pen: sum(1 for r in reg["ies"] if r["pen"] == pen) for pen in FILES if pen}


def test_ie_table_matches_registry_json():
    """The C table compiled into libngz (ie_table.inc) carries the same rows and data types."""
    with open(os.path.join(ROOT, "netgauze_amd", "data", "ie_registry.json")) as f:
        reg = json.load(f)
    types = reg["data_types"]
    rows = set()
    for m in re.finditer(r'NGZ_IE\((\d+)u, (\d+)u, (\d+), (\d+), "([^"]*)"\)',
                         open(os.path.join(ROOT, "netgauze_amd", "csrc", "ie_table.inc")).read()):
        pen, ie, dt, flags, name = int(m[1]), int(m[2]), int(m[3]), int(m[4]), m[5]
        sem = "identifier" if flags & 8 else ("flags" if flags & 16 else None)
        rows.add((pen, ie, types[dt], name, sem, bool(flags & 4)))
    exp = {(r["pen"], r["id"], r["type"], r["name"],
            r.get("semantics") if r.get("semantics") in ("identifier", "flags") else None, r["subreg"] is not None)
           for r in reg["ies"]}
    assert rows == exp
