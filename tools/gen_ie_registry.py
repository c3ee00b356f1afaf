#!/usr/bin/env python3
"""Generate the Information Element registry tables used by netgauze_amd.

Offline tool, run in the build container where /root/reference exists.  It
restates the reference's build-time code generator rules so that the
(pen, id) -> (name, data type, sub-registry) mapping is identical:

* IE record filter rules:
  crates/ipfix-code-generator/src/xml_parsers/ipfix.rs:141-291
  (skip "Assigned for NetFlow v9 compatibility" / "Unassigned" / "Reserved",
  missing dataType / elementId(u16) / status / description / revision(u32) /
  date; samplerId and forwardingStatus forced to unsigned32).
* sub-registry discovery: xml_parsers/ipfix.rs:62-100 (children of the IE
  registry whose id contains "ipfix-", classification-engine-ids,
  forwarding-status as a 2-bit reason-code nested registry) plus the external
  sub-registries configured in crates/flow-pkt/build.rs:32-132 (flowDirection
  61, protocol numbers 4, segment routing 502, psamp 304; VMware 954/880).
* sub-registry record rules: xml_parsers/sub_registries.rs:118-256 and the
  enum-name derivation xml_common.rs:122-177.
* vendors: build.rs:137-255 (nokia 637, huawei 2011, netgauze 3746,
  vmware 6876), in the order of build.rs:271.

Outputs (committed, since /root/reference does not travel to the GPU box):
  netgauze_amd/data/ie_registry.json   full registry incl. sub-registry names
  netgauze_amd/csrc/ie_table.inc       C table (pen, id, data type, flags)
"""
import json
import os
import re
import sys
import xml.etree.ElementTree as ET

NS = "{http://www.iana.org/assignments}"
REG = "/root/reference/crates/flow-pkt/registry"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

DATA_TYPES = [
    "octetArray", "unsigned8", "unsigned16", "unsigned32", "unsigned64",
    "signed8", "signed16", "signed32", "signed64", "float32", "float64",
    "boolean", "macAddress", "string", "dateTimeSeconds",
    "dateTimeMilliseconds", "dateTimeMicroseconds", "dateTimeNanoseconds",
    "ipv4Address", "ipv6Address", "basicList", "subTemplateList",
    "subTemplateMultiList", "unsigned256",
]  # crates/flow-pkt/src/ie.rs:14-110 (repr(u8) order)


def child_text(node, tag):
    """roxmltree get_string_child: first child with the tag, its text trimmed,
    None if the child is absent or has no text (xml_common.rs:86-92)."""
    for c in node:
        if c.tag == NS + tag:
            if c.text is None:
                return None
            return c.text.strip()
    return None


def has_child(node, tag):
    return any(c.tag == NS + tag for c in node)


def find_by_id(node, ident):
    for n in node.iter():
        if n.attrib.get("id") == ident:
            return n
    return None


def rfc_link(text):
    text = re.sub(r"\[RFC(\d+)]", lambda m: "[RFC%s](https://datatracker.ietf.org/doc/rfc%s)" % (m.group(1), m.group(1)), text, count=1)
    return text


def http_link(text):
    pat = r"(https?://(www\.)?[-a-zA-Z0-9@:%._\+~#=]{2,256}\.[a-z]{2,4}\b([-a-zA-Z0-9@:%_\+.~#?&//=]*))"
    return re.sub(pat, lambda m: "<" + m.group(1) + ">", text, count=1)


def simple_description(node):
    """xml_common.rs:179-195 parse_simple_description_string."""
    for c in node:
        if c.tag == NS + "description":
            body = c.text.strip() if c.text is not None else None
            desc = body if body else ""
            desc = rfc_link(desc)
            desc = http_link(desc)
            return desc
    return None


PUNCT = set("!\"#$%&'()*+,-./:;<=>?@[\\]^_`{|}~")
DIGIT_WORD = {"0": "Zero", "1": "One", "2": "Two", "3": "Three", "4": "Four",
              "5": "Five", "6": "Six", "7": "Seven", "8": "Eight", "9": "Nine"}


def to_enum_type(s):
    """xml_common.rs:122-177 xml_string_to_enum_type -> (words, name)."""
    one = " ".join(line.strip() for line in s.splitlines())
    before = one.split(":")[0].strip()
    words = len(before.split())
    out = "".join(ch for ch in before if not ch.isspace() and ch not in PUNCT)
    if out and out[0].isnumeric():
        out = DIGIT_WORD.get(out[0], out[0]) + out[1:]
    return words, out


def parse_u8(x):
    try:
        if x.startswith("0x"):
            v = int(x[2:], 16)
        elif x.startswith("0b"):
            v = int(x[2:], 2)
        elif x.endswith("b"):
            v = int(x[:-1], 2)
        else:
            if not re.fullmatch(r"\+?\d+", x):
                return None
            v = int(x)
    except ValueError:
        return None
    if v > 255:
        return None
    return v


def parse_vnd(node):
    """sub_registries.rs:118-234 parse_val_name_desc_u8_registry."""
    title = child_text(node, "title") or ""
    m = re.search(r"Value (\d+)", title)
    ie_id = int(m.group(1)) if m else 0
    if ie_id > 65535:
        ie_id = 0
    out = []
    for rec in node:
        if rec.tag != NS + "record":
            continue
        vtxt = child_text(rec, "value")
        if has_child(rec, "value"):
            value = parse_u8(vtxt) if vtxt is not None else None
            value_present = True
        else:
            value_present = False
            value = None
        if not value_present:
            itxt = child_text(rec, "id")
            if has_child(rec, "id"):
                value_present = True
                value = parse_u8(itxt) if itxt is not None else None
        # get_string_child returns None when the child element has no text
        if vtxt is None and has_child(rec, "value"):
            value_present = False
            itxt = child_text(rec, "id")
            if itxt is not None:
                value_present = True
                value = parse_u8(itxt)
        name_parsed = child_text(rec, "name")
        if name_parsed is not None and (name_parsed == "Unassigned" or "experimentation" in name_parsed):
            continue
        desc = simple_description(rec)
        if desc is not None and (desc == "Unassigned" or "experimentation" in desc):
            continue
        if not value_present or value is None:
            continue
        if value == 255:
            continue
        if name_parsed is not None:
            display = name_parsed
            _, name = to_enum_type(name_parsed)
        elif desc is not None:
            words, dname = to_enum_type(desc)
            if words < 10:
                name = dname
            else:
                name = "Value%d" % value
        else:
            continue
        if name in ("Reserved", "Private"):
            name = "%s%d" % (name, value)
        out.append([value, name])
    return ie_id, out


def parse_nested(node):
    """sub_registries.rs:236-292 parse_reason_code_nested_u8_registry_2bit."""
    ie_id, sub = parse_vnd(node)
    out = []
    for value, name in sub:
        pat = re.compile(r".*-%sb" % format(value, "02b"))
        target = None
        for c in node:
            cid = c.attrib.get("id")
            if cid is not None and pat.match(cid):
                target = c
                break
        _, reasons = parse_vnd(target)
        out.append([(value << 6) & 0xFF, name, reasons])
    return ie_id, out


def parse_ie_subregistries(ie_node):
    subs = {}
    for c in ie_node:
        cid = c.attrib.get("id")
        if cid is not None and "ipfix-" in cid:
            i, r = parse_vnd(c)
            subs[i] = {"kind": "vnd", "entries": r}
    ce = find_by_id(ie_node, "classification-engine-ids")
    if ce is not None:
        i, r = parse_vnd(ce)
        subs[i] = {"kind": "vnd", "entries": r}
    fw = find_by_id(ie_node, "forwarding-status")
    if fw is not None:
        i, r = parse_nested(fw)
        subs[i] = {"kind": "nested", "entries": r}
    return subs


def parse_ies(ie_node, pen, ext):
    subs = parse_ie_subregistries(ie_node)
    subs.update(ext)
    out = []
    for rec in ie_node:
        if rec.tag != NS + "record":
            continue
        name = child_text(rec, "name")
        if name is None:
            continue
        if name in ("Assigned for NetFlow v9 compatibility", "Unassigned", "Reserved"):
            continue
        dt = child_text(rec, "dataType")
        if dt is None:
            continue
        if name == "samplerId" or name.lower() == "forwardingstatus":
            dt = "unsigned32"
        eid = child_text(rec, "elementId")
        if eid is None or not re.fullmatch(r"\+?\d+", eid) or int(eid) > 65535:
            continue
        eid = int(eid)
        if child_text(rec, "status") is None:
            continue
        if not has_child(rec, "description"):
            continue
        rev = child_text(rec, "revision")
        if rev is None or not re.fullmatch(r"\+?\d+", rev) or int(rev) > 0xFFFFFFFF:
            continue
        if child_text(rec, "date") is None:
            continue
        # dataTypeSemantics (xml_parsers/ipfix.rs:194-195): identifier / flags IEs do not
        # support arithmetic (generator.rs:584-589, IE::supports_arithmetic_ops :1176-1180)
        out.append({"pen": pen, "id": eid, "name": name, "type": dt,
                    "semantics": child_text(rec, "dataTypeSemantics"), "subreg": subs.get(eid)})
    return out


def ext_subreg(path, reg_id, kind="vnd"):
    root = ET.parse(path).getroot()
    node = find_by_id(root, reg_id)
    if kind == "vnd":
        return {"kind": "vnd", "entries": parse_vnd(node)[1]}
    return {"kind": "nested", "entries": parse_nested(node)[1]}


def main():
    sub = os.path.join(REG, "subregistry")
    iana_ext = {
        61: ext_subreg(os.path.join(sub, "iana_flow_direction.xml"), "ipfix-flow-direction"),
        4: ext_subreg(os.path.join(sub, "iana_protocol_numbers.xml"), "protocol-numbers-1"),
        502: ext_subreg(os.path.join(sub, "iana_segment_routing.xml"), "srv6-endpoint-behaviors"),
        304: ext_subreg(os.path.join(sub, "iana_psamp_parameters.xml"), "psamp-parameters-1"),
    }
    root = ET.parse(os.path.join(REG, "iana_ipfix_information_elements.xml")).getroot()
    iana = parse_ies(find_by_id(root, "ipfix-information-elements"), 0, iana_ext)
    vendors = []
    all_ies = list(iana)
    vendor_cfg = [
        ("Nokia", "nokia", 637, "nokia.xml", {}),
        ("Huawei", "huawei", 2011, "huawei.xml", {}),
        ("NetGauze", "netgauze", 3746, "netgauze.xml", {}),
        ("VMWare", "vmware", 6876, "vmware.xml", {
            954: ext_subreg(os.path.join(sub, "iana_flow_direction.xml"), "ipfix-flow-direction"),
            880: ext_subreg(os.path.join(sub, "iana_protocol_numbers.xml"), "protocol-numbers-1"),
        }),
    ]
    for name, mod, pen, fname, ext in vendor_cfg:
        vroot = ET.parse(os.path.join(REG, fname)).getroot()
        ies = parse_ies(find_by_id(vroot, "ipfix-information-elements"), pen, ext)
        vendors.append({"name": name, "mod": mod, "pen": pen, "count": len(ies)})
        all_ies.extend(ies)
    for ie in all_ies:
        if ie["type"] not in DATA_TYPES:
            raise SystemExit("unknown data type %r" % ie["type"])
    data = {
        "generator": "tools/gen_ie_registry.py",
        "source": "crates/flow-pkt/registry/*.xml (NetGauze v0.13.0)",
        "data_types": DATA_TYPES,
        "vendors": vendors,
        "ies": all_ies,
    }
    out_json = os.path.join(REPO, "netgauze_amd", "data", "ie_registry.json")
    with open(out_json, "w") as f:
        json.dump(data, f, indent=0, sort_keys=True)
        f.write("\n")
    write_c_table(all_ies, vendors, os.path.join(REPO, "netgauze_amd", "csrc", "ie_table.inc"))
    print("IANA %d, vendors %s" % (len(iana), [(v["name"], v["count"]) for v in vendors]))


def write_c_table(ies, vendors, path):
    lines = [
        "/* GENERATED by tools/gen_ie_registry.py from the reference IE registry XML.",
        " * Do not edit. One row per registered IE: {pen, id, data type, flags, name}.",
        " * flags: bit0 MPLS label ([u8;3], generator.rs:2753-2755),",
        " *        bit1 tcpControlBits (TCPHeaderFlags::from truncates to u8, iana/src/tcp.rs:165-168),",
        " *        bit2 has sub-registry (lossless enum wrap, generator_sub_registries.rs:215-247),",
        " *        bit3 dataTypeSemantics identifier, bit4 dataTypeSemantics flags (generator.rs:584-589). */",
    ]
    for ie in ies:
        flags = 0
        if ie["name"] == "mplsTopLabelStackSection" or ie["name"].startswith("mplsLabelStackSection"):
            flags |= 1
        if ie["name"] == "tcpControlBits" and ie["pen"] == 0:
            flags |= 2
        if ie["subreg"] is not None:
            flags |= 4
        if ie.get("semantics") == "identifier":
            flags |= 8
        if ie.get("semantics") == "flags":
            flags |= 16
        lines.append('NGZ_IE(%du, %du, %d, %d, "%s")' % (ie["pen"], ie["id"], DATA_TYPES.index(ie["type"]), flags, ie["name"]))
    lines.append("")
    lines.append("/* vendor PENs with their own IE package (build.rs:271); other PENs decode as IE::Unknown. */")
    for v in vendors:
        lines.append('NGZ_VENDOR(%du, "%s")' % (v["pen"], v["name"]))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
