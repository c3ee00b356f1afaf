"""INTEGRATION.md's Rust binding against include/ngz/*.h (CPU, no device).

The reference-side FFI a netgauze-flow-pkt maintainer would add is
text: no Rust toolchain is in this image to compile it.  This test keeps it from drifting
from the headers, which is what it must bind (the reference surface it stands in for is
`impl Decoder for FlowInfoCodec`, crates/flow-pkt/src/codec.rs:189-220):

- every `extern "C"` function of the ```rust blocks exists in a header with the same
  parameter count and the same parameter and return types (C types mapped to their Rust
  FFI spelling), and every header function is bound;
- every non-opaque struct typedef of the headers has a `#[repr(C)]` mirror with the same
  field names in the same order and the same field types, and the repr(C) layout the Rust
  declaration implies (sizes and offsets computed here) equals the C layout reported by a
  small `offsetof` probe compiled with gcc; opaque handles are zero-sized;
- every integer `#define NGZ_*` of the headers is a `pub const` of the same value, and the
  safe wrapper checks the ABI versions against those constants, not against literals.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR_DIR = os.path.join(ROOT, "include", "ngz")
HEADERS = [os.path.join(HDR_DIR, h) for h in ("flow_decode.h", "flow_ingest.h", "flow_aggregate.h")]
DOC = os.path.join(ROOT, "INTEGRATION.md")

C_SCALARS = {"int": "c_int", "uint8_t": "u8", "uint16_t": "u16", "uint32_t": "u32", "uint64_t": "u64",
             "int64_t": "i64", "size_t": "usize", "float": "f32", "char": "c_char", "void": "c_void"}
RUST_SIZES = {"u8": 1, "u16": 2, "u32": 4, "u64": 8, "i64": 8, "i32": 4, "f32": 4, "f64": 8, "c_int": 4,
              "c_char": 1, "usize": 8}


def camel(c_name):
    return "".join(p.capitalize() for p in c_name.split("_"))


def strip_c(text):
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    return text


def split_top(s, sep=","):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "([{<":
            depth += 1
        elif ch in ")]}>" and not (ch == ">" and cur.endswith("-")):
            depth -= 1
        if ch == sep and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def c_decl_type(decl, fnptrs):
    """'const uint8_t *bytes' -> Rust FFI type ('*const u8'); returns (name, rust_type)."""
    decl = " ".join(decl.replace("*", " * ").split())
    arr = re.match(r"(.*?)\s*\[\s*(\w+)\s*\]$", decl)
    n_arr = None
    if arr:
        decl, n_arr = arr.group(1), arr.group(2)
    toks = decl.split()
    name = None
    # every parameter and field of the headers is named: the last identifier after the type
    if len(toks) >= 2 and re.match(r"^[A-Za-z_]\w*$", toks[-1]) and toks[:-1] != ["const"]:
        name = toks.pop()
    const = toks[0] == "const"
    if const:
        toks = toks[1:]
    base, stars = toks[0], toks[1:].count("*")
    if base in fnptrs:
        r = camel(base)
    elif base in C_SCALARS:
        r = C_SCALARS[base]
    else:
        assert base.startswith("ngz_"), decl
        r = camel(base)
    for i in range(stars):
        # the const binds to the innermost pointee
        r = ("*const " if (i == 0 and const) else "*mut ") + r
    if n_arr:
        r = f"[{r}; {n_arr}]"
    return name, r


def parse_headers():
    funcs, structs, opaque, fnptrs, consts = {}, {}, set(), {}, {}
    for h in HEADERS:
        raw = open(h).read()
        for m in re.finditer(r"^#define\s+(NGZ_\w+)\s+\(?(-?\d+)u?\)?", raw, re.M):
            consts[m.group(1)] = int(m.group(2))
        text = strip_c(raw)
        text = "\n".join(l for l in text.splitlines() if not l.strip().startswith("#"))
        text = text.replace('extern "C" {', " ")
        for m in re.finditer(r"typedef\s+struct\s*\{(.*?)\}\s*(\w+)\s*;", text, re.S):
            structs[m.group(2)] = [f.strip() for f in m.group(1).split(";") if f.strip()]
        text = re.sub(r"typedef\s+struct\s*\{.*?\}\s*\w+\s*;", " ", text, flags=re.S)
        for m in re.finditer(r"typedef\s+struct\s+(\w+)\s+(\w+)\s*;", text):
            opaque.add(m.group(2))
        text = re.sub(r"typedef\s+struct\s+\w+\s+\w+\s*;", " ", text)
        for m in re.finditer(r"typedef\s+([\w\s\*]+?)\s*\(\s*\*\s*(\w+)\s*\)\s*\((.*?)\)\s*;", text, re.S):
            fnptrs[m.group(2)] = (m.group(1), m.group(3))
        text = re.sub(r"typedef\s+[\w\s\*]+?\(\s*\*\s*\w+\s*\)\s*\(.*?\)\s*;", " ", text, flags=re.S)
        for m in re.finditer(r"([\w\s\*]+?)\b(ngz_\w+)\s*\(([^;]*?)\)\s*;", text, re.S):
            funcs[m.group(2)] = (m.group(1).strip(), m.group(3).strip())
    return funcs, structs, opaque, fnptrs, consts


def c_signature(ret, params, fnptrs):
    ps = [] if params.strip() in ("", "void") else [c_decl_type(p, fnptrs)[1] for p in split_top(params)]
    _, r = c_decl_type(ret + " x", fnptrs)
    return ps, (None if r == "c_void" else r)


def rust_blocks():
    return re.findall(r"```rust\n(.*?)```", open(DOC).read(), re.S)


def parse_rust():
    structs, fns, aliases, consts = {}, {}, {}, {}
    code = "\n".join(rust_blocks())
    code_nc = re.sub(r"//[^\n]*", " ", code)
    for m in re.finditer(r"#\[repr\(C\)\]\s*pub struct (\w+)\s*\{(.*?)\}", code_nc, re.S):
        fields = []
        for f in split_top(m.group(2)):
            f = f.strip()
            if not f:
                continue
            name, ty = f.split(":", 1)
            fields.append((name.replace("pub ", "").strip(), " ".join(ty.split())))
        assert m.group(1) not in structs, m.group(1)
        structs[m.group(1)] = fields
    for m in re.finditer(r"pub type (\w+)\s*=\s*(?:unsafe\s+)?extern \"C\" fn\((.*?)\)\s*(?:->\s*([\w\s\*]+?))?\s*;",
                         code_nc, re.S):
        aliases[m.group(1)] = ([" ".join(p.split()) for p in split_top(m.group(2))],
                               " ".join(m.group(3).split()) if m.group(3) else None)
    for m in re.finditer(r"pub const (NGZ_\w+)\s*:\s*\w+\s*=\s*(-?\d+)\s*;", code_nc):
        consts[m.group(1)] = int(m.group(2))
    for blk in re.finditer(r"extern \"C\"\s*\{(.*?)\n\}", code_nc, re.S):
        for m in re.finditer(r"pub fn (\w+)\s*\((.*?)\)\s*(?:->\s*([^;]+?))?\s*;", blk.group(1), re.S):
            params = []
            for p in split_top(m.group(2)):
                name, ty = p.split(":", 1)
                params.append(" ".join(ty.split()))
            assert m.group(1) not in fns, f"{m.group(1)} bound twice"
            fns[m.group(1)] = (params, " ".join(m.group(3).split()) if m.group(3) else None)
    return structs, fns, aliases, consts, code


def test_every_header_function_is_bound_with_its_signature():
    funcs, _, _, fnptrs, _ = parse_headers()
    _, fns, aliases, _, _ = parse_rust()
    assert len(funcs) > 40
    missing = sorted(set(funcs) - set(fns))
    assert not missing, f"INTEGRATION.md binds no extern fn for {missing}"
    extra = sorted(set(fns) - set(funcs))
    assert not extra, f"INTEGRATION.md binds functions no header declares: {extra}"
    for name, (ret, params) in funcs.items():
        want_p, want_r = c_signature(ret, params, fnptrs)
        got_p, got_r = fns[name]
        assert len(got_p) == len(want_p), (name, got_p, want_p)
        assert got_p == want_p, (name, got_p, want_p)
        assert got_r == want_r, (name, got_r, want_r)
    for c_name, (ret, params) in fnptrs.items():
        assert camel(c_name) in aliases, f"no `pub type {camel(c_name)}` for {c_name}"
        want_p, want_r = c_signature(ret, params, fnptrs)
        assert aliases[camel(c_name)] == (want_p, want_r), c_name


def rust_layout(name, structs, opaque_rust):
    """(size, align, [(field, offset)]) of a #[repr(C)] struct as the Rust declaration implies."""
    def size_align(ty):
        ty = ty.strip()
        if ty.startswith("*"):
            return 8, 8
        m = re.match(r"\[(.*);\s*(\d+)\]$", ty)
        if m:
            s, a = size_align(m.group(1))
            return s * int(m.group(2)), a
        if ty in RUST_SIZES:
            return RUST_SIZES[ty], RUST_SIZES[ty]
        if ty in opaque_rust:
            return 0, 1
        s, a, _ = rust_layout(ty, structs, opaque_rust)
        return s, a
    off, align, offs = 0, 1, []
    for f, ty in structs[name]:
        s, a = size_align(ty)
        off = (off + a - 1) // a * a
        offs.append((f, off))
        off += s
        align = max(align, a)
    return (off + align - 1) // align * align, align, offs


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc missing")
def test_repr_c_structs_match_c_layout():
    _, cstructs, opaque, fnptrs, _ = parse_headers()
    rstructs, _, _, _, _ = parse_rust()
    opaque_rust = {camel(o) for o in opaque}
    for o in opaque:
        assert camel(o) in rstructs, f"no opaque #[repr(C)] {camel(o)} for {o}"
        assert rstructs[camel(o)] == [("_p", "[u8; 0]")], camel(o)
    probe = ["#include <stdio.h>", "#include <stddef.h>"] + \
        [f'#include "ngz/{os.path.basename(h)}"' for h in HEADERS] + ["int main(void) {"]
    want = {}
    for cname, fields in cstructs.items():
        rname = camel(cname)
        assert rname in rstructs, f"INTEGRATION.md has no #[repr(C)] {rname} mirroring {cname}"
        cf = [c_decl_type(f, fnptrs) for f in fields]
        assert [(n, t) for n, t in cf] == rstructs[rname], (rname, cf, rstructs[rname])
        size, _, offs = rust_layout(rname, rstructs, opaque_rust)
        want[cname] = (size, offs)
        probe.append(f'  printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in offs:
            probe.append(f'  printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    probe += ["  return 0;", "}"]
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "probe.c"), os.path.join(d, "probe")
        open(src, "w").write("\n".join(probe) + "\n")
        subprocess.check_call(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), src, "-o", exe])
        out = subprocess.check_output([exe], text=True)
    got = {}
    for line in out.splitlines():
        s, f, v = line.split()
        got[(s, f)] = int(v)
    for cname, (size, offs) in want.items():
        assert got[(cname, "size")] == size, (cname, got[(cname, "size")], size)
        for f, o in offs:
            assert got[(cname, f)] == o, (cname, f, got[(cname, f)], o)


def test_constants_mirror_headers_and_versions_are_checked_by_name():
    _, _, _, _, hconsts = parse_headers()
    _, _, _, rconsts, code = parse_rust()
    assert hconsts["NGZ_ABI_VERSION"] >= 4
    missing = sorted(set(hconsts) - set(rconsts))
    assert not missing, f"INTEGRATION.md lacks pub const {missing}"
    wrong = {k: (rconsts[k], v) for k, v in hconsts.items() if rconsts[k] != v}
    assert not wrong, wrong
    assert not set(rconsts) - set(hconsts), set(rconsts) - set(hconsts)
    # the wrapper refuses a library built from other headers, by constant, not by a literal
    assert re.search(r"ngz_abi_version\(\)\s*\}?\s*!=\s*(?:ffi::)?NGZ_ABI_VERSION\b", code)
    assert re.search(r"ngz_agg_abi_version\(\)\s*\}?\s*!=\s*(?:ffi::)?NGZ_AGG_ABI_VERSION\b", code)
    assert not re.search(r"abi_version\(\)\s*\}?\s*!=\s*\d", code)


def test_doc_table_names_every_entry_point():
    """§1's tables cite a reference interface (or say there is none) for each header function."""
    funcs, _, _, _, _ = parse_headers()
    table = open(DOC).read().split("## 2.")[0]
    missing = [f for f in funcs if not re.search(r"`" + f + r"\b", table)]
    assert not missing, f"INTEGRATION.md §1 does not list {missing}"
