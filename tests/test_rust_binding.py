"""The Rust binding crate (bindings/rpkt-gpu) against include/rpkt_gpu.h.

No Rust toolchain exists in this image, so the crate cannot be compiled here; these
checks keep it from drifting away from the C ABI it binds:
  * every function the header declares is declared in src/ffi.rs with the same
    number of parameters, and nothing else is;
  * every #[repr(C)] struct of src/ffi.rs has the C struct's fields in the same order
    with the same offsets and widths (offsetof / sizeof from a compiled C probe);
  * the status / error / flag constants equal the header's values.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "rpkt_gpu.h")
FFI = os.path.join(ROOT, "bindings", "rpkt-gpu", "src", "ffi.rs")
LIB = os.path.join(ROOT, "bindings", "rpkt-gpu", "src", "lib.rs")

RUST_SCALARS = {"u8": 1, "u16": 2, "u32": 4, "u64": 8, "usize": 8, "i32": 4, "c_int": 4}


def _strip_c_comments(s):
    return re.sub(r"/\*.*?\*/", "", s, flags=re.S)


def _arity(params):
    params = params.strip()
    if params in ("", "void"):
        return 0
    depth, n = 0, 1
    for ch in params:
        depth += ch in "([<"
        depth -= ch in ")]>"
        n += ch == "," and depth == 0
    return n


def c_functions():
    src = _strip_c_comments(open(HDR).read())
    out = {}
    for m in re.finditer(r"\b(rpkt_\w+)\s*\(([^;{]*?)\)\s*;", src):
        out[m.group(1)] = _arity(m.group(2))
    return out


def rust_functions():
    src = open(FFI).read()
    block = src[src.index('extern "C" {'):]
    out = {}
    for m in re.finditer(r"pub fn (\w+)\s*\(([^)]*)\)", block, flags=re.S):
        out[m.group(1)] = _arity(re.sub(r"//[^\n]*", "", m.group(2)))
    return out


def rust_structs():
    """{name: [(field, rust type)]} for every #[repr(C)] struct of ffi.rs."""
    src = open(FFI).read()
    out = {}
    for m in re.finditer(r"#\[repr\(C\)\][^{]*?pub struct (\w+)\s*\{(.*?)\n\}", src, flags=re.S):
        fields = re.findall(r"pub (\w+):\s*([^,\n]+),", m.group(2))
        out[m.group(1)] = [(f, t.strip()) for f, t in fields]
    return out


def rust_align(t):
    a = re.fullmatch(r"\[(\w+);.*\]", t)
    if a:
        return RUST_SCALARS[a.group(1)]
    if t.startswith("*"):
        return 8
    if t in RUST_SCALARS:
        return RUST_SCALARS[t]
    return max(rust_align(ft) for _, ft in rust_structs()[t])      # a nested struct


def rust_size(t):
    a = re.fullmatch(r"\[(\w+);\s*(\w+)\]", t)
    if a:
        n = {"RPKT_MAX_LAYERS": 16}.get(a.group(2)) or int(a.group(2))
        return RUST_SCALARS[a.group(1)] * n
    if t.startswith("*"):
        return 8
    if t in RUST_SCALARS:
        return RUST_SCALARS[t]
    fields = rust_structs()[t]                                        # a nested struct
    _, off, size = rust_layout(fields)[-1]
    al = rust_align(t)
    return (off + size + al - 1) // al * al


def rust_layout(fields):
    """C layout rules (what #[repr(C)] guarantees): offset aligned to the element size."""
    off, out = 0, []
    for f, t in fields:
        size = rust_size(t)
        align = rust_align(t)
        off = (off + align - 1) // align * align
        out.append((f, off, size))
        off += size
    return out


def test_ffi_declares_exactly_the_header_functions():
    c, r = c_functions(), rust_functions()
    assert len(c) >= 25
    assert sorted(r) == sorted(c), set(r) ^ set(c)
    for name in c:
        assert r[name] == c[name], "%s: %d params in Rust, %d in C" % (name, r[name], c[name])


def test_every_header_struct_is_bound():
    src = _strip_c_comments(open(HDR).read())
    c_structs = set(re.findall(r"\}\s*(rpkt_\w+_t);", src))
    assert c_structs == set(rust_structs())


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    structs = rust_structs()
    lines = ['#include <stddef.h>', '#include <stdio.h>', '#include "rpkt_gpu.h"',
             'int main(void) {']
    for s, fields in structs.items():
        lines.append('printf("%s size %%zu\\n", sizeof(%s));' % (s, s))
        for f, _ in fields:
            lines.append('printf("%s %s %%zu %%zu\\n", offsetof(%s, %s), sizeof(((%s*)0)->%s));'
                         % (s, f, s, f, s, f))
    lines.append("return 0; }")
    d = tmp_path_factory.mktemp("probe")
    c = d / "probe.c"
    c.write_text("\n".join(lines))
    exe = d / "probe"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    lay = {}
    for ln in out.splitlines():
        p = ln.split()
        if p[1] == "size":
            lay[(p[0], "__size__")] = int(p[2])
        else:
            lay[(p[0], p[1])] = (int(p[2]), int(p[3]))
    return lay


def test_struct_layouts_match_c(c_layout):
    for s, fields in rust_structs().items():
        lay = rust_layout(fields)
        for f, off, size in lay:
            assert (s, f) in c_layout, "%s.%s is not a field of the C struct" % (s, f)
            assert c_layout[(s, f)] == (off, size), "%s.%s: Rust (%d, %d), C %s" % (
                s, f, off, size, c_layout[(s, f)])
        last_f, last_off, last_size = lay[-1]
        end = last_off + last_size
        align = max(rust_align(t) for _, t in fields)
        assert (end + align - 1) // align * align == c_layout[(s, "__size__")], s


def test_field_order_matches_c(c_layout):
    """Offsets strictly increase in Rust declaration order, and every C field is bound."""
    src = _strip_c_comments(open(HDR).read())
    for s, fields in rust_structs().items():
        body = src[:src.index("} %s;" % s)]
        body = body[body.rindex("typedef struct"):]
        c_fields = re.findall(r"\b(\w+)(?:\[[^\]]*\])?\s*;", body)
        assert [f for f, _ in fields] == c_fields, s


def test_constants_match_header():
    src = _strip_c_comments(open(HDR).read())
    c = {m.group(1): int(m.group(2), 0) for m in
         re.finditer(r"\b(RPKT_[A-Z0-9_]+)\s*=\s*(-?(?:0x)?[0-9a-f]+)u?\b", src)}
    c.update({m.group(1): int(m.group(2).rstrip("u"), 0) for m in
              re.finditer(r"#define (RPKT_[A-Z0-9_]+)\s+(\d+u?)\b", src)})
    rs = {m.group(1): int(m.group(2)) for m in
          re.finditer(r"pub const (RPKT_[A-Z0-9_]+):\s*\w+\s*=\s*(-?\d+);", open(FFI).read())}
    shared = set(c) & set(rs)
    assert len(shared) >= 30
    for k in shared:
        assert rs[k] == c[k], k


def test_views_cover_the_reference_getters():
    """lib.rs re-exposes every getter of the five views on the path under rpkt's names
    (rpkt/src/{ether,vlan,ipv4,udp,tcp}/generated.rs)."""
    src = open(LIB).read()
    want = {
        "EtherFrame": ["parse", "dst_addr", "src_addr", "ethertype", "payload"],
        "VlanFrame": ["parse", "priority", "dei_flag", "vlan_id", "ethertype", "payload"],
        "Ipv4": ["parse", "version", "dscp", "ecn", "ident", "flag_reserved", "dont_frag",
                 "more_frag", "frag_offset", "ttl", "protocol", "checksum", "header_len",
                 "packet_len", "src_addr", "dst_addr", "payload"],
        "Udp": ["parse", "src_port", "dst_port", "checksum", "packet_len", "payload"],
        "Tcp": ["parse", "src_port", "dst_port", "seq_num", "ack_num", "reserved", "cwr", "ece",
                "urg", "ack", "psh", "rst", "syn", "fin", "window_size", "checksum",
                "urgent_pointer", "header_len", "payload"],
    }
    for view, getters in want.items():
        body = src[src.index("impl<'a> %s<'a> {" % view):]
        body = body[:body.index("\n}\n")]
        have = set(re.findall(r"pub fn (\w+)", body))
        assert set(getters) <= have, (view, set(getters) - have)
