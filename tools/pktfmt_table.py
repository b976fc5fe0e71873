"""Derive the device protocol table from the reference's pktfmt specs.

Reads /root/reference/pktfmt/protocols/*.pktfmt (the protocol descriptions rpkt's
generated header views are produced from) and writes, for every packet the layer
walker can visit, the numbers the generated `parse()` / `payload()` /
`group_parse()` are functions of (pktfmt/src/codegen/parse.rs:138-244,
payload.rs:23-87; the group dispatch as in the generated group_parse functions):

  hdr        fixed header bytes (sum of the header field widths / 8)
  hl         header_len: none | linear expression of one field | custom (gre,
             gre_pptp, gtpv1, gtpv2: the hand-written header_len functions the
             specs leave undefined) ; `fixed` when that field's default is pinned
             with '@' (parse then checks header_len == the pinned value)
  pl         payload_len or packet_len: linear expression of one field
  cond       the group-dispatch condition: per field, a set of closed ranges

Outputs (generated and committed; the GPU box has no /root/reference):
  rpkt_amd/csrc/rpkt_proto_table.h   C table compiled into the layer-walk kernel
  include/rpkt_protocols.h           protocol / group ids for the C ABI
  tests/golden/proto_table.json      the same data, for the tests

The oracle (oracle/rpkt_oracle_layers.c) does NOT use this table: it restates each
protocol's generated parse function by hand, so the two cross-check each other.

Usage: python tools/pktfmt_table.py [reference_root]
"""
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

# Walker groups, in id order: (name, spec file, member packets).  A plain packet is
# a group of one.  Members of the spec's own groups are listed in its order.
# icmpv6.pktfmt is not compiled into rpkt (no rpkt/src/icmpv6), so it is left out.
GROUPS = [
    ("ETHER", "ether", "group:EtherGroup"),
    ("VLAN", "vlan", "group:VlanGroup"),
    ("IPV4", "ipv4", ["Ipv4"]),
    ("IPV6", "ipv6", ["Ipv6"]),
    ("IPV6_HOPBYHOP", "ipv6", ["HopByHopOption"]),
    ("IPV6_DESTOPTS", "ipv6", ["DestOptions"]),
    ("IPV6_ROUTING", "ipv6", ["RoutingHeader"]),
    ("IPV6_FRAGMENT", "ipv6", ["FragmentHeader"]),
    ("IPV6_AUTH", "ipv6", ["AuthenticationHeader"]),
    ("UDP", "udp", ["Udp"]),
    ("TCP", "tcp", ["Tcp"]),
    ("ICMPV4", "icmpv4", "group:Icmpv4"),
    ("GRE", "gre", "group:GreGroup"),
    ("VXLAN", "vxlan", ["Vxlan"]),
    ("GTPV1", "gtpv1", ["Gtpv1"]),
    ("GTPV2", "gtpv2", ["Gtpv2"]),
    ("MPLS", "mpls", ["Mpls"]),
    ("ARP", "arp", ["Arp"]),
    ("LLC", "llc", ["Llc"]),
    ("PPPOE", "pppoe", "group:PppoeGroup"),
    ("STP", "stp", "group:StpGroup"),
]
CUSTOM_HL = {"Gre": 1, "GreForPPTP": 2, "Gtpv1": 3, "Gtpv2": 4}   # header_len= (undefined)
FORMS = {"ident": 0, "add": 1, "mult": 2, "addmult": 3, "multadd": 4}


def strip_code(text):
    """Drop the %% ... %% Rust code blocks and // comments."""
    text = re.sub(r"%%.*?%%", "", text, flags=re.S)
    return re.sub(r"//[^\n]*", "", text)


def blocks(text, kind):
    out = {}
    for m in re.finditer(r"\b%s\s+(\w+)\s*=?\s*\{" % kind, text):
        i, depth = m.end(), 1
        while depth:
            depth += {"{": 1, "}": -1}.get(text[i], 0)
            i += 1
        out[m.group(1)] = text[m.end():i - 1]
    return out


def num(s):
    s = s.strip()
    return int(s, 16) if s.lower().startswith("0x") else int(s)


def parse_fields(body):
    hdr = body[body.index("header"):]
    hdr = hdr[hdr.index("[") + 1:]
    depth, i = 1, 0
    while depth:
        depth += {"[": 1, "]": -1}.get(hdr[i], 0)
        i += 1
    hdr = hdr[:i - 1]
    fields, off = {}, 0
    for m in re.finditer(r"(\w+)\s*=\s*Field\s*\{([^}]*)\}", hdr):
        attrs = m.group(2)
        bits = num(re.search(r"bit\s*=\s*(\w+)", attrs).group(1))
        d = re.search(r"default\s*=\s*(@?)\s*(0x[0-9a-fA-F]+|\d+)", attrs)
        fields[m.group(1)] = {"off": off, "bits": bits,
                              "fixed": bool(d and d.group(1)),
                              "default": num(d.group(2)) if d else None}
        off += bits
    assert off % 8 == 0, off
    return fields, off // 8


def parse_expr(e, fields):
    """pktfmt's UsableAlgExpr subset (pktfmt/src/ast/length.rs:244-259)."""
    e = e.replace(" ", "")
    m = re.fullmatch(r"\(?(\w+)\)?", e)
    if m and m.group(1) in fields:
        return m.group(1), "ident", 0, 0
    for pat, form, ga, gb, fi in (
            (r"(\w+)\+(\d+)", "add", 2, None, 1), (r"(\d+)\+(\w+)", "add", 1, None, 2),
            (r"(\w+)\*(\d+)", "mult", 2, None, 1), (r"(\d+)\*(\w+)", "mult", 1, None, 2),
            (r"\((\w+)\+(\d+)\)\*(\d+)", "addmult", 2, 3, 1),
            (r"(\w+)\*(\d+)\+(\d+)", "multadd", 2, 3, 1),
            (r"(\d+)\*(\w+)\+(\d+)", "multadd", 1, 3, 2),
            (r"(\d+)\+(\w+)\*(\d+)", "multadd", 3, 1, 2)):
        m = re.fullmatch(pat, e)
        if m and m.group(fi) in fields:
            return m.group(fi), form, int(m.group(ga)), int(m.group(gb)) if gb else 0
    raise ValueError("length expression not understood: %r" % e)


def parse_length(body, fields):
    hl = pl = None
    m = re.search(r"length\s*=\s*\[(.*?)\]", body, re.S)
    if not m:
        return hl, pl
    for part in m.group(1).split(","):
        part = part.strip()
        if not part:
            continue
        key, _, expr = part.partition("=")
        key, expr = key.strip(), expr.strip()
        if key == "header_len":
            hl = ("custom", None) if not expr else ("expr", parse_expr(expr, fields))
        elif key in ("payload_len", "packet_len"):
            pl = (key, parse_expr(expr, fields))
    return hl, pl


def parse_cond(body, fields):
    m = re.search(r"cond\s*=\s*\((.*)\)", body, re.S)
    if not m:
        return []
    terms = []
    for t in re.split(r"\)\s*&&\s*\(", m.group(1)):
        f, _, rng = t.strip("() \n").partition("==")
        f = f.strip()
        ranges = []
        for r in rng.split("||"):
            r = r.strip()
            if "..=" in r:
                lo, hi = r.split("..=")
                ranges.append((num(lo) if lo.strip() else 0, num(hi)))
            elif ".." in r:
                lo, hi = r.split("..")
                ranges.append((num(lo) if lo.strip() else 0,
                               num(hi) - 1 if hi.strip() else (1 << fields[f]["bits"]) - 1))
            else:
                ranges.append((num(r), num(r)))
        terms.append({"field": f, "off": fields[f]["off"], "bits": fields[f]["bits"],
                      "ranges": ranges})
    return terms


def build(ref):
    spec_dir = os.path.join(ref, "pktfmt", "protocols")
    specs = {}
    for fn in sorted(os.listdir(spec_dir)):
        if fn.endswith(".pktfmt"):
            text = strip_code(open(os.path.join(spec_dir, fn)).read())
            specs[fn[:-7]] = (blocks(text, "packet"), blocks(text, "group"))
    packets, groups = [], []
    for gname, spec, members in GROUPS:
        pk, gr = specs[spec]
        if isinstance(members, str):
            body = gr[members.split(":")[1]]
            members = re.findall(r"\w+", body[body.index("[") + 1:body.index("]")])
        ids = []
        for name in members:
            body = pk[name]
            fields, hdr = parse_fields(body)
            hl, pl = parse_length(body, fields)
            ent = {"id": len(packets), "spec": spec, "name": name, "hdr": hdr,
                   "hl_kind": 0, "hl": None, "hl_fixed": None, "pl_kind": 0, "pl": None,
                   "cond": parse_cond(body, fields),
                   "fields": {k: [v["off"], v["bits"]] for k, v in fields.items()}}
            if hl and hl[0] == "custom":
                ent["hl_kind"] = 1 + CUSTOM_HL[name]
            elif hl:
                f, form, a, b = hl[1]
                ent["hl_kind"] = 1
                ent["hl"] = {"field": f, "off": fields[f]["off"], "bits": fields[f]["bits"],
                             "form": form, "a": a, "b": b}
                if fields[f]["fixed"]:
                    ent["hl_fixed"] = evaluate(form, a, b, fields[f]["default"])
            if pl:
                f, form, a, b = pl[1]
                ent["pl_kind"] = 1 if pl[0] == "payload_len" else 2
                ent["pl"] = {"field": f, "off": fields[f]["off"], "bits": fields[f]["bits"],
                             "form": form, "a": a, "b": b}
            packets.append(ent)
            ids.append(ent["id"])
        cond_bytes = max([(c["off"] + c["bits"] + 7) // 8 for i in ids
                          for c in packets[i]["cond"]] or [0])
        groups.append({"name": gname, "members": ids, "cond_bytes": cond_bytes})
    return {"packets": packets, "groups": groups}


def evaluate(form, a, b, x):
    return {"ident": x, "add": x + a, "mult": x * a, "addmult": (x + a) * b,
            "multadd": x * a + b}[form]


def c_header(t):
    L = ["// GENERATED by tools/pktfmt_table.py from the reference's pktfmt specs",
         "// (pktfmt/protocols/*.pktfmt); do not edit.  See that script for the meaning.",
         "#pragma once", "#include <stdint.h>", "",
         "struct RpktLenExpr { uint16_t off; uint8_t bits; uint8_t form; uint16_t a, b; };",
         "struct RpktCond { uint16_t off; uint8_t bits; uint8_t n; uint16_t lo[3], hi[3]; };",
         "struct RpktProto {",
         "    uint16_t hdr;          // fixed header bytes",
         "    uint8_t hl_kind;       // 0 none, 1 expr, 2 gre, 3 gre_pptp, 4 gtpv1, 5 gtpv2",
         "    uint8_t pl_kind;       // 0 none, 1 payload_len, 2 packet_len",
         "    int32_t hl_fixed;      // >= 0: header_len must equal this (pinned field)",
         "    RpktLenExpr hl, pl;",
         "    uint8_t n_cond;",
         "    RpktCond cond[5];",
         "};",
         "// lut 0xff: none; key: byte offset of the dword the member tests read",
         "struct RpktGroup { uint8_t first, count, cond_bytes, lut, key; };",
         "struct RpktMember { uint32_t mask, lo, span; };", ""]
    for g in t["groups"]:
        L.append("#define RPKT_G_%s %d" % (g["name"], t["groups"].index(g)))
    L.append("#define RPKT_N_GROUPS %d" % len(t["groups"]))
    L.append("#define RPKT_N_PROTOS %d" % len(t["packets"]))
    L.append("")
    L.append("__device__ __constant__ const RpktProto kProtos[RPKT_N_PROTOS] = {")

    def ex(e):
        if not e:
            return "{0, 0, 0, 0, 0}"
        return "{%d, %d, %d, %d, %d}" % (e["off"], e["bits"], FORMS[e["form"]], e["a"], e["b"])

    for p in t["packets"]:
        conds = []
        for c in p["cond"]:
            rs = c["ranges"] + [(1, 0)] * (3 - len(c["ranges"]))
            conds.append("{%d, %d, %d, {%s}, {%s}}" % (
                c["off"], c["bits"], len(c["ranges"]), ", ".join(str(r[0]) for r in rs),
                ", ".join(str(r[1]) for r in rs)))
        while len(conds) < 5:
            conds.append("{0, 0, 0, {0, 0, 0}, {0, 0, 0}}")
        L.append("    {%d, %d, %d, %d, %s, %s, %d, {%s}},  // %d %s::%s" % (
            p["hdr"], p["hl_kind"], p["pl_kind"],
            -1 if p["hl_fixed"] is None else p["hl_fixed"], ex(p["hl"]), ex(p["pl"]),
            len(p["cond"]), ", ".join(conds), p["id"], p["spec"], p["name"]))
    L.append("};")
    # Groups whose members each test one condition on the same field of <= 8 bits
    # (ICMPv4 types, PPPoE codes) also get a 256-entry lookup: field value -> the
    # first member whose ranges hold it (0xff: none), so a walk resolves them with one
    # table read instead of a loop over the members.
    luts = []
    for g in t["groups"]:
        ms = [t["packets"][i] for i in g["members"]]
        f0 = ms[0]["cond"][0] if ms[0]["cond"] else None
        if (len(ms) > 1 and f0 and f0["bits"] == 8 and f0["off"] % 8 == 0 and
                all(len(m["cond"]) == 1 and m["cond"][0]["off"] == f0["off"] and
                    m["cond"][0]["bits"] == f0["bits"] for m in ms)):
            row = []
            for v in range(256):
                hit = [m["id"] for m in ms if any(lo <= v <= hi for lo, hi in m["cond"][0]["ranges"])]
                row.append(hit[0] if hit else 0xFF)
            g["lut"] = len(luts)
            luts.append((f0["off"], f0["bits"], row))
        else:
            g["lut"] = 0xFF
    L.append("#define RPKT_N_LUT %d" % len(luts))
    L.append("__device__ __constant__ const uint32_t kGroupLutField[RPKT_N_LUT] = {%s};  // off | bits << 16" %
             ", ".join("%d" % (o | (b << 16)) for o, b, _ in luts))
    L.append("__device__ __constant__ const uint8_t kGroupLut[RPKT_N_LUT][256] = {")
    for _, _, row in luts:
        L.append("    {%s}," % ", ".join(str(x) for x in row))
    L.append("};")
    L.append("__device__ __constant__ const RpktGroup kGroups[RPKT_N_GROUPS] = {")
    for g in t["groups"]:
        L.append("    {%d, %d, %d, %d, %d},  // %s" % (g["members"][0], len(g["members"]),
                                                      g["cond_bytes"], g["lut"], g["key"],
                                                      g["name"]))
    L.append("};")
    # Every member's condition as one test on the big-endian dword at its group's key
    # byte: (key & mask) - lo <= span (unsigned).  A single-range condition on one field
    # is that field's range shifted into place; several conditions compile only when
    # each is one exact value (GreForPPTP, the STP BPDUs), which merge into one masked
    # equality.  A member with no condition has mask 0: it always matches.
    L.append("#define RPKT_MAX_MEMBERS %d" % max(
        len(g["members"]) for g in t["groups"] if g["lut"] == 0xFF))
    L.append("__device__ __constant__ const RpktMember kMembers[RPKT_N_PROTOS] = {")
    for p in t["packets"]:
        m = p["member"]
        L.append("    {0x%08x, 0x%08x, 0x%08x},  // %d %s" % (m[0], m[1], m[2], p["id"], p["name"]))
    L.append("};")
    return "\n".join(L) + "\n"


def member_tests(t):
    """Compile each group's member conditions into masked-dword range tests."""
    for g in t["groups"]:
        ms = [t["packets"][i] for i in g["members"]]
        conds = [c for m in ms for c in m["cond"]]
        g["key"] = min([c["off"] // 8 for c in conds] or [0])
        assert g["key"] < 16, g                # the key dword lies in the 20-B header prefix
        for m in ms:
            mask = lo = hi = 0
            for c in m["cond"]:
                rel = c["off"] - 8 * g["key"]
                assert rel + c["bits"] <= 32, (m["name"], c)
                sh = 32 - rel - c["bits"]
                assert len(c["ranges"]) == 1, (m["name"], c)
                clo, chi = c["ranges"][0]
                if len(m["cond"]) > 1:
                    assert clo == chi, (m["name"], c)
                mask |= ((1 << c["bits"]) - 1) << sh
                lo |= clo << sh
                hi |= chi << sh
            m["member"] = (mask, lo, hi - lo)


def host_header(t):
    """include/rpkt_protocols.h: protocol and group ids for rpkt_layers_t users."""
    L = ["/* GENERATED by tools/pktfmt_table.py from the reference's pktfmt specs; do not",
         " * edit.  Protocol ids (rpkt_layers_t.proto[k]) and walker groups (err_group). */",
         "#ifndef RPKT_PROTOCOLS_H", "#define RPKT_PROTOCOLS_H", ""]
    for p in t["packets"]:
        L.append("#define RPKT_P_%s_%s %d" % (p["spec"].upper(), p["name"].upper(), p["id"]))
    L.append("#define RPKT_N_PROTOCOLS %d" % len(t["packets"]))
    L.append("")
    for k, g in enumerate(t["groups"]):
        L.append("#define RPKT_GROUP_%s %d" % (g["name"], k))
    L.append("#define RPKT_N_GROUPS_HOST %d" % len(t["groups"]))
    L += ["", "#endif"]
    return "\n".join(L) + "\n"


def main(ref="/root/reference"):
    t = build(ref)
    for g in t["groups"]:                      # members must be consecutive ids
        assert g["members"] == list(range(g["members"][0], g["members"][0] + len(g["members"])))
    for p in t["packets"]:                     # the kernel reads fields through 4 bytes
        for f in [c for c in p["cond"]] + [e for e in (p["hl"], p["pl"]) if e]:
            assert f["off"] % 8 + f["bits"] <= 32, (p["name"], f)
        for c in p["cond"]:                    # condition fields and ranges are 16-bit
            assert c["bits"] <= 16 and all(0 <= v < 1 << 16 for r in c["ranges"] for v in r)
        if p["pl"]:                            # payload fields lie in the 20-B prefix
            assert p["pl"]["off"] // 8 < 16, p["name"]
    member_tests(t)
    with open(os.path.join(ROOT, "rpkt_amd", "csrc", "rpkt_proto_table.h"), "w") as fh:
        fh.write(c_header(t))
    with open(os.path.join(ROOT, "include", "rpkt_protocols.h"), "w") as fh:
        fh.write(host_header(t))
    for g in t["groups"]:
        g.pop("lut", None)
        g.pop("key", None)
    for p in t["packets"]:
        p.pop("member", None)
    with open(os.path.join(ROOT, "rpkt_amd", "proto_fields.json"), "w") as fh:
        json.dump({"%s_%s" % (p["spec"].upper(), p["name"].upper()):
                   {"id": p["id"], "hdr": p["hdr"], "fields": p["fields"]}
                   for p in t["packets"]}, fh, indent=1)
    with open(os.path.join(ROOT, "tests", "golden", "proto_table.json"), "w") as fh:
        json.dump(t, fh, indent=1)
    print("%d packets in %d groups" % (len(t["packets"]), len(t["groups"])))


if __name__ == "__main__":
    main(*sys.argv[1:])
