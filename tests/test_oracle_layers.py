"""The protocol layer walk: the hand-written oracle (oracle/rpkt_oracle_layers.c)
against what the reference's own tests assert on its captures, and the
pktfmt-derived table (tests/golden/proto_table.json, tools/pktfmt_table.py) --
interpreted here in Python with the pktfmt codegen rules -- against the oracle on
fuzzed traffic.  The two derivations are independent: the oracle is restated from
rpkt's generated views, the table from the pktfmt specs."""
import json
import os

import numpy as np

from oracle import oracle
from rpkt_amd import gen
from rpkt_amd.records import LAYER_STOP, LAYERS_DTYPE, protocol_names

HERE = os.path.dirname(os.path.abspath(__file__))
PKTS = os.path.join(HERE, "golden", "packets")
TABLE = json.load(open(os.path.join(HERE, "golden", "proto_table.json")))
NAMES = protocol_names()
GID = {g["name"]: k for k, g in enumerate(TABLE["groups"])}


def walk(name):
    f = oracle.load_dat(os.path.join(PKTS, name))
    o = oracle.layers_batch(np.frombuffer(f, np.uint8), 1,
                            offsets=np.array([0, len(f)], np.uint32))[0]
    return [(NAMES[int(o["proto"][k])], int(o["off"][k])) for k in range(o["n"])], o


def test_layer_kats_from_reference_tests():
    # vlan_mpls_tests.rs:224-240: Ether / Ipv4 / Udp / Vxlan / Ether / ...
    lay, o = walk("Vxlan1.dat")
    assert [p for p, _ in lay][:5] == ["ETHER_ETHERFRAME", "IPV4_IPV4", "UDP_UDP",
                                       "VXLAN_VXLAN", "ETHER_ETHERFRAME"]
    # gre_test.rs:185-200: GreGroup -> Gre with header_len 8 carrying Ethernet
    lay, o = walk("GREv0_4.dat")
    assert lay[2] == ("GRE_GRE", 34) and lay[3] == ("ETHER_ETHERFRAME", 42)
    # gre_test.rs:100-115: GreForPPTP, header_len 12, payload_len 0
    lay, o = walk("GREv1_1.dat")
    assert lay[-1] == ("GRE_GREFORPPTP", 34) and o["payload_off"] == 46 and o["payload_len"] == 0
    # gtpv1_test.rs:200-210: Gtpv1 packet_len 92 + 8, 12-byte header (extension bit)
    lay, o = walk("gtp-u-1ext.dat")
    assert lay[-1] == ("GTPV1_GTPV1", 42) and o["payload_off"] == 54 and o["payload_len"] == 88
    # gtpv2_test.rs:17-30: Gtpv2 packet_len 4 + 107, teid present (12-byte header)
    lay, o = walk("gtpv2-with-teid.dat")
    assert lay[-1] == ("GTPV2_GTPV2", 42) and o["payload_off"] == 54 and o["payload_len"] == 99
    # pppoe_test.rs:12-30: PppoeSession packet_len 26, data_type 0xc021 (not IP)
    lay, o = walk("PPPoESession1.dat")
    assert lay[-1] == ("PPPOE_PPPOESESSION", 14) and o["stop"] == LAYER_STOP["UNKNOWN"]
    assert o["next_key"] == 0xC021 and (o["payload_off"], o["payload_len"]) == (22, 18)
    # pppoe_test.rs:60-75: PppoeDiscovery packet_len 46
    lay, o = walk("PPPoEDiscovery2.dat")
    assert lay[-1] == ("PPPOE_PPPOEDISCOVERY", 14) and o["payload_len"] == 40
    # vlan_mpls_tests.rs:134-150: Ether / Vlan / Vlan / Mpls / (IPv4 after bottom of stack)
    lay, o = walk("MplsPackets1.dat")
    assert [p for p, _ in lay][:4] == ["ETHER_ETHERFRAME", "VLAN_VLANFRAME", "VLAN_VLANFRAME",
                                       "MPLS_MPLS"]
    # vlan_mpls_tests.rs:156-173: two labels, then a payload starting 0x00 0x00
    lay, o = walk("MplsPackets2.dat")
    assert [p for p, _ in lay] == ["ETHER_ETHERFRAME", "MPLS_MPLS", "MPLS_MPLS"]
    assert o["stop"] == LAYER_STOP["UNKNOWN"] and o["next_key"] == 0
    # llc_test.rs:40-55: VlanGroup -> VlanDot3Frame (payload_len 357) -> Llc
    lay, o = walk("llc_vlan.dat")
    assert [p for p, _ in lay] == ["ETHER_ETHERFRAME", "VLAN_VLANDOT3FRAME", "LLC_LLC"]
    assert o["payload_off"] == 21 and o["payload_len"] == 357 - 3
    # stp_test.rs: EtherDot3Frame -> Llc -> StpGroup members
    assert walk("StpTcn.dat")[0][-1] == ("STP_STPTCNBPDU", 17)
    assert walk("StpRapid.dat")[0][-1] == ("STP_RSTPCONFBPDU", 17)
    assert walk("StpMultiple.dat")[0][-1] == ("STP_MSTPCONFBPDU", 17)
    # eth_and_arp_test.rs: Ether / Arp, and Ether / Vlan / Vlan / Arp
    assert [p for p, _ in walk("ArpRequestWithVlan.dat")[0]] == [
        "ETHER_ETHERFRAME", "VLAN_VLANFRAME", "VLAN_VLANFRAME", "ARP_ARP"]
    # ipv6_test.rs: the extension-header chain of ipv6_options_multi
    lay, o = walk("ipv6_options_multi.dat")
    assert [p for p, _ in lay][1:] == ["IPV6_IPV6", "IPV6_HOPBYHOPOPTION", "IPV6_DESTOPTIONS",
                                       "IPV6_ROUTINGHEADER", "IPV6_AUTHENTICATIONHEADER"]


# ---- the pktfmt-derived table, interpreted in Python -------------------------------

def field(f, x, off, bits):
    b0, b1 = off // 8, (off + bits - 1) // 8
    v = 0
    for b in range(b0, b1 + 1):
        v = (v << 8) | f[x + b]
    return (v >> (7 - (off + bits - 1) % 8)) & ((1 << bits) - 1)


def expr(e, x):
    return {"ident": x, "add": x + e["a"], "mult": x * e["a"], "addmult": (x + e["a"]) * e["b"],
            "multadd": x * e["a"] + e["b"]}[e["form"]]


def table_group(f, g, s, e):
    """group_parse + parse + payload of group g by the table (pktfmt codegen rules)."""
    G = TABLE["groups"][g]
    r = e - s
    if r < G["cond_bytes"]:
        return None
    m = None
    for pid in G["members"]:
        P = TABLE["packets"][pid]
        if all(any(lo <= field(f, s, c["off"], c["bits"]) <= hi for lo, hi in c["ranges"])
               for c in P["cond"]):
            m = P
            break
    if m is None or r < m["hdr"]:
        return None
    h = m["hdr"]
    kind = m["hl_kind"]
    if kind == 1:
        h = expr(m["hl"], field(f, s, m["hl"]["off"], m["hl"]["bits"]))
    elif kind in (2, 3):
        ind = (f[s] << 8) | f[s + 1]
        h = (4 + 4 * bool(ind & 0xC000) + 4 * bool(ind & 0x2000) + 4 * bool(ind & 0x1000)) \
            if kind == 2 else (8 + 4 * bool(ind & 0x1000) + 4 * bool(ind & 0x80))
    elif kind == 4:
        h = 12 if f[s] & 7 else 8
    elif kind == 5:
        h = 12 if f[s] & 8 else 8
    if kind and (h < m["hdr"] or h > r):
        return None
    end = e
    if m["pl_kind"] == 1:
        pay = expr(m["pl"], field(f, s, m["pl"]["off"], m["pl"]["bits"]))
        if pay + h > r:
            return None
        end = s + h + pay
    elif m["pl_kind"] == 2:
        pkt = expr(m["pl"], field(f, s, m["pl"]["off"], m["pl"]["bits"]))
        if pkt < h or pkt > r:
            return None
        end = s + pkt
    return m["id"], h, end


ETHERTYPE = {0x0800: "IPV4", 0x86DD: "IPV6", 0x8100: "VLAN", 0x88A8: "VLAN", 0x0806: "ARP",
             0x8847: "MPLS", 0x8848: "MPLS", 0x8863: "PPPOE", 0x8864: "PPPOE"}
IPPROTO = {0: "IPV6_HOPBYHOP", 1: "ICMPV4", 4: "IPV4", 6: "TCP", 17: "UDP", 41: "IPV6",
           43: "IPV6_ROUTING", 44: "IPV6_FRAGMENT", 47: "GRE", 51: "IPV6_AUTH", 59: "END",
           60: "IPV6_DESTOPTS"}


def nxt(f, p, h, s, e):
    """The dispatch documented in include/rpkt_gpu.h (same graph as the oracle)."""
    n = NAMES[p]
    be16 = lambda x: (f[x] << 8) | f[x + 1]   # noqa: E731

    def ip(v):
        return IPPROTO.get(v, "UNKNOWN"), v
    if n in ("ETHER_ETHERFRAME", "VLAN_VLANFRAME"):
        k = be16(h + (12 if n.startswith("ETHER") else 2))
        return ETHERTYPE.get(k, "UNKNOWN"), k
    if n in ("ETHER_ETHERDOT3FRAME", "VLAN_VLANDOT3FRAME"):
        return "LLC", 0
    if n == "IPV4_IPV4":
        return ("END", 0) if be16(h + 6) & 0x1FFF else ip(f[h + 9])
    if n == "IPV6_IPV6":
        return ip(f[h + 6])
    if n == "IPV6_FRAGMENTHEADER":
        return ("END", 0) if be16(h + 2) >> 3 else ip(f[h])
    if n in ("IPV6_HOPBYHOPOPTION", "IPV6_DESTOPTIONS", "IPV6_ROUTINGHEADER",
             "IPV6_AUTHENTICATIONHEADER"):
        return ip(f[h])
    if n == "UDP_UDP":
        dp, sp = be16(h + 2), be16(h)
        port = dp if dp in (4789, 2152, 2123) else (sp if sp in (4789, 2152, 2123) else 0)
        if not port:
            return "END", 0
        if port == 4789:
            return "VXLAN", port
        if e <= s:
            return "END", 0
        v = f[s] >> 5
        return {1: "GTPV1", 2: "GTPV2"}.get(v, "UNKNOWN"), v
    if n == "GRE_GRE":
        k = be16(h + 2)
        return ("ETHER", k) if k == 0x6558 else (ETHERTYPE.get(k, "UNKNOWN"), k)
    if n == "VXLAN_VXLAN":
        return "ETHER", 0
    if n in ("GTPV1_GTPV1", "MPLS_MPLS"):
        if n == "GTPV1_GTPV1" and ((f[h] & 4) or f[h + 1] != 255):
            return "END", 0
        if n == "MPLS_MPLS" and not (f[h + 2] & 1):
            return "MPLS", 0
        if e <= s:
            return "END", 0
        v = f[s] >> 4
        return {4: "IPV4", 6: "IPV6"}.get(v, "UNKNOWN"), v
    if n == "PPPOE_PPPOESESSION":
        k = be16(h + 6)
        return {0x21: "IPV4", 0x57: "IPV6"}.get(k, "UNKNOWN"), k
    if n == "LLC_LLC":
        return ("STP", 0) if f[h] == 0x42 and f[h + 1] == 0x42 else ("END", 0)
    return "END", 0


def table_walk(f):
    o = np.zeros(1, LAYERS_DTYPE)[0]
    s, e, g = 0, len(f), GID["ETHER"]
    while True:
        if o["n"] == 16:
            o["stop"] = LAYER_STOP["MAX"]
            break
        res = table_group(f, g, s, e)
        if res is None:
            o["stop"], o["err_group"] = LAYER_STOP["ERR"], g
            break
        p, h, end = res
        o["proto"][o["n"]], o["off"][o["n"]] = p, s
        o["n"] += 1
        hs, e, s = s, end, s + h
        nx, key = nxt(f, p, hs, s, e)
        if nx == "END":
            o["stop"] = LAYER_STOP["END"]
            break
        if nx == "UNKNOWN":
            o["stop"], o["next_key"], o["key_proto"] = LAYER_STOP["UNKNOWN"], key, p
            break
        g = GID[nx]
    o["payload_off"], o["payload_len"] = s, e - s
    return o


def test_table_matches_oracle_on_fixtures_and_fuzz():
    hb = gen.make_mix(6000, seed=21)
    got = oracle.layers_batch(hb.frames, hb.n, offsets=hb.offsets)
    for i in range(hb.n):
        f = hb.frames[hb.offsets[i]:hb.offsets[i + 1]].tobytes()
        want = table_walk(f)
        assert got[i].tobytes() == want.tobytes(), (i, got[i], want)
    stops = set(got["stop"].tolist())
    assert stops == {1, 2, 3}
    assert len(set(got["proto"][got["n"] > 0, 0].tolist())) >= 2


def test_table_shape():
    """The generated table carries the generated views' constants (spot checks
    against rpkt/src/*/generated.rs)."""
    P = {(p["spec"], p["name"]): p for p in TABLE["packets"]}
    assert P[("ipv4", "Ipv4")]["hdr"] == 20 and P[("ipv4", "Ipv4")]["hl"]["a"] == 4
    assert P[("ipv6", "Ipv6")]["hdr"] == 40 and P[("ipv6", "Ipv6")]["pl_kind"] == 1
    assert P[("stp", "MstpConfBpdu")]["hdr"] == 102                 # stp/generated.rs:787
    assert P[("stp", "MstpConfBpdu")]["hl"]["off"] == 36 * 8        # version3_len, :1065
    assert P[("gtpv1", "Gtpv1")]["pl"]["a"] == 8                    # packet_len = 8 + len
    assert P[("pppoe", "PppoeSession")]["hdr"] == 8                 # pppoe/generated.rs:33
    assert {g["name"]: g["cond_bytes"] for g in TABLE["groups"]}["ETHER"] == 14
