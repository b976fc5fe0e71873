"""Pin the oracle's IPv6 chain (RPKT_F_IPV6) against the reference's own IPv6 tests.

Every assert of the *_parse tests of rpkt/tests/ipv6_test.rs is replayed here through
the oracle's record and the host views (rpkt_amd/views.py), on the same captures
(tests/golden/packets/ipv6_options_*.dat, byte copies of rpkt/tests/packet_examples).
The L4 sums are pinned by the checksums the capturing stacks stored: a correct sum over
a valid segment is 0xffff.  ipv6_options_routing2.dat (Routing type 0, segments_left 1,
UDP) is 0xffff only when the pseudo header uses the routing header's final address
(RFC 8200 section 8.1), the policy include/rpkt_gpu.h documents.  CPU only.
"""
import ipaddress
import os

import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import gen
from rpkt_amd.records import (STATUS, F_IPV6, OPT_STOP, IP6_OPT_KINDS, ip6_block, ip6_opts_view,
                              is_ip6, project16, trace_kinds, MAX_IP6_EXT)
from rpkt_amd.views import (EtherFrame, Ipv4, Ipv6, DestOptions, HopByHopOption, RoutingHeader,
                            FragmentHeader, AuthenticationHeader, Udp, Packet, EtherType,
                            IpProtocol)

HERE = os.path.dirname(os.path.abspath(__file__))
PKTS = os.path.join(HERE, "golden", "packets")
FLAGS6 = 3 | F_IPV6


def load(name):
    return oracle.load_dat(os.path.join(PKTS, name))


def chain(name):
    frame = load(name)
    rec = oracle.parse_one(frame, FLAGS6)
    eth = EtherFrame.parse(Packet(rec, frame)).unwrap()
    assert eth.ethertype() == EtherType.IPV6
    return frame, rec, Ipv6.parse(eth.payload()).unwrap()


def A(s):
    return ipaddress.IPv6Address(s)


def test_destination_options_parse():
    """ipv6_test.rs:20-76"""
    frame, rec, ip = chain("ipv6_options_destination.dat")
    assert (ip.version(), ip.traffic_class(), ip.flow_label()) == (6, 0, 0)
    assert ip.payload_len() == 26
    assert ip.next_header() == IpProtocol.IPV6_DEST_OPTS
    assert ip.hop_limit() == 64
    assert ip.src_addr() == A("2a01:e35:8bd9:8bb0:a0a7:ea9c:74e8:d397")
    assert ip.dst_addr() == A("2001:4b98:dc0:41:216:3eff:fece:1902")
    d = DestOptions.parse(ip.payload()).unwrap()
    assert d.next_header() == IpProtocol.UDP and d.header_len() == 8
    udp = Udp.parse(d.payload()).unwrap()
    assert udp.packet_len() == 18
    assert len(udp.payload().chunk()) == 10
    # the stored UDP checksum (0x6889) verifies with the IPv6 pseudo header
    assert udp.checksum() == 0x6889 and udp.sum() == 0xffff and udp.verify_checksum()
    assert int(rec["status"]) == STATUS["OK"] and int(ip6_block(np.array([rec]))[0]["ip6_n_ext"]) == 1


def test_hop_by_hop_parse():
    """ipv6_test.rs:129-179"""
    frame, rec, ip = chain("ipv6_options_hop_by_hop.dat")
    assert (ip.version(), ip.traffic_class(), ip.flow_label()) == (6, 0, 0)
    assert ip.payload_len() == 36
    assert ip.next_header() == IpProtocol.IPV6_HOP_BY_HOP_OPTS
    assert ip.hop_limit() == 1
    assert ip.src_addr() == A("fe80::9c09:b416:768:ff42")
    assert ip.dst_addr() == A("ff02::16")
    h = HopByHopOption.parse(ip.payload()).unwrap()
    assert h.next_header() == IpProtocol.ICMPV6 and h.header_len() == 8
    assert len(h.payload().chunk()) == 28
    # ICMPv6 is not on the path: the walk stops there with the upper-layer region
    assert int(rec["status"]) == STATUS["L4_OTHER"] and int(rec["ip_protocol"]) == 58
    assert (int(rec["l4_off"]), int(rec["payload_len"])) == (62, 28)


def test_routing1_parse():
    """ipv6_test.rs:225-270"""
    frame, rec, ip = chain("ipv6_options_routing1.dat")
    assert ip.payload_len() == 48 and ip.next_header() == IpProtocol.IPV6_ROUTE
    assert ip.hop_limit() == 5
    assert ip.src_addr() == A("2200::244:212:3fff:feae:22f7")
    assert ip.dst_addr() == A("2200::211:2:0:0:2")
    r = RoutingHeader.parse(ip.payload()).unwrap()
    assert r.next_header() == IpProtocol.ICMPV6 and r.header_len() == 40
    assert (r.type_(), r.segments_left(), r.type_specific_data()) == (0, 2, 0)
    v = r.var_header_slice()
    assert ipaddress.IPv6Address(v[0:16]) == A("2200::210:2:0:0:4")
    assert ipaddress.IPv6Address(v[16:32]) == A("2200::240:2:0:0:4")
    assert len(r.payload().chunk()) == 8
    # the pseudo-header destination: the last address of the type-0 list
    b = ip6_block(np.array([rec]))[0]
    assert int(b["ip6_pdst_off"]) == 14 + 40 + 8 + 16


def test_routing2_l4_sum_uses_final_address():
    """ipv6_options_routing2.dat: Routing type 0, segments_left 1 -> UDP.  0xffff with
    the final address; with dst_addr the sum would be 0x0030."""
    frame, rec, ip = chain("ipv6_options_routing2.dat")
    r = RoutingHeader.parse(ip.payload()).unwrap()
    assert (r.type_(), r.segments_left()) == (0, 1)
    udp = Udp.parse(r.payload()).unwrap()
    assert udp.sum() == 0xffff
    # recompute both ways independently of the oracle's composition
    l3 = int(rec["l3_off"])
    src, dst = frame[l3 + 8:l3 + 24], frame[l3 + 24:l3 + 40]
    final = frame[l3 + 40 + 8:l3 + 40 + 24]
    seg = frame[int(rec["l4_off"]):int(rec["l4_off"]) + udp.packet_len()]

    def v6sum(d):
        ph = src + d + len(seg).to_bytes(4, "big") + bytes([0, 0, 0, 17])
        return oracle.combine([oracle.from_slice(ph), oracle.from_slice(seg)])
    assert v6sum(final) == 0xffff and v6sum(dst) == 0x0030


def test_fragment_parse():
    """ipv6_test.rs:319-353: a non-first fragment stops the walk (IP6_FRAGMENT)."""
    frame, rec, ip = chain("ipv6_options_fragments.dat")
    assert ip.flow_label() == 0x21289 and ip.payload_len() == 1456
    assert ip.next_header() == IpProtocol.IPV6_FRAG and ip.hop_limit() == 64
    assert ip.src_addr() == A("2607:f010:3f9::1001")
    assert ip.dst_addr() == A("2607:f010:3f9::11:0")
    f = FragmentHeader.parse(ip.payload()).unwrap()
    assert f.next_header() == IpProtocol.UDP
    assert (f.reserved(), f.offset(), f.reserved1(), f.more_frag()) == (0, 181, 0, True)
    assert f.ident() == 0xf88eb466
    assert len(f.payload().chunk()) == 1448
    assert int(rec["status"]) == STATUS["IP6_FRAGMENT"]
    assert (int(rec["ip_protocol"]), int(rec["payload_off"]), int(rec["payload_len"])) == (17, 62, 1448)
    assert int(rec["l4_sum"]) == 0


def test_ah_parse():
    """ipv6_test.rs:391-422"""
    frame, rec, ip = chain("ipv6_options_ah.dat")
    assert ip.traffic_class() == 0b11100000 and ip.flow_label() == 0
    assert ip.payload_len() == 64 and ip.next_header() == IpProtocol.AH and ip.hop_limit() == 1
    assert ip.src_addr() == A("fe80::2") and ip.dst_addr() == A("ff02::5")
    ah = AuthenticationHeader.parse(ip.payload()).unwrap()
    assert ah.next_header() == 89 and ah.header_len() == 24 and ah.reserved() == 0
    assert ah.security_parameters_index() == 0x100 and ah.seq_num_field() == 32
    assert ah.var_header_slice() == bytes([0x35, 0x48, 0x21, 0x48, 0xb2, 0x43, 0x5a, 0x23,
                                           0xdc, 0xdd, 0x55, 0x36])
    assert len(ah.payload().chunk()) == 40
    assert int(rec["status"]) == STATUS["L4_OTHER"] and int(rec["ip_protocol"]) == 89


def test_multi_extension_chain():
    """ipv6_options_multi.dat: HopByHop -> DestOptions -> Routing -> AH -> OSPF (89)."""
    frame, rec, ip = chain("ipv6_options_multi.dat")
    c = ip.payload()
    kinds = []
    for view in (HopByHopOption, DestOptions, RoutingHeader, AuthenticationHeader):
        h = view.parse(c).unwrap()
        kinds.append(h.next_header())
        c = h.payload()
    assert kinds == [60, 43, 51, 89]
    assert c.cursor() == int(rec["l4_off"]) == 118
    b = ip6_block(np.array([rec]))[0]
    assert int(b["ip6_n_ext"]) == 4 and int(rec["ip_protocol"]) == 89


def test_without_flag_ipv6_stays_not_ipv4():
    for name in sorted(os.listdir(PKTS)):
        if name.startswith("ipv6"):
            rec = oracle.parse_one(load(name), 3)
            assert int(rec["status"]) == STATUS["NOT_IPV4"], name


def test_flag_leaves_ipv4_records_unchanged():
    """RPKT_F_IPV6 changes nothing for frames that are not dispatched on 0x86DD."""
    for cfg in (5, 6):
        hb = gen.make_batch(cfg, 20000, seed=3)
        a = oracle.parse_batch(hb.frames, hb.n, flags=3, offsets=hb.offsets)
        b = oracle.parse_batch(hb.frames, hb.n, flags=FLAGS6, offsets=hb.offsets)
        v6 = is_ip6(b)
        assert np.array_equal(a[~v6], b[~v6]), cfg
        # fault 6 frames (0x86DD over an IPv4 body) become IPv6 records
        assert (a["status"][v6] == STATUS["NOT_IPV4"]).all()


def test_ip4_records_never_flagged_ip6():
    hb = gen.make_batch(6, 20000, seed=4)
    r = oracle.parse_batch(hb.frames, hb.n, flags=3, offsets=hb.offsets)
    assert not is_ip6(r).any()


# ---- an independent Python model of the IPv6 walk (cross-checks the C restatement) ----

EXT = {0: (2, 2), 60: (2, 2), 43: (8, 8), 44: (8, 8), 51: (12, 12)}   # fixed, min header_len


def model_ip6(f, flags):
    """Status, l4_off, protocol and the pseudo-destination offset of one frame, or None
    when the frame is not dispatched to Ipv6::parse."""
    if len(f) < 14:
        return None
    et, c, nv = int.from_bytes(f[12:14], "big"), 14, 0
    while et in (0x8100, 0x88a8) and nv < 2:
        if len(f) - c < 4:
            return None
        et = int.from_bytes(f[c + 2:c + 4], "big")
        c += 4
        nv += 1
    if et != 0x86DD or not flags & F_IPV6:
        return None
    l3 = c
    if len(f) - l3 < 40:
        return ("IP6_SHORT",)
    plen = int.from_bytes(f[l3 + 4:l3 + 6], "big")
    if plen + 40 > len(f) - l3:
        return ("IP6_BAD_LEN",)
    end, c, nh, pdst = l3 + 40 + plen, l3 + 40, f[l3 + 6], l3 + 24
    for _ in range(MAX_IP6_EXT):
        if nh not in EXT:
            break
        fixed, mn = EXT[nh]
        if end - c < fixed:
            return ("IP6_EXT_SHORT", c, nh, pdst)
        hl = 8 if nh == 44 else (f[c + 1] * 4 + 8 if nh == 51 else f[c + 1] * 8 + 8)
        if nh != 44 and (hl < mn or hl > end - c):
            return ("IP6_EXT_BAD_LEN", c, nh, pdst)
        if nh == 43 and f[c + 3] > 0:
            n = (hl - 8) // 16
            if n and f[c + 2] in (0, 2):
                pdst = c + 8 + 16 * (n - 1)
            elif n and f[c + 2] == 4:
                pdst = c + 8
        frag = nh == 44 and (int.from_bytes(f[c + 2:c + 4], "big") & 0xfff9)
        nh, c = f[c], c + hl
        if frag:
            return ("IP6_FRAGMENT", c, nh, pdst)
    if nh in EXT:
        return ("L4_OTHER", c, nh, pdst)
    if nh == 17:
        if end - c < 8:
            return ("UDP_SHORT", c, nh, pdst)
        ul = int.from_bytes(f[c + 4:c + 6], "big")
        return ("UDP_BAD_LEN" if ul < 8 or ul > end - c else "OK", c, nh, pdst)
    if nh == 6:
        if end - c < 20:
            return ("TCP_SHORT", c, nh, pdst)
        hl = (f[c + 12] >> 4) * 4
        return ("TCP_BAD_DOFF" if hl < 20 or hl > end - c else "OK", c, nh, pdst)
    return ("L4_OTHER", c, nh, pdst)


def test_python_model_agrees_on_dual_stack_fuzz():
    hb = gen.make_batch(12, 6000, seed=12)
    recs = oracle.parse_batch(hb.frames, hb.n, flags=FLAGS6, offsets=hb.offsets)
    blk = ip6_block(recs)
    seen = set()
    for i in range(hb.n):
        f = hb.frames[int(hb.offsets[i]):int(hb.offsets[i + 1])].tobytes()
        m = model_ip6(f, FLAGS6)
        r = recs[i]
        if m is None:
            assert not is_ip6(recs[i:i + 1])[0], i
            continue
        seen.add(m[0])
        assert int(r["status"]) == STATUS[m[0]], (i, m, int(r["status"]))
        if len(m) > 1:
            assert (int(r["l4_off"]), int(r["ip_protocol"]), int(blk[i]["ip6_pdst_off"])) == \
                m[1:], (i, m)
    assert {"OK", "IP6_SHORT", "IP6_BAD_LEN", "IP6_EXT_BAD_LEN", "IP6_FRAGMENT",
            "L4_OTHER"} <= seen


@pytest.mark.parametrize("cfg", [10, 11])
def test_dual_stack_configs_verify(cfg):
    """The generator stamps every L4 checksum with its own IPv6 pseudo-header code
    (independent of the oracle); only the ~1 % injected bad sums fail."""
    hb = gen.make_batch(cfg, 40000)
    r = oracle.parse_batch(hb.frames, hb.n, flags=FLAGS6, stride=hb.stride, threads=8)
    v6 = is_ip6(r)
    assert (r["status"] == 0).all()
    assert 0.45 < v6.mean() < 0.55
    good = r["l4_sum"] == 0xffff
    assert 0.98 < good[v6].mean() < 0.997 and 0.98 < good[~v6].mean() < 0.997


def test_compact_projection_verdicts():
    hb = gen.make_batch(12, 20000, seed=5)
    r = oracle.parse_batch(hb.frames, hb.n, flags=FLAGS6, offsets=hb.offsets)
    p = project16(r, FLAGS6)
    v6 = is_ip6(r)
    assert ((p["verdict"] >> 2 & 1).astype(bool) == v6).all()
    # IPv6 with the header parsed: bit 0 set without any header checksum
    parsed6 = v6 & ~np.isin(r["status"], [STATUS["IP6_SHORT"], STATUS["IP6_BAD_LEN"]])
    assert (p["verdict"][parsed6] & 1).all()
    # a UDP checksum of 0 over IPv6 does not verify
    z = v6 & (r["status"] == 0) & (r["ip_protocol"] == 17) & (r["l4_checksum"] == 0)
    assert z.any() and not (p["verdict"][z] & 2).any()


def test_flow_events_ip6():
    hb = gen.make_batch(12, 20000, seed=6)
    r, ev = oracle.parse_batch(hb.frames, hb.n, flags=FLAGS6, offsets=hb.offsets,
                               n_buckets=4096, flow_ev=True)
    v6 = is_ip6(r)
    assert not ((ev[v6] >> np.uint64(48)) & np.uint64(1)).any()       # no IPv6 header sum
    ok6 = v6 & (r["status"] == 0)
    b = (ev >> np.uint64(32)) & np.uint64(0xffff)
    assert (b[ok6] < 4096).all() and (b[v6 & (r["status"] != 0)] == 4096).all()


def test_build_rebuilds_ip6_records_in_place():
    """IPv6 records are built (round 5: Ipv6::prepend_header + setters): over frames that
    already hold those headers with valid sums, the build changes nothing."""
    hb = gen.make_batch(11, 2000)
    r = oracle.parse_batch(hb.frames, hb.n, flags=FLAGS6, stride=hb.stride)
    out, built = oracle.build_batch(hb.frames, hb.n, r, flags=3, stride=hb.stride)
    v6 = is_ip6(r)
    good = v6 & (r["l4_sum"] == 0xFFFF)
    assert built[v6].all() and built[~v6].all() and good.sum() > 900
    f = out.reshape(hb.n, hb.stride)
    assert np.array_equal(f[good], hb.frames.reshape(hb.n, hb.stride)[good])


def test_ipv4_view_refuses_ip6_record():
    frame = load("ipv6_options_destination.dat")
    rec = oracle.parse_one(frame, FLAGS6)
    eth = EtherFrame.parse(Packet(rec, frame)).unwrap()
    assert Ipv4.parse(eth.payload()).is_err()


# ---- Ipv6OptionsIter (the IPv6 half of rpkt_opts_t) ----

def opts_of(name):
    f = load(name)
    r = np.array([oracle.parse_one(f, FLAGS6)])
    o = oracle.options_batch(np.frombuffer(f, dtype=np.uint8), 1, r,
                             offsets=np.array([0, len(f)], dtype=np.uint32))
    return o[0], ip6_opts_view(o)[0]


def test_ip6_options_destination():
    """ipv6_test.rs:47-69: Generic (type 11, header_len 3, var_header_slice()[0] == 9),
    then PadN (header_len 3, var_header_slice()[0] == 0), then None."""
    o, v = opts_of("ipv6_options_destination.dat")
    assert trace_kinds(o["ip_trace"], o["ip_count"], IP6_OPT_KINDS) == ["Generic", "Padn"]
    assert int(v["stop"]) == OPT_STOP["END"] and int(v["end"]) == 6        # 3 + 3 bytes
    assert (int(v["generic_type"]), int(v["generic_len"]) + 2) == (11, 3)
    assert int(v["generic_data"]) >> 24 == 9
    assert (int(v["n_hdrs"]), int(v["first_hdr"])) == (1, 60)
    assert int(o["tcp_stop"]) == OPT_STOP["NONE"]                          # UDP


def test_ip6_options_hop_by_hop():
    """ipv6_test.rs:154-175: RouterAlert (type 5, header_len 4, router_alert 0), then PadN
    (header_len 2), then None."""
    o, v = opts_of("ipv6_options_hop_by_hop.dat")
    assert trace_kinds(o["ip_trace"], o["ip_count"], IP6_OPT_KINDS) == ["RouterAlert", "Padn"]
    assert int(v["router_alert"]) == 0 and int(v["end"]) == 6              # 4 + 2 bytes
    assert int(v["stop"]) == OPT_STOP["END"] and (int(v["n_hdrs"]), int(v["first_hdr"])) == (1, 0)


def test_ip6_options_every_options_header():
    """ipv6_options_multi.dat: HopByHop then DestOptions are both walked, in order."""
    o, v = opts_of("ipv6_options_multi.dat")
    assert trace_kinds(o["ip_trace"], o["ip_count"], IP6_OPT_KINDS) == \
        ["RouterAlert", "Padn", "Generic", "Padn"]
    assert (int(v["n_hdrs"]), int(v["first_hdr"])) == (2, 0)
    o, v = opts_of("ipv6_options_routing1.dat")                           # no options header
    assert int(v["stop"]) == OPT_STOP["NONE"] and int(o["ip_count"]) == 0


def model_ip6_opts(f, l3, l4):
    """Independent Python restatement of the walk (ipv6/generated.rs:1568-1615)."""
    c, nh, out, stop, hdrs = l3 + 40, f[l3 + 6], [], 0, 0
    for _ in range(MAX_IP6_EXT):
        if c >= l4:
            break
        hl = 8 if nh == 44 else (f[c + 1] * 4 + 8 if nh == 51 else f[c + 1] * 8 + 8)
        if nh in (0, 60):
            hdrs += 1
            b, pos, stop = f[c + 2:c + hl], 0, 1
            while pos < len(b):
                t, rem = b[pos], len(b) - pos
                if t == 0:
                    out.append("Pad0"); pos += 1; continue
                ln = b[pos + 1] + 2 if rem >= 2 else 0
                ok = (rem >= 4 and ln == 4) if t == 5 else (rem >= 2 and ln <= rem)
                if not ok:
                    stop = 3
                    break
                out.append("Padn" if t == 1 else "RouterAlert" if t == 5 else "Generic")
                pos += ln
            if stop == 3:
                break
        nh, c = f[c], c + hl
    return out, stop, hdrs


def test_ip6_options_model_on_fuzz():
    hb = gen.make_batch(12, 6000, seed=21)
    r = oracle.parse_batch(hb.frames, hb.n, flags=FLAGS6, offsets=hb.offsets)
    o = oracle.options_batch(hb.frames, hb.n, r, offsets=hb.offsets)
    v = ip6_opts_view(o)
    stops = set()
    for i in np.nonzero(is_ip6(r) & ~np.isin(r["status"], [14, 15]))[0]:
        f = hb.frames[int(hb.offsets[i]):int(hb.offsets[i + 1])].tobytes()
        kinds, stop, hdrs = model_ip6_opts(f, int(r[i]["l3_off"]), int(r[i]["l4_off"]))
        assert trace_kinds(o[i]["ip_trace"], o[i]["ip_count"], IP6_OPT_KINDS) == kinds[:16], i
        assert int(o[i]["ip_count"]) == len(kinds) and int(v[i]["stop"]) == stop, i
        assert int(v[i]["n_hdrs"]) == hdrs, i
        stops.add(stop)
    assert stops == {0, 1, 3}
