"""The encapsulation build (rpkt_gpu_build_tunnel_batch) on the CPU, through the build
oracle (oracle/rpkt_oracle_build.c oracle_build_tunnel_one): the reference's own build
tests run with the host views (rpkt_amd/txviews.py Vxlan / Gtpv1 / Gre) give its captures
back byte for byte -- vlan_mpls_tests.rs:254-300 (Vxlan2.dat), gtpv1_test.rs:236-282
(gtp-u-1ext.dat), gre_test.rs:255-287 (GREv0_4.dat) -- and every tunnel capture is
rebuilt from its parsed getters (the records rpkt_gpu_parse_tunnel_batch returns)."""
import os

import numpy as np

from oracle import oracle
from rpkt_amd import txviews as tv
from rpkt_amd.records import F_IPV6, TUN_DTYPE, TUN_STATUS
from rpkt_amd.views import EtherType, IpProtocol

HERE = os.path.dirname(os.path.abspath(__file__))
PKTS = os.path.join(HERE, "golden", "packets")


def chain_batch(chains, payloads):
    """(frames buffer, offsets, records, tunnels) of finished cursors, the payload of each
    placed at the frame's end and every `extra` byte the views list."""
    recs_extra, tuns = [], []
    for buf in chains:
        rec, extra = buf.record()
        t, textra = tv.tunnel_record(buf)
        recs_extra.append((rec, extra + textra))
        tuns.append(t)
    lens = [c.frame_len - c.start for c in chains]
    buf, offs, recs = tv.assemble(recs_extra, lens, payloads)
    return buf, offs, recs, np.array(tuns, dtype=TUN_DTYPE)


def vxlan2_chain(pkt_bytes):
    """vlan_mpls_tests.rs:254-300, statement for statement."""
    pkt = tv.CursorMut(148)
    pkt.advance(14 + 20 + 8 + 8)
    vx = tv.Vxlan.prepend_header(pkt, tv.VXLAN_HEADER_TEMPLATE)
    vx.set_vni_present(True)
    vx.set_policy_applied(True)
    vx.set_group_id(32639)
    vx.set_vni(300)
    udp = tv.Udp.prepend_header(vx.release(), tv.UDP_HEADER_TEMPLATE)
    udp.set_src_port(45149)
    udp.set_dst_port(4789)
    udp.set_checksum(0xad94)
    ip = tv.Ipv4.prepend_header(udp.release(), tv.IPV4_HEADER_TEMPLATE)
    ip.set_dscp(0)
    ip.set_ident(0xd2c2)
    ip.set_dont_frag(True)
    ip.set_ttl(64)
    ip.set_protocol(IpProtocol.UDP)
    ip.set_checksum(0x5150)
    ip.set_src_addr("192.168.203.1")
    ip.set_dst_addr("192.168.202.1")
    eth = tv.EtherFrame.prepend_header(ip.release(), tv.ETHER_FRAME_HEADER_TEMPLATE)
    eth.set_dst_addr([0x00, 0x16, 0x3e, 0x08, 0x71, 0xcf])
    eth.set_src_addr([0x36, 0xdc, 0x85, 0x1e, 0xb3, 0x40])
    eth.set_ethertype(EtherType.IPV4)
    return eth.release(), pkt_bytes[50:]


def gtpu1_chain(pkt_bytes):
    """gtpv1_test.rs:236-282: ExtPduNumber placed by the caller (move_back), then the
    Gtpv1 header built from a header array with E and S set."""
    pkt = tv.CursorMut(len(pkt_bytes))
    pkt.advance(len(pkt_bytes) - 84)
    pkt.move_back(4, bytes([0x01, 0x09, 0x04, 0x00]))          # ExtPduNumber 2308, NO_EXTENTION
    hdr = tv.Gtpv1.set_header_flags(tv.GTPV1_HEADER_TEMPLATE, extention_header_present=True,
                                    sequence_present=True, message_type=255, teid=1)
    g = tv.Gtpv1.prepend_header(pkt, hdr)
    g.set_sequence(10461)
    g.set_next_extention_header(0xc0)                           # PDU_NUMBER
    udp = tv.Udp.prepend_header(g.release(), tv.UDP_HEADER_TEMPLATE)
    udp.set_checksum(0xb58d)
    udp.set_dst_port(2152)
    udp.set_src_port(2152)
    ip = tv.Ipv4.prepend_header(udp.release(), tv.IPV4_HEADER_TEMPLATE)
    ip.set_ident(0)
    ip.set_ttl(64)
    ip.set_dont_frag(True)
    ip.set_protocol(IpProtocol.UDP)
    ip.set_checksum(0x67b7)
    ip.set_src_addr("192.168.40.179")
    ip.set_dst_addr("192.168.40.178")
    eth = tv.EtherFrame.prepend_header(ip.release(), tv.ETHER_FRAME_HEADER_TEMPLATE)
    eth.set_dst_addr([0x00, 0x0c, 0x29, 0xda, 0xd1, 0xde])
    eth.set_src_addr([0x00, 0x0c, 0x29, 0xe3, 0xc6, 0x4d])
    eth.set_ethertype(EtherType.IPV4)
    return eth.release(), pkt_bytes[-84:]


def grev0_4_chain(pkt_bytes):
    """gre_test.rs:255-287: a Gre header array with key_present, protocol type
    TRANS_ETH_BRIDGE, key 0xfde8."""
    pkt = tv.CursorMut(len(pkt_bytes))
    pkt.advance(14 + 20 + 8)
    hdr = tv.Gre.set_header_flags(tv.GRE_HEADER_TEMPLATE, key_present=True)
    gre = tv.Gre.prepend_header(pkt, hdr)
    gre.set_protocol_type(0x6558)
    gre.set_key(0x0000fde8)
    ip = tv.Ipv4.prepend_header(gre.release(), tv.IPV4_HEADER_TEMPLATE)
    ip.set_ident(0x0001)
    ip.set_ttl(64)
    ip.set_protocol(IpProtocol.GRE)
    ip.set_checksum(0x7073)
    ip.set_src_addr("1.2.3.4")
    ip.set_dst_addr("4.3.2.1")
    eth = tv.EtherFrame.prepend_header(ip.release(), tv.ETHER_FRAME_HEADER_TEMPLATE)
    eth.set_dst_addr([0x00, 0xae, 0xf3, 0x52, 0xaa, 0xd1])
    eth.set_src_addr([0x00, 0x02, 0x15, 0x37, 0xa2, 0x44])
    eth.set_ethertype(EtherType.IPV4)
    return eth.release(), pkt_bytes[42:]


REFERENCE_BUILDS = (("Vxlan2.dat", vxlan2_chain), ("gtp-u-1ext.dat", gtpu1_chain),
                    ("GREv0_4.dat", grev0_4_chain))


def reference_build_batch():
    frames, chains, payloads = [], [], []
    for name, fn in REFERENCE_BUILDS:
        f = oracle.load_dat(os.path.join(PKTS, name))
        c, p = fn(f)
        frames.append(f)
        chains.append(c)
        payloads.append(p)
    return frames, chain_batch(chains, payloads)


def test_reference_build_tests_give_their_captures():
    frames, (buf, offs, recs, tuns) = reference_build_batch()
    for flags in (0, 3):                                  # setter checksums / filled ones
        out, built = oracle.build_tunnel_batch(buf, len(frames), recs, tuns, flags, offsets=offs)
        assert built.all()
        for i, f in enumerate(frames):
            got = bytes(out[offs[i]:offs[i + 1]])
            assert got == f, (REFERENCE_BUILDS[i][0], flags,
                              [k for k in range(len(f)) if got[k] != f[k]][:8])


def test_captures_rebuilt_from_their_tunnel_getters():
    """Every capture with a decodable tunnel: zero the outer and tunnel header bytes the
    build writes, rebuild them from the parse's outer and tunnel records with both sums
    filled, and get the capture back where its stored checksums were valid."""
    names = [n for n in sorted(os.listdir(PKTS)) if n.endswith(".dat")]
    done = 0
    for name in names:
        f = oracle.load_dat(os.path.join(PKTS, name))
        o, t, i = oracle.tunnel_one(f, 3 | F_IPV6)
        if int(t["status"]) not in (TUN_STATUS["OK"], TUN_STATUS["INNER_UNKNOWN"]) or \
                int(t["inner_type"]) == 0x880b:
            continue
        buf = np.frombuffer(f, np.uint8).copy()
        ts = int(t["tun_off"])
        buf[:14] = 0
        buf[14:14 + 20] = 0
        buf[ts:ts + 4] = 0
        offs = np.array([0, len(f)], np.uint32)
        for flags in (0, 3):
            out, built = oracle.build_tunnel_batch(buf, 1, np.array([o]), np.array([t]), flags,
                                                   offsets=offs)
            assert built[0] == 1, name
            if flags == 0 or (int(o["ip_sum"]) == 0xffff and int(o["l4_sum"]) in (0, 0xffff)):
                assert bytes(out) == f, (name, flags)
        done += 1
    assert done >= 9


def test_tunnel_build_refusals():
    """A kind that does not match the outer protocol, a header past the frame or past
    RPKT_TUN_BUILD_MAX_END, an unknown kind: the frame is left untouched."""
    frames, (buf, offs, recs, tuns) = reference_build_batch()
    t2 = tuns.copy()
    t2["kind"] = [3, 3, 1]                                    # GRE on UDP (x2), VXLAN on GRE
    out, built = oracle.build_tunnel_batch(buf, 3, recs, t2, 3, offsets=offs)
    assert not built.any() and np.array_equal(out, buf)
    t2["kind"] = 7
    assert not oracle.build_tunnel_batch(buf, 3, recs, t2, 3, offsets=offs)[1].any()
    r2 = recs.copy()
    r2["n_vlan"] = 2                                           # pushes the headers along
    r2["ip_vhl"] = 0x4f                                        # 60-B IPv4 headers
    out, built = oracle.build_tunnel_batch(buf, 3, r2, tuns, 3, offsets=offs)
    assert built.all()                                         # VXLAN ends at 98, GTP 102, GRE 90
    r2 = recs.copy()
    r2["ethertype"] = 0x86dd                                   # IPv6 records whose upper layer
    r2["l4_off"] = [106, 92, 113]                              # starts past extension headers
    out, built = oracle.build_tunnel_batch(buf, 3, r2, tuns, 3, offsets=offs)
    assert built.tolist() == [0, 1, 0]                        # ends 122, 112 (<= 113), 121
