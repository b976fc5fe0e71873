"""The host-side build views (rpkt_amd/txviews.py: rpkt's prepend_header + setters composing
rpkt_gpu_build_batch records) on CPU, through the build oracle (oracle/rpkt_oracle_build.c):
the reference's own build callers give the bytes their code writes, and the reference's
captures are rebuilt byte for byte from views driven by their parsed getters."""
import os

import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import txviews as tv
from rpkt_amd.records import F_IPV6, STATUS, ip6_block, is_ip6
from rpkt_amd.views import EtherType, IpProtocol

HERE = os.path.dirname(os.path.abspath(__file__))
PKTS = os.path.join(HERE, "golden", "packets")
F6 = 3 | F_IPV6


def build(chains, lens, flags, payloads=None):
    buf, offs, recs = tv.assemble(chains, lens, payloads)
    out, built = oracle.build_batch(buf, len(lens), recs, flags, offsets=offs)
    return out, offs, built, recs


def test_rpkt_build_bench_packet():
    """benches/rpkt/rpkt_build.rs:9-28 packet_build(buf, 66): the 42 header bytes its
    prepend_header + setters leave (IPv4 protocol never set: 0, so the UDP header is
    carried as written), with the lengths prepend_header takes from remaining()."""
    pkt = tv.CursorMut(42 + 66)
    pkt.advance(42)
    udp = tv.Udp.prepend_header(pkt, tv.UDP_HEADER_TEMPLATE)
    udp.set_src_port(60376)
    udp.set_dst_port(161)
    udp.set_checksum(0xbc86)
    ip = tv.Ipv4.prepend_header(udp.release(), tv.IPV4_HEADER_TEMPLATE)
    ip.set_ident(0x5c65)
    ip.set_ttl(128)
    ip.set_src_addr("192.168.29.58")
    ip.set_dst_addr("192.168.29.160")
    eth = tv.EtherFrame.prepend_header(ip.release(), tv.ETHER_FRAME_HEADER_TEMPLATE)
    eth.set_dst_addr([0x00, 0x0b, 0x86, 0x64, 0x8b, 0xa0])
    eth.set_src_addr([0x00, 0x50, 0x56, 0xae, 0x76, 0xf5])
    eth.set_ethertype(EtherType.IPV4)
    out, _, built, _ = build([eth.release().record()], [108], 0)
    want = bytes([0x00, 0x0b, 0x86, 0x64, 0x8b, 0xa0, 0x00, 0x50, 0x56, 0xae, 0x76, 0xf5,
                  0x08, 0x00,                                         # Ether
                  0x45, 0x00, 0x00, 94, 0x5c, 0x65, 0, 0, 128, 0, 0, 0,
                  192, 168, 29, 58, 192, 168, 29, 160,                # IPv4, packet_len 94
                  0xeb, 0xd8, 0x00, 0xa1, 0x00, 74, 0xbc, 0x86])      # UDP, length 74
    assert built[0] == 1 and bytes(out[:42]) == want


def loopback_tx_chain(src):
    """rpkt-dpdk/examples/loopback_tx.rs:70-99 fill_packet_template, then the per-packet
    source address of the flow (:160-170), 1500-B frames of PAYLOAD_BYTE."""
    pbuf = tv.CursorMut(1500)
    pbuf.advance(14 + 20 + 8)
    udp = tv.Udp.prepend_header(pbuf, tv.UDP_HEADER_TEMPLATE)
    udp.set_src_port(60376)
    udp.set_dst_port(161)
    udp.set_checksum(0)
    ip = tv.Ipv4.prepend_header(udp.release(), tv.IPV4_HEADER_TEMPLATE)
    ip.set_src_addr(src)
    ip.set_dst_addr("192.168.23.2")
    ip.set_protocol(IpProtocol.UDP)
    ip.set_ttl(128)
    ip.set_checksum(0)
    eth = tv.EtherFrame.prepend_header(ip.release(), tv.ETHER_FRAME_HEADER_TEMPLATE)
    eth.set_src_addr([0xac, 0xdc, 0xca, 0x79, 0xca, 0x86])
    eth.set_dst_addr([0xac, 0xdc, 0xca, 0x79, 0xe5, 0xc6])
    eth.set_ethertype(EtherType.IPV4)
    return eth.release().record()


def test_loopback_tx_frames_with_checksum_offload():
    """The loopback_tx frames over 64 flows, TX checksums filled (the offload the example
    requests): every frame parses OK with valid IPv4 and UDP sums and the set getters."""
    srcs = ["172.74.%d.%d" % (2 + k // 250, 2 + k % 250) for k in range(64)]
    chains = [loopback_tx_chain(s) for s in srcs]
    out, offs, built, _ = build(chains, [1500] * 64, 3, [b"\xae" * 1458] * 64)
    assert built.all()
    r = oracle.parse_batch(out, 64, 3, offsets=offs)
    assert (r["status"] == STATUS["OK"]).all()
    assert (r["ip_sum"] == 0xffff).all() and (r["l4_sum"] == 0xffff).all()
    assert (r["src_port"] == 60376).all() and (r["dst_port"] == 161).all()
    assert (r["ip_ttl"] == 128).all() and (r["ip_packet_len"] == 1486).all()
    assert [int(x) for x in r["ip_src"][:2]] == [(172 << 24) | (74 << 16) | (2 << 8) | 2,
                                                 (172 << 24) | (74 << 16) | (2 << 8) | 3]


def chain_from_capture(f, r):
    """A build chain that writes the capture's fixed headers: its parsed getters fed to
    the setters, extension headers and option bytes placed with move_back /
    var_header_slice_mut as the capture holds them."""
    l3, l4, end = int(r["l3_off"]), int(r["l4_off"]), len(f)
    six = bool(is_ip6(np.array([r]))[0])
    proto = int(r["ip_protocol"])
    pkt = tv.CursorMut(end)
    pkt.advance(l4 + (8 if proto == 17 else (int(r["l4_word6"]) >> 12) * 4))
    if proto == 17:
        l4v = tv.Udp.prepend_header(pkt)
        l4v.set_checksum(int(r["l4_checksum"]))
    else:
        t = bytearray(tv.TCP_HEADER_TEMPLATE)
        t[12] = (int(r["l4_word6"]) >> 8) & 0xf0
        l4v = tv.Tcp.prepend_header(pkt, bytes(t))
        l4v.set_seq_num(int(r["tcp_seq"]))
        l4v.set_ack_num(int(r["tcp_ack"]))
        l4v.set_reserved((int(r["l4_word6"]) >> 8) & 0xf)
        flags = int(r["l4_word6"]) & 0xff
        for bit, fn in enumerate((l4v.set_fin, l4v.set_syn, l4v.set_rst, l4v.set_psh,
                                  l4v.set_ack, l4v.set_urg, l4v.set_ece, l4v.set_cwr)):
            fn(bool(flags >> bit & 1))
        l4v.set_window_size(int(r["tcp_window"]))
        l4v.set_checksum(int(r["l4_checksum"]))
        l4v.set_urgent_pointer(int(r["tcp_urgent"]))
        l4v.var_header_slice_mut()[:] = f[l4 + 20:l4 + l4v.header_len()]
    l4v.set_src_port(int(r["src_port"]))
    l4v.set_dst_port(int(r["dst_port"]))
    buf = l4v.release()
    if six:
        if l4 > l3 + 40:
            buf.move_back(l4 - l3 - 40, f[l3 + 40:l4])            # the extension chain
        b = ip6_block(np.array([r]))[0]
        ip = tv.Ipv6.prepend_header(buf)
        v = int(b["ip6_vtcfl"])
        ip.set_traffic_class((v >> 20) & 0xff)
        ip.set_flow_label(v & 0xfffff)
        ip.set_next_header(int(b["ip6_next_header"]))
        ip.set_hop_limit(int(b["ip6_hop_limit"]))
        ip.set_src_addr(bytes(f[l3 + 8:l3 + 24]))
        ip.set_dst_addr(bytes(f[l3 + 24:l3 + 40]))
        if int(b["ip6_pdst_off"]) != l3 + 24:
            ip.set_pseudo_dst_offset(int(b["ip6_pdst_off"]))
    else:
        hdr = bytearray(tv.IPV4_HEADER_TEMPLATE)
        hdr[0] = 0x40 | (int(r["ip_vhl"]) & 0xf)
        ip = tv.Ipv4.prepend_header(buf, bytes(hdr))
        ip.set_dscp(int(r["ip_tos"]) >> 2)
        ip.set_ecn(int(r["ip_tos"]) & 3)
        ip.set_ident(int(r["ip_ident"]))
        fr = int(r["ip_frag"])
        ip.set_flag_reserved(fr >> 15)
        ip.set_dont_frag(bool(fr & 0x4000))
        ip.set_more_frag(bool(fr & 0x2000))
        ip.set_frag_offset(fr & 0x1fff)
        ip.set_ttl(int(r["ip_ttl"]))
        ip.set_protocol(proto)
        ip.set_checksum(int(r["ip_checksum"]))
        ip.set_src_addr(int(r["ip_src"]))
        ip.set_dst_addr(int(r["ip_dst"]))
        ip.var_header_slice_mut()[:] = f[l3 + 20:l4]
    buf = ip.release()
    for k in reversed(range(int(r["n_vlan"]))):                # innermost tag first
        v = tv.VlanFrame.prepend_header(buf)
        tci = int(r["vlan_tci"][k])
        v.set_priority(tci >> 13)
        v.set_dei_flag(bool(tci & 0x1000))
        v.set_vlan_id(tci & 0xfff)
        v.set_ethertype(int(r["vlan_ethertype"][k]))
        buf = v.release()
    eth = tv.EtherFrame.prepend_header(buf)
    eth.set_dst_addr(bytes(r["dst_addr"]))
    eth.set_src_addr(bytes(r["src_addr"]))
    eth.set_ethertype(int(r["ethertype"]))
    return eth.release().record()


def test_captures_rebuilt_from_their_getters():
    """Every capture that parses OK to UDP or TCP (IPv4 and IPv6, tagged, with IPv4 or
    TCP options and IPv6 extension headers) and whose length fields span it: a chain of
    views fed with its parsed getters rebuilds it byte for byte on a buffer holding only
    its payload; with the checksum fill, those whose stored sums verify are reproduced
    too."""
    names = sorted(f for f in os.listdir(PKTS) if f.endswith(".dat"))
    n = n6 = n_ck = 0
    for name in names:
        f = oracle.load_dat(os.path.join(PKTS, name))
        r = oracle.parse_one(f, F6)
        if r["status"] != STATUS["OK"] or int(r["ip_protocol"]) not in (6, 17):
            continue
        six = bool(is_ip6(np.array([r]))[0])
        l3 = int(r["l3_off"])
        span = l3 + (40 + int(ip6_block(np.array([r]))[0]["ip6_payload_len"]) if six
                     else int(r["ip_packet_len"]))
        if span != len(f) or (int(r["ip_protocol"]) == 17 and
                              int(r["l4_word6"]) != len(f) - int(r["l4_off"])):
            continue                                   # trailer bytes / a trimmed UDP length
        f = bytes(f)
        chain = chain_from_capture(f, r)
        pay = f[int(r["payload_off"]):]
        out, offs, built, _ = build([chain], [len(f)], 0, [pay])
        assert built[0] == 1 and bytes(out) == f, name
        ok = r["l4_sum"] == 0xffff and (six or r["ip_sum"] == 0xffff)
        if ok:
            out, offs, built, _ = build([chain], [len(f)], 3, [pay])
            assert bytes(out) == f, name
            n_ck += 1
        n += 1
        n6 += six
    assert n >= 15 and n6 >= 2 and n_ck >= 8, (n, n6, n_ck)


def test_vlan_ipv6_tcp_options_parse_back():
    """QinQ + IPv6 + a routing header (final address in the pseudo header) + TCP with
    options: built with both sums filled, the frame parses back to every value set."""
    pkt = tv.CursorMut(200)
    pkt.advance(14 + 8 + 40 + 24 + 28)
    t = bytearray(tv.TCP_HEADER_TEMPLATE)
    t[12] = 7 << 4                                           # doff 7: 8 option bytes
    tcp = tv.Tcp.prepend_header(pkt, bytes(t))
    tcp.set_src_port(443)
    tcp.set_dst_port(51000)
    tcp.set_seq_num(0x01020304)
    tcp.set_ack_num(0xa0b0c0d0)
    tcp.set_syn(True)
    tcp.set_ack(True)
    tcp.set_window_size(29200)
    tcp.var_header_slice_mut()[:] = bytes([2, 4, 0x05, 0xb4, 1, 1, 4, 2])   # MSS, NOP, SACK-perm
    final = bytes(range(0xf0, 0x100))
    rt = bytes([6, 2, 0, 1, 0, 0, 0, 0]) + final             # type 0, 1 segment left
    buf = tcp.release()
    buf.move_back(24, rt)
    ip = tv.Ipv6.prepend_header(buf)
    ip.set_traffic_class(0xb8)
    ip.set_flow_label(0x12345)
    ip.set_next_header(IpProtocol.IPV6_ROUTE)
    ip.set_hop_limit(63)
    ip.set_src_addr("2001:db8::1")
    ip.set_dst_addr("2001:db8::2")
    ip.set_pseudo_dst_offset(14 + 8 + 40 + 8)
    buf = ip.release()
    inner = tv.VlanFrame.prepend_header(buf)
    inner.set_vlan_id(100)
    inner.set_ethertype(EtherType.IPV6)
    outer = tv.VlanFrame.prepend_header(inner.release())
    outer.set_priority(5)
    outer.set_vlan_id(30)
    outer.set_ethertype(EtherType.VLAN)
    eth = tv.EtherFrame.prepend_header(outer.release())
    eth.set_dst_addr(bytes(range(6)))
    eth.set_src_addr(bytes(range(6, 12)))
    eth.set_ethertype(EtherType.QINQ)
    out, offs, built, recs = build([eth.release().record()], [200], 3, [b"\x5a" * 86])
    assert built[0] == 1
    r = oracle.parse_one(bytes(out), F6)
    b = ip6_block(np.array([r]))[0]
    assert r["status"] == STATUS["OK"] and r["l4_sum"] == 0xffff
    assert int(r["n_vlan"]) == 2 and [int(x) for x in r["vlan_tci"]] == [(5 << 13) | 30, 100]
    assert int(b["ip6_vtcfl"]) == (6 << 28) | (0xb8 << 20) | 0x12345
    assert int(b["ip6_hop_limit"]) == 63 and int(b["ip6_n_ext"]) == 1
    assert int(b["ip6_pdst_off"]) == 14 + 8 + 40 + 8
    assert (int(r["src_port"]), int(r["dst_port"]), int(r["tcp_seq"]), int(r["tcp_ack"])) == \
        (443, 51000, 0x01020304, 0xa0b0c0d0)
    assert int(r["l4_word6"]) == (7 << 12) | 0x12 and int(r["tcp_window"]) == 29200


def test_reference_asserts_hold():
    """prepend_header's and the setters' assert!s (a Rust panic) are AssertionError."""
    pkt = tv.CursorMut(64)
    pkt.advance(6)
    with pytest.raises(AssertionError):
        tv.Udp.prepend_header(pkt)                           # chunk_headroom() < 8
    pkt = tv.CursorMut(64)
    pkt.advance(18)
    v = tv.VlanFrame.prepend_header(pkt)
    with pytest.raises(AssertionError):
        v.set_vlan_id(0x1000)
    ip = tv.Ipv4.prepend_header(_headroom(40))
    with pytest.raises(AssertionError):
        ip.set_header_len(62)
    with pytest.raises(AssertionError):
        tv.Ipv6.prepend_header(_headroom(40)).set_flow_label(0x100000)


def _headroom(n):
    c = tv.CursorMut(n + 10)
    c.advance(n)
    return c


def test_cursor_mut_positions_and_panics():
    """cursors.rs:321-412 (test_cursor_mut and the *_too_much should_panic tests) on the
    host mirror: cursor / remaining after advance, move_back and trim_off over a 1000-B
    buffer, and an AssertionError where rpkt panics."""
    for c_pos in range(0, 1001, 37):
        c = tv.CursorMut(1000)
        c.advance(c_pos)
        assert c.cursor() == c_pos and c.remaining() == 1000 - c_pos
        c = tv.CursorMut(1000)
        c.advance(1000)
        c.move_back(c_pos)
        assert c.cursor() == 1000 - c_pos and c.remaining() == c_pos
    for c_pos in range(0, 701, 29):
        c = tv.CursorMut(1000)
        c.advance(300)
        c.trim_off(c_pos)
        assert c.remaining() == 1000 - 300 - c_pos
    for op in ("advance", "move_back", "trim_off"):
        c = tv.CursorMut(1000)
        c.advance(407)
        with pytest.raises(AssertionError):
            getattr(c, op)(10000)


def test_ipv6_without_l4_view_leaves_caller_bytes():
    """An IPv6 next_header of 17 with the UDP header written by the caller (move_back, no
    Udp view): the build writes no L4 header over it (prepend_header leaves those bytes),
    even with the L4 checksum fill requested; the next_header byte stays 17."""
    udp = bytes([0x12, 0x34, 0x00, 0x35, 0x00, 0x10, 0xab, 0xcd])    # hand-made UDP header
    pkt = tv.CursorMut(14 + 40 + 8 + 8)
    pkt.advance(14 + 40 + 8)
    buf = pkt
    buf.move_back(8, udp)
    ip = tv.Ipv6.prepend_header(buf)
    ip.set_next_header(IpProtocol.UDP)
    ip.set_hop_limit(9)
    ip.set_src_addr("2001:db8::5")
    ip.set_dst_addr("2001:db8::6")
    eth = tv.EtherFrame.prepend_header(ip.release())
    eth.set_ethertype(EtherType.IPV6)
    rec, extra = eth.release().record()
    b = ip6_block(np.array([rec]))[0]
    assert int(rec["ip_protocol"]) == 59 and int(b["ip6_next_header"]) == 17
    assert int(rec["l4_off"]) == 14 + 40 + 8 and int(b["ip6_n_ext"]) == 1
    out, _, built, _ = build([(rec, extra)], [70], 3, [b"\x77" * 8])
    assert built[0] == 1
    f = bytes(out[:70])
    assert f[54:62] == udp and f[20] == 17 and f[21] == 9 and f[62:70] == b"\x77" * 8


def test_ipv4_udp_protocol_without_udp_view_is_refused():
    """IPv4 protocol 17 with no Udp view: the record cannot say "leave the L4 bytes", so the
    host view refuses it rather than let the build overwrite them."""
    pkt = tv.CursorMut(14 + 20 + 8)
    pkt.advance(14 + 20)
    ip = tv.Ipv4.prepend_header(pkt, tv.IPV4_HEADER_TEMPLATE)
    ip.set_protocol(IpProtocol.UDP)
    eth = tv.EtherFrame.prepend_header(ip.release(), tv.ETHER_FRAME_HEADER_TEMPLATE)
    eth.set_ethertype(EtherType.IPV4)
    with pytest.raises(ValueError):
        eth.release().record()


def test_ipv6_build_checksums_match_rfc8200_fixture():
    """The IPv6 build's L4 checksum fill against frames whose checksums were worked out
    from RFC 8200 section 8.1 + RFC 1071 alone (tests/golden/make_ip6_tx_golden.py, no
    engine or oracle code): each parses with a valid sum, and a build from its own parse
    record with the checksum field zeroed writes it back byte for byte (the reference has no
    IPv6 pseudo-header code: this pins the extension to the RFC, not to the oracle)."""
    import json
    cases = json.load(open(os.path.join(HERE, "golden", "ip6_tx.json")))
    for c in cases:
        f = bytes.fromhex(c["frame"])
        r = oracle.parse_one(f, F6)
        assert r["status"] == STATUS["OK"] and r["l4_sum"] == 0xffff, c["kind"]
        assert int(r["l4_checksum"]) == c["checksum"]
        z = bytearray(f)
        ck = int(r["l4_off"]) + (6 if c["kind"] == "udp" else 16)
        z[ck:ck + 2] = b"\0\0"
        buf = np.frombuffer(bytes(z), np.uint8)
        offs = np.array([0, len(f)], np.uint32)
        out, built = oracle.build_batch(buf, 1, np.array([r]), 3, offsets=offs)
        assert built[0] == 1 and bytes(out) == f, c
