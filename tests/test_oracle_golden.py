"""Pin the CPU oracle against the reference's own fixtures and asserted values.

Each check below restates an assert from the reference's tests (cited in
tests/golden/expected.json) or a checksum property of the captured frames.
Runs on CPU only.
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle
from rpkt_amd.records import STATUS
from rpkt_amd.views import EtherFrame, VlanFrame, Ipv4, Udp, Tcp, Packet, EtherType, IpProtocol

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
PKTS = os.path.join(GOLD, "packets")
with open(os.path.join(GOLD, "expected.json")) as fh:
    EXPECTED = json.load(fh)

# the l4 / ip sums of the offload-captured (invalid) frames.
APPENDIX_A_INVALID = {
    "bench_frame.dat": {"ip_sum": 0xde00, "l4_sum": 0xb49d},
}


def derived(rec, key):
    vhl, frag, w6 = int(rec["ip_vhl"]), int(rec["ip_frag"]), int(rec["l4_word6"])
    d = {
        "ip_header_len": (vhl & 0xf) * 4, "ip_version": vhl >> 4,
        "ip_dscp": int(rec["ip_tos"]) >> 2, "ip_ecn": int(rec["ip_tos"]) & 3,
        "ip_flag_reserved": frag >> 15, "ip_dont_frag": (frag >> 14) & 1,
        "ip_more_frag": (frag >> 13) & 1, "ip_frag_offset": frag & 0x1fff,
        "tcp_header_len": (w6 >> 12) * 4, "tcp_flags": w6 & 0xff,
        "vlan0_id": int(rec["vlan_tci"][0]) & 0xfff,
        "vlan0_priority": int(rec["vlan_tci"][0]) >> 13,
        "vlan0_dei": (int(rec["vlan_tci"][0]) >> 12) & 1,
        "vlan0_ethertype": int(rec["vlan_ethertype"][0]),
        "vlan1_id": int(rec["vlan_tci"][1]) & 0xfff,
        "vlan1_priority": int(rec["vlan_tci"][1]) >> 13,
        "vlan1_dei": (int(rec["vlan_tci"][1]) >> 12) & 1,
        "vlan1_ethertype": int(rec["vlan_ethertype"][1]),
    }
    if key in d:
        return d[key]
    v = rec[key]
    if isinstance(v, np.ndarray):
        return [int(x) for x in v]
    return int(v)


@pytest.mark.parametrize("name", sorted(EXPECTED))
def test_fixture_getters(name):
    frame = oracle.load_dat(os.path.join(PKTS, name))
    rec = oracle.parse_one(frame, flags=3)
    exp = EXPECTED[name]
    assert int(rec["status"]) == STATUS[exp["status"]], name
    assert int(rec["frame_len"]) == len(frame)
    for k, v in exp.items():
        if k in ("cite", "status", "sums", "l4_sum"):
            continue
        assert derived(rec, k) == v, (name, k)
    sums = exp.get("sums")
    if sums == "valid":
        assert int(rec["ip_sum"]) == 0xffff and int(rec["l4_sum"]) == 0xffff, name
    elif sums == "ip_valid":
        assert int(rec["ip_sum"]) == 0xffff and int(rec["l4_sum"]) == 0, name
    elif sums in ("ip_valid_l4_invalid", "ip_valid_udp_zero"):
        assert int(rec["ip_sum"]) == 0xffff
        assert int(rec["l4_sum"]) == exp["l4_sum"], name
    elif sums == "invalid":
        assert int(rec["ip_sum"]) == APPENDIX_A_INVALID[name]["ip_sum"]
        assert int(rec["l4_sum"]) == APPENDIX_A_INVALID[name]["l4_sum"]


def test_every_fixture_parses_without_abort():
    for f in sorted(os.listdir(PKTS)):
        frame = oracle.load_dat(os.path.join(PKTS, f))
        rec = oracle.parse_one(frame, flags=3)
        assert int(rec["status"]) in STATUS.values()
        for cut in range(0, len(frame) + 1, 7):       # every truncation is a clean status
            r = oracle.parse_one(frame[:cut], flags=3)
            assert int(r["status"]) in STATUS.values()


def test_views_read_like_reference_bench():
    """benches/rpkt/rpkt_parse.rs:62-106 through the host views."""
    frame = oracle.load_dat(os.path.join(PKTS, "bench_frame.dat"))
    rec = oracle.parse_one(frame, flags=3)
    eth = EtherFrame.parse(Packet(rec, frame)).unwrap()
    assert eth.ethertype() == EtherType.IPV4
    assert eth.dst_addr() == frame[0:6] and eth.src_addr() == frame[6:12]
    ip = Ipv4.parse(eth.payload()).unwrap()
    assert ip.protocol() == IpProtocol.UDP
    assert ip.src_addr() == "192.168.29.58" and ip.dst_addr() == "192.168.29.160"
    assert ip.checksum() == 0x0000 and ip.ident() == 0x5c65
    udp = Udp.parse(ip.payload()).unwrap()
    assert udp.src_port() == 60376 and udp.dst_port() == 161
    assert udp.packet_len() == 74 and udp.checksum() == 0xbc86
    payload = udp.payload()
    assert payload.chunk() == frame[42:108]
    assert Tcp.parse(ip.payload()).is_err()
    assert not ip.verify_checksum() and not udp.verify_checksum()


def test_views_qinq_chain():
    """rpkt/tests/vlan_mpls_tests.rs:96-130 through the host views."""
    frame = oracle.load_dat(os.path.join(PKTS, "QinQ_802.1_AD.dat"))
    rec = oracle.parse_one(frame, flags=3)
    eth = EtherFrame.parse(Packet(rec, frame)).unwrap()
    assert eth.ethertype() == EtherType.QINQ
    q = VlanFrame.parse(eth.payload()).unwrap()
    assert q.vlan_id() == 30 and q.ethertype() == EtherType.VLAN
    v = VlanFrame.parse(q.payload()).unwrap()
    assert v.priority() == 0 and v.dei_flag() is False and v.vlan_id() == 100
    assert v.ethertype() == EtherType.IPV4
    assert Ipv4.parse(q.payload()).is_err()          # IPv4 is after the inner tag
    ip = Ipv4.parse(v.payload()).unwrap()
    assert ip.version() == 4 and ip.header_len() == 20 and ip.packet_len() == 1474
    assert ip.ttl() == 255 and ip.protocol() == 253 and ip.checksum() == 0xddbf
    assert len(ip.payload().chunk()) == 1454
    assert ip.verify_checksum()


def test_views_tcp_options():
    """rpkt/tests/tcp_test.rs:17-43 through the host views."""
    frame = oracle.load_dat(os.path.join(PKTS, "TcpPacketWithOptions.dat"))
    rec = oracle.parse_one(frame, flags=3)
    eth = EtherFrame.parse(Packet(rec, frame)).unwrap()
    ip = Ipv4.parse(eth.payload()).unwrap()
    tcp = Tcp.parse(ip.payload()).unwrap()
    assert tcp.src_port() == 44147 and tcp.dst_port() == 80
    assert tcp.seq_num() == 777047406 and tcp.ack_num() == 3761117865
    assert tcp.header_len() - 20 == 12
    assert (tcp.cwr(), tcp.ece(), tcp.urg(), tcp.ack(), tcp.psh(), tcp.rst(), tcp.syn(),
            tcp.fin()) == (False, False, False, True, True, False, False, False)
    assert tcp.window_size() == 913 and tcp.checksum() == 0xac20 and tcp.urgent_pointer() == 0
    assert tcp.payload().cursor() == 14 + 20 + 32


# ---- checksum.rs known answers -------------------------------------------------

def test_from_slice_basic():
    assert oracle.from_slice(b"") == 0
    assert oracle.from_slice(b"\x00\x01") == 1
    assert oracle.from_slice(b"\xff") == 0xff00            # odd tail << 8, checksum.rs:57-59
    assert oracle.from_slice(b"\xff\xff\x00\x01") == 1     # end-around carry
    assert oracle.from_slice(b"\x00\x00" * 40) == 0        # zero only for all-zero input
    assert oracle.from_slice(b"\xff\xff" * 3) == 0xffff


def test_from_buf_matches_from_slice_for_any_chunking():
    rng = np.random.default_rng(7)
    for trial in range(200):
        n = int(rng.integers(0, 300))
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        cuts = sorted(set(int(c) for c in rng.integers(0, n + 1, int(rng.integers(0, 6)))))
        segs, prev = [], 0
        for c in cuts + [n]:
            segs.append(data[prev:c])
            prev = c
        assert oracle.from_buf(segs) == oracle.from_slice(data), (trial, cuts)


def test_combine_is_order_free_and_matches_concatenation():
    rng = np.random.default_rng(8)
    for _ in range(200):
        a = rng.integers(0, 256, 2 * int(rng.integers(0, 40)), dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, int(rng.integers(0, 80)), dtype=np.uint8).tobytes()
        assert oracle.combine([oracle.from_slice(a), oracle.from_slice(b)]) == \
            oracle.from_slice(a + b)


def test_icmp_style_roundtrip():
    """Stamping the complement of the sum makes the sum 0xffff (the KAT pattern of
    rpkt/tests/icmpv4_test.rs:82-96)."""
    rng = np.random.default_rng(9)
    for _ in range(100):
        n = 2 * int(rng.integers(2, 200))
        data = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
        data[2:4] = b"\x00\x00"
        ck = (~oracle.from_slice(bytes(data))) & 0xffff
        data[2:4] = bytes([ck >> 8, ck & 0xff])
        assert oracle.from_slice(bytes(data)) == 0xffff


def test_views_group_parse_dot3():
    """rpkt/tests/eth_and_arp_test.rs:114-142: EtherGroup::group_parse -> EtherDot3Frame."""
    from rpkt_amd.views import EtherGroup, EtherDot3Frame
    frame = oracle.load_dat(os.path.join(PKTS, "EthDot3.dat"))
    rec = oracle.parse_one(frame, flags=3)
    d3 = EtherGroup.group_parse(Packet(rec, frame)).unwrap()
    assert isinstance(d3, EtherDot3Frame)
    assert d3.src_addr() == bytes.fromhex("0013f7115edb")
    assert d3.dst_addr() == bytes.fromhex("0180c2000000")
    assert d3.payload_len() == 38
    llc = d3.payload().chunk()
    assert llc[0] == 0x42 and llc[1] == 0x42 and llc[2] == 0x03   # BPDU dsap/ssap, control
    assert len(llc) - 3 == 35
    # an Ethernet II frame dispatches to EtherFrame
    f2 = oracle.load_dat(os.path.join(PKTS, "bench_frame.dat"))
    assert isinstance(EtherGroup.group_parse(Packet(oracle.parse_one(f2), f2)).unwrap(),
                      EtherFrame)


def test_views_vlan_group_parse_dot3():
    """rpkt/tests/llc_test.rs:39-61: VlanGroup::group_parse -> VlanDot3Frame."""
    from rpkt_amd.views import VlanGroup, VlanDot3Frame
    frame = oracle.load_dat(os.path.join(PKTS, "llc_vlan.dat"))
    rec = oracle.parse_one(frame, flags=3)
    eth = EtherFrame.parse(Packet(rec, frame)).unwrap()
    assert eth.ethertype() == EtherType.VLAN
    vd = VlanGroup.group_parse(eth.payload()).unwrap()
    assert isinstance(vd, VlanDot3Frame) and vd.payload_len() == 357
    llc = vd.payload().chunk()
    assert (llc[0], llc[1], llc[2]) == (0xaa, 0xaa, 0x03)


BENCH_WANT = ((192 << 24) | (168 << 16) | (29 << 8) | 58, (192 << 24) | (168 << 16) | (29 << 8) | 160,
              0x0000, 0x5c65, 60376, 161, 74, 0xbc86)     # benches/rpkt/rpkt_parse.rs:62-80


def test_packet_l4_on_bench_frame():
    """Config 1's harness body (`packet_l4`, rpkt_parse.rs:62-80) holds on the reference's
    own 110-B frame with the values it asserts, and fails on any other value."""
    frame = oracle.load_dat(os.path.join(PKTS, "bench_frame.dat"))
    assert oracle.packet_l4(frame, BENCH_WANT) == 0
    for k in range(len(BENCH_WANT)):
        w = list(BENCH_WANT)
        w[k] ^= 1
        assert oracle.packet_l4(frame, tuple(w)) != 0, k
    assert oracle.packet_l4(frame[:40], BENCH_WANT) != 0          # Udp::parse fails


def config1_want(hb):
    """The values config 1's frames carry (rpkt_build.rs:13-27 headers), for packet_l4."""
    r = oracle.parse_batch(hb.frames, hb.n, flags=3, stride=hb.stride)
    keys = ("ip_src", "ip_dst", "ip_checksum", "ip_ident", "src_port", "dst_port", "l4_word6",
            "l4_checksum")
    assert all((r[k] == r[k][0]).all() for k in keys)            # 1000 identical frames
    return tuple(int(r[k][0]) for k in keys)


def test_packet_l4_loop_over_config1():
    from rpkt_amd import gen
    hb = gen.make_batch(1)
    want = config1_want(hb)
    assert want[6] == 30 and want[4] == 60376
    assert oracle.packet_l4_loop(hb.frames, hb.n, hb.stride, hb.frame_len or hb.stride, 3,
                                 want) == 0
    bad = list(want)
    bad[3] ^= 0x100
    assert oracle.packet_l4_loop(hb.frames, hb.n, hb.stride, hb.frame_len or hb.stride, 2,
                                 tuple(bad)) == 2 * hb.n


def test_cursor_positions_and_panics():
    """cursors.rs:288-320 (test_cursor) and its *_too_much should_panic tests on the host
    view's Cursor over a 1000-B frame: cursor / remaining / chunk after advance, move_back
    and trim_off; an AssertionError where rpkt panics."""
    from rpkt_amd import views
    from rpkt_amd.records import REC_DTYPE
    rec = np.zeros(1, dtype=REC_DTYPE)[0]
    rec["frame_len"] = 1000
    b = bytes([10]) * 1000
    for c_pos in range(0, 1001, 41):
        c = views.Packet(rec, b)
        c.advance(c_pos)
        assert c.cursor() == c_pos and c.remaining() == 1000 - c_pos and c.chunk() == b[c_pos:]
        c = views.Packet(rec, b)
        c.advance(1000)
        c.move_back(c_pos)
        assert c.cursor() == 1000 - c_pos and c.remaining() == c_pos
        assert c.chunk() == b[1000 - c_pos:]
    for c_pos in range(0, 701, 23):
        c = views.Packet(rec, b)
        c.advance(300)
        c.trim_off(c_pos)
        assert c.remaining() == 700 - c_pos and c.chunk() == b[300:1000 - c_pos]
    for op in ("advance", "move_back", "trim_off"):
        c = views.Packet(rec, b)
        c.advance(407)
        with pytest.raises(AssertionError):
            getattr(c, op)(10000)
    c = views.Packet(rec, b)
    c.advance(0)
    assert not views.EtherFrame.parse(c).is_ok()          # a moved cursor is no parse start


def test_icmp_checksum_kat_and_relation_to_from_slice():
    """rpkt/tests/icmpv4_test.rs:82-96: the Echo Request's checksum is non-zero, and the
    message carrying it checks to 0.  calculate_icmp_checksum(d) == !from_slice(d) on any
    non-empty slice (so a record's ICMP l4_sum of 0xffff <=> the reference's check returns
    0), and the empty slice, where the reference panics, is refused."""
    import numpy as np
    data = bytearray([0x08, 0x00, 0x00, 0x00, 0x12, 0x34, 0x00, 0x01])
    ck = oracle.icmp_checksum(data)
    assert ck != 0
    data[2], data[3] = ck >> 8, ck & 0xff
    assert oracle.icmp_checksum(data) == 0
    assert oracle.from_slice(bytes(data)) == 0xffff
    assert oracle.icmp_checksum(b"") is None
    rng = np.random.default_rng(11)
    for n in list(range(1, 40)) + [1499, 1500, 65535]:
        for _ in range(3):
            d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            assert oracle.icmp_checksum(d) == (~oracle.from_slice(d)) & 0xffff, n
    assert oracle.icmp_checksum(b"\xff" * 4) == 0 and oracle.icmp_checksum(b"\0" * 6) == 0xffff


def test_icmp_and_gre_sums_in_records():
    """IPv4 protocol 1 and GRE-with-checksum frames (status L4_OTHER) carry the sum of
    their IP payload in l4_sum under RPKT_F_L4_SUM: the reference's ICMP captures
    (ipv4_test.rs IPv4Option1/2/6/7) and GREv0_1 (checksum 30719, gre_test.rs:35-41) and
    GREv0_3 verify as 0xffff; GRE without the C bit and every frame without the flag carry
    0; an empty ICMP payload is RPKT_S_ICMP_EMPTY."""
    for name in ("IPv4Option1.dat", "IPv4Option2.dat", "IPv4Option6.dat", "IPv4Option7.dat",
                 "GREv0_1.dat", "GREv0_3.dat"):
        f = oracle.load_dat(os.path.join(PKTS, name))
        r = oracle.parse_one(f, flags=3)
        assert int(r["status"]) == STATUS["L4_OTHER"] and int(r["l4_sum"]) == 0xffff, name
        assert int(oracle.parse_one(f, flags=1)["l4_sum"]) == 0
        if int(r["ip_protocol"]) == 1:
            msg = f[int(r["l4_off"]):int(r["l3_off"]) + int(r["ip_packet_len"])]
            assert oracle.icmp_checksum(msg) == 0, name
    g = oracle.load_dat(os.path.join(PKTS, "GREv0_1.dat"))
    gre = g[int(oracle.parse_one(g, 3)["l4_off"]):]
    assert (gre[4] << 8) | gre[5] == 30719                     # gre_test.rs:41
    for name in ("GREv0_2.dat", "GREv0_4.dat", "GREv1_1.dat"):   # no checksum_present
        r = oracle.parse_one(oracle.load_dat(os.path.join(PKTS, name)), flags=3)
        assert int(r["l4_sum"]) == 0, name
    # an ICMP packet of just its IPv4 header: the empty message
    f = bytearray(oracle.load_dat(os.path.join(PKTS, "IPv4Option6.dat")))
    ihl = (f[14] & 0xf) * 4
    f[16:18] = ihl.to_bytes(2, "big")
    r = oracle.parse_one(bytes(f[:14 + ihl]), flags=3)
    assert int(r["status"]) == STATUS["ICMP_EMPTY"] and int(r["l4_sum"]) == 0
    assert int(r["ip_ttl"]) == 64 and int(r["l4_off"]) == 14 + ihl
