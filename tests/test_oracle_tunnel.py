"""The tunnel oracle (oracle/rpkt_oracle_tunnel.c) pinned by the reference's own tests:
every assert the reference makes on its VXLAN, GTP-U and GRE captures
(rpkt/tests/vlan_mpls_tests.rs:224-251, gtpv1_test.rs:199-231, 284-320, 377-412,
468-505, gre_test.rs:20-210) holds on the oracle's tunnel and inner records, and the
inner sums of the captures whose stored checksums are valid are 0xffff."""
import os

import numpy as np
import pytest

from oracle import oracle
from rpkt_amd.records import F_IPV6, STATUS, TUN_KIND, TUN_STATUS

HERE = os.path.dirname(os.path.abspath(__file__))
PKTS = os.path.join(HERE, "golden", "packets")
F6 = 3 | F_IPV6


def cap(name, flags=F6):
    return oracle.tunnel_one(oracle.load_dat(os.path.join(PKTS, name)), flags)


def test_vxlan_captures():
    """vlan_mpls_tests.rs:224-251: Vxlan1's flags, group_id 100, vni 3000001, and the inner
    EtherFrame (ethertype IPv4) parsed from vxlan.payload(); Vxlan2 the same header shape.
    Both inner frames are IPv4/ICMP with valid sums."""
    for name in ("Vxlan1.dat", "Vxlan2.dat"):
        o, t, i = cap(name)
        assert int(o["status"]) == STATUS["OK"] and int(o["dst_port"]) == 4789
        assert int(t["kind"]) == TUN_KIND["VXLAN"] and int(t["status"]) == TUN_STATUS["OK"]
        assert int(t["tun_off"]) == 14 + 20 + 8 and int(t["inner_off"]) == 14 + 20 + 8 + 8
        assert int(t["inner_type"]) == 0x6558
        assert int(i["ethertype"]) == 0x0800 and int(i["l3_off"]) == 50 + 14
        assert int(i["frame_len"]) == int(o["payload_len"]) - 8
        assert int(i["ip_sum"]) == 0xffff
    _, t, i = cap("Vxlan1.dat")
    h0, h1 = int(t["hdr0"]), int(t["hdr1"])
    assert h0 & 0x80 and h0 & 0x08 and (h0 >> 4) & 7 == 0          # gbp, vni_present, reserved_0
    assert h1 & 0x40 and h1 & 0x08 and h1 & 0x37 == 0               # dont_learn, policy_applied
    assert int(t["aux"]) == 100 and int(t["id"]) == 3000001         # group_id, vni
    assert int(i["status"]) == STATUS["L4_OTHER"] and int(i["ip_protocol"]) == 1   # ICMP inside
    assert int(i["l4_sum"]) == 0xffff                                   # the inner ICMP sum


@pytest.mark.parametrize("name,plen,seq,ext,ttl_proto", [
    ("gtp-u-1ext.dat", 92 + 8, 10461, 4, 1),           # gtpv1_test.rs:199-231 (ICMP inside)
    ("gtp-u-2ext.dat", 96 + 8, 10461, 8, 1),           # :284-320 (PDU number + UDP port)
])
def test_gtpu_extension_captures(name, plen, seq, ext, ttl_proto):
    o, t, i = cap(name)
    assert int(t["kind"]) == TUN_KIND["GTPU"] and int(t["status"]) == TUN_STATUS["OK"]
    h0 = int(t["hdr0"])
    assert h0 >> 5 == 1 and h0 & 0x4 and h0 & 0x2 and not h0 & 0x1   # E, S, no PN
    assert int(t["hdr1"]) == 255                                      # G_PDU
    assert int(t["id"]) == 1 and int(t["aux"]) == seq                 # teid, sequence
    ts = int(t["tun_off"])
    f = oracle.load_dat(os.path.join(PKTS, name))
    assert ((f[ts + 2] << 8) | f[ts + 3]) + 8 == plen                 # packet_len
    assert int(t["inner_off"]) == ts + 12 + ext
    assert int(t["inner_type"]) == 0x0800
    assert int(i["ip_protocol"]) == ttl_proto                         # Ipv4 protocol ICMP
    assert int(i["l3_off"]) == int(t["inner_off"])
    assert int(i["ip_sum"]) == 0xffff and int(i["l4_sum"]) == 0xffff  # inner ICMP valid
    if name == "gtp-u-2ext.dat":                                       # ExtUdpPort 1308
        p = int(t["inner_off"]) - 4
        assert (f[p + 1] << 8) | f[p + 2] == 1308


def test_gtpu_pdu_session_container():
    """gtpv1_test.rs:468-505: no sequence, teid 14872, PduSessionUp (UlPduSessionInfo,
    header_len 4, qfi 1), then an IPv4/TCP packet."""
    o, t, i = cap("gtp_pdu_session_container.dat")
    assert int(t["status"]) == TUN_STATUS["OK"] and int(t["id"]) == 14872
    assert not int(t["hdr0"]) & 0x2 and int(t["aux"]) == 0
    assert int(t["inner_off"]) == int(t["tun_off"]) + 12 + 4
    f = oracle.load_dat(os.path.join(PKTS, "gtp_pdu_session_container.dat"))
    assert f[int(t["tun_off"]) + 12 + 2] & 0x3f == 1                   # qos_flow_identifier
    assert int(i["status"]) == STATUS["OK"] and int(i["ip_protocol"]) == 6


def test_gtpu_nr_container_has_no_tpdu():
    """gtpv1_test.rs:377-412: NrUp DlDataDeliveryStatus, then an empty payload: no inner."""
    o, t, i = cap("gtp_nr_container.dat")
    assert int(t["kind"]) == TUN_KIND["GTPU"]
    assert int(t["status"]) == TUN_STATUS["INNER_UNKNOWN"] and int(t["inner_type"]) == 0
    assert int(i["status"]) == STATUS["NO_INNER"]
    assert int(t["inner_off"]) == int(o["payload_off"]) + int(o["payload_len"])


def test_gtp_c_is_not_a_tunnel():
    """gtp-c1 (port 2123, gtpv1_test.rs:22-34): the control plane carries no T-PDU."""
    o, t, i = cap("gtp-c1.dat")
    assert int(t["kind"]) == TUN_KIND["NONE"] and int(t["status"]) == TUN_STATUS["NONE"]
    assert int(i["status"]) == STATUS["NO_INNER"] and i.tobytes()[1:] == bytes(79)


def test_gre_captures():
    """gre_test.rs:20-99, 180-210: GREv0_1 (C bit, checksum 30719, inner IPv4 ttl 64 ident
    0x4c0f), GREv0_2 (4-B header, inner IPv4 whose protocol is GRE again: one level),
    GREv0_4 (K bit, key 0xfde8, transparent Ethernet bridging), GREv1_1 (PPTP: PPP)."""
    o, t, i = cap("GREv0_1.dat")
    assert int(o["l4_sum"]) == 0xffff                                  # the GRE checksum
    assert int(t["kind"]) == TUN_KIND["GRE"] and int(t["status"]) == TUN_STATUS["OK"]
    assert int(t["hdr0"]) & 0x80 and int(t["aux"]) == 30719 and int(t["inner_type"]) == 0x0800
    assert int(t["inner_off"]) == int(t["tun_off"]) + 8
    assert int(i["ip_ttl"]) == 64 and int(i["ip_ident"]) == 0x4c0f and int(i["ip_sum"]) == 0xffff
    o, t, i = cap("GREv0_2.dat")
    assert int(t["status"]) == TUN_STATUS["OK"] and int(t["inner_off"]) == int(t["tun_off"]) + 4
    assert int(i["ip_protocol"]) == 47 and int(i["status"]) == STATUS["L4_OTHER"]
    o, t, i = cap("GREv0_4.dat")
    assert int(t["hdr0"]) & 0x20 and int(t["id"]) == 0xfde8 and int(t["inner_type"]) == 0x6558
    assert int(t["inner_off"]) == int(t["tun_off"]) + 8
    o, t, i = cap("GREv1_1.dat")
    assert int(t["status"]) == TUN_STATUS["INNER_UNKNOWN"] and int(t["inner_type"]) == 0x880b
    assert int(t["id"]) & 0xffff == 6 and int(t["id"]) >> 16 == 0    # key_call_id, payload_len
    assert int(t["inner_off"]) == int(t["tun_off"]) + 12
    o, t, i = cap("GREv0_3.dat")
    assert int(o["l4_sum"]) == 0xffff and int(t["status"]) in (TUN_STATUS["OK"],
                                                              TUN_STATUS["INNER_UNKNOWN"])


def test_every_capture_inner_record_is_a_parse_of_its_bytes():
    """For every capture the inner record equals the parse of the tunnel payload's bytes
    (oracle_parse_one / parse_at_ip), offsets moved by inner_off; all statuses are known."""
    for name in sorted(os.listdir(PKTS)):
        f = oracle.load_dat(os.path.join(PKTS, name))
        for flags in (0, 3, F6):
            o, t, i = oracle.tunnel_one(f, flags)
            assert o.tobytes() == oracle.parse_one(f, flags).tobytes()
            assert int(t["status"]) in TUN_STATUS.values()
            if int(t["status"]) != TUN_STATUS["OK"]:
                assert int(i["status"]) == STATUS["NO_INNER"]
                continue
            a = int(t["inner_off"])
            if int(t["inner_type"]) == 0x6558:
                ref = oracle.parse_one(f[a:a + int(i["frame_len"])], flags)
                assert int(i["l3_off"]) == int(ref["l3_off"]) + a or int(ref["l3_off"]) == 0
            assert int(i["frame_len"]) <= len(f) - a


def test_truncations_and_fuzz_never_abort():
    """Every truncation of every tunnel capture, and random mutations of its tunnel
    header bytes, give known statuses (the oracle aborts on a cursor misuse)."""
    rng = np.random.default_rng(5)
    names = [n for n in sorted(os.listdir(PKTS)) if n.startswith(("Vxlan", "gtp", "GRE"))]
    for name in names:
        f = oracle.load_dat(os.path.join(PKTS, name))
        for cut in range(len(f) + 1):
            o, t, i = oracle.tunnel_one(f[:cut], F6)
            assert int(t["status"]) in TUN_STATUS.values()
        for _ in range(300):
            g = bytearray(f)
            for _ in range(3):
                g[int(rng.integers(34, min(len(g), 110)))] = int(rng.integers(0, 256))
            o, t, i = oracle.tunnel_one(bytes(g), F6)
            assert int(t["status"]) in TUN_STATUS.values()


def test_odd_tunnel_frames_decode():
    """tests/tunnel_frames.py's shapes (checksums made there from RFC 1071): VXLAN over
    IPv6 and over QinQ, GTP-U chains of 1..8 extension headers (a 9th is EXT_BAD), GTP-U
    and GRE over IPv6 with IPv6 inside, GRE transparent bridging: every level's sums valid."""
    import tunnel_frames as tf
    frames = tf.odd_frames(n=0)
    want = ["OK", "OK", "OK", "OK", "OK", "OK", "EXT_BAD", "OK", "OK", "OK", "OK"]
    for f, w in zip(frames, want):
        o, t, i = oracle.tunnel_one(f, F6)
        assert int(t["status"]) == TUN_STATUS[w], (w, t)
        assert int(o["l4_sum"]) in (0, 0xffff)
        if w == "OK":
            assert int(i["status"]) == STATUS["OK"] and int(i["l4_sum"]) == 0xffff, i
            assert int(i["ip_sum"]) in (0, 0xffff)
    o, t, i = oracle.tunnel_one(frames[5], F6)                # 8 extensions: past the window
    assert int(t["inner_off"]) > 128
    o, t, i = oracle.tunnel_one(frames[0], 3)                 # IPv6 outer without the flag
    assert int(o["status"]) == STATUS["NOT_IPV4"] and int(t["kind"]) == TUN_KIND["NONE"]
    o, t, i = oracle.tunnel_one(frames[7], 3)                 # IPv6 T-PDU without the flag
    assert int(t["kind"]) == TUN_KIND["NONE"]                 #   (outer IPv6 too)
    o, t, i = oracle.tunnel_one(frames[1], 3)
    assert int(o["n_vlan"]) == 2 and int(t["status"]) == TUN_STATUS["OK"]


def test_tunnel_flow_events_are_the_inner_or_outer_record_events():
    """oracle.tunnel_flow_events: a frame without a decoded tunnel gets exactly
    rpkt_gpu_parse_batch's event of its outer record; a tunnel frame the event of its inner
    record (its 5-tuple and length), which differs from the outer one."""
    from rpkt_amd import gen
    hb = gen.make_batch(14, 3000, seed=77)
    o, t, i = oracle.tunnel_batch(hb.frames, hb.n, F6, offsets=hb.offsets, stride=hb.stride,
                                  frame_len=hb.frame_len)
    ev = oracle.tunnel_flow_events(o, t, i, 8192)
    _, pev = oracle.parse_batch(hb.frames, hb.n, flags=F6, offsets=hb.offsets, stride=hb.stride,
                                frame_len=hb.frame_len, n_buckets=8192, flow_ev=True)
    tun = t["status"] == TUN_STATUS["OK"]
    assert tun.any() and (~tun).any()
    assert np.array_equal(ev[~tun], pev[~tun])
    assert np.array_equal(ev[tun] & 0xffffffff, i["frame_len"][tun].astype(np.uint64))
    assert (ev[tun] != pev[tun]).mean() > 0.9

