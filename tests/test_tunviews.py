"""The host tunnel views (rpkt_amd/tunviews.py) over the oracle's tunnel records, walked
as the reference's tests walk their captures, with the same asserts
(rpkt/tests/vlan_mpls_tests.rs:224-251, gtpv1_test.rs:199-231, 468-505,
gre_test.rs:20-99)."""
import os

import pytest

from oracle import oracle
from rpkt_amd.records import F_IPV6
from rpkt_amd.tunviews import (ExtContainer, ExtPduNumber, ExtUdpPort, Gre, Gtpv1, PduSessionUp,
                               TunnelPacket, UlPduSessionInfo, Vxlan)
from rpkt_amd.views import EtherFrame, EtherType, IpProtocol, Ipv4, Tcp, Udp

HERE = os.path.dirname(os.path.abspath(__file__))
PKTS = os.path.join(HERE, "golden", "packets")


def packet(name, flags=3 | F_IPV6):
    f = oracle.load_dat(os.path.join(PKTS, name))
    o, t, i = oracle.tunnel_one(f, flags)
    return TunnelPacket(o, t, i, f)


def test_vxlan1_chain():
    """vlan_mpls_tests.rs:224-251, assert for assert."""
    eth_pkt = EtherFrame.parse(packet("Vxlan1.dat")).unwrap()
    assert eth_pkt.ethertype() == EtherType.IPV4
    ip_pkt = Ipv4.parse(eth_pkt.payload()).unwrap()
    assert ip_pkt.protocol() == IpProtocol.UDP
    udp_pkt = Udp.parse(ip_pkt.payload()).unwrap()
    assert udp_pkt.dst_port() == 4789 and udp_pkt.src_port() == 45149
    vxlan_pkt = Vxlan.parse(udp_pkt.payload()).unwrap()
    assert vxlan_pkt.gbp_extention() and vxlan_pkt.vni_present()
    assert vxlan_pkt.dont_learn() and vxlan_pkt.policy_applied()
    assert (vxlan_pkt.reserved_0(), vxlan_pkt.reserved_1(), vxlan_pkt.reserved_2(),
            vxlan_pkt.reserved_3(), vxlan_pkt.reserved_4()) == (0, 0, 0, 0, 0)
    assert vxlan_pkt.group_id() == 100 and vxlan_pkt.vni() == 3000001
    eth_pkt = EtherFrame.parse(vxlan_pkt.payload()).unwrap()
    assert eth_pkt.ethertype() == EtherType.IPV4
    # beyond the reference test: the inner IPv4 header and its sum, from the inner record
    inner_ip = Ipv4.parse(eth_pkt.payload()).unwrap()
    assert inner_ip.protocol() == IpProtocol.ICMP and inner_ip.verify_checksum()


def test_gtp_u1_ext_chain():
    """gtpv1_test.rs:199-231: the GTPv1 getters, then the T-PDU (the reference walks
    ExtPduNumber::parse(gtp.payload()) -> Ipv4::parse(ext.payload()))."""
    eth = EtherFrame.parse(packet("gtp-u-1ext.dat")).unwrap()
    assert eth.ethertype() == EtherType.IPV4
    ipv4 = Ipv4.parse(eth.payload()).unwrap()
    assert ipv4.protocol() == IpProtocol.UDP
    udp = Udp.parse(ipv4.payload()).unwrap()
    assert udp.src_port() == 2152 and udp.dst_port() == 2152
    gtp = Gtpv1.parse(udp.payload()).unwrap()
    assert gtp.extention_header_present() and gtp.sequence_present() and not gtp.npdu_present()
    assert gtp.message_type() == 255                                   # G_PDU
    assert gtp.packet_len() == 92 + 8 and gtp.teid() == 1 and gtp.sequence() == 10461
    assert gtp.next_extention_header() == 0xc0                         # PDU_NUMBER
    assert gtp.payload().cursor() == gtp.buf.cursor() + 12             # the extension header
    ext = ExtPduNumber.parse(gtp.payload()).unwrap()
    assert ext.pdcp_number() == 2308 and ext.next_extention_header() == 0   # NO_EXTENTION
    ipv4 = Ipv4.parse(ext.payload()).unwrap()
    assert ipv4.protocol() == IpProtocol.ICMP and ipv4.verify_checksum()
    assert Ipv4.parse(gtp.t_pdu()).unwrap().buf.cursor() == ipv4.buf.cursor()


def test_gtp_u2_ext_chain():
    """gtpv1_test.rs:284-320: ExtPduNumber -> ExtUdpPort -> the T-PDU."""
    eth = EtherFrame.parse(packet("gtp-u-2ext.dat")).unwrap()
    udp = Udp.parse(Ipv4.parse(eth.payload()).unwrap().payload()).unwrap()
    gtp = Gtpv1.parse(udp.payload()).unwrap()
    assert gtp.next_extention_header() == 0xc0                         # PDU_NUMBER
    ext = ExtPduNumber.parse(gtp.payload()).unwrap()
    assert ext.pdcp_number() == 2308 and ext.next_extention_header() == 0x40   # UDP_PORT
    assert Ipv4.parse(ext.payload()).is_err()                          # not the T-PDU yet
    ext = ExtUdpPort.parse(ext.payload()).unwrap()
    assert ext.udp_port() == 1308 and ext.next_extention_header() == 0
    assert Ipv4.parse(ext.payload()).unwrap().verify_checksum()


def test_gtp_pdu_session_container_chain():
    """gtpv1_test.rs:468-505: no sequence, teid 14872, then IPv4 / TCP inside."""
    eth = EtherFrame.parse(packet("gtp_pdu_session_container.dat")).unwrap()
    udp = Udp.parse(Ipv4.parse(eth.payload()).unwrap().payload()).unwrap()
    gtp = Gtpv1.parse(udp.payload()).unwrap()
    assert gtp.teid() == 14872 and gtp.extention_header_present()
    assert gtp.packet_len() == 159 + 8 and gtp.next_extention_header() == 0x85
    pkt = PduSessionUp.group_parse(gtp.payload()).unwrap()
    assert isinstance(pkt, UlPduSessionInfo)
    assert pkt.qos_flow_identifier() == 1 and pkt.next_extention_header() == 0
    assert pkt.header_len() == 4
    ipv4 = Ipv4.parse(pkt.payload()).unwrap()
    assert ipv4.protocol() == IpProtocol.TCP
    tcp = Tcp.parse(ipv4.payload()).unwrap()
    assert tcp.payload().cursor() > tcp.buf.cursor()


def test_gtp_nr_container_chain():
    """gtpv1_test.rs:377-416: a G-PDU carrying only an NR RAN container (no T-PDU: the
    engine's tunnel status is not OK, the views still walk the header chain); the
    container's payload is empty."""
    eth = EtherFrame.parse(packet("gtp_nr_container.dat")).unwrap()
    udp = Udp.parse(Ipv4.parse(eth.payload()).unwrap().payload()).unwrap()
    gtp = Gtpv1.parse(udp.payload()).unwrap()
    assert not gtp.sequence_present() and gtp.packet_len() == 16 + 8 and gtp.teid() == 1
    assert gtp.next_extention_header() == 0x84                         # NR_RAN_CONTAINER
    c = ExtContainer.parse(gtp.payload()).unwrap()
    assert c.next_extention_header() == 0 and c.payload().remaining() == 0
    v = c.var_header_slice()              # DlDataDeliveryStatus (generated.rs:1802-1890)
    assert v[0] >> 4 == 1 and (v[0] >> 3) & 1 == 1                    # PDU type, highest_trans_nr_pdcp_sn_ind
    assert int.from_bytes(v[2:6], "big") == 0                          # buf_size_for_data_radio_bearer
    assert ExtPduNumber.parse(c.payload()).is_err()


def test_grev0_1_chain():
    """gre_test.rs:20-44, assert for assert."""
    eth = EtherFrame.parse(packet("GREv0_1.dat")).unwrap()
    ipv4 = Ipv4.parse(eth.payload()).unwrap()
    assert ipv4.protocol() == IpProtocol.GRE
    gre = Gre.parse(ipv4.payload()).unwrap()
    assert gre.header_len() == 8 and gre.checksum_present() and not gre.routing_present()
    assert not gre.sequence_present() and gre.recursion_control() == 0 and gre.flags() == 0
    assert gre.protocol_type() == EtherType.IPV4
    assert gre.checksum() == 30719 and gre.offset() == 0
    assert gre.verify_checksum()                                       # beyond the test
    ipv4 = Ipv4.parse(gre.payload()).unwrap()
    assert ipv4.ttl() == 64 and ipv4.ident() == 0x4c0f


def test_views_refuse_what_the_engine_did_not_decode():
    """Err where the reference parse fails or the dispatch does not reach the view: a
    non-tunnel UDP payload, the wrong tunnel kind, a cursor elsewhere."""
    eth = EtherFrame.parse(packet("Vxlan1.dat")).unwrap()
    udp = Udp.parse(Ipv4.parse(eth.payload()).unwrap().payload()).unwrap()
    assert Gtpv1.parse(udp.payload()).is_err() and Gre.parse(udp.payload()).is_err()
    assert Vxlan.parse(eth.payload()).is_err()
    eth = EtherFrame.parse(packet("gtp-c1.dat")).unwrap()
    udp = Udp.parse(Ipv4.parse(eth.payload()).unwrap().payload()).unwrap()
    assert Gtpv1.parse(udp.payload()).is_err()                         # GTP-C: no tunnel
    with pytest.raises(ValueError):
        Vxlan.parse(TunnelPacket(*oracle.tunnel_one(b"\0" * 20))).unwrap()
