"""Host-side header views over engine records — the rpkt API surface for the path.

The reference exposes header views over a byte buffer (`T: Buf`) with
`parse(buf) -> Result<View, buf>`, getters and `payload()`:
  EtherFrame  rpkt/src/ether/generated.rs:17-67
  VlanFrame   rpkt/src/vlan/generated.rs:15-69
  Ipv4        rpkt/src/ipv4/generated.rs:17-127, 269-288
  Udp         rpkt/src/udp/generated.rs:13-76
  Tcp         rpkt/src/tcp/generated.rs:16-131
  Ipv6 and its extension headers (RPKT_F_IPV6 records)
              rpkt/src/ipv6/generated.rs:22-216, 224-999
The engine already walked that chain on the GPU and left one rpkt_rec_t per
frame; these classes re-expose it under the same names, argument meaning and
Ok/Err behaviour, so code written against rpkt's chain reads the same:

    eth = EtherFrame.parse(Packet(rec)).unwrap()
    assert eth.ethertype() == EtherType.IPV4
    ip = Ipv4.parse(eth.payload()).unwrap()
    udp = Udp.parse(ip.payload()).unwrap()

`parse` returns Ok(view) exactly when the reference `parse` at that position
returned Ok for this frame, and Err(buf) otherwise (buf = the unchanged
cursor, as in ipv4/generated.rs:37,48).  Payload cursors carry (offset, len)
within the frame; `chunk()` needs the frame bytes to have been supplied.
"""
import ipaddress

import numpy as np

from .records import STATUS, MAX_VLAN, ip6_block, is_ip6


class EtherType:
    """rpkt/src/ether/mod.rs:12-36"""
    ARP = 0x0806
    IPV4 = 0x0800
    IPV6 = 0x86DD
    VLAN = 0x8100
    QINQ = 0x88a8
    MPLS = 0x8847
    PPPOE_SESSION = 0x8864
    PPPOE_DISCOVERY = 0x8863
    PPP = 0x880b
    TRANS_ETH_BRIDGE = 0x6558


class IpProtocol:
    """rpkt/src/ipv4/mod.rs:107-155 (subset on the path + common values)"""
    IPV6_HOP_BY_HOP_OPTS = 0
    ICMP = 1
    IGMP = 2
    IPIP = 4
    TCP = 6
    UDP = 17
    IPV6_ROUTE = 43
    IPV6_FRAG = 44
    GRE = 47
    ESP = 50
    AH = 51
    ICMPV6 = 58
    IPV6_NO_NXT = 59
    IPV6_DEST_OPTS = 60


class Result:
    __slots__ = ("_ok", "_v")

    def __init__(self, ok, v):
        self._ok, self._v = ok, v

    def is_ok(self):
        return self._ok

    def is_err(self):
        return not self._ok

    def unwrap(self):
        if not self._ok:
            raise ValueError("called unwrap() on an Err value (status %s)"
                             % _status_name(self._v))
        return self._v

    def unwrap_err(self):
        if self._ok:
            raise ValueError("called unwrap_err() on an Ok value")
        return self._v


def _status_name(v):
    from .records import STATUS_NAME
    try:
        return STATUS_NAME[int(v.rec["status"])]
    except Exception:
        return "?"


def Ok(v):
    return Result(True, v)


def Err(v):
    return Result(False, v)


class Cursor:
    """Position in the frame the chain has reached (cursors.rs:34-60): `stage`
    names which header starts here, `cursor()` its frame offset."""
    __slots__ = ("rec", "frame", "stage", "vlan_idx", "off", "length")

    def __init__(self, rec, frame, stage, vlan_idx, off, length):
        self.rec, self.frame, self.stage = rec, frame, stage
        self.vlan_idx, self.off, self.length = vlan_idx, off, length

    def cursor(self):
        return self.off

    def remaining(self):
        return self.length

    # The raw moves of cursors.rs Cursor (:63-99), in place as rpkt's `&mut self`
    # methods: the position leaves the parsed chain (a header view parses only where the
    # record placed one), so a moved cursor's stage is "raw".  rpkt panics past the
    # bounds; here an AssertionError.
    def advance(self, n):
        assert 0 <= n <= self.length, "advance past the end"
        self.stage, self.off, self.length = "raw", self.off + n, self.length - n

    def move_back(self, n):
        assert 0 <= n <= self.off, "move_back past the start"
        self.stage, self.off, self.length = "raw", self.off - n, self.length + n

    def trim_off(self, n):
        assert 0 <= n <= self.length, "trim_off past the cursor"
        self.stage, self.length = "raw", self.length - n

    def chunk(self):
        if self.frame is None:
            raise ValueError("frame bytes were not supplied to Packet()")
        return bytes(self.frame[self.off:self.off + self.length])


def Packet(rec, frame=None):
    """Cursor::new(frame) for one parsed frame: the start of the chain."""
    return Cursor(rec, frame, "ether", 0, 0, int(rec["frame_len"]))


def _st(rec):
    return int(rec["status"])


_IP_FAIL = {STATUS[k] for k in ("IP_SHORT", "IP_BAD_IHL", "IP_IHL_GT_LEN", "IP_TOT_LT_IHL",
                                 "IP_TOT_GT_LEN")}
_PRE_IP = {STATUS["ETH_SHORT"], STATUS["VLAN_SHORT"], STATUS["NOT_IPV4"]} | _IP_FAIL
_IP6_FAIL = {STATUS["IP6_SHORT"], STATUS["IP6_BAD_LEN"]}


def _rec_is_ip6(rec):
    return bool(is_ip6(np.asarray(rec).reshape(1))[0])


class EtherFrame:
    def __init__(self, buf):
        self.buf, self.rec = buf, buf.rec

    @staticmethod
    def parse(buf):
        """ether/generated.rs:34-41 — Err iff chunk_len < 14."""
        if buf.stage != "ether" or _st(buf.rec) == STATUS["ETH_SHORT"]:
            return Err(buf)
        return Ok(EtherFrame(buf))

    def dst_addr(self):
        return bytes(int(x) for x in self.rec["dst_addr"])

    def src_addr(self):
        return bytes(int(x) for x in self.rec["src_addr"])

    def ethertype(self):
        return int(self.rec["ethertype"])

    def payload(self):
        """ether/generated.rs:63-67 — advance(14) (from the cursor: an inner frame of a
        tunnel starts past the outer headers, rpkt_amd.tunviews)."""
        b = self.buf
        return Cursor(b.rec, b.frame, "l3", 0, b.off + 14, b.length - 14)


class EtherDot3Frame:
    """IEEE 802.3 frame: the type field is a payload length (ether/generated.rs:137-200)."""

    def __init__(self, buf):
        self.buf, self.rec = buf, buf.rec

    @staticmethod
    def parse(buf):
        """Err iff chunk_len < 14 or payload_len + 14 > remaining (ether/generated.rs:162-173)."""
        rec = buf.rec
        if buf.stage != "ether" or _st(rec) == STATUS["ETH_SHORT"]:
            return Err(buf)
        if int(rec["ethertype"]) + 14 > buf.length:
            return Err(buf)
        return Ok(EtherDot3Frame(buf))

    def dst_addr(self):
        return bytes(int(x) for x in self.rec["dst_addr"])

    def src_addr(self):
        return bytes(int(x) for x in self.rec["src_addr"])

    def payload_len(self):
        return int(self.rec["ethertype"])

    def payload(self):
        b = self.buf
        return Cursor(b.rec, b.frame, "dot3", 0, 14, self.payload_len())


class EtherGroup:
    """EtherGroup::group_parse (ether/generated.rs:292-302): Ethernet II when the
    type field is >= 1536, IEEE 802.3 when <= 1500, Err otherwise."""

    @staticmethod
    def group_parse(buf):
        rec = buf.rec
        if buf.stage != "ether" or _st(rec) == STATUS["ETH_SHORT"]:
            return Err(buf)
        v = int(rec["ethertype"])
        if v >= 1536:
            return EtherFrame.parse(buf)
        if v <= 1500:
            return EtherDot3Frame.parse(buf)
        return Err(buf)


class VlanDot3Frame:
    """802.1Q tag whose type field is a payload length (vlan/generated.rs:153-205)."""

    def __init__(self, buf):
        self.buf, self.rec, self.i = buf, buf.rec, buf.vlan_idx

    @staticmethod
    def parse(buf):
        rec = buf.rec
        if buf.stage != "l3" or buf.vlan_idx >= int(rec["n_vlan"]):
            return Err(buf)
        if int(rec["vlan_ethertype"][buf.vlan_idx]) + 4 > buf.length:
            return Err(buf)
        return Ok(VlanDot3Frame(buf))

    def _tci(self):
        return int(self.rec["vlan_tci"][self.i])

    def priority(self):
        return self._tci() >> 13

    def dei_flag(self):
        return bool(self._tci() & 0x1000)

    def vlan_id(self):
        return self._tci() & 0xfff

    def payload_len(self):
        return int(self.rec["vlan_ethertype"][self.i])

    def payload(self):
        b = self.buf
        return Cursor(b.rec, b.frame, "dot3", self.i + 1, b.off + 4, self.payload_len())


class VlanGroup:
    """VlanGroup::group_parse (vlan/generated.rs:312-322)."""

    @staticmethod
    def group_parse(buf):
        rec = buf.rec
        if buf.stage != "l3" or buf.vlan_idx >= int(rec["n_vlan"]):
            return Err(buf)
        v = int(rec["vlan_ethertype"][buf.vlan_idx])
        if v >= 1536:
            return VlanFrame.parse(buf)
        if v <= 1500:
            return VlanDot3Frame.parse(buf)
        return Err(buf)


class VlanFrame:
    def __init__(self, buf):
        self.buf, self.rec, self.i = buf, buf.rec, buf.vlan_idx

    @staticmethod
    def parse(buf):
        """vlan/generated.rs:32-39 — Ok for each tag the engine walked."""
        rec = buf.rec
        if buf.stage != "l3" or buf.vlan_idx >= int(rec["n_vlan"]):
            return Err(buf)
        return Ok(VlanFrame(buf))

    def _tci(self):
        return int(self.rec["vlan_tci"][self.i])

    def priority(self):
        return self._tci() >> 13

    def dei_flag(self):
        return bool(self._tci() & 0x1000)

    def vlan_id(self):
        return self._tci() & 0xfff

    def ethertype(self):
        return int(self.rec["vlan_ethertype"][self.i])

    def payload(self):
        b = self.buf
        return Cursor(b.rec, b.frame, "l3", self.i + 1, b.off + 4, b.length - 4)


class Ipv4:
    def __init__(self, buf):
        self.buf, self.rec = buf, buf.rec

    @staticmethod
    def parse(buf):
        """ipv4/generated.rs:35-51."""
        rec = buf.rec
        if (buf.stage != "l3" or buf.vlan_idx != int(rec["n_vlan"])
                or _st(rec) in _PRE_IP or _rec_is_ip6(rec)):
            return Err(buf)
        return Ok(Ipv4(buf))

    def version(self):
        return int(self.rec["ip_vhl"]) >> 4

    def header_len(self):
        return (int(self.rec["ip_vhl"]) & 0xf) * 4

    def dscp(self):
        return int(self.rec["ip_tos"]) >> 2

    def ecn(self):
        return int(self.rec["ip_tos"]) & 3

    def packet_len(self):
        return int(self.rec["ip_packet_len"])

    def ident(self):
        return int(self.rec["ip_ident"])

    def flag_reserved(self):
        return int(self.rec["ip_frag"]) >> 15

    def dont_frag(self):
        return bool(int(self.rec["ip_frag"]) & 0x4000)

    def more_frag(self):
        return bool(int(self.rec["ip_frag"]) & 0x2000)

    def frag_offset(self):
        return int(self.rec["ip_frag"]) & 0x1fff

    def ttl(self):
        return int(self.rec["ip_ttl"])

    def protocol(self):
        return int(self.rec["ip_protocol"])

    def checksum(self):
        return int(self.rec["ip_checksum"])

    def src_addr(self):
        v = int(self.rec["ip_src"])
        return "%d.%d.%d.%d" % (v >> 24, (v >> 16) & 255, (v >> 8) & 255, v & 255)

    def dst_addr(self):
        v = int(self.rec["ip_dst"])
        return "%d.%d.%d.%d" % (v >> 24, (v >> 16) & 255, (v >> 8) & 255, v & 255)

    def header_sum(self):
        """checksum::from_slice(header[0..header_len]) computed by the engine."""
        return int(self.rec["ip_sum"])

    def verify_checksum(self):
        return self.header_sum() == 0xffff

    def payload(self):
        """ipv4/generated.rs:115-127 — trim to packet_len, advance header_len."""
        b = self.buf
        off = int(self.rec["l4_off"])
        return Cursor(b.rec, b.frame, "l4", b.vlan_idx, off, self.packet_len() - self.header_len())


class Ipv6:
    """ipv6/generated.rs:22-216 over an IPv6 record (the record's IPv6 block,
    include/rpkt_gpu.h); the addresses are read from the frame bytes."""

    def __init__(self, buf):
        self.buf, self.rec = buf, buf.rec
        self.b = ip6_block(np.asarray(buf.rec).reshape(1))[0]

    @staticmethod
    def parse(buf):
        """ipv6/generated.rs:40-51 -- Err iff chunk_len < 40 or payload_len + 40 >
        remaining (the engine's IP6_SHORT / IP6_BAD_LEN)."""
        rec = buf.rec
        if (buf.stage != "l3" or buf.vlan_idx != int(rec["n_vlan"]) or not _rec_is_ip6(rec)
                or _st(rec) in _IP6_FAIL):
            return Err(buf)
        return Ok(Ipv6(buf))

    def version(self):
        return int(self.b["ip6_vtcfl"]) >> 28

    def traffic_class(self):
        return (int(self.b["ip6_vtcfl"]) >> 20) & 0xff

    def flow_label(self):
        return int(self.b["ip6_vtcfl"]) & 0xfffff

    def payload_len(self):
        return int(self.b["ip6_payload_len"])

    def next_header(self):
        return int(self.b["ip6_next_header"])

    def hop_limit(self):
        return int(self.b["ip6_hop_limit"])

    def _addr(self, at):
        l3 = int(self.rec["l3_off"])
        return ipaddress.IPv6Address(bytes(self.buf.frame[l3 + at:l3 + at + 16]))

    def src_addr(self):
        return self._addr(8)

    def dst_addr(self):
        return self._addr(24)

    def payload(self):
        """ipv6/generated.rs:83-92 -- trim to payload_len, advance 40."""
        b = self.buf
        return Cursor(b.rec, b.frame, "ip6ext", b.vlan_idx, b.off + 40, self.payload_len())


class _Ip6Ext:
    """An IPv6 extension header view over the frame bytes at a cursor (the generated
    parse of its type; ipv6/generated.rs).  FIXED: fixed header bytes; min_len: the
    smallest header_len its parse accepts."""
    FIXED = 2
    MIN_LEN = 2

    def __init__(self, buf):
        self.buf, self.rec = buf, buf.rec
        self.h = bytes(buf.frame[buf.off:buf.off + buf.length])

    @classmethod
    def parse(cls, buf):
        if buf.stage != "ip6ext" or buf.frame is None or buf.length < cls.FIXED:
            return Err(buf)
        v = cls(buf)
        hl = v.header_len()
        if hl < cls.MIN_LEN or hl > buf.length:
            return Err(buf)
        return Ok(v)

    def next_header(self):
        return self.h[0]

    def header_len(self):
        return self.h[1] * 8 + 8

    def var_header_slice(self):
        return self.h[self.FIXED:self.header_len()]

    def payload(self):
        b, hl = self.buf, self.header_len()
        return Cursor(b.rec, b.frame, "ip6ext", b.vlan_idx, b.off + hl, b.length - hl)


class HopByHopOption(_Ip6Ext):
    """ipv6/generated.rs:367-421"""


class DestOptions(_Ip6Ext):
    """ipv6/generated.rs:224-279"""


class RoutingHeader(_Ip6Ext):
    """ipv6/generated.rs:511-577"""
    FIXED = 8
    MIN_LEN = 8

    def type_(self):
        return self.h[2]

    def segments_left(self):
        return self.h[3]

    def type_specific_data(self):
        return int.from_bytes(self.h[4:8], "big")


class FragmentHeader(_Ip6Ext):
    """ipv6/generated.rs:679-739"""
    FIXED = 8
    MIN_LEN = 8

    def header_len(self):
        return 8

    def reserved(self):
        return self.h[1]

    def offset(self):
        return int.from_bytes(self.h[2:4], "big") >> 3

    def reserved1(self):
        return (self.h[3] >> 1) & 3

    def more_frag(self):
        return bool(self.h[3] & 1)

    def ident(self):
        return int.from_bytes(self.h[4:8], "big")


class AuthenticationHeader(_Ip6Ext):
    """ipv6/generated.rs:833-899"""
    FIXED = 12
    MIN_LEN = 12

    def header_len(self):
        return self.h[1] * 4 + 8

    def reserved(self):
        return int.from_bytes(self.h[2:4], "big")

    def security_parameters_index(self):
        return int.from_bytes(self.h[4:8], "big")

    def seq_num_field(self):
        return int.from_bytes(self.h[8:12], "big")


class _L4:
    PROTO = None

    def __init__(self, buf):
        self.buf, self.rec = buf, buf.rec

    @classmethod
    def parse(cls, buf):
        """Ok where the engine's chain parsed this protocol: after Ipv4::payload(), or
        at the cursor where the IPv6 extension headers ended (the record's l4_off)."""
        rec = buf.rec
        at_l4 = buf.stage == "l4" or (buf.stage == "ip6ext" and buf.off == int(rec["l4_off"]))
        if not at_l4 or _st(rec) != STATUS["OK"] or int(rec["ip_protocol"]) != cls.PROTO:
            return Err(buf)
        return Ok(cls(buf))

    def src_port(self):
        return int(self.rec["src_port"])

    def dst_port(self):
        return int(self.rec["dst_port"])

    def checksum(self):
        return int(self.rec["l4_checksum"])

    def sum(self):
        """checksum::combine(&[pseudo_header, from_slice(l4)]) computed by the engine."""
        return int(self.rec["l4_sum"])

    def payload(self):
        b = self.buf
        return Cursor(b.rec, b.frame, "app", b.vlan_idx, int(self.rec["payload_off"]),
                      int(self.rec["payload_len"]))


class Udp(_L4):
    """udp/generated.rs:31-76"""
    PROTO = IpProtocol.UDP

    def packet_len(self):
        return int(self.rec["l4_word6"])

    def verify_checksum(self):
        # smoltcp policy: a zero UDP checksum means "not computed" (SURVEY §8a A12), over
        # IPv4 only (RFC 8200 section 8.1 makes it mandatory over IPv6)
        if self.checksum() == 0 and not _rec_is_ip6(self.rec):
            return True
        return self.sum() == 0xffff


class Tcp(_L4):
    """tcp/generated.rs:34-131"""
    PROTO = IpProtocol.TCP

    def _w6(self):
        return int(self.rec["l4_word6"])

    def seq_num(self):
        return int(self.rec["tcp_seq"])

    def ack_num(self):
        return int(self.rec["tcp_ack"])

    def header_len(self):
        return (self._w6() >> 12) * 4

    def reserved(self):
        return (self._w6() >> 8) & 0xf

    def cwr(self):
        return bool(self._w6() & 0x80)

    def ece(self):
        return bool(self._w6() & 0x40)

    def urg(self):
        return bool(self._w6() & 0x20)

    def ack(self):
        return bool(self._w6() & 0x10)

    def psh(self):
        return bool(self._w6() & 0x08)

    def rst(self):
        return bool(self._w6() & 0x04)

    def syn(self):
        return bool(self._w6() & 0x02)

    def fin(self):
        return bool(self._w6() & 0x01)

    def window_size(self):
        return int(self.rec["tcp_window"])

    def urgent_pointer(self):
        return int(self.rec["tcp_urgent"])

    def verify_checksum(self):
        return self.sum() == 0xffff


__all__ = ["EtherType", "IpProtocol", "Result", "Ok", "Err", "Cursor", "Packet",
           "EtherFrame", "EtherDot3Frame", "EtherGroup", "VlanFrame", "VlanDot3Frame",
           "VlanGroup", "Ipv4", "Ipv6", "HopByHopOption", "DestOptions", "RoutingHeader",
           "FragmentHeader", "AuthenticationHeader", "Udp", "Tcp", "MAX_VLAN"]
