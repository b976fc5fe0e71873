"""Host-side header views over engine records — the rpkt API surface for the path.

The reference exposes header views over a byte buffer (`T: Buf`) with
`parse(buf) -> Result<View, buf>`, getters and `payload()`:
  EtherFrame  rpkt/src/ether/generated.rs:17-67
  VlanFrame   rpkt/src/vlan/generated.rs:15-69
  Ipv4        rpkt/src/ipv4/generated.rs:17-127, 269-288
  Udp         rpkt/src/udp/generated.rs:13-76
  Tcp         rpkt/src/tcp/generated.rs:16-131
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
from .records import STATUS, MAX_VLAN


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
    ICMP = 1
    IGMP = 2
    IPIP = 4
    TCP = 6
    UDP = 17
    GRE = 47


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
        """ether/generated.rs:63-67 — advance(14)."""
        b = self.buf
        return Cursor(b.rec, b.frame, "l3", 0, 14, b.length - 14)


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
                or _st(rec) in _PRE_IP):
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


class _L4:
    PROTO = None

    def __init__(self, buf):
        self.buf, self.rec = buf, buf.rec

    @classmethod
    def parse(cls, buf):
        rec = buf.rec
        if buf.stage != "l4" or _st(rec) != STATUS["OK"] or int(rec["ip_protocol"]) != cls.PROTO:
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
        # smoltcp policy: a zero UDP checksum means "not computed" 
        return self.checksum() == 0 or self.sum() == 0xffff


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
           "VlanGroup", "Ipv4", "Udp", "Tcp", "MAX_VLAN"]
