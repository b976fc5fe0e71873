"""Host-side views of one tunnel level over rpkt_gpu_parse_tunnel_batch's three records
(outer rpkt_rec_t, rpkt_tun_t, inner rpkt_rec_t) -- the read side of the reference's
tunnel API, so a receive loop written against rpkt's chain reads the same:

    pkt = TunnelPacket(outer, tun, inner, frame)
    udp = Udp.parse(Ipv4.parse(EtherFrame.parse(pkt).unwrap().payload()).unwrap()
                    .payload()).unwrap()
    vxlan = Vxlan.parse(udp.payload()).unwrap()          # vxlan/generated.rs:32-39
    assert vxlan.vni() == 3000001
    inner_eth = EtherFrame.parse(vxlan.payload()).unwrap()   # vlan_mpls_tests.rs:237-251

The reference views and the chains its tests walk:
  Vxlan     rpkt/src/vxlan/generated.rs:17-103 (getters :45-84, payload :97-103)
  Gtpv1     rpkt/src/gtpv1/generated.rs:17-120, 233-290 (header_len, sequence, npdu,
            next_extention_header); its extension headers (ExtPduNumber, ExtUdpPort,
            ExtLongPduNumber, ExtServiceClassIndicator, ExtContainer, PduSessionUp's
            Dl/UlPduSessionInfo: :319-1517) walk to the T-PDU as gtpv1_test.rs:199-231,
            284-320, 468-505 do; `Gtpv1.t_pdu()` jumps there directly
  Gre       rpkt/src/gre/generated.rs:17-110, 222-280 (checksum, offset, key, sequence)
Ok / Err follow the engine's decode (rpkt_tun_t.kind / status): `parse` is Ok exactly
where the reference parse returned Ok for this frame.  Getters come from the tunnel
record; the few the record does not carry (GTP packet_len / npdu / next extension, GRE
offset / sequence) are read from the frame bytes, which must then be supplied.
"""
import numpy as np

from .records import TUN_KIND, TUN_STATUS
from .views import Cursor, Err, EtherType, Ok


class _TunRec:
    """The outer record as the outer views see it, carrying its tunnel and inner records
    (so the payload cursor a Udp / Ipv4 view returns still knows them)."""
    __slots__ = ("rec", "tun", "inner")

    def __init__(self, rec, tun, inner):
        self.rec, self.tun, self.inner = rec, tun, inner

    def __getitem__(self, k):
        return self.rec[k]

    def __array__(self, dtype=None, copy=None):
        return np.asarray(self.rec)


def TunnelPacket(outer, tun, inner, frame=None):
    """Cursor::new(frame) over a frame rpkt_gpu_parse_tunnel_batch parsed: the outer chain
    starts here; the tunnel views take their cursors from its payloads."""
    return Cursor(_TunRec(outer, tun, inner), frame, "ether", 0, 0, int(outer["frame_len"]))


def _tun(buf):
    return getattr(buf.rec, "tun", None)


def _inner_cursor(buf, t):
    """The inner frame's cursor: an Ethernet frame (VXLAN, GRE 0x6558) starts a chain at
    "ether", an IP packet (GTP-U T-PDU, GRE 0x0800 / 0x86DD) at "l3", over the inner
    record (offsets in the outer frame); anything else is a raw cursor."""
    inner = buf.rec.inner
    off, n = int(t["inner_off"]), int(inner["frame_len"])
    if int(t["status"]) != TUN_STATUS["OK"]:
        end = int(buf.rec["payload_off"]) + int(buf.rec["payload_len"]) \
            if int(t["kind"]) != TUN_KIND["GRE"] else int(buf.rec["l3_off"]) + \
            int(buf.rec["ip_packet_len"])
        return Cursor(buf.rec, buf.frame, "raw", 0, off, max(0, end - off))
    stage = "ether" if int(t["inner_type"]) == EtherType.TRANS_ETH_BRIDGE or \
        int(t["kind"]) == TUN_KIND["VXLAN"] else "l3"
    return Cursor(inner, buf.frame, stage, 0, off, n)


def _frame_bytes(buf, off, n):
    if buf.frame is None:
        raise ValueError("frame bytes were not supplied to TunnelPacket()")
    return bytes(buf.frame[off:off + n])


class _Tunnel:
    KIND = None

    def __init__(self, buf, t):
        self.buf, self.t = buf, t

    @classmethod
    def _at(cls, buf, stage):
        t = _tun(buf)
        if t is None or buf.stage != stage or int(t["kind"]) != cls.KIND or \
                int(t["status"]) in (TUN_STATUS["BAD"], TUN_STATUS["NONE"]) or \
                buf.off != int(t["tun_off"]):
            return Err(buf)
        return Ok(cls(buf, t))

    def _h0(self):
        return int(self.t["hdr0"])

    def _h1(self):
        return int(self.t["hdr1"])

    def payload(self):
        """The tunnel's payload cursor (an Ethernet frame or an IP packet parses from it)."""
        return _inner_cursor(self.buf, self.t)


class Vxlan(_Tunnel):
    """vxlan/generated.rs:17-103 in a UDP payload (the engine's dispatch: port 4789)."""
    KIND = TUN_KIND["VXLAN"]

    @classmethod
    def parse(cls, buf):
        """vxlan/generated.rs:32-39 -- Err iff chunk_len < 8."""
        return cls._at(buf, "app")

    def gbp_extention(self):
        return bool(self._h0() & 0x80)

    def reserved_0(self):
        return (self._h0() >> 4) & 0x7

    def reserved_1(self):
        return (((self._h0() << 8) | self._h1()) >> 7) & 0xf

    def reserved_2(self):
        return (self._h1() >> 4) & 0x3

    def reserved_3(self):
        return self._h1() & 0x7

    def reserved_4(self):
        """Byte 7, read from the frame (the tunnel record does not carry it)."""
        return _frame_bytes(self.buf, int(self.t["tun_off"]) + 7, 1)[0]

    def vni_present(self):
        return bool(self._h0() & 0x08)

    def dont_learn(self):
        return bool(self._h1() & 0x40)

    def policy_applied(self):
        return bool(self._h1() & 0x08)

    def group_id(self):
        return int(self.t["aux"])

    def vni(self):
        return int(self.t["id"])


class Gtpv1(_Tunnel):
    """gtpv1/generated.rs:17-120, 233-290 in a UDP payload (port 2152)."""
    KIND = TUN_KIND["GTPU"]

    @classmethod
    def parse(cls, buf):
        """gtpv1/generated.rs:33-49 -- Err iff chunk_len < 8, header_len > chunk_len or
        packet_len + 8 > remaining."""
        return cls._at(buf, "app")

    def version(self):
        return self._h0() >> 5

    def protocol_type(self):
        return (self._h0() >> 4) & 1

    def reserved(self):
        return (self._h0() >> 3) & 1

    def extention_header_present(self):
        return bool(self._h0() & 0x04)

    def sequence_present(self):
        return bool(self._h0() & 0x02)

    def npdu_present(self):
        return bool(self._h0() & 0x01)

    def message_type(self):
        return self._h1()

    def teid(self):
        return int(self.t["id"])

    def header_len(self):
        """:239-249 -- 12 when any of E / S / PN is set, else 8."""
        return 12 if self._h0() & 7 else 8

    def packet_len(self):
        """:92-94 -- the length field + 8 (the whole GTPv1 packet)."""
        b = _frame_bytes(self.buf, int(self.t["tun_off"]) + 2, 2)
        return int.from_bytes(b, "big") + 8

    def sequence(self):
        """:255-258 -- asserts header_len() == 12."""
        assert self.header_len() == 12, "sequence() of an 8-byte GTPv1 header"
        return int(self.t["aux"])

    def npdu(self):
        assert self.header_len() == 12, "npdu() of an 8-byte GTPv1 header"
        return _frame_bytes(self.buf, int(self.t["tun_off"]) + 10, 1)[0]

    def next_extention_header(self):
        assert self.header_len() == 12, "next_extention_header() of an 8-byte GTPv1 header"
        return _frame_bytes(self.buf, int(self.t["tun_off"]) + 11, 1)[0]

    def t_pdu(self):
        """The T-PDU after the extension headers (the chain gtpv1_test.rs:199-231 walks
        header by header: ExtPduNumber / ExtUdpPort / ... / PduSessionUp, each payload()):
        Ipv4 / Ipv6 parse from it when the engine found a G-PDU carrying one."""
        return _inner_cursor(self.buf, self.t)

    def payload(self):
        """:98-108 -- trim to packet_len, advance header_len: the first extension header
        when E is set (a raw cursor), else the T-PDU."""
        if not self.extention_header_present():
            return self.t_pdu()
        at = int(self.t["tun_off"]) + 12
        end = int(self.t["tun_off"]) + self.packet_len()
        return Cursor(self.buf.rec, self.buf.frame, "raw", 0, at, max(0, end - at))


class _GtpExt:
    """A GTP-U extension header in the chain Gtpv1.payload() starts (gtpv1/generated.rs
    :319-1300), read from the frame bytes as views.py reads IPv6 extension headers: the
    engine walked the same chain to find the T-PDU (rpkt_tun_t.inner_off).  FIXED is the
    view's fixed header length; variable-length headers are 4 * byte 0 long; the next
    extension type is the header's last byte.  payload() advances header_len; the cursor it
    returns is the T-PDU's (Ipv4 / Ipv6 parse from it) where the engine found the inner
    packet, else a raw cursor the next extension header parses from."""
    FIXED = 4
    VARIABLE = False

    def __init__(self, buf):
        self.buf = buf
        self.h = _frame_bytes(buf, buf.off, buf.length)

    @classmethod
    def parse(cls, buf):
        """Err iff chunk_len < FIXED (and, variable-length, header_len < FIXED or
        header_len > chunk_len), or the cursor is not one the chain reached."""
        if buf.stage != "raw" or _tun(buf) is None or buf.frame is None or buf.length < cls.FIXED:
            return Err(buf)
        v = cls(buf)
        if cls.VARIABLE and not (cls.FIXED <= v.header_len() <= buf.length):
            return Err(buf)
        return Ok(v)

    def header_len(self):
        return self.h[0] * 4 if self.VARIABLE else self.FIXED

    def len(self):
        return self.h[0]

    def next_extention_header(self):
        return self.h[self.header_len() - 1]

    def payload(self):
        b, t, hl = self.buf, _tun(self.buf), self.header_len()
        if int(t["status"]) == TUN_STATUS["OK"] and b.off + hl == int(t["inner_off"]):
            return _inner_cursor(b, t)
        return Cursor(b.rec, b.frame, "raw", 0, b.off + hl, b.length - hl)


class ExtUdpPort(_GtpExt):
    """gtpv1/generated.rs:319-366 (type 0x40)."""

    def udp_port(self):
        return int.from_bytes(self.h[1:3], "big")


class ExtPduNumber(_GtpExt):
    """gtpv1/generated.rs:444-492 (type 0xc0)."""

    def pdcp_number(self):
        return int.from_bytes(self.h[1:3], "big")


class ExtLongPduNumber(_GtpExt):
    """gtpv1/generated.rs:570-634 (types 0x03 / 0x82)."""
    FIXED = 8

    def spare1(self):
        return self.h[1] >> 2

    def pdu_number(self):
        return int.from_bytes(self.h[1:4], "big") & 0x3ffff

    def spare2(self):
        return self.h[4]

    def spare3(self):
        return self.h[5]

    def spare4(self):
        return self.h[6]


class ExtServiceClassIndicator(_GtpExt):
    """gtpv1/generated.rs:730-782 (type 0x20)."""

    def service_class_indicator(self):
        return self.h[1]

    def spare(self):
        return self.h[2]


class ExtContainer(_GtpExt):
    """gtpv1/generated.rs:863-935: any container (RAN / Xw RAN / NR RAN / PDU session,
    types 0x81 / 0x83 / 0x84 / 0x85) as its length-prefixed bytes."""
    FIXED = 1
    VARIABLE = True

    def var_header_slice(self):
        return self.h[1:self.header_len()]


class DlPduSessionInfo(_GtpExt):
    """gtpv1/generated.rs:1029-1130: the PDU session container, PDU type 0."""
    FIXED = 3
    VARIABLE = True

    def pdu_type(self):
        return self.h[1] >> 4

    def qmp(self):
        return bool(self.h[1] & 0x8)

    def snp(self):
        return bool(self.h[1] & 0x4)

    def msnp(self):
        return bool(self.h[1] & 0x2)

    def spare(self):
        return self.h[1] & 0x1

    def ppp(self):
        return bool(self.h[2] & 0x80)

    def rqi(self):
        return bool(self.h[2] & 0x40)

    def qos_flow_identifier(self):
        return self.h[2] & 0x3f


class UlPduSessionInfo(_GtpExt):
    """gtpv1/generated.rs:1268-1330: the PDU session container, PDU type 1."""
    FIXED = 3
    VARIABLE = True

    def pdu_type(self):
        return self.h[1] >> 4

    def qmp(self):
        return (self.h[1] >> 3) & 1

    def dl_delay_ind(self):
        return (self.h[1] >> 2) & 1

    def ul_delay_ind(self):
        return (self.h[1] >> 1) & 1

    def snp(self):
        return self.h[1] & 1

    def n3_n9_delay_ind(self):
        return self.h[2] >> 7

    def new_ie_flag(self):
        return (self.h[2] >> 6) & 1

    def qos_flow_identifier(self):
        return self.h[2] & 0x3f


class PduSessionUp:
    """PduSessionUp::group_parse (gtpv1/generated.rs:1507-1517): dispatch on the PDU type
    (byte 1 >> 4): 0 DlPduSessionInfo, 1 UlPduSessionInfo, else Err.  The Ok value is the
    view itself (match on its class where rpkt matches the enum variant)."""

    @staticmethod
    def group_parse(buf):
        if buf.stage != "raw" or buf.frame is None or buf.length < 2:
            return Err(buf)
        kind = _frame_bytes(buf, buf.off + 1, 1)[0] >> 4
        cls = {0: DlPduSessionInfo, 1: UlPduSessionInfo}.get(kind)
        return cls.parse(buf) if cls else Err(buf)


class Gre(_Tunnel):
    """gre/generated.rs:17-110, 222-280 in an IPv4 / IPv6 payload (protocol 47)."""
    KIND = TUN_KIND["GRE"]

    @classmethod
    def parse(cls, buf):
        """GreGroup::group_parse (gre/generated.rs:800-820): the version 0 (RFC 2784/2890)
        or version 1 (PPTP) header."""
        # (after IPv4::payload, or where an IPv6 extension chain ended)
        return cls._at(buf, "ip6ext" if buf.stage == "ip6ext" else "l4")

    def checksum_present(self):
        return bool(self._h0() & 0x80)

    def routing_present(self):
        return bool(self._h0() & 0x40)

    def key_present(self):
        return bool(self._h0() & 0x20)

    def sequence_present(self):
        return bool(self._h0() & 0x10)

    def strict_source_route(self):
        return bool(self._h0() & 0x08)

    def recursion_control(self):
        return self._h0() & 0x07

    def flags(self):
        return self._h1() >> 3

    def version(self):
        return self._h1() & 0x07

    def protocol_type(self):
        return int(self.t["inner_type"])

    def header_len(self):
        """:228-238 -- 4 + 4 per optional word (checksum/offset, key, sequence)."""
        h = self._h0()
        return 4 + 4 * bool(h & 0xc0) + 4 * bool(h & 0x20) + 4 * bool(h & 0x10)

    def checksum(self):
        assert self._h0() & 0xc0, "checksum() without the C or R bit"
        return int(self.t["aux"])

    def offset(self):
        """:250-253 -- bytes 6..8, with the C or R bit (read from the frame)."""
        assert self._h0() & 0xc0, "offset() without the C or R bit"
        return int.from_bytes(_frame_bytes(self.buf, int(self.t["tun_off"]) + 6, 2), "big")

    def key(self):
        assert self._h0() & 0x20, "key() without the K bit"
        return int(self.t["id"])

    def sequence(self):
        assert self._h0() & 0x10, "sequence() without the S bit"
        at = int(self.t["tun_off"]) + 4 + 4 * bool(self._h0() & 0xc0) + 4 * bool(self._h0() & 0x20)
        return int.from_bytes(_frame_bytes(self.buf, at, 4), "big")

    def verify_checksum(self):
        """The RFC 2784 sum over the GRE header and payload, from the outer record's l4_sum
        (the engine's RPKT_F_L4_SUM): valid iff 0xffff."""
        return int(self.buf.rec["l4_sum"]) == 0xffff


__all__ = ["TunnelPacket", "Vxlan", "Gtpv1", "Gre", "ExtUdpPort", "ExtPduNumber",
           "ExtLongPduNumber", "ExtServiceClassIndicator", "ExtContainer", "DlPduSessionInfo",
           "UlPduSessionInfo", "PduSessionUp"]
