"""Host-side build views: rpkt's write-side API (prepend_header + setters) composing the
records rpkt_gpu_build_batch takes.

The reference builds a frame inside-out on a mutable cursor that starts at the payload
(benches/rpkt/rpkt_build.rs:9-28, rpkt-dpdk/examples/loopback_tx.rs:70-99):

    pkt = CursorMut(frame_len); pkt.advance(42)
    udp = Udp.prepend_header(pkt, UDP_HEADER_TEMPLATE)
    udp.set_src_port(60376); udp.set_dst_port(161)
    ip = Ipv4.prepend_header(udp.release(), IPV4_HEADER_TEMPLATE)
    ip.set_ident(0x5c65); ip.set_ttl(128); ip.set_src_addr("192.168.29.58"); ...
    eth = EtherFrame.prepend_header(ip.release(), ETHER_FRAME_HEADER_TEMPLATE)
    eth.set_dst_addr(...); eth.set_src_addr(...); eth.set_ethertype(EtherType.IPV4)
    rec, extra = eth.release().record()

Each view holds the header bytes exactly as the reference's prepend_header (template
copied, length field set from remaining()) and setters (the same masks and asserts:
rpkt/src/{udp,tcp,ipv4,ipv6,vlan,ether}/generated.rs, cited per method) would leave them
in the frame.  `record()` turns the finished chain into the rpkt_rec_t
rpkt_gpu_build_batch writes back (include/rpkt_gpu.h), and `extra` lists the frame bytes
a record does not carry and the caller places in the frame buffer with the payload: IPv6
addresses (the record keeps them folded), and whatever the caller wrote into option or
extension-header space (`var_header_slice_mut`, `CursorMut.move_back`).  Length fields
(IPv4 packet_len, IPv6 payload_len, UDP length) are the build's: from the frame span,
as prepend_header sets them from remaining().  The build writes the L4 header a record's
IP protocol names (6, 17); an L4 view under an IPv4 header whose protocol field names
something else (rpkt_build.rs never sets it) is carried in `extra` as written.
"""
import ipaddress

import numpy as np

from .records import REC_DTYPE

# rpkt/src/{udp,tcp,ipv4,ipv6,vlan,ether}/generated.rs header templates
UDP_HEADER_TEMPLATE = bytes([0x00, 0x00, 0x00, 0x00, 0x00, 0x08, 0x00, 0x00])
TCP_HEADER_TEMPLATE = bytes([0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x50, 0, 0, 0, 0, 0, 0, 0])
IPV4_HEADER_TEMPLATE = bytes([0x45, 0, 0, 0x14] + [0] * 16)
IPV6_HEADER_TEMPLATE = bytes([0x60, 0, 0, 0, 0, 0, 0x04, 0]) + bytes(32)
VLAN_FRAME_HEADER_TEMPLATE = bytes([0x00, 0x01, 0x08, 0x00])
ETHER_FRAME_HEADER_TEMPLATE = bytes([0] * 12 + [0x08, 0x00])


def _be16(b, at):
    return (b[at] << 8) | b[at + 1]


def _be32(b, at):
    return (b[at] << 24) | (b[at + 1] << 16) | (b[at + 2] << 8) | b[at + 3]


def _put16(b, at, v):
    b[at:at + 2] = int(v).to_bytes(2, "big")


class CursorMut:
    """CursorMut::new(&mut buf[..frame_len]) (rpkt/src/cursors.rs): the build's cursor over
    one frame of `frame_len` bytes.  `advance(n)` makes headroom for the headers,
    `move_back(n)` claims n bytes of it the caller fills itself (extension headers)."""

    def __init__(self, frame_len):
        self.frame_len = int(frame_len)
        self.start = 0
        self.layers = []             # (kind, offset, header view), outermost last
        self.extra = []              # (offset, bytes) the caller places in the frame

    def advance(self, n):
        """cursors.rs CursorMut::advance: assert!(cnt <= self.remaining())."""
        assert 0 <= n <= self.frame_len - self.start, "advance past the end"
        self.start += n

    def cursor(self):
        return self.start

    def chunk_headroom(self):
        return self.start

    def remaining(self):
        return self.frame_len - self.start

    def trim_off(self, n):
        """cursors.rs CursorMut::trim_off: the last n bytes leave the chunk
        (assert!(cnt <= self.remaining()))."""
        assert 0 <= n <= self.frame_len - self.start, "trim_off past the cursor"
        self.frame_len -= n

    def move_back(self, n, data=None):
        """PktBufMut::move_back: n bytes of headroom become part of the packet (an
        extension header the caller writes: `data`, if given, is placed there)."""
        assert 0 <= n <= self.start, "move_back past the start"
        self.start -= n
        if data is not None:
            assert len(data) == n
            self.extra.append((self.start, bytes(data)))
        self.layers.append(("raw", self.start, n))

    def _push(self, kind, view, hl):
        assert hl <= self.start, "prepend_header: chunk_headroom() < header length"
        self.start -= hl
        self.layers.append((kind, self.start, view))
        return self.start

    def record(self):
        """(rpkt_rec_t, extra frame bytes) of the finished chain; the frame is
        [start, frame_len) of the buffer (start == 0 when the headroom was exact)."""
        arr = np.zeros(1, dtype=REC_DTYPE)
        r = arr[0]
        base = self.start
        kinds = [k for k, _, _ in self.layers]
        assert kinds and kinds[-1] == "ether", "the chain ends with EtherFrame.prepend_header"
        extra = [(o - base, b) for o, b in self.extra]
        vlans = [v for k, _, v in reversed(self.layers) if k == "vlan"]   # frame order
        assert len(vlans) <= 2, "at most RPKT_MAX_VLAN tags"
        eth = self.layers[-1][2].b
        r["dst_addr"] = list(eth[0:6])
        r["src_addr"] = list(eth[6:12])
        r["ethertype"] = _be16(eth, 12)
        r["n_vlan"] = len(vlans)
        for k, v in enumerate(vlans):
            r["vlan_tci"][k] = _be16(v.b, 0)
            r["vlan_ethertype"][k] = _be16(v.b, 2)
        l3 = 14 + 4 * len(vlans)
        r["l3_off"] = l3
        raw = arr.view(np.uint8)
        for kind, off, v in self.layers:
            if kind == "ipv4":
                b = v.b
                assert off - base == l3, "the IPv4 header follows the link layer"
                r["ip_vhl"], r["ip_tos"] = b[0], b[1]
                r["ip_ident"], r["ip_frag"] = _be16(b, 4), _be16(b, 6)
                r["ip_ttl"], r["ip_protocol"] = b[8], b[9]
                r["ip_checksum"] = _be16(b, 10)
                r["ip_src"], r["ip_dst"] = _be32(b, 12), _be32(b, 16)
                r["l4_off"] = l3 + v.header_len()
                if b[9] in (6, 17) and not any(k in ("udp", "tcp") for k, _, _ in self.layers):
                    # the record's ip_protocol is both the header byte and what the build
                    # writes at l4_off (a UDP / TCP header): with no Udp / Tcp view the build
                    # would overwrite the caller's bytes there, which prepend_header leaves
                    raise ValueError("IPv4 protocol %d without a Udp/Tcp view: the build "
                                     "writes that header; prepend it with its view" % b[9])
                if v.header_len() > 20:
                    extra.append((off - base + 20, bytes(v.b[20:])))
            elif kind == "ipv6":
                b = v.b
                assert off - base == l3, "the IPv6 header follows the link layer"
                # the IPv6 block (include/rpkt_gpu.h bytes 24..43): vtcfl, next_header,
                # hop_limit, the upper-layer protocol, the pseudo header's destination
                raw[24:28] = np.frombuffer(_be32(b, 0).to_bytes(4, "little"), np.uint8)
                raw[30], raw[31] = b[6], b[7]
                extra.append((off - base + 8, bytes(b[8:40])))
                up = [x for x in self.layers if x[0] in ("udp", "tcp")]
                raws = [(o, n) for k, o, n in self.layers if k == "raw" and o >= off]
                # with no Udp / Tcp view the upper layer starts after the extension headers
                # placed with move_back, and the record's upper-layer protocol (byte 33) is
                # 59, No Next Header: the build writes no L4 header over the caller's bytes
                # there (next_header, byte 30, stays the header's own)
                l4 = (up[0][1] - base) if up else max([v.end - base] +
                                                      [o + n - base for o, n in raws])
                raw[32] = len(raws)
                r["ip_protocol"] = up[0][2].proto if up else 59
                pd = l3 + 24 if v.pdst is None else v.pdst
                raw[34:36] = np.frombuffer(int(pd).to_bytes(2, "little"), np.uint8)
                r["l4_off"] = l4
        ip_proto = int(r["ip_protocol"])
        for kind, off, v in self.layers:
            if kind in ("udp", "tcp"):
                b = v.b
                if ip_proto != v.proto:
                    # an L4 header under an IPv4 protocol field that does not name it (the
                    # reference bench leaves protocol 0): the build writes L4 headers by the
                    # record's protocol, so these bytes travel with the payload instead
                    extra.append((off - base, bytes(b)))
                r["src_port"], r["dst_port"] = _be16(b, 0), _be16(b, 2)
                if kind == "udp":
                    r["l4_checksum"] = _be16(b, 6)
                    r["l4_word6"] = _be16(b, 4)
                else:
                    r["tcp_seq"], r["tcp_ack"] = _be32(b, 4), _be32(b, 8)
                    r["l4_word6"], r["tcp_window"] = _be16(b, 12), _be16(b, 14)
                    r["l4_checksum"], r["tcp_urgent"] = _be16(b, 16), _be16(b, 18)
                    if v.header_len() > 20:
                        extra.append((off - base + 20, bytes(v.b[20:])))
        r["frame_len"] = self.frame_len - base
        return arr[0], extra


class _View:
    def __init__(self, buf, b):
        self.buf, self.b = buf, b

    def release(self):
        return self.buf


class Udp(_View):
    proto = 17

    @classmethod
    def prepend_header(cls, buf, header=UDP_HEADER_TEMPLATE):
        """udp/generated.rs:79-88: 8 bytes, packet_len = remaining()"""
        assert len(header) == 8
        v = cls(buf, bytearray(header))
        buf._push("udp", v, 8)
        assert buf.remaining() <= 65535
        _put16(v.b, 4, buf.remaining())
        return v

    def set_src_port(self, value):              # :90
        _put16(self.b, 0, value)

    def set_dst_port(self, value):              # :94
        _put16(self.b, 2, value)

    def set_checksum(self, value):              # :98
        _put16(self.b, 6, value)

    def set_packet_len(self, value):            # :102 (the build sets it from the span)
        _put16(self.b, 4, value)


class Tcp(_View):
    proto = 6

    @classmethod
    def prepend_header(cls, buf, header=TCP_HEADER_TEMPLATE):
        """tcp/generated.rs:135-141: header_len (the template's doff) bytes; the option
        bytes past 20 are the caller's (var_header_slice_mut)"""
        assert len(header) == 20
        hl = (header[12] >> 4) * 4
        assert hl >= 20
        v = cls(buf, bytearray(header) + bytearray(hl - 20))
        buf._push("tcp", v, hl)
        return v

    def header_len(self):
        return (self.b[12] >> 4) * 4

    def var_header_slice_mut(self):
        return memoryview(self.b)[20:self.header_len()]

    def set_src_port(self, value):              # :148
        _put16(self.b, 0, value)

    def set_dst_port(self, value):              # :152
        _put16(self.b, 2, value)

    def set_seq_num(self, value):               # :156
        self.b[4:8] = int(value).to_bytes(4, "big")

    def set_ack_num(self, value):               # :160
        self.b[8:12] = int(value).to_bytes(4, "big")

    def set_reserved(self, value):              # :164
        assert value <= 0xf
        self.b[12] = (self.b[12] & 0xf0) | value

    def _flag(self, bit, value):                # :169-207
        self.b[13] = (self.b[13] & ~(1 << bit) & 0xff) | ((1 if value else 0) << bit)

    def set_cwr(self, v): self._flag(7, v)
    def set_ece(self, v): self._flag(6, v)
    def set_urg(self, v): self._flag(5, v)
    def set_ack(self, v): self._flag(4, v)
    def set_psh(self, v): self._flag(3, v)
    def set_rst(self, v): self._flag(2, v)
    def set_syn(self, v): self._flag(1, v)
    def set_fin(self, v): self._flag(0, v)

    def set_window_size(self, value):           # :209
        _put16(self.b, 14, value)

    def set_checksum(self, value):              # :213
        _put16(self.b, 16, value)

    def set_urgent_pointer(self, value):        # :217
        _put16(self.b, 18, value)


class Ipv4(_View):
    @classmethod
    def prepend_header(cls, buf, header=IPV4_HEADER_TEMPLATE):
        """ipv4/generated.rs:130-140: header_len (the template's IHL) bytes, packet_len =
        remaining(); option bytes past 20 are the caller's"""
        assert len(header) == 20
        hl = (header[0] & 0xf) * 4
        assert hl >= 20
        v = cls(buf, bytearray(header) + bytearray(hl - 20))
        buf._push("ipv4", v, hl)
        assert buf.remaining() <= 65535
        _put16(v.b, 2, buf.remaining())
        return v

    def header_len(self):
        return (self.b[0] & 0xf) * 4

    def var_header_slice_mut(self):
        return memoryview(self.b)[20:self.header_len()]

    def set_version(self, value):               # :147
        assert value == 4
        self.b[0] = (self.b[0] & 0x0f) | (value << 4)

    def set_dscp(self, value):                  # :152
        assert value <= 0x3f
        self.b[1] = (self.b[1] & 0x03) | (value << 2)

    def set_ecn(self, value):                   # :157
        assert value <= 0x3
        self.b[1] = (self.b[1] & 0xfc) | value

    def set_ident(self, value):                 # :162
        _put16(self.b, 4, value)

    def set_flag_reserved(self, value):         # :166
        assert value <= 1
        self.b[6] = (self.b[6] & 0x7f) | (value << 7)

    def set_dont_frag(self, value):             # :171
        self.b[6] = (self.b[6] & 0xbf) | ((1 if value else 0) << 6)

    def set_more_frag(self, value):             # :176
        self.b[6] = (self.b[6] & 0xdf) | ((1 if value else 0) << 5)

    def set_frag_offset(self, value):           # :181
        assert value <= 0x1fff
        _put16(self.b, 6, value | ((self.b[6] & 0xe0) << 8))

    def set_ttl(self, value):                   # :187
        self.b[8] = value

    def set_protocol(self, value):              # :191
        self.b[9] = value

    def set_checksum(self, value):              # :195
        _put16(self.b, 10, value)

    def set_header_len(self, value):            # :199
        assert value <= 60 and value % 4 == 0
        self.b[0] = (self.b[0] & 0xf0) | (value // 4)

    def set_packet_len(self, value):            # :204 (the build sets it from the span)
        _put16(self.b, 2, value)

    def set_src_addr(self, value):              # :291
        self.b[12:16] = ipaddress.IPv4Address(value).packed

    def set_dst_addr(self, value):              # :295
        self.b[16:20] = ipaddress.IPv4Address(value).packed


class Ipv6(_View):
    @classmethod
    def prepend_header(cls, buf, header=IPV6_HEADER_TEMPLATE):
        """ipv6/generated.rs:96-105: 40 bytes, payload_len = remaining()"""
        assert len(header) == 40
        end = buf.start
        v = cls(buf, bytearray(header))
        v.end, v.pdst = end, None
        assert buf.remaining() <= 65535
        _put16(v.b, 4, buf.remaining())
        buf._push("ipv6", v, 40)
        return v

    def set_version(self, value):               # :107
        assert value == 6
        self.b[0] = (self.b[0] & 0x0f) | (value << 4)

    def set_traffic_class(self, value):         # :112
        w = (value << 4) | ((self.b[0] & 0xf0) << 8) | (self.b[1] & 0xf)
        _put16(self.b, 0, w)

    def set_flow_label(self, value):            # :119
        assert value <= 0xfffff
        w = value | ((self.b[1] & 0xf0) << 16)
        self.b[1:4] = w.to_bytes(3, "big")

    def set_next_header(self, value):           # :125
        self.b[6] = value

    def set_hop_limit(self, value):             # :129
        self.b[7] = value

    def set_payload_len(self, value):           # :133 (the build sets it from the span)
        _put16(self.b, 4, value)

    def set_src_addr(self, value):
        self.b[8:24] = ipaddress.IPv6Address(value).packed

    def set_dst_addr(self, value):
        self.b[24:40] = ipaddress.IPv6Address(value).packed

    def set_pseudo_dst_offset(self, frame_off):
        """Not an rpkt setter: the frame offset of the address the L4 checksum's pseudo
        header uses as destination when a routing header with segments left was placed
        with move_back (RFC 8200 section 8.1; the record's ip6_pdst_off)."""
        self.pdst = int(frame_off)


class VlanFrame(_View):
    @classmethod
    def prepend_header(cls, buf, header=VLAN_FRAME_HEADER_TEMPLATE):
        """vlan/generated.rs:73-78"""
        assert len(header) == 4
        v = cls(buf, bytearray(header))
        buf._push("vlan", v, 4)
        return v

    def set_priority(self, value):              # :80
        assert value <= 7
        self.b[0] = (self.b[0] & 0x1f) | (value << 5)

    def set_dei_flag(self, value):              # :85
        self.b[0] = (self.b[0] & 0xef) | ((1 if value else 0) << 4)

    def set_vlan_id(self, value):               # :90
        assert value <= 0xfff
        _put16(self.b, 0, value | ((self.b[0] & 0xf0) << 8))

    def set_ethertype(self, value):             # :96
        _put16(self.b, 2, value)


class EtherFrame(_View):
    @classmethod
    def prepend_header(cls, buf, header=ETHER_FRAME_HEADER_TEMPLATE):
        """ether/generated.rs:71-76"""
        assert len(header) == 14
        v = cls(buf, bytearray(header))
        buf._push("ether", v, 14)
        return v

    def set_dst_addr(self, value):              # :78
        self.b[0:6] = bytes(value)

    def set_src_addr(self, value):              # :82
        self.b[6:12] = bytes(value)

    def set_ethertype(self, value):             # :86
        _put16(self.b, 12, value)


# rpkt/src/vxlan/generated.rs:12, gtpv1/generated.rs (GTPV1_HEADER_TEMPLATE), gre/generated.rs
VXLAN_HEADER_TEMPLATE = bytes(8)
GTPV1_HEADER_TEMPLATE = bytes([0x30, 0xff, 0x00, 0x00, 0x00, 0x00, 0x00, 0x00])   # :13
GRE_HEADER_TEMPLATE = bytes(4)                                                    # :13


class Vxlan(_View):
    """vxlan/generated.rs:99-161: Vxlan::prepend_header + setters (the encapsulation build,
    rpkt_gpu_build_tunnel_batch, vlan_mpls_tests.rs:254-300)."""
    kind = 1

    @classmethod
    def prepend_header(cls, buf, header=VXLAN_HEADER_TEMPLATE):
        assert len(header) == 8                              # :101 chunk_headroom >= 8
        v = cls(buf, bytearray(header))
        buf._push("vxlan", v, 8)
        return v

    def _bit(self, byte, bit, value):
        self.b[byte] = (self.b[byte] & ~(1 << bit) & 0xff) | ((1 if value else 0) << bit)

    def set_gbp_extention(self, v): self._bit(0, 7, v)          # :106
    def set_vni_present(self, v): self._bit(0, 3, v)            # :116
    def set_dont_learn(self, v): self._bit(1, 6, v)             # :129
    def set_policy_applied(self, v): self._bit(1, 3, v)         # :139

    def set_reserved_0(self, value):                           # :111
        assert value <= 0x7
        self.b[0] = (self.b[0] & 0x8f) | (value << 4)

    def set_reserved_1(self, value):                           # :121
        assert value <= 0xf
        w = (value << 7) | ((self.b[0] & 0xf8) << 8) | (self.b[1] & 0x7f)
        _put16(self.b, 0, w)

    def set_reserved_2(self, value):                           # :134
        assert value <= 0x3
        self.b[1] = (self.b[1] & 0xcf) | (value << 4)

    def set_reserved_3(self, value):                           # :144
        assert value <= 0x7
        self.b[1] = (self.b[1] & 0xf8) | value

    def set_group_id(self, value):                             # :149
        _put16(self.b, 2, value)

    def set_vni(self, value):                                  # :153
        assert value <= 0xffffff
        self.b[4:7] = int(value).to_bytes(3, "big")

    def set_reserved_4(self, value):                           # :158 (the build writes 0)
        self.b[7] = value

    def tun_fields(self):
        assert self.b[7] == 0, "reserved_4: the build writes the template's 0"
        return {"hdr0": self.b[0], "hdr1": self.b[1], "aux": _be16(self.b, 2),
                "id": (self.b[4] << 16) | (self.b[5] << 8) | self.b[6]}, []


class Gtpv1(_View):
    """gtpv1/generated.rs:110-170, 254-310: Gtpv1::prepend_header(header) + setters
    (gtpv1_test.rs:236-282); the extension headers after it are the caller's
    (CursorMut.move_back with their bytes, as ExtPduNumber::prepend_header writes them)."""
    kind = 2

    @staticmethod
    def header_len_of(header):
        return 8 if (header[0] & 0x7) == 0 else 12          # :239-250

    @classmethod
    def prepend_header(cls, buf, header=GTPV1_HEADER_TEMPLATE):
        assert len(header) == 8
        hl = cls.header_len_of(header)
        v = cls(buf, bytearray(header) + bytearray(hl - 8))
        buf._push("gtpv1", v, hl)
        assert buf.remaining() <= 65543                      # :116
        _put16(v.b, 2, buf.remaining() - 8)                  # set_packet_len(remaining)
        return v

    @staticmethod
    def set_header_flags(header, extention_header_present=None, sequence_present=None,
                         npdu_present=None, message_type=None, teid=None):
        """The setters on a header array (Gtpv1::from_header_array_mut, gtpv1_test.rs:249-256)."""
        h = bytearray(header)
        for bit, val in ((2, extention_header_present), (1, sequence_present), (0, npdu_present)):
            if val is not None:
                h[0] = (h[0] & ~(1 << bit) & 0xff) | ((1 if val else 0) << bit)
        if message_type is not None:
            h[1] = message_type
        if teid is not None:
            h[4:8] = int(teid).to_bytes(4, "big")
        return bytes(h)

    def header_len(self):
        return self.header_len_of(self.b)

    def set_teid(self, value):                                 # :163
        self.b[4:8] = int(value).to_bytes(4, "big")

    def set_message_type(self, value):                         # :159
        self.b[1] = value

    def set_sequence(self, value):                             # :287
        assert self.header_len() == 12
        _put16(self.b, 8, value)

    def set_npdu(self, value):                                 # :297
        assert self.header_len() == 12
        self.b[10] = value

    def set_next_extention_header(self, value):                # :307
        assert self.header_len() == 12
        self.b[11] = value

    def tun_fields(self):
        long = self.header_len() == 12
        f = {"hdr0": self.b[0], "hdr1": self.b[1], "id": _be32(self.b, 4),
             "aux": _be16(self.b, 8) if long else 0}
        # npdu and next_extention_header are not in the record: the caller's bytes
        return f, ([(10, bytes(self.b[10:12]))] if long else [])


class Gre(_View):
    """gre/generated.rs:104-340: Gre::prepend_header(header) + setters
    (gre_test.rs:213-278); a GRE header follows an IPv4 / IPv6 header of protocol 47."""
    kind = 3

    @staticmethod
    def header_len_of(header):                                 # gre/mod.rs:68-85
        ind = _be16(header, 0)
        return 4 + (4 if ind & 0xc000 else 0) + (4 if ind & 0x2000 else 0) + (4 if ind & 0x1000 else 0)

    @classmethod
    def prepend_header(cls, buf, header=GRE_HEADER_TEMPLATE):
        assert len(header) == 4
        hl = cls.header_len_of(header)
        v = cls(buf, bytearray(header) + bytearray(hl - 4))
        buf._push("gre", v, hl)
        return v

    def header_len(self):
        return self.header_len_of(self.b)

    @staticmethod
    def set_header_flags(header, checksum_present=None, routing_present=None,
                         key_present=None, sequence_present=None):
        """The flag setters on a header array (Gre::from_header_array_mut + set_*_present,
        :117-135, gre_test.rs:262-266): they decide the header's length."""
        h = bytearray(header)
        for bit, val in ((7, checksum_present), (6, routing_present), (5, key_present),
                         (4, sequence_present)):
            if val is not None:
                h[0] = (h[0] & ~(1 << bit) & 0xff) | ((1 if val else 0) << bit)
        return bytes(h)

    def set_protocol_type(self, value):                        # :157
        _put16(self.b, 2, value)

    def set_checksum(self, value):                             # :297
        assert self.b[0] & 0xc0
        _put16(self.b, 4, value)

    def set_offset(self, value):                               # :308
        assert self.b[0] & 0xc0
        _put16(self.b, 6, value)

    def set_key(self, value):                                  # :318
        assert self.b[0] & 0x20
        at = 8 if self.b[0] & 0xc0 else 4
        self.b[at:at + 4] = int(value).to_bytes(4, "big")

    def set_sequence(self, value):                             # :332
        assert self.b[0] & 0x10
        at = 4 + (4 if self.b[0] & 0xc0 else 0) + (4 if self.b[0] & 0x20 else 0)
        self.b[at:at + 4] = int(value).to_bytes(4, "big")

    def tun_fields(self):
        cr = 4 if self.b[0] & 0xc0 else 0
        f = {"hdr0": self.b[0], "hdr1": self.b[1], "inner_type": _be16(self.b, 2),
             "aux": _be16(self.b, 4) if cr else 0,
             "id": _be32(self.b, 4 + cr) if self.b[0] & 0x20 else 0}
        extra = [(6, bytes(self.b[6:8]))] if cr else []          # offset: the caller's
        if self.b[0] & 0x10:                                      # sequence: the caller's
            at = 4 + cr + (4 if self.b[0] & 0x20 else 0)
            extra.append((at, bytes(self.b[at:at + 4])))
        return f, extra


def tunnel_record(buf):
    """The rpkt_tun_t rpkt_gpu_build_tunnel_batch takes for a finished chain (kind NONE
    without a tunnel view), and the frame bytes of the tunnel header the build leaves as
    the buffer holds them (GTP npdu / next extension type, GRE offset / sequence)."""
    from .records import TUN_DTYPE
    t = np.zeros(1, dtype=TUN_DTYPE)[0]
    base = buf.start
    views = [(o, v) for k, o, v in buf.layers if k in ("vxlan", "gtpv1", "gre")]
    assert len(views) <= 1, "one tunnel level"
    extra = []
    if views:
        o, v = views[0]
        fields, left = v.tun_fields()
        t["kind"] = v.kind
        t["tun_off"] = o - base
        for k, x in fields.items():
            t[k] = x
        extra = [(o - base + at, b) for at, b in left]
    return t, extra


def assemble(records_extra, frame_lens, payloads=None):
    """A packed batch for rpkt_gpu_build_batch from finished chains: (frames buffer,
    u32 offsets, records).  Each frame is frame_len bytes: its payload (placed at the end)
    and the `extra` bytes its chain lists; the fixed header bytes are left zero for the
    build to write."""
    lens = np.asarray(frame_lens, dtype=np.int64)
    offs = np.zeros(lens.size + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    buf = np.zeros(int(offs[-1]), dtype=np.uint8)
    recs = np.zeros(lens.size, dtype=REC_DTYPE)
    for i, (r, extra) in enumerate(records_extra):
        recs[i] = r
        o = int(offs[i])
        if payloads is not None and payloads[i]:
            p = np.frombuffer(bytes(payloads[i]), np.uint8)
            buf[o + int(lens[i]) - p.size:o + int(lens[i])] = p
        for at, b in extra:
            buf[o + at:o + at + len(b)] = np.frombuffer(b, np.uint8)
    return buf, offs.astype(np.uint32), recs
