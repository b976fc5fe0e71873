"""Writes tests/golden/ip6_tx.json: IPv6 frames whose UDP / TCP checksums are worked out
here, independently of the engine and of its oracle, from RFC 8200 section 8.1 (the
pseudo header: source, final destination, 32-bit upper-layer length, 3 zero bytes and
the next header) and RFC 1071 (the one's-complement sum, complemented; a UDP result of 0
sent as 0xffff).  The reference has no IPv6 pseudo-header code, so these pin the IPv6
build / forward checksums of this repository to the RFC
rather than to the oracle written beside the kernels.

Run: python tests/golden/make_ip6_tx_golden.py (deterministic; no reference code used).
"""
import ipaddress
import json
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))


def rfc1071(data):
    if len(data) % 2:
        data += b"\0"
    s = sum(struct.unpack("!%dH" % (len(data) // 2), data))
    while s >> 16:
        s = (s & 0xffff) + (s >> 16)
    return (~s) & 0xffff


def frame(kind, payload, routing_final=None):
    src = ipaddress.IPv6Address("2001:db8:1::10").packed
    dst = ipaddress.IPv6Address("2001:db8:2::20").packed
    ext = b""
    nh_l4 = 17 if kind == "udp" else 6
    first_nh = nh_l4
    pdst = dst
    if routing_final is not None:
        fin = ipaddress.IPv6Address(routing_final).packed
        # Routing header type 0, 1 segment left, one address (RFC 8200 section 4.4)
        ext = bytes([nh_l4, 2, 0, 1, 0, 0, 0, 0]) + fin
        first_nh = 43
        pdst = fin
    if kind == "udp":
        l4 = struct.pack("!HHHH", 40000, 4789, 8 + len(payload), 0) + payload
        ck_off = 6
    else:
        l4 = struct.pack("!HHIIBBHHH", 443, 51000, 0x01020304, 0x0a0b0c0d, 5 << 4, 0x18,
                         8192, 0, 0) + payload
        ck_off = 16
    pseudo = src + pdst + struct.pack("!I", len(l4)) + b"\0\0\0" + bytes([nh_l4])
    ck = rfc1071(pseudo + l4)
    if kind == "udp" and ck == 0:
        ck = 0xffff
    l4 = l4[:ck_off] + struct.pack("!H", ck) + l4[ck_off + 2:]
    ip = struct.pack("!IHBB", (6 << 28) | (0x2e << 20) | 0xbeef, len(ext) + len(l4), first_nh,
                     64) + src + dst
    eth = bytes.fromhex("020000000001" "020000000002" "86dd")
    return eth + ip + ext + l4, ck


def main():
    cases = []
    for kind, payload, rt in (("udp", bytes(range(37)), None),
                              ("udp", b"\xff" * 18, "2001:db8:3::30"),
                              ("tcp", bytes(range(200, 256)) * 3, None),
                              ("tcp", b"abc", "2001:db8:3::30")):
        f, ck = frame(kind, payload, rt)
        cases.append({"kind": kind, "routing_final": rt, "frame": f.hex(), "checksum": ck})
    with open(os.path.join(HERE, "ip6_tx.json"), "w") as fh:
        json.dump(cases, fh, indent=1)


if __name__ == "__main__":
    main()
