"""Tunnel frames the generator (configs 13/14) does not make: VXLAN / GTP-U / GRE over an
IPv6 or VLAN-tagged outer frame, GTP-U extension chains that run past the 128-B header
window, and GRE over IPv6.  Built in numpy-free Python (checksums from RFC 1071 here,
independent of the engine and the oracle), shared by the oracle and the GPU tests."""
import struct

import numpy as np


def rfc1071(data):
    if len(data) % 2:
        data += b"\0"
    s = sum(struct.unpack("!%dH" % (len(data) // 2), data))
    while s >> 16:
        s = (s & 0xffff) + (s >> 16)
    return (~s) & 0xffff


def ipv4_packet(proto, payload, src=0x0a000001, dst=0x0a000002, ttl=64):
    h = bytearray(struct.pack("!BBHHHBBHII", 0x45, 0, 20 + len(payload), 0x1234, 0x4000, ttl,
                              proto, 0, src, dst))
    h[10:12] = struct.pack("!H", rfc1071(bytes(h)))
    if proto == 17:
        u = bytearray(payload)
        ps = struct.pack("!IIBBH", src, dst, 0, 17, len(u))
        ck = rfc1071(ps + bytes(u[:6]) + b"\0\0" + bytes(u[8:])) or 0xffff
        u[6:8] = struct.pack("!H", ck)
        payload = bytes(u)
    return bytes(h) + payload


def ipv6_packet(nh, payload, src=b"\x20\x01\x0d\xb8" + bytes(11) + b"\x01",
                dst=b"\x20\x01\x0d\xb8" + bytes(11) + b"\x02"):
    h = struct.pack("!IHBB", 6 << 28, len(payload), nh, 64) + src + dst
    if nh == 17:
        u = bytearray(payload)
        ps = src + dst + struct.pack("!I", len(u)) + b"\0\0\0\x11"
        ck = rfc1071(ps + bytes(u[:6]) + b"\0\0" + bytes(u[8:])) or 0xffff
        u[6:8] = struct.pack("!H", ck)
        payload = bytes(u)
    return h + payload


def udp(sport, dport, payload):
    return struct.pack("!HHHH", sport, dport, 8 + len(payload), 0) + payload


def ether(et, payload, tags=()):
    b = bytes.fromhex("020000000001020000000002")
    for tpid, tci in tags:
        b += struct.pack("!HH", tpid, tci)
    return b + struct.pack("!H", et) + payload


def inner_udp4(n):
    return ipv4_packet(17, udp(5000, 53, bytes((k * 7 + 3) & 0xff for k in range(n))),
                       src=0xc0a80001, dst=0xc0a80002)


def vxlan(inner_frame, vni=0x123456):
    return struct.pack("!BBHI", 0x08, 0, 0, vni << 8) + inner_frame


def gtpu(tpdu, exts=(), teid=0xdeadbeef, seq=None):
    """GTPv1 G-PDU with extension headers [(type, body bytes)], each padded to 4n bytes
    with its next type last."""
    flags = 0x30 | (0x04 if exts else 0) | (0x02 if seq is not None else 0)
    opt = b""
    if exts or seq is not None:
        opt = struct.pack("!HBB", seq or 0, 0, exts[0][0] if exts else 0)
        for k, (t, body) in enumerate(exts):
            nxt = exts[k + 1][0] if k + 1 < len(exts) else 0
            n = (len(body) + 2 + 3) // 4 * 4
            opt += bytes([n // 4]) + body + bytes(n - 2 - len(body)) + bytes([nxt])
    rest = opt + tpdu
    return struct.pack("!BBHI", flags, 255, len(rest), teid) + rest


def gre(inner, proto=0x0800, checksum=False, key=None):
    b0 = (0x80 if checksum else 0) | (0x20 if key is not None else 0)
    h = struct.pack("!BBH", b0, 0, proto)
    if checksum:
        h += b"\0\0\0\0"
    if key is not None:
        h += struct.pack("!I", key)
    pkt = bytearray(h + inner)
    if checksum:
        pkt[4:6] = struct.pack("!H", rfc1071(bytes(pkt)))
    return bytes(pkt)


def odd_frames(seed=0, n=64):
    """A list of frames: outer IPv6 / VLAN-tagged, long GTP extension chains, GRE over IPv6,
    and random cuts and byte flips of them."""
    rng = np.random.default_rng(seed)
    base = []
    inner_eth = ether(0x0800, inner_udp4(40))
    base.append(ether(0x86dd, ipv6_packet(17, udp(40000, 4789, vxlan(inner_eth)))))
    base.append(ether(0x0800, ipv4_packet(17, udp(40000, 4789, vxlan(inner_eth))),
                      tags=((0x88a8, 30), (0x8100, 100))))
    for n_ext in (1, 3, 5, 8, 9):
        exts = [(0x81, bytes(range(30)))] * (n_ext - 1) + [(0x85, bytes([0x10, 1]))]
        base.append(ether(0x0800, ipv4_packet(17, udp(2152, 2152, gtpu(inner_udp4(60), exts,
                                                                         seq=77)))))
    base.append(ether(0x86dd, ipv6_packet(17, udp(2152, 2152, gtpu(
        ipv6_packet(17, udp(1, 2, b"abcdefgh")), [(0xc0, b"\x09\x04")])))))
    base.append(ether(0x86dd, ipv6_packet(47, gre(inner_udp4(100), checksum=True, key=7))))
    base.append(ether(0x86dd, ipv6_packet(47, gre(ipv6_packet(17, udp(9, 9, b"x" * 33)),
                                                  proto=0x86dd, checksum=True))))
    base.append(ether(0x0800, ipv4_packet(47, gre(inner_eth, proto=0x6558, key=0xfde8))))
    out = list(base)
    while len(out) < n:
        f = bytearray(base[int(rng.integers(len(base)))])
        if rng.integers(2):
            f = f[:int(rng.integers(0, len(f) + 1))]
        for _ in range(int(rng.integers(0, 3))):
            if len(f) > 40:
                f[int(rng.integers(34, len(f)))] = int(rng.integers(0, 256))
        out.append(bytes(f))
    return out


def jumbo_frames(seed=0, n=48):
    """Tunnelled jumbo frames (inner payloads of 1.4 KB to 60 KB: the long-stream and
    tail-line paths of the tunnel parse), mixed with short tunnel frames, and cuts of them."""
    rng = np.random.default_rng(seed)
    base = []
    for p in (1400, 8950, 16000, 60000):
        inner = inner_udp4(p)
        base.append(ether(0x0800, ipv4_packet(17, udp(40000, 4789, vxlan(ether(0x0800, inner))))))
        base.append(ether(0x0800, ipv4_packet(47, gre(inner, checksum=True, key=9))))
        if p <= 30000:
            base.append(ether(0x0800, ipv4_packet(17, udp(2152, 2152, gtpu(
                inner, [(0xc0, b"\x09\x04"), (0x85, bytes([0x10, 1]))], seq=5)))))
            base.append(ether(0x86dd, ipv6_packet(17, udp(40000, 4789, vxlan(ether(0x0800, inner))))))
    base.append(ether(0x0800, ipv4_packet(17, udp(40000, 4789, vxlan(ether(0x0800, inner_udp4(40)))))))
    out = list(base)
    while len(out) < n:
        f = bytes(base[int(rng.integers(len(base)))])
        if rng.integers(2):
            f = f[:int(rng.integers(0, len(f) + 1))]
        out.append(f)
    order = rng.permutation(len(out))
    return [out[k] for k in order]
