"""Synthetic IPv6 frames for the IPv6 tests (host side, no GPU): Ether [+ 802.1Q] +
IPv6 + extension headers + UDP/TCP with a valid L4 sum over the final address."""
import numpy as np

from oracle import oracle


def ip6_opts(rng, n, bad=False):
    """n bytes of IPv6 options (Pad0 / PadN / RouterAlert / Generic), optionally ending in
    a malformed one."""
    out = bytearray()
    while len(out) < n:
        left = n - len(out)
        k = int(rng.integers(0, 4))
        if k == 1 and left >= 4:
            out += bytes([5, 2]) + int(rng.integers(0, 3)).to_bytes(2, "big")
        elif k == 2 and left >= 3:
            dl = int(min(left - 2, rng.integers(1, 9)))
            out += bytes([int(rng.choice([2, 11, 0xc2])), dl]) + \
                rng.integers(0, 256, dl, dtype=np.uint8).tobytes()
        elif k == 3 and left >= 2:
            dl = int(min(left - 2, rng.integers(0, 6)))
            out += bytes([1, dl]) + bytes(dl)
        else:
            out += b"\x00"
    if bad and n >= 2:
        out[-2:] = bytes([11, 9])                      # header_len past the slice
    return bytes(out)


def ip6_frame(rng, exts, proto, payload, tag=False, opts=False):
    """Ether [+ 802.1Q] + IPv6 + extension headers (type, header_len) + UDP/TCP + payload
    bytes; the L4 checksum is stamped valid with the pseudo header over the final address."""
    f = bytearray(b"\x02\x00\x00\x00\x00\x01\x02\x00\x00\x00\x00\x02")
    if tag:
        f += b"\x81\x00" + bytes([0x20, 0x07])
    f += b"\x86\xdd"
    l3 = len(f)
    src = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
    dst = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
    chain = bytearray()
    types = [t for t, _ in exts] + [proto]
    pdst = dst
    for k, (t, hl) in enumerate(exts):
        h = bytearray(rng.integers(0, 256, hl, dtype=np.uint8).tobytes())
        h[0] = types[k + 1]
        if t in (0, 60, 43):
            h[1] = hl // 8 - 1
        if t in (0, 60):
            h[2:hl] = (ip6_opts(rng, hl - 2, bad=rng.integers(0, 8) == 0) if opts
                       else bytes(hl - 2))                               # Pad0 options
        if t == 43:
            h[2], h[3] = 0, 1                                            # type 0, 1 left
            n = (hl - 8) // 16
            pdst = bytes(h[8 + 16 * (n - 1):8 + 16 * n])
        if t == 44:
            h[1], h[2], h[3] = 0, 0, 0                                   # atomic
        if t == 51:
            h[1] = hl // 4 - 2
        chain += h
    l4h = 8 if proto == 17 else 20
    seg = bytearray(l4h) + bytearray(payload)
    seg[0:4] = b"\x13\x88\x01\xbb"
    if proto == 17:
        seg[4:6] = len(seg).to_bytes(2, "big")
    else:
        seg[12] = 0x50
    ph = src + pdst + len(seg).to_bytes(4, "big") + bytes([0, 0, 0, proto])
    ck = ~oracle.combine([oracle.from_slice(ph), oracle.from_slice(bytes(seg))]) & 0xffff
    at = 6 if proto == 17 else 16
    seg[at:at + 2] = ck.to_bytes(2, "big")
    ip = bytearray(40)
    ip[0] = 0x60
    ip[4:6] = (len(chain) + len(seg)).to_bytes(2, "big")
    ip[6] = types[0]
    ip[7] = 64
    ip[8:24], ip[24:40] = src, dst
    return bytes(f + ip + chain + seg)
