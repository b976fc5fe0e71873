"""Header-field getters over the layer walk (rpkt_gpu_fields_batch's checker,
oracle/rpkt_oracle_fields.c): pinned by the getter values the reference's own tests
assert on its captures, and checked against pktfmt's shift-and-mask form
(pktfmt/src/codegen/field.rs:115-250, restated below in Python) for every field of
every protocol the walk reaches on fuzzed traffic."""
import os

import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import fields, gen

HERE = os.path.dirname(os.path.abspath(__file__))
PKTS = os.path.join(HERE, "golden", "packets")


def get(name, items):
    f = oracle.load_dat(os.path.join(PKTS, name))
    frames = np.frombuffer(f, np.uint8)
    offs = np.array([0, len(f)], np.uint32)
    lay = oracle.layers_batch(frames, 1, offsets=offs)
    v, p = oracle.fields_batch(frames, 1, lay, fields.requests(items), offsets=offs)
    assert p[0] == (1 << len(items)) - 1, (name, bin(int(p[0])))
    return [int(x) for x in v[0]]


def test_field_kats_from_reference_tests():
    # ipv6_test.rs:20-45 (ipv6_options_destination.dat)
    v = get("ipv6_options_destination.dat", [
        ("IPV6_IPV6", "version"), ("IPV6_IPV6", "traffic_class"), ("IPV6_IPV6", "flow_label"),
        ("IPV6_IPV6", "payload_len_"), ("IPV6_IPV6", "next_header"), ("IPV6_IPV6", "hop_limit"),
        ("IPV6_IPV6", "src_addr", 0, "hi"), ("IPV6_IPV6", "src_addr", 0, "lo"),
        ("IPV6_IPV6", "dst_addr", 0, "hi"), ("IPV6_IPV6", "dst_addr", 0, "lo"),
        ("IPV6_DESTOPTIONS", "next_header")])
    assert v[:6] == [6, 0, 0, 26, 60, 64] and v[10] == 17
    import ipaddress
    assert fields.join128(v[6], v[7]) == ipaddress.IPv6Address(
        "2a01:e35:8bd9:8bb0:a0a7:ea9c:74e8:d397").packed
    assert fields.join128(v[8], v[9]) == ipaddress.IPv6Address(
        "2001:4b98:dc0:41:216:3eff:fece:1902").packed
    # ipv6_test.rs:320-350 (ipv6_options_fragments.dat): the 13-bit offset, 1-bit flag
    v = get("ipv6_options_fragments.dat", [
        ("IPV6_IPV6", "flow_label"), ("IPV6_IPV6", "payload_len_"),
        ("IPV6_FRAGMENTHEADER", "next_header"), ("IPV6_FRAGMENTHEADER", "reserved"),
        ("IPV6_FRAGMENTHEADER", "offset"), ("IPV6_FRAGMENTHEADER", "reserved1"),
        ("IPV6_FRAGMENTHEADER", "more_frag"), ("IPV6_FRAGMENTHEADER", "ident")])
    assert v == [0x21289, 1456, 17, 0, 181, 0, 1, 0xf88eb466]
    # eth_and_arp_test.rs:15-45 (ArpResponsePacket.dat)
    v = get("ArpResponsePacket.dat", [
        ("ARP_ARP", "hardware_type"), ("ARP_ARP", "protocol_type"),
        ("ARP_ARP", "hardware_addr_len"), ("ARP_ARP", "protocol_addr_len"),
        ("ARP_ARP", "operation"), ("ARP_ARP", "sender_ipv4_addr"),
        ("ARP_ARP", "target_ether_addr"), ("ETHER_ETHERFRAME", "dst_addr")])
    assert v[:6] == [1, 0x0800, 6, 4, 2, int.from_bytes(bytes([10, 0, 0, 138]), "big")]
    assert v[6] == v[7] == 0x6cf049b2de6e
    # gtpv1_test.rs:15-46 (gtp-c1.dat)
    v = get("gtp-c1.dat", [
        ("UDP_UDP", "src_port"), ("UDP_UDP", "dst_port"), ("GTPV1_GTPV1", "version"),
        ("GTPV1_GTPV1", "protocol_type"), ("GTPV1_GTPV1", "extention_header_present"),
        ("GTPV1_GTPV1", "sequence_present"), ("GTPV1_GTPV1", "npdu_present"),
        ("GTPV1_GTPV1", "teid")])
    assert v == [2123, 2123, 1, 1, 0, 1, 0, 0x09fe4b60]
    # gtpv2_test.rs:10-36 (gtpv2-with-teid.dat)
    v = get("gtpv2-with-teid.dat", [
        ("GTPV2_GTPV2", "version"), ("GTPV2_GTPV2", "piggybacking_flag"),
        ("GTPV2_GTPV2", "teid_present"), ("GTPV2_GTPV2", "message_priority_present"),
        ("GTPV2_GTPV2", "message_type")])
    assert v == [2, 0, 1, 0, 34]
    # vlan_mpls_tests.rs:224-248 (Vxlan1.dat): vni_present, vni; the inner Ethernet
    # frame is the second ETHERFRAME layer (nth = 1)
    v = get("Vxlan1.dat", [("VXLAN_VXLAN", "vni_present"), ("VXLAN_VXLAN", "vni"),
                           ("ETHER_ETHERFRAME", "ethertype", 0),
                           ("ETHER_ETHERFRAME", "ethertype", 1)])
    assert v[:2] == [1, 3000001] and v[2] == 0x0800


def shift_mask(h, off, bits):
    """pktfmt's generated getter (field.rs:115-160): the big-endian integer of bytes
    [start, end], >> (7 - end bit), & ones(bits)."""
    sb, eb = off // 8, (off + bits - 1) // 8
    x = int.from_bytes(h[sb:eb + 1], "big") >> (7 - (off + bits - 1) % 8)
    return x & ((1 << bits) - 1)


def all_requests():
    """Every field of every protocol, 128-bit ones as halves, in batches of <= 32."""
    out = []
    for name, p in fields.table().items():
        for fname, (off, bits) in p["fields"].items():
            for nth in (0, 1):
                if bits == 128:
                    out += [fields.field(name, fname, nth, "hi"), fields.field(name, fname, nth, "lo")]
                elif bits <= 64:
                    out.append(fields.field(name, fname, nth))
    return [out[k:k + 32] for k in range(0, len(out), 32)]


def test_oracle_matches_pktfmt_getters_on_fuzz():
    hb = gen.make_mix(3000, seed=23)
    lay = oracle.layers_batch(hb.frames, hb.n, offsets=hb.offsets)
    hits = 0
    for chunk in all_requests():
        reqs = fields.requests(chunk)
        v, pres = oracle.fields_batch(hb.frames, hb.n, lay, reqs, offsets=hb.offsets)
        for i in range(hb.n):
            f = hb.frames[hb.offsets[i]:hb.offsets[i + 1]].tobytes()
            L = lay[i]
            for r, (pid, nth, bits, off) in enumerate(chunk):
                ks = [k for k in range(L["n"]) if L["proto"][k] == pid]
                want, ok = 0, False
                if len(ks) > nth:
                    lo = int(L["off"][ks[nth]])
                    if lo + (off + bits - 1) // 8 < len(f):
                        want, ok = shift_mask(f[lo:], off, bits), True
                assert bool(pres[i] >> r & 1) == ok and int(v[i, r]) == want, (i, chunk[r])
                hits += ok
    assert hits > 20000


def test_unaligned_64bit_field_spans_nine_bytes():
    """A 64-bit request at a nonzero bit phase reads 9 bytes (the kernel's two-part
    form); the oracle's bitwise walk and the shift-and-mask form agree."""
    hb = gen.make_mix(200, seed=5)
    lay = oracle.layers_batch(hb.frames, hb.n, offsets=hb.offsets)
    chunk = [(0, 0, 64, s) for s in range(1, 8)] + [(0, 0, 33, 3), (0, 0, 1, 111)]
    v, pres = oracle.fields_batch(hb.frames, hb.n, lay, fields.requests(chunk), offsets=hb.offsets)
    for i in range(hb.n):
        f = hb.frames[hb.offsets[i]:hb.offsets[i + 1]].tobytes()
        for r, (_, _, bits, off) in enumerate(chunk):
            if pres[i] >> r & 1:
                assert int(v[i, r]) == shift_mask(f, off, bits)


def test_request_builder_rejects_bad_widths():
    with pytest.raises(ValueError):
        fields.field("IPV6_IPV6", "src_addr")
    with pytest.raises(ValueError):
        fields.field("IPV4_IPV4", "ttl", 0, "hi")
    with pytest.raises(ValueError):
        fields.requests([("IPV4_IPV4", "ttl")] * 33)


def random_requests(rng, k=32, max_bit=8 * 160):
    """Requests past the fixed headers too: any protocol, bit offset and width, so
    fields that cross or pass the frame's end (and the buffer's last dword) occur."""
    names = list(fields.table())
    out = []
    for _ in range(k):
        p = fields.table()[names[rng.integers(len(names))]]
        out.append((p["id"], int(rng.integers(2)), int(rng.integers(1, 65)),
                    int(rng.integers(0, max_bit))))
    return out


def test_oracle_matches_pktfmt_form_on_random_requests():
    rng = np.random.default_rng(77)
    hb = gen.make_mix(1500, seed=41)
    lay = oracle.layers_batch(hb.frames, hb.n, offsets=hb.offsets)
    hits = misses = 0
    for _ in range(6):
        chunk = random_requests(rng)
        v, pres = oracle.fields_batch(hb.frames, hb.n, lay, fields.requests(chunk),
                                      offsets=hb.offsets)
        for i in range(hb.n):
            f = hb.frames[hb.offsets[i]:hb.offsets[i + 1]].tobytes()
            L = lay[i]
            for r, (pid, nth, bits, off) in enumerate(chunk):
                ks = [k for k in range(L["n"]) if L["proto"][k] == pid]
                ok = len(ks) > nth and int(L["off"][ks[nth]]) + (off + bits - 1) // 8 < len(f)
                want = shift_mask(f[int(L["off"][ks[nth]]):], off, bits) if ok else 0
                assert bool(pres[i] >> r & 1) == ok and int(v[i, r]) == want, (i, chunk[r])
                hits += ok
                misses += (len(ks) > nth) and not ok
    assert hits > 1000 and misses > 1000
