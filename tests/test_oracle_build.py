"""The TX-side oracle (oracle/rpkt_oracle_build.c) pinned on the reference's own
captures: rebuilding a fixture's headers from its parse record, on a buffer whose
fixed header bytes were wiped, must give back the captured bytes (setter layout),
and filling the checksums must give back the checksums real stacks computed."""
import os
import sys

import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import gen
from rpkt_amd.records import STATUS

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
PKTS = os.path.join(HERE, "golden", "packets")
UDP, TCP = 17, 6


def fixture_frames():
    out = []
    for name in sorted(os.listdir(PKTS)):
        f = oracle.load_dat(os.path.join(PKTS, name))
        r = oracle.parse_one(f, 3)
        if r["status"] in (STATUS["OK"], STATUS["L4_OTHER"]):
            out.append((name, f, r))
    return out


def fixed_ranges(r):
    """The bytes prepend_header + setters write (option bytes excluded)."""
    l3, l4, p = int(r["l3_off"]), int(r["l4_off"]), int(r["ip_protocol"])
    rng = [(0, l3 + 20)]
    if r["status"] == STATUS["OK"]:
        rng.append((l4, l4 + (8 if p == UDP else 20)))
    return rng


def rebuild(f, r, flags):
    """Wipe the fixed header bytes of the frame cut to its IPv4 packet, rebuild."""
    cut = int(r["l3_off"]) + int(r["ip_packet_len"])
    work = bytearray(f[:cut])
    for a, b in fixed_ranges(r):
        work[a:b] = bytes(b - a)
    rec = np.array([r])
    out, built = oracle.build_batch(np.frombuffer(bytes(work), np.uint8), 1, rec, flags,
                                    offsets=np.array([0, cut], np.uint32))
    return bytes(out), int(built[0]), f[:cut]


def length_consistent(r):
    if r["status"] != STATUS["OK"] or r["ip_protocol"] != UDP:
        return True
    return int(r["l4_word6"]) == int(r["ip_packet_len"]) - (int(r["l4_off"]) - int(r["l3_off"]))


def test_rebuild_fixtures_setter_layout():
    n = 0
    for name, f, r in fixture_frames():
        if not length_consistent(r):
            continue
        out, built, want = rebuild(f, r, 0)
        assert built == 1, name
        assert out == want, name
        n += 1
    assert n >= 25


def test_rebuild_fixtures_checksum_fill():
    """The TX checksum fill recomputes what the capturing stacks stored: every
    fixture whose stored checksums verify is reproduced byte for byte."""
    n_ip = n_l4 = 0
    for name, f, r in fixture_frames():
        if not length_consistent(r):
            continue
        ip_ok = r["ip_sum"] == 0xFFFF
        l4_ok = (r["status"] == STATUS["OK"] and r["l4_sum"] == 0xFFFF and
                 not (r["ip_protocol"] == UDP and r["l4_checksum"] == 0))
        flags = (1 if ip_ok else 0) | (2 if l4_ok else 0)
        out, built, want = rebuild(f, r, flags)
        assert built == 1 and out == want, name
        n_ip += ip_ok
        n_l4 += l4_ok
    assert n_ip >= 25 and n_l4 >= 8


def test_build_rejects_frames_too_short():
    f = gen.make_batch(3, n=1).frames[:1500].tobytes()
    r = oracle.parse_one(f, 3)
    rec = np.array([r, r, r])
    frames = np.frombuffer(f[:53] + f[:54] + f[:33], np.uint8)
    offs = np.array([0, 53, 107, 140], np.uint32)
    out, built = oracle.build_batch(frames, 3, rec, 3, offsets=offs)
    assert built.tolist() == [0, 1, 0]
    assert bytes(out[:53]) == f[:53] and bytes(out[107:]) == f[:33]


def test_built_frames_parse_back():
    """Round trip at batch scale: records of a config-5 batch (VLAN/QinQ, IPv4 and
    TCP options) rebuilt onto wiped headers parse back to the same records, with
    filled checksums that verify."""
    hb = gen.make_batch(5, n=3000)
    recs = oracle.parse_batch(hb.frames, hb.n, 3, offsets=hb.offsets)
    work = hb.frames.copy()
    for i, r in enumerate(recs):
        if r["status"] == STATUS["OK"]:
            for a, b in fixed_ranges(r):
                o = int(hb.offsets[i])
                work[o + a:o + b] = 0
    out, built = oracle.build_batch(work, hb.n, recs, 3, offsets=hb.offsets)
    back = oracle.parse_batch(out, hb.n, 3, offsets=hb.offsets)
    ok = recs["status"] == STATUS["OK"]
    pad = recs["ip_packet_len"] + recs["l3_off"] != np.diff(hb.offsets.astype(np.int64))
    sel = ok & ~pad
    assert sel.sum() > 2500 and built[sel].all()
    assert (back["ip_sum"][sel] == 0xFFFF).all() and (back["l4_sum"][sel] == 0xFFFF).all()
    for k in ("src_port", "dst_port", "tcp_seq", "tcp_ack", "l4_word6", "ip_src", "ip_dst",
              "ip_ident", "ip_ttl", "vlan_tci", "n_vlan", "payload_off", "payload_len"):
        assert np.array_equal(back[k][sel], recs[k][sel]), k


def test_forward_rewrites_like_loopback_rx():
    hb = gen.make_batch(2, n=4000)
    recs = oracle.parse_batch(hb.frames, hb.n, 3, stride=hb.stride)
    dmac, smac = bytes([0xAC, 0xDC, 0xCA, 0x79, 0xCA, 0x86]), bytes([0xAC, 0xDC, 0xCA, 0x79, 0xE5, 0xC6])
    forbid = np.unique(recs["ip_src"][:50])
    out, keep = oracle.forward_batch(hb.frames, hb.n, recs, dmac, smac, forbid, stride=hb.stride)
    back = oracle.parse_batch(out, hb.n, 3, stride=hb.stride)
    k = keep.astype(bool)
    want_keep = (recs["ip_sum"] == 0xFFFF) & ~np.isin(recs["ip_src"], forbid)
    assert np.array_equal(k, want_keep)
    assert 0.9 < k.mean() < 0.99
    assert (back["ip_src"][k] == recs["ip_dst"][k]).all()
    assert (back["src_port"][k] == recs["dst_port"][k]).all()
    assert (back["ip_ttl"][k] == (recs["ip_ttl"][k].astype(np.int64) - 1) % 256).all()
    assert (back["ip_sum"][k] == 0xFFFF).all() and (back["l4_sum"][k] == 0xFFFF).all()
    assert (back["dst_addr"][k] == np.frombuffer(dmac, np.uint8)).all()
    frames = out.reshape(-1, 64)
    assert np.array_equal(frames[~k], hb.frames.reshape(-1, 64)[~k])


# ---- IPv6 records (Ipv6::prepend_header + setters, ipv6/generated.rs:94-135) ----
F_IPV6 = 8


def fixed_ranges6(r):
    """Bytes the IPv6 build writes: link layer, IPv6 bytes 0..7 (addresses and extension
    headers are the buffer's), the fixed L4 header."""
    l3, l4, p = int(r["l3_off"]), int(r["l4_off"]), int(r["ip_protocol"])
    rng = [(0, l3 + 8)]
    if r["status"] == STATUS["OK"]:
        rng.append((l4, l4 + (8 if p == UDP else 20)))
    return rng


def ip6_payload_len(r):
    b = np.array([r]).view(np.uint8)
    return int(b[28]) | int(b[29]) << 8


def rebuild6(f, r, flags):
    cut = int(r["l3_off"]) + 40 + ip6_payload_len(r)
    work = bytearray(f[:cut])
    for a, b in fixed_ranges6(r):
        work[a:b] = bytes(b - a)
    out, built = oracle.build_batch(np.frombuffer(bytes(work), np.uint8), 1, np.array([r]), flags,
                                    offsets=np.array([0, cut], np.uint32))
    return bytes(out), int(built[0]), f[:cut]


def ip6_fixtures():
    out = []
    for name in sorted(os.listdir(PKTS)):
        f = oracle.load_dat(os.path.join(PKTS, name))
        r = oracle.parse_one(f, 3 | F_IPV6)
        if oracle_is6(r) and int(r["l4_off"]) >= int(r["l3_off"]) + 40 and \
                r["status"] in (STATUS["OK"], STATUS["L4_OTHER"]):
            out.append((name, f, r))
    return out


def test_rebuild_ip6_fixtures():
    """The reference's IPv6 captures rebuilt from their records onto wiped headers give
    back the captured bytes; with the L4 fill, those whose stored checksum verifies
    (the routing-header one over its final address) are reproduced byte for byte."""
    fx = ip6_fixtures()
    assert len(fx) >= 5, [n for n, _, _ in fx]
    n_l4 = 0
    for name, f, r in fx:
        out, built, want = rebuild6(f, r, 0)
        assert built == 1 and out == want, name
        l4_ok = r["status"] == STATUS["OK"] and r["l4_sum"] == 0xFFFF
        out, built, want = rebuild6(f, r, 3 if l4_ok else 1)
        assert built == 1 and out == want, name
        n_l4 += l4_ok
    assert n_l4 >= 2


@pytest.mark.parametrize("cfg", [10, 11])
def test_ip6_built_frames_parse_back(cfg):
    """Dual-stack batches (configs 10, 11: IPv6 with 0-3 extension headers): every record
    rebuilt onto wiped headers parses back to the same record, and the filled L4
    checksums verify, for the IPv4 and the IPv6 frames alike."""
    hb = gen.make_batch(cfg, n=4000)
    fl = 3 | F_IPV6
    recs = oracle.parse_batch(hb.frames, hb.n, fl, stride=hb.stride)
    work = hb.frames.copy()
    ok = recs["status"] == STATUS["OK"]
    is6 = np.array([oracle_is6(r) for r in recs])
    for i, r in enumerate(recs):
        if ok[i]:
            o = i * hb.stride
            for a, b in (fixed_ranges6(r) if is6[i] else fixed_ranges(r)):
                work[o + a:o + b] = 0
    out, built = oracle.build_batch(work, hb.n, recs, 3, stride=hb.stride)
    back = oracle.parse_batch(out, hb.n, fl, stride=hb.stride)
    assert is6[ok].sum() > 1000 and (~is6[ok]).sum() > 1000
    assert built[ok].all()
    assert (back["l4_sum"][ok] == 0xFFFF).all()
    # frames whose stored sums verified come back byte-identical (the injected bad sums
    # and IPv4's "not computed" UDP zero are refilled)
    good = ok & (recs["l4_sum"] == 0xFFFF) & (is6 | ((recs["ip_sum"] == 0xFFFF) &
                                                      (recs["l4_checksum"] != 0)))
    assert good.sum() > 0.9 * ok.sum()
    assert back[good].tobytes() == recs[good].tobytes()


def oracle_is6(r):
    et = int(r["vlan_ethertype"][r["n_vlan"] - 1]) if r["n_vlan"] else int(r["ethertype"])
    return et == 0x86DD and r["status"] not in (STATUS["ETH_SHORT"], STATUS["VLAN_SHORT"],
                                                STATUS["NOT_IPV4"])


def test_ip6_build_rejects_short_and_keeps_addresses():
    """An IPv6 record whose frame cannot hold its headers is not built; a built frame
    keeps the buffer's address and extension-header bytes."""
    import ip6_frames
    rng = np.random.default_rng(3)
    f = ip6_frames.ip6_frame(rng, [(43, 24), (60, 16)], 17, bytes(30))
    r = oracle.parse_one(f, 3 | F_IPV6)
    assert r["status"] == STATUS["OK"]
    l4 = int(r["l4_off"])
    buf = np.frombuffer(f + f[:l4 + 7], np.uint8)
    out, built = oracle.build_batch(buf, 2, np.array([r, r]), 3,
                                    offsets=np.array([0, len(f), len(f) + l4 + 7], np.uint32))
    assert built.tolist() == [1, 0]
    assert bytes(out[:len(f)]) == f and bytes(out[len(f):]) == f[:l4 + 7]


def test_forward_ip6_like_loopback_rx():
    """rpkt_fwd_t.flags = RPKT_F_IPV6: untagged IPv6/UDP frames with a valid L4 sum are
    forwarded (addresses and ports swapped, hop_limit - 1, MACs, UDP checksum valid over
    the new pseudo header, the routing header's final address kept); without the flag
    they are not.  IPv4 frames are forwarded as before either way."""
    import ip6_frames
    rng = np.random.default_rng(11)
    frames = []
    for k in range(300):
        exts = [[], [(43, 24)], [(0, 8), (43, 40)], [(60, 16)]][k % 4]
        f = bytearray(ip6_frames.ip6_frame(rng, exts, 17 if k % 5 else 6, bytes(20 + k % 7),
                                           tag=(k % 11 == 0)))
        if k % 13 == 0:
            f[-1] ^= 0x5a                                  # bad L4 sum
        frames.append(bytes(f))
    hb4 = gen.make_batch(2, n=100)
    frames += [hb4.frames[i * 64:(i + 1) * 64].tobytes() for i in range(100)]
    offs = np.concatenate([[0], np.cumsum([len(f) for f in frames])]).astype(np.uint32)
    buf = np.frombuffer(b"".join(frames), np.uint8)
    recs = oracle.parse_batch(buf, len(frames), 3 | F_IPV6, offsets=offs)
    dmac, smac = bytes(range(1, 7)), bytes(range(7, 13))
    out, keep = oracle.forward_batch(buf, len(frames), recs, dmac, smac, offsets=offs, flags=F_IPV6)
    _, keep4 = oracle.forward_batch(buf, len(frames), recs, dmac, smac, offsets=offs)
    k = keep.astype(bool)
    is6 = np.array([oracle_is6(r) for r in recs])
    want = (recs["status"] == STATUS["OK"]) & (recs["ip_protocol"] == UDP) & \
        (recs["l4_sum"] == 0xFFFF) & (recs["n_vlan"] == 0)
    assert np.array_equal(k[is6], want[is6]) and k[is6].sum() > 100
    assert not keep4[is6].any() and np.array_equal(keep4[~is6], keep[~is6])
    back = oracle.parse_batch(out, len(frames), 3 | F_IPV6, offsets=offs)
    assert (back["l4_sum"][k] == 0xFFFF).all()
    assert (back["src_port"][k] == recs["dst_port"][k]).all()
    for i in np.nonzero(k & is6)[0]:
        o, f = int(offs[i]), frames[i]
        g = out[o:o + len(f)].tobytes()
        l3 = int(recs["l3_off"][i])
        assert g[:12] == dmac + smac
        assert g[l3 + 8:l3 + 24] == f[l3 + 24:l3 + 40] and g[l3 + 24:l3 + 40] == f[l3 + 8:l3 + 24]
        assert g[l3 + 7] == (f[l3 + 7] - 1) % 256
        assert g[l3 + 40:int(recs["l4_off"][i])] == f[l3 + 40:int(recs["l4_off"][i])]
    for i in np.nonzero(~k)[0]:
        o, f = int(offs[i]), frames[i]
        assert out[o:o + len(f)].tobytes() == f
