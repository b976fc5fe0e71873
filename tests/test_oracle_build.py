"""The TX-side oracle (oracle/rpkt_oracle_build.c) pinned on the reference's own
captures: rebuilding a fixture's headers from its parse record, on a buffer whose
fixed header bytes were wiped, must give back the captured bytes (setter layout),
and filling the checksums must give back the checksums real stacks computed."""
import os

import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import gen
from rpkt_amd.records import STATUS

HERE = os.path.dirname(os.path.abspath(__file__))
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
