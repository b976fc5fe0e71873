"""GPU parity of the IPv6 TX side: rpkt_gpu_build_batch over IPv6 records
(Ipv6::prepend_header + setters, rpkt/src/ipv6/generated.rs:94-135) and
rpkt_gpu_forward_batch with rpkt_fwd_t.flags = RPKT_F_IPV6 (the loopback_rx rewrite of
untagged IPv6/UDP frames), against oracle/rpkt_oracle_build.c on the same buffers
(pinned by tests/test_oracle_build.py on the reference's IPv6 captures).  Bit-exact."""
import os

import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, gen
from rpkt_amd.records import F_IPV6, STATUS, as_records, is_ip6

from ip6_frames import ip6_frame
from test_gpu_parity import host_batch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
PKTS = os.path.join(HERE, "golden", "packets")
F6 = 3 | F_IPV6
DMAC = bytes([0xAC, 0xDC, 0xCA, 0x79, 0xCA, 0x86])      # loopback_rx.rs:29-30
SMAC = bytes([0xAC, 0xDC, 0xCA, 0x79, 0xE5, 0xC6])


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def oracle_recs(hb):
    return oracle.parse_batch(hb.frames, hb.n, F6, offsets=hb.offsets, stride=hb.stride,
                              frame_len=hb.frame_len, threads=8)


def check_build(torch, hb, recs, flags):
    db = engine.DeviceBatch.from_host(hb)
    d = torch.from_numpy(np.ascontiguousarray(recs).view(np.uint8).copy()).cuda()
    gb = engine.build_batch(db, d, flags).cpu().numpy()
    g = db.frames.cpu().numpy()
    o, ob = oracle.build_batch(hb.frames, hb.n, recs, flags, offsets=hb.offsets,
                               stride=hb.stride, frame_len=hb.frame_len)
    assert np.array_equal(gb, ob), "built flags differ"
    if not np.array_equal(g[:o.size], o):
        bad = np.nonzero(g[:o.size] != o)[0]
        raise AssertionError("%d bytes differ, first at %d" % (bad.size, bad[0]))
    return gb


def check_forward(torch, hb, fwd_flags, forbid=None):
    db = engine.DeviceBatch.from_host(hb)
    r = as_records(engine.parse_batch(db, F6).cpu().numpy())
    fl = engine.forbid_list(forbid) if forbid is not None else None
    keep = engine.forward_batch(db, DMAC, SMAC, fl, flags=fwd_flags).cpu().numpy()
    o, ok = oracle.forward_batch(hb.frames, hb.n, r, DMAC, SMAC,
                                 () if forbid is None else forbid.astype(np.uint32),
                                 offsets=hb.offsets, stride=hb.stride, frame_len=hb.frame_len,
                                 flags=fwd_flags)
    assert np.array_equal(keep, ok), "keep flags differ"
    g = db.frames.cpu().numpy()
    if not np.array_equal(g[:o.size], o):
        bad = np.nonzero(g[:o.size] != o)[0]
        raise AssertionError("%d bytes differ, first at %d" % (bad.size, bad[0]))
    return r, ok


@pytest.mark.parametrize("cfg", [10, 11, 12])
@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_build_ip6_parity_configs(torch, cfg, flags):
    """Dual-stack batches (64 B, 1500 B with 0-3 extension headers, the fuzz config):
    IPv4 and IPv6 records built as the oracle builds them."""
    n = {10: 1 << 16, 11: 1 << 14, 12: 1 << 16}[cfg]
    hb = gen.make_batch(cfg, n, seed=700 + cfg)
    recs = oracle_recs(hb)
    built = check_build(torch, hb, recs, flags)
    six = is_ip6(recs) & (recs["status"] == STATUS["OK"])
    assert six.sum() > n // 10 and built[six].all()


def test_build_ip6_mutated_records(torch):
    """IPv6 records no parse would produce: random tag counts, l4_off, pdst_off (inside and
    outside the frame), protocol and data offset, over fuzz frames of every length."""
    hb = gen.make_batch(12, 1 << 15, seed=71)
    recs = oracle_recs(hb)
    rng = np.random.default_rng(8)
    raw = recs.view(np.uint8).reshape(hb.n, 80)
    raw[:, 1] = rng.integers(0, 3, hb.n)                                  # n_vlan 0..2
    raw[:, 33] = rng.choice([6, 17, 59, 0], hb.n)                         # protocol
    l4 = rng.integers(0, 400, hb.n).astype(np.uint16)
    raw[:, 66:68] = l4.view(np.uint8).reshape(-1, 2)                      # l4_off
    pd = rng.integers(0, 300, hb.n).astype(np.uint16)
    raw[:, 34:36] = pd.view(np.uint8).reshape(-1, 2)                      # ip6_pdst_off
    raw[:, 56:58] = rng.integers(0, 256, (hb.n, 2), dtype=np.uint8)       # l4_word6
    for flags in (0, 3):
        check_build(torch, hb, recs, flags)


@pytest.mark.parametrize("lead", list(range(16)))
def test_build_ip6_fixtures_every_alignment(torch, lead):
    """The reference's captures (IPv6 and IPv4) at every 16-B phase, records from the
    RPKT_F_IPV6 parse, both checksums filled."""
    names = sorted(f for f in os.listdir(PKTS) if f.endswith(".dat"))
    hb = host_batch([oracle.load_dat(os.path.join(PKTS, f)) for f in names], lead)
    recs = oracle_recs(hb)
    check_build(torch, hb, recs, 3)


def long_chain_batch(seed, lead=0):
    """IPv6 frames whose extension headers push the L4 header past the 128-B window (and
    to kilobytes), routing headers with segments left (pseudo header over the final
    address), tagged and untagged, UDP and TCP, some with a broken L4 sum."""
    rng = np.random.default_rng(seed)
    frames = []
    for hbh in (8, 16, 48, 72, 96, 120, 2048):
        for proto in (17, 6):
            for tail in ([], [(43, 8 + 16 * 3)], [(60, 24), (51, 12 + 8)], [(44, 8)]):
                pl = rng.integers(0, 256, int(rng.integers(0, 1500)), dtype=np.uint8).tobytes()
                f = bytearray(ip6_frame(rng, [(0, hbh)] + tail, proto, pl,
                                        tag=bool(rng.integers(0, 4) == 0)))
                if rng.integers(0, 8) == 0:
                    f[-1] ^= 0x3c
                frames.append(bytes(f))
    for k in range(64):                                       # short ones, in the window
        frames.append(ip6_frame(rng, [[], [(43, 24)], [(60, 8)]][k % 3], 17, bytes(k % 9)))
    return host_batch(frames, lead)


@pytest.mark.parametrize("lead", [0, 3, 8, 15])
def test_build_ip6_headers_past_the_window(torch, lead):
    """L4 headers past the LDS window are written to memory by their lane and their
    checksums summed from the record's values plus the streamed payload."""
    hb = long_chain_batch(90 + lead, lead)
    recs = oracle_recs(hb)
    for flags in (0, 2, 3):
        check_build(torch, hb, recs, flags)


def test_build_ip6_round_trip_full_size(torch):
    """Config 11 at BASELINE size (1M x 1500 B, IPv6 with 0-3 extension headers): wipe the
    fixed header bytes, rebuild with the L4 checksums filled, get the original frames back
    wherever the original sums verified, and every rebuilt frame verifies."""
    hb = gen.make_batch(11)
    db = engine.DeviceBatch.from_host(hb)
    recs = engine.parse_batch(db, F6)
    r = as_records(recs.cpu().numpy())
    six = is_ip6(r)
    f = db.frames.view(-1, 1500)
    f[:, :22] = 0                                             # Ethernet + IPv6 bytes 0..7
    built = engine.build_batch(db, recs, 3).cpu().numpy()
    out = db.frames.cpu().numpy().reshape(-1, 1500)
    good = six & (r["l4_sum"] == 0xFFFF)
    assert built.all() and good.mean() > 0.45
    assert np.array_equal(out[good], hb.frames.reshape(-1, 1500)[good])
    back = as_records(engine.parse_batch(db, F6).cpu().numpy())
    assert (back["l4_sum"] == 0xFFFF).all()


def test_forward_ip6_full_size(torch):
    """Config 10 at BASELINE size (1M x 64 B, half IPv6/UDP): with RPKT_F_IPV6 the IPv6
    frames are forwarded too; without it, only the IPv4 ones, as before."""
    hb = gen.make_batch(10)
    r, ok = check_forward(torch, hb, F_IPV6, forbid=np.arange(1000, 1100, dtype=np.int64))
    six = is_ip6(r)
    assert 0.9 < ok[six].mean() and 0.9 < ok[~six].mean()
    r0, ok0 = check_forward(torch, hb, 0)
    assert not ok0[six].any()


@pytest.mark.parametrize("lead", [0, 5, 9, 14])
def test_forward_ip6_long_chains(torch, lead):
    """Routing headers (delta of the pseudo header), UDP headers past the window (ports and
    checksum stored by the lane), tagged frames (never forwarded), broken sums."""
    hb = long_chain_batch(200 + lead, lead)
    forbid = np.array([0x0a000001, 0xc0a80503], dtype=np.int64)
    r, ok = check_forward(torch, hb, F_IPV6, forbid=forbid)
    assert ok.sum() > 20


@pytest.mark.parametrize("lead", list(range(16)))
def test_forward_ip6_fixtures_every_alignment(torch, lead):
    names = sorted(f for f in os.listdir(PKTS) if f.endswith(".dat"))
    hb = host_batch([oracle.load_dat(os.path.join(PKTS, f)) for f in names], lead)
    check_forward(torch, hb, F_IPV6)


@pytest.mark.parametrize("stride,flen", [(64, 64), (64, 62), (48, 48), (80, 64), (96, 96)])
def test_tx_ip6_short_strided_frames(torch, stride, flen):
    """Dual-stack fuzz frames cut to flen bytes at `stride` (the 64-B-window compile takes
    frame + phase <= 64): IPv6 records built and IPv6 frames forwarded as the oracle does,
    no byte outside a frame touched."""
    src = gen.make_batch(12, 20000, seed=stride * 7 + flen)
    lens = src.lens()
    buf = np.zeros(src.n * stride + 64, dtype=np.uint8)
    for i in range(src.n):
        a = int(src.offsets[i])
        k = min(int(lens[i]), flen)
        buf[i * stride:i * stride + k] = src.frames[a:a + k]
    hb = gen.HostBatch(12, src.n, 0, buf, None, stride, flen)
    recs = oracle_recs(hb)
    for flags in (1, 3):
        check_build(torch, hb, recs, flags)
    check_forward(torch, hb, F_IPV6)


def test_build_from_host_build_views(torch):
    """Records composed by the host-side build views (rpkt_amd/txviews.py: rpkt's
    prepend_header + setters) for the reference's captures, its loopback_tx frames and a
    QinQ/IPv6/routing/TCP-options chain, built by rpkt_gpu_build_batch with and without the
    checksum fill: the same bytes as the oracle build."""
    import test_txviews as tt
    from rpkt_amd import txviews as tv
    chains, lens, pays = [], [], []
    for name in sorted(f for f in os.listdir(PKTS) if f.endswith(".dat")):
        f = bytes(oracle.load_dat(os.path.join(PKTS, name)))
        r = oracle.parse_one(f, F6)
        if r["status"] != STATUS["OK"] or int(r["ip_protocol"]) not in (6, 17):
            continue
        chains.append(tt.chain_from_capture(f, r))
        lens.append(len(f))
        pays.append(f[int(r["payload_off"]):])
    for k in range(200):
        chains.append(tt.loopback_tx_chain("172.74.%d.%d" % (2 + k // 250, 2 + k % 250)))
        lens.append(1500)
        pays.append(b"\xae" * 1458)
    buf, offs, recs = tv.assemble(chains, lens, pays)
    hb = gen.HostBatch(0, len(lens), 0, buf, offs, 0, 0)
    for flags in (0, 3):
        check_build(torch, hb, recs, flags)


def test_build_ip6_rfc8200_fixture(torch):
    """tests/golden/ip6_tx.json (checksums from RFC 8200 section 8.1 + RFC 1071 alone, see
    tests/golden/make_ip6_tx_golden.py): the device build fills each frame's zeroed L4
    checksum with the RFC's value, at every 16-B phase."""
    import json
    cases = json.load(open(os.path.join(HERE, "golden", "ip6_tx.json")))
    frames = [bytes.fromhex(c["frame"]) for c in cases]
    for lead in range(16):
        hb = host_batch(frames, lead)
        recs = oracle_recs(hb)
        z = hb.frames.copy()
        for i, c in enumerate(cases):
            k = i + (1 if lead else 0)                       # after the lead junk frame
            ck = int(hb.offsets[k]) + int(recs[k]["l4_off"]) + (6 if c["kind"] == "udp" else 16)
            z[ck:ck + 2] = 0
        hz = gen.HostBatch(hb.config, hb.n, hb.seed, z, hb.offsets, hb.stride, hb.frame_len)
        db = engine.DeviceBatch.from_host(hz)
        d = torch.from_numpy(np.ascontiguousarray(recs).view(np.uint8).copy()).cuda()
        assert engine.build_batch(db, d, 3).cpu().numpy()[(1 if lead else 0):].all()
        assert np.array_equal(db.frames.cpu().numpy()[:hb.frames.size], hb.frames)
