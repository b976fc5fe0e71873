"""GPU parity of the encapsulation build (rpkt_gpu_build_tunnel_batch) against the build
oracle, byte for byte: the reference's VXLAN / GTP-U / GRE build tests (their captures
come back, tests/test_tunnel_build.py) at every 16-B phase, config 13 at full size
rebuilt from its tunnel parse, and mutated tunnel records over the tunnel fuzz."""
import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, gen
from rpkt_amd.records import TUN_STATUS, as_records, as_tunnels

from test_gpu_parity import host_batch
from test_tunnel_build import reference_build_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def check_build(torch, hb, recs, tuns, flags):
    db = engine.DeviceBatch.from_host(hb)
    r = torch.from_numpy(np.ascontiguousarray(recs).view(np.uint8).copy()).cuda()
    t = torch.from_numpy(np.ascontiguousarray(tuns).view(np.uint8).copy()).cuda()
    gb = engine.build_tunnel_batch(db, r, t, flags).cpu().numpy()
    g = db.frames.cpu().numpy()
    o, ob = oracle.build_tunnel_batch(hb.frames, hb.n, recs, tuns, flags, offsets=hb.offsets,
                                      stride=hb.stride, frame_len=hb.frame_len)
    assert np.array_equal(gb, ob), "built flags differ"
    if not np.array_equal(g[:o.size], o):
        bad = np.nonzero(g[:o.size] != o)[0]
        raise AssertionError("%d bytes differ, first at %d" % (bad.size, bad[0]))
    return g[:o.size], gb


@pytest.mark.parametrize("lead", list(range(16)))
def test_reference_builds_every_alignment(torch, lead):
    frames, (buf, offs, recs, tuns) = reference_build_batch()
    parts = [bytes(buf[offs[i]:offs[i + 1]]) for i in range(len(frames))]
    hb = host_batch(parts, lead)
    k = 1 if lead else 0
    recs = np.concatenate([np.zeros(k, recs.dtype), recs])
    tuns = np.concatenate([np.zeros(k, tuns.dtype), tuns])
    for flags in (0, 1, 2, 3):
        out, built = check_build(torch, hb, recs, tuns, flags)
        assert built[k:].all()
        if flags in (0, 3):                                 # the captures themselves
            for i, f in enumerate(frames):
                a = int(hb.offsets[i + k])
                assert bytes(out[a:a + len(f)]) == f


def test_config13_round_trip_full_size(torch):
    """Parse config 13 (1M x 1500 B) with the tunnel entry, zero every outer header and
    tunnel header byte the build writes, rebuild on the device with both sums filled:
    equal to the oracle's build, and to the original frames wherever every stored sum was
    valid."""
    hb = gen.make_batch(13)
    db = engine.DeviceBatch.from_host(hb)
    o, t, _ = engine.parse_tunnel_batch(db, gen.FLAGS[13])
    recs = as_records(o.cpu().numpy())
    tuns = as_tunnels(t.cpu().numpy())
    z = hb.frames.copy().reshape(hb.n, hb.stride)
    z[:, :34] = 0                                            # Ether + IPv4
    ts = tuns["tun_off"].astype(np.int64)
    rows = np.arange(hb.n)
    for k in range(4):
        z[rows, ts + k] = 0
    hz = gen.HostBatch(13, hb.n, hb.seed, z.reshape(-1), None, hb.stride, hb.frame_len)
    out, built = check_build(torch, hz, recs, tuns, 3)
    assert built.all()
    # every stored sum valid: the IPv4 header's, and the UDP one (a VXLAN checksum of 0 is
    # filled by the build) or the GRE one (0 without the C bit: nothing to fill)
    clean = (recs["ip_sum"] == 0xffff) & (
        ((recs["status"] == 0) & (recs["l4_sum"] == 0xffff) & (recs["l4_checksum"] != 0)) |
        ((recs["status"] == 9) & np.isin(recs["l4_sum"], (0, 0xffff))))
    same = (out.reshape(hb.n, -1) == hb.frames.reshape(hb.n, -1)).all(axis=1)
    assert same[clean].all() and clean.mean() > 0.7


@pytest.mark.parametrize("seed", [1, 2])
def test_mutated_tunnel_records(torch, seed):
    """Tunnel records no parse would produce over the tunnel fuzz: random kinds, flag bytes
    (header lengths), ids and aux values, with records of random VLAN counts."""
    hb = gen.make_batch(14, 1 << 14, seed=seed)
    o, t, _ = oracle.tunnel_batch(hb.frames, hb.n, 11, offsets=hb.offsets)
    rng = np.random.default_rng(seed)
    t["kind"] = rng.integers(0, 5, hb.n)
    t["hdr0"] = rng.integers(0, 256, hb.n)
    t["hdr1"] = rng.integers(0, 256, hb.n)
    t["aux"] = rng.integers(0, 65536, hb.n)
    t["id"] = rng.integers(0, 2 ** 32, hb.n, dtype=np.uint64).astype(np.uint32)
    t["inner_type"] = rng.choice([0x0800, 0x86dd, 0x6558, 0x1234], hb.n)
    o["n_vlan"] = np.where(rng.integers(0, 4, hb.n) == 0, rng.integers(0, 3, hb.n), o["n_vlan"])
    for flags in (0, 3):
        check_build(torch, hb, o, t, flags)
