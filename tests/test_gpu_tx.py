"""GPU parity of the TX side: rpkt_gpu_build_batch (rpkt_build.rs prepend_header +
setters + TX checksum fill) and rpkt_gpu_forward_batch (loopback_rx.rs firewall
rewrite) against oracle/rpkt_oracle_build.c on the same buffers, bit-exact."""
import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, gen
from rpkt_amd.records import REC_DTYPE, STATUS, as_records

pytestmark = pytest.mark.gpu

DMAC = bytes([0xAC, 0xDC, 0xCA, 0x79, 0xCA, 0x86])      # loopback_rx.rs:29-30
SMAC = bytes([0xAC, 0xDC, 0xCA, 0x79, 0xE5, 0xC6])


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def dev_recs(torch, recs):
    return torch.from_numpy(np.ascontiguousarray(recs).view(np.uint8).copy()).cuda()


def gpu_build(torch, hb, recs, flags):
    db = engine.DeviceBatch.from_host(hb)
    built = engine.build_batch(db, dev_recs(torch, recs), flags)
    return db.frames.cpu().numpy(), built.cpu().numpy()


def oracle_build(hb, recs, flags):
    return oracle.build_batch(hb.frames, hb.n, recs, flags, offsets=hb.offsets,
                              stride=hb.stride, frame_len=hb.frame_len)


def check_build(torch, hb, recs, flags):
    g, gb = gpu_build(torch, hb, recs, flags)
    o, ob = oracle_build(hb, recs, flags)
    assert np.array_equal(gb, ob)
    if not np.array_equal(g[:o.size], o):
        bad = np.nonzero(g[:o.size] != o)[0]
        raise AssertionError("%d bytes differ, first at %d" % (bad.size, bad[0]))
    return gb


@pytest.mark.parametrize("cfg", [2, 3, 5, 6])
@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_build_parity_configs(torch, cfg, flags):
    n = {2: 1 << 16, 3: 1 << 14, 5: 1 << 15, 6: 1 << 16}[cfg]
    hb = gen.make_batch(cfg, n, seed=300 + cfg)
    recs = oracle.parse_batch(hb.frames, hb.n, 3, offsets=hb.offsets, stride=hb.stride)
    built = check_build(torch, hb, recs, flags)
    if cfg != 6:
        assert built.mean() > 0.95


def test_build_parity_mutated_records(torch):
    """Records no parse would produce: random tag counts, IHL, protocol, data offset
    and checksum fields, over fuzz frames of every length (too-short frames must be
    left untouched)."""
    hb = gen.make_batch(6, 1 << 15, seed=31)
    recs = oracle.parse_batch(hb.frames, hb.n, 3, offsets=hb.offsets)
    rng = np.random.default_rng(5)
    raw = recs.view(np.uint8).reshape(hb.n, 80)
    noise = rng.integers(0, 256, size=raw.shape, dtype=np.uint8)
    raw[:, 1] = rng.integers(0, 4, hb.n)                                  # n_vlan 0..3
    raw[:, 24] = rng.integers(0, 256, hb.n)                               # ip_vhl
    raw[:, 33] = rng.choice([6, 17, 1, 47], hb.n)                         # protocol
    raw[:, 56:58] = noise[:, 56:58]                                       # l4_word6 (doff)
    raw[:, 34:36] = noise[:, 34:36]
    raw[:, 60:62] = noise[:, 60:62]
    for flags in (0, 3):
        check_build(torch, hb, recs, flags)


def test_build_round_trip_full_size(torch):
    """Config 3 at BASELINE size: wipe every fixed header byte, rebuild from the
    records with both checksums filled, get the original frames back wherever the
    original checksums were valid."""
    hb = gen.make_batch(3)
    db = engine.DeviceBatch.from_host(hb)
    recs = engine.parse_batch(db, 3)
    r = as_records(recs.cpu().numpy())
    f = db.frames.view(-1, 1500)
    f[:, :34] = 0
    f[:, 34:54] = 0
    built = engine.build_batch(db, recs, 3).cpu().numpy()
    out = db.frames.cpu().numpy().reshape(-1, 1500)
    good = (r["ip_sum"] == 0xFFFF) & (r["l4_sum"] == 0xFFFF)
    assert built.all() and good.mean() > 0.97
    assert np.array_equal(out[good], hb.frames.reshape(-1, 1500)[good])
    back = as_records(engine.parse_batch(db, 3).cpu().numpy())
    assert (back["ip_sum"] == 0xFFFF).all() and (back["l4_sum"] == 0xFFFF).all()


@pytest.mark.parametrize("cfg", [2, 4, 6])
def test_forward_parity(torch, cfg):
    n = {2: 1 << 20, 4: 1 << 20, 6: 1 << 16}[cfg]
    hb = gen.make_batch(cfg, n, seed=400 + cfg)
    db = engine.DeviceBatch.from_host(hb)
    r = as_records(engine.parse_batch(db, 3).cpu().numpy())
    forbid = np.unique(r["ip_src"][::97])[:64].astype(np.int64)
    keep = engine.forward_batch(db, DMAC, SMAC, engine.forbid_list(forbid))
    o, ok = oracle.forward_batch(hb.frames, hb.n, r, DMAC, SMAC, forbid.astype(np.uint32),
                                 offsets=hb.offsets, stride=hb.stride, frame_len=hb.frame_len)
    assert np.array_equal(keep.cpu().numpy(), ok)
    g = db.frames.cpu().numpy()
    assert np.array_equal(g[:o.size], o)
    if cfg != 6:
        assert 0.3 < ok.mean() < 0.999


def test_forward_long_forbid_list(torch):
    """More than 128 forbidden addresses: the binary search runs in global memory."""
    hb = gen.make_batch(2, 1 << 16, seed=12)
    db = engine.DeviceBatch.from_host(hb)
    r = as_records(engine.parse_batch(db, 3).cpu().numpy())
    forbid = np.unique(np.concatenate([r["ip_src"][::50], np.arange(1000, 1400)])).astype(np.int64)
    assert forbid.size > 128
    keep = engine.forward_batch(db, DMAC, SMAC, engine.forbid_list(forbid)).cpu().numpy()
    o, ok = oracle.forward_batch(hb.frames, hb.n, r, DMAC, SMAC, forbid.astype(np.uint32),
                                 stride=hb.stride)
    assert np.array_equal(keep, ok)
    assert np.array_equal(db.frames.cpu().numpy(), o)


def test_forward_empty_forbid_and_rejects(torch):
    hb = gen.make_batch(2, 4096, seed=9)
    db = engine.DeviceBatch.from_host(hb)
    recs = engine.parse_batch(db, 3)
    r = as_records(recs.cpu().numpy())
    keep = engine.forward_batch(db, DMAC, SMAC, None).cpu().numpy()
    assert np.array_equal(keep.astype(bool), r["ip_sum"] == 0xFFFF)
    with pytest.raises(engine.RpktError):
        engine.build_batch(db, recs, flags=4)


def strided_short(src, stride, flen):
    """Frames of a packed batch cut or padded to flen bytes, placed at `stride`."""
    n = src.n
    buf = np.zeros(n * stride + 64, dtype=np.uint8)
    lens = src.lens()
    for i in range(n):
        a = int(src.offsets[i])
        k = min(int(lens[i]), flen)
        buf[i * stride:i * stride + k] = src.frames[a:a + k]
    return gen.HostBatch(src.config, n, 0, buf, None, stride, flen)


@pytest.mark.parametrize("stride,flen", [(64, 64), (64, 42), (48, 48), (49, 49), (80, 64),
                                         (64, 65), (96, 96)])
def test_tx_short_strided_frames(torch, stride, flen):
    """Build and forward over strided batches around the 64-B-window compile's bound
    (frame + 16-B phase <= 64 takes it, the last two cases take the 128-B one): IMIX
    frames (TCP and UDP) cut to flen bytes, every frame rebuilt / rewritten exactly as
    the oracle does, no byte outside a frame touched."""
    hb = strided_short(gen.make_batch(4, 20000, seed=stride + flen), stride, flen)
    recs = oracle.parse_batch(hb.frames, hb.n, 3, stride=hb.stride, frame_len=hb.frame_len)
    for flags in (1, 3):
        check_build(torch, hb, recs, flags)
    db = engine.DeviceBatch.from_host(hb)
    r = as_records(engine.parse_batch(db, 3).cpu().numpy())
    forbid = np.unique(r["ip_src"][::31])[:16].astype(np.int64)
    keep = engine.forward_batch(db, DMAC, SMAC, engine.forbid_list(forbid))
    o, ok = oracle.forward_batch(hb.frames, hb.n, r, DMAC, SMAC, forbid.astype(np.uint32),
                                 stride=hb.stride, frame_len=hb.frame_len)
    assert np.array_equal(keep.cpu().numpy(), ok)
    assert np.array_equal(db.frames.cpu().numpy()[:o.size], o)
