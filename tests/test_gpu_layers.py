"""GPU parity of rpkt_gpu_layers_batch (the pktfmt-table interpreter) against the
hand-written oracle (oracle/rpkt_oracle_layers.c), bit-exact."""
import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, gen
from rpkt_amd.records import LAYER_STOP, as_records
from rpkt_amd.records import LAYERS_DTYPE

from test_gpu_parity import host_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def check(hb):
    db = engine.DeviceBatch.from_host(hb)
    g = engine.layers_batch(db).cpu().numpy().view(LAYERS_DTYPE)
    o = oracle.layers_batch(hb.frames, hb.n, offsets=hb.offsets, stride=hb.stride,
                            frame_len=hb.frame_len)
    if g.tobytes() != o.tobytes():
        bad = np.nonzero(g.view(np.uint8).reshape(-1, 64) != o.view(np.uint8).reshape(-1, 64))
        i = int(bad[0][0])
        raise AssertionError("%d frames differ, first %d: gpu %s oracle %s" % (
            len(np.unique(bad[0])), i, g[i], o[i]))
    return g


def test_layers_mix_full_size(torch):
    g = check(gen.make_mix())
    assert set(g["stop"].tolist()) >= {1, 2, 3}


@pytest.mark.parametrize("lead", [0, 1, 5, 11, 15])
def test_layers_fixtures_every_alignment(torch, lead):
    check(host_batch(gen.fixture_frames() * 2, lead))


@pytest.mark.parametrize("cfg", [2, 3, 5, 6])
def test_layers_baseline_configs(torch, cfg):
    g = check(gen.make_batch(cfg))
    if cfg in (2, 3):
        assert (g["stop"] == LAYER_STOP["END"]).mean() > 0.97


def ipv6_ext_frame(n_ext, ext_len=20, payload=b"\xab" * 10):
    """Ether / IPv6 / n_ext DestOptions of 8*ext_len+8 bytes / UDP: headers far past
    the 256-B LDS window."""
    udp = (1000).to_bytes(2, "big") + (2000).to_bytes(2, "big") + \
        (8 + len(payload)).to_bytes(2, "big") + b"\x00\x00" + payload
    body = udp
    for k in range(n_ext):
        nh = 17 if k == 0 else 60
        body = bytes([nh, ext_len]) + b"\x01" * (8 * ext_len + 6) + body
    ip6 = b"\x60\x00\x00\x00" + len(body).to_bytes(2, "big") + bytes([60 if n_ext else 17, 64]) + \
        b"\x20" * 32
    return b"\x02" * 12 + b"\x86\xdd" + ip6 + body


def test_layers_deep_stacks(torch):
    """Headers beyond the 256-B LDS window (read from global memory) and walks that
    hit the 16-layer cap (long MPLS label stacks)."""
    vx = next(f for f in gen.fixture_frames() if len(f) == 148 and f[36:38] == b"\x12\xb5")
    mpls = b"\x00\x11\x22\x33\x44\x55" * 2 + b"\x88\x47" + b"\x00\x01\x00\x40" * 30 + \
        b"\x00\x01\x01\x40" + vx[14:]
    frames = [ipv6_ext_frame(k) for k in range(0, 6)] + [ipv6_ext_frame(3)[:300]]
    frames += [mpls, mpls[:70], mpls[:200]]
    g = check(host_batch(frames, 3))[1:]              # [0] is the 3-byte lead frame
    assert g["n"][:6].tolist() == [3, 4, 5, 6, 7, 8]
    assert (g["stop"][:6] == LAYER_STOP["END"]).all() and g["off"][5][7] > 600
    assert (g["stop"] == LAYER_STOP["MAX"]).sum() == 2


@pytest.mark.parametrize("n", [1, 63, 64, 65, 255, 256, 257, 1000, 4097])
def test_layers_ragged_batch_sizes(torch, n):
    """A lane walks frames base + L + 64 k in turn (kLayFrames per lane): batch sizes
    around the 64-frame tile and the 256-frame wave; no record past n is written."""
    hb = gen.make_mix(n, seed=900 + n)
    db = engine.DeviceBatch.from_host(hb)
    out = torch.full(((n + 64) * 64,), 0xAB, dtype=torch.uint8, device="cuda")
    engine.layers_batch(db, out=out)
    o = oracle.layers_batch(hb.frames, hb.n, offsets=hb.offsets)
    got = out.cpu().numpy()
    assert got[:n * 64].tobytes() == o.tobytes()
    assert (got[n * 64:] == 0xAB).all()


def test_layers_frames_per_lane_variants(torch):
    """The walk with 1, 2, 4 and 8 frames per lane (development hook behind
    tools/ablate_layers.py) gives the product kernel's records byte for byte."""
    import ctypes
    L = engine.ablate_lib()          # the variants are development hooks
    L.rpkt_gpu_debug_layers_variant.argtypes = [ctypes.POINTER(engine.Batch), ctypes.c_void_p,
                                                ctypes.c_int, ctypes.c_void_p]
    L.rpkt_gpu_debug_layers_variant.restype = ctypes.c_int
    hb = gen.make_mix(20000, seed=77)
    db = engine.DeviceBatch.from_host(hb)
    ref = engine.layers_batch(db).cpu().numpy()
    d = db.desc()
    for f in (1, 2, 4, 8):
        out = torch.zeros(hb.n * 64, dtype=torch.uint8, device="cuda")
        assert L.rpkt_gpu_debug_layers_variant(ctypes.byref(d), out.data_ptr(), f, None) == 0
        torch.cuda.synchronize()
        assert out.cpu().numpy().tobytes() == ref.tobytes(), f
