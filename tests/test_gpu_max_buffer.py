"""The largest batch the descriptor allows: a strided config-3 batch (1500-B TCP frames,
1 % bad checksums) filling all but a few hundred bytes of the 32-bit offset range
(kMaxFrameBytes = 0xffffff00), so the last tiles load, stream and write at buffer
offsets just below 4 GiB.  Parse (full and compact records), the layer walk and the
header build are bit-exact against the oracle over the whole batch."""
import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, gen
from rpkt_amd.records import LAYERS_DTYPE, as_records, project16

from test_gpu_parity import assert_same, assert_same16, THREADS

pytestmark = pytest.mark.gpu

MAX_FRAME_BYTES = 0xFFFFFF00                 # rpkt_common.h kMaxFrameBytes


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


@pytest.fixture(scope="module")
def big(torch):
    n = MAX_FRAME_BYTES // 1500              # 2,863,311 frames, 4,294,966,500 bytes
    hb = gen.make_batch(3, n)
    assert hb.offsets is None and hb.stride == 1500
    assert MAX_FRAME_BYTES - hb.frames.size < 1500
    db = engine.DeviceBatch.from_host(hb)
    assert db.frames.numel() == hb.frames.size
    return hb, db


def test_max_buffer_parse(big):
    hb, db = big
    recs = engine.parse_batch(db, 3)
    g = as_records(recs.cpu().numpy())
    o = oracle.parse_batch(hb.frames, hb.n, flags=3, stride=hb.stride, threads=THREADS)
    assert_same(g, o)
    assert (g["status"] == 0).mean() > 0.99
    from rpkt_amd.records import as_records16
    g16 = as_records16(engine.parse_batch_compact(db, 3).cpu().numpy())
    assert_same16(g16, project16(o, 3))


def test_max_buffer_layers(big):
    hb, db = big
    g = engine.layers_batch(db).cpu().numpy().view(LAYERS_DTYPE)
    o = oracle.layers_batch(hb.frames, hb.n, stride=hb.stride)
    assert g.tobytes() == o.tobytes()


def test_max_buffer_build(big):
    """Headers rebuilt with both checksums filled: the 1 % of frames with bad stored
    sums change, everything else is rewritten with its own bytes; the whole 4 GiB
    buffer equals the oracle's."""
    hb, db = big
    recs = engine.parse_batch(db, 3)
    r = as_records(recs.cpu().numpy())
    built = engine.build_batch(db, recs, 3)
    ob, obuilt = oracle.build_batch(hb.frames, hb.n, r, 3, stride=hb.stride)
    assert np.array_equal(built.cpu().numpy(), obuilt)
    gf = db.frames.cpu().numpy()
    assert gf.size == ob.size
    step = 1 << 28                            # compare in 256 MiB slices
    for a in range(0, ob.size, step):
        if not np.array_equal(gf[a:a + step], ob[a:a + step]):
            bad = np.nonzero(gf[a:a + step] != ob[a:a + step])[0]
            raise AssertionError("%d bytes differ from offset %d" % (bad.size, a + int(bad[0])))
