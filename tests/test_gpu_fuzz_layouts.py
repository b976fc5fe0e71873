"""Randomised batch layouts (tests/fuzz_layouts.py) through every per-frame entry point,
bit-exact against the oracle.  Each seed runs the parse (a random flag combination,
with flow events), the compact records, both option-walk entry points and the layer
walk over the same buffers."""
import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine
from rpkt_amd.records import F_FLOW_EV, LAYERS_DTYPE, as_opts, as_records, project16

from fuzz_layouts import packed_layout, strided_layout
from test_gpu_parity import assert_same, assert_same16, gpu_records, gpu_records16, oracle_records

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def check_all(hb, rng):
    flags = int(rng.integers(0, 4))
    nb = int(rng.integers(1, 9000))
    g, gev = gpu_records(hb, flags | F_FLOW_EV, nb)
    o, oev = oracle_records(hb, flags, nb, flow=True)
    assert_same(g, o)
    assert np.array_equal(gev, oev)
    assert_same16(gpu_records16(hb, flags), project16(o, flags))
    # option walks from full and from compact records (located by a flags-3 parse)
    db = engine.DeviceBatch.from_host(hb)
    recs = engine.parse_batch(db, 3)
    r3 = as_records(recs.cpu().numpy())
    oo = oracle.options_batch(hb.frames, hb.n, r3, offsets=hb.offsets, stride=hb.stride,
                              frame_len=hb.frame_len)
    go = as_opts(engine.options_batch(db, recs).cpu().numpy())
    gc = as_opts(engine.options_batch(db, engine.parse_batch_compact(db, 3), compact=True)
                 .cpu().numpy())
    assert go.tobytes() == oo.tobytes(), "options (full records) differ"
    assert gc.tobytes() == oo.tobytes(), "options (compact records) differ"
    gl = engine.layers_batch(db).cpu().numpy().view(LAYERS_DTYPE)
    ol = oracle.layers_batch(hb.frames, hb.n, offsets=hb.offsets, stride=hb.stride,
                             frame_len=hb.frame_len)
    assert gl.tobytes() == ol.tobytes(), "layer walks differ"


@pytest.mark.parametrize("seed", range(10))
def test_fuzz_packed_layouts(torch, seed):
    rng = np.random.default_rng(9000 + seed)
    check_all(packed_layout(rng, int(rng.integers(1, 4000))), rng)


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_strided_layouts(torch, seed):
    rng = np.random.default_rng(7000 + seed)
    check_all(strided_layout(rng, int(rng.integers(1, 3000))), rng)
