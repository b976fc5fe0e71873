"""The oracle over random batch layouts (tests/fuzz_layouts.py) on the CPU: parse (with
flow events), option walks and layer walk run without fault on overlapping, empty,
negative and past-the-end descriptors and odd strides, and the multi-threaded parse
equals the single-threaded one.  test_oracle_asan.py runs this file again under
ASan/UBSan, where an out-of-range read in the C restatement fails it."""
import numpy as np
import pytest

from oracle import oracle
from fuzz_layouts import packed_layout, strided_layout


def run(hb, rng):
    flags = int(rng.integers(0, 4))
    nb = int(rng.integers(1, 9000))
    kw = dict(offsets=hb.offsets, stride=hb.stride, frame_len=hb.frame_len)
    r1, ev1 = oracle.parse_batch(hb.frames, hb.n, flags=flags, n_buckets=nb, flow_ev=True,
                                 threads=1, **kw)
    r4, ev4 = oracle.parse_batch(hb.frames, hb.n, flags=flags, n_buckets=nb, flow_ev=True,
                                 threads=4, **kw)
    assert r1.tobytes() == r4.tobytes() and np.array_equal(ev1, ev4)
    r3 = oracle.parse_batch(hb.frames, hb.n, flags=3, **kw)
    o = oracle.options_batch(hb.frames, hb.n, r3, **kw)
    lay = oracle.layers_batch(hb.frames, hb.n, **kw)
    assert o.size == hb.n and lay.size == hb.n
    return r3


@pytest.mark.parametrize("seed", range(6))
def test_oracle_packed_layouts(seed):
    rng = np.random.default_rng(9000 + seed)
    r = run(packed_layout(rng, int(rng.integers(1, 4000))), rng)
    assert len(set(r["status"].tolist())) > 3


@pytest.mark.parametrize("seed", range(4))
def test_oracle_strided_layouts(seed):
    rng = np.random.default_rng(7000 + seed)
    run(strided_layout(rng, int(rng.integers(1, 3000))), rng)
