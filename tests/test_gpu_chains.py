"""GPU parity over mbuf chains (rpkt_gpu_parse_chains): every record byte equals the
chain oracle's (oracle/rpkt_oracle_chain.c, a field-for-field restatement of
rpkt-dpdk's Pbuf pinned by rpkt-dpdk/tests/pbuf.rs) on the same segments."""
import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, gen
from rpkt_amd.records import F_FLOW_EV, STATUS, as_records

from test_gpu_parity import assert_same
from test_oracle_chain import _chains_of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def gpu_chain_records(buf, segs, first, flags=3, n_buckets=0):
    hc = gen.HostChains(0, len(first) - 1, 0, buf, np.ascontiguousarray(segs, np.uint32),
                        np.ascontiguousarray(first, np.uint32), None)
    dc = engine.DeviceChains.from_host(hc)
    if flags & F_FLOW_EV:
        recs, ev = engine.parse_chains(dc, flags, n_buckets=n_buckets)
        return as_records(recs.cpu().numpy()), ev.cpu().numpy().view(np.uint64)
    return as_records(engine.parse_chains(dc, flags).cpu().numpy())


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_chain_fuzz_parity(torch, flags):
    hc = gen.make_chains(8)
    g = gpu_chain_records(hc.buf, hc.segs, hc.chain_first, flags)
    o = oracle.parse_chains(hc.buf, hc.segs, hc.chain_first, flags)
    assert_same(g, o)
    assert len(set(o["status"].tolist())) == 15


def test_chain_fuzz_flow_events(torch):
    hc = gen.make_chains(8, n=20000, seed=81)
    g, gev = gpu_chain_records(hc.buf, hc.segs, hc.chain_first, 3 | F_FLOW_EV, 4096)
    o, oev = oracle.parse_chains(hc.buf, hc.segs, hc.chain_first, 3 | F_FLOW_EV, 4096, True)
    assert_same(g, o)
    assert np.array_equal(gev, oev)


def test_jumbo_mbuf_chains_full_size(torch):
    """Config 7 at BASELINE size: 262,144 x 8000 B in 2048-B segments; equal to the
    chain oracle and, since the headers sit in segment 0, to the contiguous parse."""
    hc = gen.make_chains(7)
    g = gpu_chain_records(hc.buf, hc.segs, hc.chain_first, 3)
    o = oracle.parse_chains(hc.buf, hc.segs, hc.chain_first, 3)
    assert_same(g, o)
    ok = g["status"] == STATUS["OK"]
    assert ok.mean() > 0.97
    good_l4 = (g["l4_sum"][ok] == 0xFFFF).mean()
    assert 0.97 < good_l4 < 1.0                      # 1 % injected bad L4 checksums


def test_chain_edge_cases(torch):
    f = gen.make_batch(3, n=1).frames[:1500].tobytes()
    u = gen.make_batch(2, n=1).frames[:64].tobytes()
    layouts = [[1500], [14, 1486], [13, 1487], [0, 1500], [14, 0, 1486], [30, 1470], [34, 1466],
               [40, 1460], [34, 10, 1456], [34, 20, 1446], [20, 14, 1466], [14, 20, 1466],
               [1500, 0, 0], [100, 100, 100, 1200], [1, 1499], [54, 1446], [53, 1, 1446],
               [14, 4, 16, 20, 1446], [18, 1482], [22, 1478]]
    frames = [f] * len(layouts)
    layouts += [[64], [42, 22], [34, 8, 22], [34, 7, 23], [14, 20, 8, 22], [33, 31]]
    frames += [u] * 6
    # many tiny segments: the stream's items exceed one 64-item round per chain
    layouts += [[54] + [7] * 206 + [4], [128] + [3] * 457 + [1], [14] + [1] * 1486, [2] * 750]
    frames += [f, f, f, f]
    buf, segs, first = _chains_of(frames, layouts)
    for flags in (1, 3):
        assert_same(gpu_chain_records(buf, segs, first, flags),
                    oracle.parse_chains(buf, segs, first, flags))


def test_chain_descriptor_edge_cases(torch):
    f = gen.make_batch(3, n=1).frames[:1500].tobytes()
    buf, segs, first = _chains_of([f, f, f], [[700, 800], [1500], [34, 1466]])
    weird = np.array([0, 0, 2, 1, 99, 3, 4, 5], np.uint32)   # empty, decreasing, past n_segs
    assert_same(gpu_chain_records(buf, segs, weird, 3), oracle.parse_chains(buf, segs, weird, 3))
    # a segment running past the arena is clamped like a frame
    segs2 = segs.copy()
    segs2[-1, 1] = 100000
    assert_same(gpu_chain_records(buf, segs2, first, 3), oracle.parse_chains(buf, segs2, first, 3))


def test_single_segment_chains_equal_parse_batch(torch):
    hb = gen.make_batch(6, n=5000, seed=66)
    frames = [hb.frames[hb.offsets[i]:hb.offsets[i + 1]].tobytes() for i in range(hb.n)]
    buf, segs, first = _chains_of(frames, [[len(x)] for x in frames])
    g = gpu_chain_records(buf, segs, first, 3)
    db = engine.DeviceBatch.from_host(hb)
    assert_same(g, as_records(engine.parse_batch(db, 3).cpu().numpy()))


@pytest.mark.parametrize("n", [1, 63, 65, 257])
def test_chain_ragged_sizes(torch, n):
    hc = gen.make_chains(8, n=n, seed=800 + n)
    assert_same(gpu_chain_records(hc.buf, hc.segs, hc.chain_first, 3),
                oracle.parse_chains(hc.buf, hc.segs, hc.chain_first, 3))


def test_parse_chains_rejects_bad_descriptors(torch):
    hc = gen.make_chains(8, n=64)
    dc = engine.DeviceChains.from_host(hc)
    with pytest.raises(engine.RpktError):
        engine.parse_chains(dc, flags=3 | 64)
    odd = engine.DeviceChains(dc.buf, dc.segs[1:], dc.chain_first, dc.n)   # 4-byte aligned segs
    with pytest.raises(engine.RpktError):
        engine.parse_chains(odd, flags=3)
