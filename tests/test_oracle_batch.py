"""Oracle batch drivers: single-thread, multi-thread, strided and packed layouts,
clamping of descriptors that point past the buffer, flow counters."""
import numpy as np

from oracle import oracle
from rpkt_amd import gen
from rpkt_amd.records import REC_DTYPE


def test_mt_equals_st():
    b = gen.make_batch(6, 30000)
    a = oracle.parse_batch(b.frames, b.n, offsets=b.offsets)
    m = oracle.parse_batch(b.frames, b.n, offsets=b.offsets, threads=7)
    assert a.tobytes() == m.tobytes()
    s = gen.make_batch(3, 3000)
    a = oracle.parse_batch(s.frames, s.n, stride=s.stride)
    m = oracle.parse_batch(s.frames, s.n, stride=s.stride, threads=5)
    assert a.tobytes() == m.tobytes()


def test_packed_equals_per_frame():
    b = gen.make_batch(6, 2000)
    r = oracle.parse_batch(b.frames, b.n, offsets=b.offsets)
    for i in range(0, b.n, 37):
        f = b.frames[b.offsets[i]:b.offsets[i + 1]].tobytes()
        assert oracle.parse_one(f).tobytes() == r[i].tobytes()


def test_descriptor_clamping():
    frames = np.arange(300, dtype=np.uint8)
    offs = np.array([0, 100, 50, 400, 500], dtype=np.uint32)   # decreasing + past the end
    r = oracle.parse_batch(frames, 4, offsets=offs)
    assert [int(x) for x in r["frame_len"]] == [100, 0, 250, 0]


def test_flow_counts_conserve_packets_and_bytes():
    b = gen.make_batch(4, 50000)
    r, ev = oracle.parse_batch(b.frames, b.n, offsets=b.offsets, n_buckets=8192, flow_ev=True)
    c = oracle.flow_count(ev, 8192).reshape(-1, 4)
    assert int(c[:, 0].sum()) == b.n
    assert int(c[:, 1].sum()) == int(b.lens().sum())
    assert int(c[:, 2].sum()) == int((r["ip_sum"] != 0xffff).sum())
    assert c[8192, 0] == 0                       # every IMIX frame parses to L4
    nz = (c[:8192, 0] > 0).sum()
    assert nz > 6000                             # flows spread over the buckets
