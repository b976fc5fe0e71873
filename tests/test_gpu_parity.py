"""GPU parity: every record byte of the HIP path equals the oracle's on the same
buffers (bit-exact; integer/byte work has no tolerance), at the BASELINE.json
full sizes and on the edge cases rpkt's own tests exercise."""
import os

import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, gen
from rpkt_amd.records import REC_DTYPE, STATUS, F_FLOW_EV, as_records

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
PKTS = os.path.join(HERE, "golden", "packets")
THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def gpu_records(hb, flags=3, n_buckets=0):
    db = engine.DeviceBatch.from_host(hb)
    if flags & F_FLOW_EV:
        recs, ev = engine.parse_batch(db, flags, n_buckets=n_buckets)
        return as_records(recs.cpu().numpy()), ev.cpu().numpy().view(np.uint64)
    return as_records(engine.parse_batch(db, flags).cpu().numpy())


def oracle_records(hb, flags=3, n_buckets=0, flow=False):
    return oracle.parse_batch(hb.frames, hb.n, flags=flags, offsets=hb.offsets,
                              stride=hb.stride, frame_len=hb.frame_len, n_buckets=n_buckets,
                              threads=THREADS, flow_ev=flow)


def assert_same(g, o):
    if g.tobytes() == o.tobytes():
        return
    bad = np.nonzero(g.view(np.uint8).reshape(-1, 80) != o.view(np.uint8).reshape(-1, 80))
    i = int(bad[0][0])
    fields = [f for f in REC_DTYPE.names if not np.array_equal(g[i][f], o[i][f])]
    raise AssertionError("%d records differ; first #%d fields %s gpu=%s oracle=%s" % (
        len(np.unique(bad[0])), i, fields, [g[i][f] for f in fields], [o[i][f] for f in fields]))


def host_batch(frames_list, lead=0):
    """Packed HostBatch from a list of byte strings; a `lead`-byte junk frame first
    shifts every following frame's alignment."""
    parts = ([b"\xee" * lead] if lead else []) + list(frames_list)
    lens = np.array([len(p) for p in parts], dtype=np.uint64)
    offs = np.zeros(len(parts) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    blob = np.frombuffer(b"".join(parts), dtype=np.uint8).copy()
    return gen.HostBatch(0, len(parts), 0, blob, offs.astype(np.uint32), 0, 0)


# ---- full-size BASELINE configs --------------------------------------------------

@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5, 6])
def test_parity_baseline_configs(torch, cfg):
    hb = gen.make_batch(cfg)
    flags = 3
    g = gpu_records(hb, flags)
    o = oracle_records(hb, flags)
    assert_same(g, o)
    if cfg in (2, 3, 4):
        assert (g["status"] == STATUS["OK"]).all()


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
@pytest.mark.parametrize("cfg", [3, 5, 6])
def test_parity_flag_combinations(torch, cfg, flags):
    hb = gen.make_batch(cfg, 50000, seed=100 + cfg)
    assert_same(gpu_records(hb, flags), oracle_records(hb, flags))


def test_parity_flow_events_and_counters(torch):
    hb = gen.make_batch(4, 1 << 20, seed=41)
    nb = 8192
    g, gev = gpu_records(hb, 3 | F_FLOW_EV, nb)
    o, oev = oracle_records(hb, 3, nb, flow=True)
    assert_same(g, o)
    assert np.array_equal(gev, oev)
    dev = torch.from_numpy(gev.view(np.int64)).cuda()
    c = engine.flow_count(dev, hb.n, nb).cpu().numpy().view(np.uint64)
    assert np.array_equal(c, oracle.flow_count(oev, nb))
    # calls accumulate
    c2 = engine.flow_count(dev, hb.n, nb, counters=torch.from_numpy(c.view(np.int64)).cuda())
    assert np.array_equal(c2.cpu().numpy().view(np.uint64), 2 * oracle.flow_count(oev, nb))


def test_flow_counters_large_bucket_count(torch):
    hb = gen.make_batch(4, 200000, seed=43)
    nb = 50000                                     # beyond the LDS-privatised range
    g, gev = gpu_records(hb, 3 | F_FLOW_EV, nb)
    _, oev = oracle_records(hb, 3, nb, flow=True)
    assert np.array_equal(gev, oev)
    dev = torch.from_numpy(gev.view(np.int64)).cuda()
    c = engine.flow_count(dev, hb.n, nb).cpu().numpy().view(np.uint64)
    assert np.array_equal(c, oracle.flow_count(oev, nb))


# ---- reference fixtures at every alignment ---------------------------------------

def fixtures():
    names = sorted(f for f in os.listdir(PKTS) if f.endswith(".dat"))
    return names, [oracle.load_dat(os.path.join(PKTS, f)) for f in names]


@pytest.mark.parametrize("lead", list(range(16)))
def test_fixtures_every_alignment(torch, lead):
    names, frames = fixtures()
    hb = host_batch(frames, lead)
    g, o = gpu_records(hb), oracle_records(hb)
    assert_same(g, o)
    base = 1 if lead else 0
    i = base + names.index("TcpPacketWithOptions2.dat")
    assert g[i]["ip_sum"] == 0xffff and g[i]["l4_sum"] == 0xffff


def test_views_over_gpu_records(torch):
    from rpkt_amd.views import EtherFrame, Ipv4, Udp, Packet, EtherType, IpProtocol
    frame = oracle.load_dat(os.path.join(PKTS, "bench_frame.dat"))
    g = gpu_records(host_batch([frame] * 3))
    eth = EtherFrame.parse(Packet(g[1], frame)).unwrap()
    assert eth.ethertype() == EtherType.IPV4
    ip = Ipv4.parse(eth.payload()).unwrap()
    assert ip.protocol() == IpProtocol.UDP and ip.ident() == 0x5c65 and ip.checksum() == 0
    udp = Udp.parse(ip.payload()).unwrap()
    assert (udp.src_port(), udp.dst_port(), udp.packet_len(), udp.checksum()) == \
        (60376, 161, 74, 0xbc86)
    assert udp.payload().chunk() == frame[42:108]


# ---- edge cases --------------------------------------------------------------------

@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 255, 256, 257, 1000])
def test_ragged_batch_sizes(torch, n):
    hb = gen.make_batch(6, n, seed=n)
    assert_same(gpu_records(hb), oracle_records(hb))


def test_empty_batch(torch):
    db = engine.DeviceBatch(torch.zeros(16, dtype=torch.uint8, device="cuda"), 0, None, 64)
    out = engine.alloc_records(1)
    engine.parse_batch(db, 3, recs=out)          # no launch, no error


def test_unpadded_buffer_end(torch):
    """Last frame ends at the last byte of an allocation that is not a multiple of 16."""
    for cfg in (3, 5, 6):
        hb = gen.make_batch(cfg, 777, seed=9)
        hb.frames = hb.frames[:int(hb.offsets[-1])] if hb.offsets is not None else hb.frames
        assert_same(gpu_records(hb), oracle_records(hb))


def test_descriptor_past_buffer_is_clamped(torch):
    hb = gen.make_batch(6, 1000, seed=5)
    offs = hb.offsets.copy()
    offs[500] = offs[-1] + 1000                  # one frame starts past the end
    offs[700] = offs[699] - 5                    # one negative length
    hb.offsets = offs
    assert_same(gpu_records(hb), oracle_records(hb))


def test_long_tiles_with_ragged_offsets(torch):
    """1500-B frames packed (tiles over the 64-KB threshold, so the edge lines are
    summed before the parse) with shifted, empty, negative, overlapping and past-the-end
    offsets, and IPv4 total lengths short of the frame (Ethernet padding)."""
    rng = np.random.default_rng(33)
    base = gen.make_batch(3, 4096, seed=33)
    offs = (np.arange(base.n + 1, dtype=np.int64) * base.stride)
    offs[100:] += 7                                   # odd phase from here on
    offs[200] = offs[199]                             # empty frame
    offs[300] = offs[299] - 100                       # negative length
    offs[400] = offs[401] + 3000                      # overlapping the next frames
    offs[500] = int(offs[-1]) + 10000                 # past the end
    frames = np.zeros(int(offs[-1]) + 64, dtype=np.uint8)
    src = base.frames.reshape(base.n, base.stride)
    for k in range(base.n):                           # lay frame k at its (new) offset
        o = int(offs[k])
        if 0 <= o and o + base.stride <= frames.size:
            frames[o:o + base.stride] = src[k]
    for k in rng.choice(base.n, 200, replace=False):  # IPv4 tot short of the frame
        o = int(offs[k])
        if 0 <= o and o + 18 <= frames.size:
            frames[o + 16:o + 18] = [0x04, 0x00]
    offs = np.clip(offs, 0, None).astype(np.uint32)
    hb = gen.HostBatch(0, base.n, 0, frames, offs, 0, 0)
    assert_same(gpu_records(hb), oracle_records(hb))


def test_jumbo_and_max_length_frames(torch):
    rng = np.random.default_rng(1)
    frames = []
    for L in (9000, 9001, 16384, 65535, 65549):
        base = gen.make_batch(3, 1, seed=L)          # 1500-B TCP frame as a template
        f = bytearray(base.frames.tobytes()) + bytearray(rng.integers(0, 256, L - 1500,
                                                                      dtype=np.uint8).tobytes())
        tot = min(L - 14, 65535)
        f[16:18] = bytes([tot >> 8, tot & 0xff])
        frames.append(bytes(f))
    hb = host_batch(frames, lead=3)
    g, o = gpu_records(hb), oracle_records(hb)
    assert_same(g, o)
    assert (g["status"][1:] == 0).all()


def test_repeat_launches_identical(torch):
    hb = gen.make_batch(5, 100000, seed=77)
    db = engine.DeviceBatch.from_host(hb)
    a = engine.parse_batch(db, 3).cpu().numpy()
    for _ in range(3):
        assert np.array_equal(engine.parse_batch(db, 3).cpu().numpy(), a)


def test_checksum_ranges_match_from_slice(torch):
    rng = np.random.default_rng(2)
    buf = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    n = 20000
    starts = rng.integers(0, buf.size, n)
    lens = rng.integers(0, 4000, n)
    lens[::10] = rng.integers(0, 20, n // 10)
    lens[::97] = 65535
    lens = np.minimum(lens, buf.size - starts)
    ranges = np.stack([starts, lens], 1).astype(np.uint32)
    out = engine.checksum_ranges(torch.from_numpy(buf).cuda(),
                                 torch.from_numpy(ranges.view(np.int32)).cuda())
    got = out.cpu().numpy().view(np.uint16)
    want = [oracle.from_slice(buf[s:s + l]) for s, l in ranges[:3000]]
    assert got[:3000].tolist() == want


def test_checksum_ranges_at_buffer_end(torch):
    """Every (start, len) range inside the last 48 bytes of buffers whose size is not
    a multiple of 16: the edge chunks of the stream straddle the descriptor's end
    (the hardware drops such a dwordx4 whole; the kernel re-reads it), at every phase."""
    rng = np.random.default_rng(21)
    for size in (1001, 1024 + 7, 4093, 33, 7):
        buf = rng.integers(0, 256, size, dtype=np.uint8)
        lo = max(0, size - 48)
        ranges = np.array([(s, l) for s in range(lo, size + 1) for l in range(0, size - s + 1)],
                          dtype=np.uint32)
        out = engine.checksum_ranges(torch.from_numpy(buf).cuda(),
                                     torch.from_numpy(ranges.view(np.int32)).cuda())
        got = out.cpu().numpy().view(np.uint16).tolist()
        want = [oracle.from_slice(buf[s:s + l]) for s, l in ranges]
        assert got == want, size


def test_cpp_host_example_through_c_abi(torch):
    """examples/parse_batch: a non-Python host (plain hipMalloc) drives the C ABI."""
    import subprocess
    from rpkt_amd.build import build_example
    exe = build_example()[0]
    r = subprocess.run([exe, "100000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "status=OK" in r.stdout and "sport=60376" in r.stdout


def test_cpp_flow_reduce_through_c_abi(torch):
    """examples/flow_reduce: a C++ host shards frames over the visible GPUs, parses with
    flow events, counts, and sums the counters with rpkt_gpu_flow_reduce over an
    ncclCommInitAll communicator; every counter word must equal the host's count."""
    import subprocess
    from rpkt_amd.build import FLOW_REDUCE_BIN
    r = subprocess.run([FLOW_REDUCE_BIN, "300000", "8192"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "differing from the host count on any GPU: 0" in r.stdout, r.stdout


def test_checksum_chains_match_from_buf(torch):
    """Multi-segment (mbuf chain) sums vs the oracle's from_buf (checksum.rs:8-27):
    segments of odd and even lengths at arbitrary buffer offsets, chains of 0..9."""
    rng = np.random.default_rng(4)
    buf = rng.integers(0, 256, 4 << 20, dtype=np.uint8)
    n_chains = 5000
    counts = rng.integers(0, 10, n_chains)
    first = np.zeros(n_chains + 1, dtype=np.uint32)
    first[1:] = np.cumsum(counts)
    n_segs = int(first[-1])
    starts = rng.integers(0, buf.size - 3000, n_segs)
    lens = rng.integers(0, 3000, n_segs)
    lens[::7] = rng.integers(0, 3, (n_segs + 6) // 7)           # tiny segments
    segs = np.stack([starts, lens], 1).astype(np.uint32)
    out = engine.checksum_chains(torch.from_numpy(buf).cuda(),
                                 torch.from_numpy(segs.view(np.int32)).cuda(),
                                 torch.from_numpy(first.view(np.int32)).cuda())
    got = out.cpu().numpy().view(np.uint16)
    for p in range(0, n_chains, 3):
        parts = [buf[s:s + l].tobytes() for s, l in segs[first[p]:first[p + 1]]]
        assert got[p] == oracle.from_buf(parts), p


# ---- compact records (rpkt_gpu_parse_batch_compact) ---------------------------------

def gpu_records16(hb, flags=3, n_buckets=0):
    from rpkt_amd.records import as_records16
    db = engine.DeviceBatch.from_host(hb)
    if flags & F_FLOW_EV:
        recs, ev = engine.parse_batch_compact(db, flags, n_buckets=n_buckets)
        return as_records16(recs.cpu().numpy()), ev.cpu().numpy().view(np.uint64)
    return as_records16(engine.parse_batch_compact(db, flags).cpu().numpy())


def assert_same16(g, o):
    if g.tobytes() == o.tobytes():
        return
    bad = np.nonzero(g != o)[0]
    i = int(bad[0])
    fields = [f for f in g.dtype.names if g[i][f] != o[i][f]]
    raise AssertionError("%d compact records differ; first #%d fields %s gpu=%s oracle=%s" % (
        bad.size, i, fields, [g[i][f] for f in fields], [o[i][f] for f in fields]))


@pytest.mark.parametrize("cfg", [2, 3, 4, 5, 6])
def test_compact_records_equal_projected_oracle(torch, cfg):
    """The 16-byte records equal the oracle's full records projected (status, offsets,
    sums, verdict bits), full BASELINE sizes for configs 2-5, the fuzz mix for 6."""
    from rpkt_amd.records import project16
    hb = gen.make_batch(cfg)
    flags = gen.FLAGS.get(cfg, 3)
    assert_same16(gpu_records16(hb, flags), project16(oracle_records(hb, flags), flags))


@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_compact_flag_combinations_and_flow_events(torch, flags):
    from rpkt_amd.records import project16
    hb = gen.make_batch(6, 60000, seed=77)
    nb = 4096
    g, gev = gpu_records16(hb, flags | F_FLOW_EV, nb)
    o, oev = oracle_records(hb, flags, nb, flow=True)
    assert_same16(g, project16(o, flags))
    assert np.array_equal(gev, oev)


@pytest.mark.parametrize("lead", [0, 1, 3, 7, 13])
def test_compact_fixtures_alignment(torch, lead):
    from rpkt_amd.records import project16
    _, frames = fixtures()
    hb = host_batch(frames, lead)
    assert_same16(gpu_records16(hb), project16(oracle_records(hb), 3))


# ---- strided batches of short frames at every stride phase -----------------------------

@pytest.mark.parametrize("stride,flen", [(64, 64), (64, 60), (64, 14), (48, 48), (49, 49),
                                         (40, 40), (80, 64), (32, 20), (64, 65), (96, 96),
                                         (112, 112), (128, 128), (113, 113), (129, 129),
                                         (144, 128)])
def test_short_strided_frames(torch, stride, flen):
    """Strided batches of short frames (strides that are and are not multiples of 16, so
    every 16-B phase of a window occurs): fuzzed headers of every status cut to flen
    bytes, records bit-exact vs the oracle, full and compact.  Batches whose frames all
    lie in their 128-B (64-B) windows take the in-window L4 instantiation (no stream
    past the window); (129, 129) and (64, 65) just miss it."""
    from rpkt_amd.records import project16
    src = gen.make_batch(6, 20000, seed=stride * 131 + flen)
    n = src.n
    buf = np.zeros(n * stride + 64, dtype=np.uint8)
    lens = src.lens()
    for i in range(n):
        a = int(src.offsets[i])
        k = min(int(lens[i]), flen)
        buf[i * stride:i * stride + k] = src.frames[a:a + k]
    hb = gen.HostBatch(6, n, 0, buf, None, stride, flen)
    for flags in (1, 3):
        o = oracle_records(hb, flags)
        assert_same(gpu_records(hb, flags), o)
        assert_same16(gpu_records16(hb, flags), project16(o, flags))
    # compact records with flow events (frames inside a 64-B window take the 64-B-window
    # compile of the compact parse)
    g, gev = gpu_records16(hb, 3 | F_FLOW_EV, 4096)
    o, oev = oracle_records(hb, 3, 4096, flow=True)
    assert_same16(g, project16(o, 3))
    assert np.array_equal(gev, oev)


@pytest.mark.parametrize("stride,flen", [(64, 64), (80, 80), (113, 113), (128, 128), (130, 130)])
def test_short_strided_dual_stack(torch, stride, flen):
    """The same over the dual-stack fuzz (IPv6 extension chains cut at any byte): full and
    compact records, flow events, and a receive ring of such batches, against the oracle."""
    from rpkt_amd.records import F_IPV6, project16
    src = gen.make_batch(12, 12000, seed=stride * 7 + flen)
    n = src.n
    buf = np.zeros(n * stride + 64, dtype=np.uint8)
    lens = src.lens()
    for i in range(n):
        a = int(src.offsets[i])
        k = min(int(lens[i]), flen)
        buf[i * stride:i * stride + k] = src.frames[a:a + k]
    hb = gen.HostBatch(12, n, 0, buf, None, stride, flen)
    for flags in (F_IPV6 | 3, F_IPV6 | 2):
        o = oracle_records(hb, flags)
        assert_same(gpu_records(hb, flags), o)
        assert_same16(gpu_records16(hb, flags), project16(o, flags))
    g, gev = gpu_records16(hb, F_IPV6 | 3 | F_FLOW_EV, 4096)
    o, oev = oracle_records(hb, F_IPV6 | 3, 4096, flow=True)
    assert_same16(g, project16(o, F_IPV6 | 3))
    assert np.array_equal(gev, oev)
    db = engine.DeviceBatch.from_host(hb)
    recs = [engine.alloc_records(n), engine.alloc_records(n)]
    engine.parse_ring(engine.ring_slots([db, db], recs), F_IPV6 | 3)
    o = oracle_records(hb, F_IPV6 | 3)
    for r in recs:
        assert_same(as_records(r.cpu().numpy()), o)
