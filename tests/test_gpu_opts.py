"""GPU parity of rpkt_gpu_options_batch (TcpOptionsIter / Ipv4OptionsIter) against
oracle/rpkt_oracle_opts.c, bit-exact, on the reference captures and full batches;
every case also walks from compact records (rpkt_gpu_options_batch_compact) and in the
fused pass (rpkt_gpu_parse_options_batch[_compact]: records, flow events and option
walks of one launch, each byte-identical to the oracle's parse + walks)."""
import os

import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, gen
from rpkt_amd.records import F_FLOW_EV, OPT_STOP, as_opts, as_records, as_records16, project16

from test_gpu_parity import host_batch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
PKTS = os.path.join(HERE, "golden", "packets")


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def gpu_opts(hb):
    db = engine.DeviceBatch.from_host(hb)
    recs = engine.parse_batch(db, 3)
    o = as_opts(engine.options_batch(db, recs).cpu().numpy())
    r16 = engine.parse_batch_compact(db, 3)
    oc = as_opts(engine.options_batch(db, r16, compact=True).cpu().numpy())
    return o, oc, as_records(recs.cpu().numpy())


def diff_records(what, g, o):
    if g.tobytes() != o.tobytes():
        i = int(np.nonzero(g != o)[0][0])
        raise AssertionError("%s: record %d differs: gpu %s oracle %s" % (what, i, g[i], o[i]))


def fused(hb, flags=3, n_buckets=0):
    """The fused entry points (full and compact records), checked against the oracle's
    parse; returns their option walks."""
    db = engine.DeviceBatch.from_host(hb)
    o = oracle.parse_batch(hb.frames, hb.n, flags & 3, offsets=hb.offsets, stride=hb.stride,
                           frame_len=hb.frame_len)
    outs = []
    for compact in (False, True):
        res = engine.parse_options_batch(db, flags, n_buckets=n_buckets, compact=compact)
        if compact:
            diff_records("fused compact records", as_records16(res[0].cpu().numpy()),
                         project16(o, flags & 3))
        else:
            diff_records("fused records", as_records(res[0].cpu().numpy()), o)
        if flags & F_FLOW_EV:                      # the same events as the parse alone
            _, ev = engine.parse_batch(db, flags, n_buckets=n_buckets)
            assert np.array_equal(res[2].cpu().numpy(), ev.cpu().numpy()), "flow events differ"
        outs.append(as_opts(res[1].cpu().numpy()))
    return outs


def check(hb):
    g, gc, r = gpu_opts(hb)
    o = oracle.options_batch(hb.frames, hb.n, r, offsets=hb.offsets, stride=hb.stride,
                             frame_len=hb.frame_len)
    f, fc = fused(hb)
    for what, x in (("full records", g), ("compact records", gc), ("fused", f),
                    ("fused compact", fc)):
        if x.tobytes() != o.tobytes():
            bad = np.nonzero(x.view(np.uint8).reshape(-1, 64) != o.view(np.uint8).reshape(-1, 64))
            i = int(bad[0][0])
            raise AssertionError("%s: %d frames differ, first %d: gpu %s oracle %s" % (
                what, len(np.unique(bad[0])), i, x[i], o[i]))
    return g, r


@pytest.mark.parametrize("cfg", [2, 3, 5, 6])
def test_options_parity_configs(torch, cfg):
    hb = gen.make_batch(cfg)
    g, r = check(hb)
    if cfg == 5:
        ok = r["status"] == 0
        assert (g["tcp_stop"][ok] == OPT_STOP["END"]).all()


@pytest.mark.parametrize("lead", [0, 1, 3, 7, 13, 15])
def test_options_fixtures_every_alignment(torch, lead):
    frames = [oracle.load_dat(os.path.join(PKTS, n)) for n in sorted(os.listdir(PKTS))]
    check(host_batch(frames * 3, lead))


def test_options_random_option_bytes(torch):
    """Random bytes in every option slice (config 5 frames with their IPv4 and TCP
    option areas overwritten): unknown types, bad lengths, truncated options."""
    hb = gen.make_batch(5, 1 << 16, seed=77)
    r = oracle.parse_batch(hb.frames, hb.n, 3, offsets=hb.offsets)
    rng = np.random.default_rng(3)
    f = hb.frames
    for i in np.nonzero(r["status"] == 0)[0]:
        o = int(hb.offsets[i])
        a, b = o + int(r["l3_off"][i]) + 20, o + int(r["l4_off"][i])
        f[a:b] = rng.integers(0, 256, b - a, dtype=np.uint8) if rng.integers(0, 2) else \
            rng.choice([0, 1, 7, 68, 148, 134, 137, 131, 2, 3, 40], b - a).astype(np.uint8)
        c, d = o + int(r["l4_off"][i]) + 20, o + int(r["payload_off"][i])
        f[c:d] = rng.choice([0, 1, 2, 3, 4, 5, 8, 34, 10, 12, 99], d - c).astype(np.uint8)
    g, _ = check(hb)
    assert set(g["tcp_stop"].tolist()) >= {1, 2, 3} and set(g["ip_stop"].tolist()) >= {1, 2, 3}


@pytest.mark.parametrize("flags", [0, 1, 2, 3, 3 | F_FLOW_EV])
def test_fused_flags(torch, flags):
    """Every flag set of the fused pass: records and events as the parse alone, option
    walks as the standalone walk (which needs only the offsets every flag set fills)."""
    hb = gen.make_batch(6, 1 << 15, seed=11)
    r = oracle.parse_batch(hb.frames, hb.n, 3, offsets=hb.offsets)
    o = oracle.options_batch(hb.frames, hb.n, r, offsets=hb.offsets)
    for x in fused(hb, flags, n_buckets=8192 if flags & F_FLOW_EV else 0):
        assert x.tobytes() == o.tobytes()


@pytest.mark.parametrize("n", [1, 63, 64, 65, 257, 1000])
def test_fused_ragged(torch, n):
    hb = gen.make_batch(5, n, seed=100 + n)
    check(hb)


def test_fused_window_overflow(torch):
    """Option slices that end past the 128-B header window (QinQ + 60-B IPv4 header +
    60-B TCP header at every 16-B phase): the fused pass refills those slots."""
    frames = []
    rng = np.random.default_rng(5)
    for k in range(512):
        ihl, doff = 15 - (k % 3), 15 - (k // 3) % 3
        l3 = 22
        tot = ihl * 4 + doff * 4 + int(rng.integers(0, 40))
        f = np.zeros(l3 + tot + int(rng.integers(0, 9)), np.uint8)
        f[12:14] = (0x88, 0xa8)
        f[16:18] = (0x81, 0x00)
        f[20:22] = (0x08, 0x00)
        f[l3] = 0x40 | ihl
        f[l3 + 2:l3 + 4] = (tot >> 8, tot & 0xff)
        f[l3 + 9] = 6
        f[l3 + 20:l3 + ihl * 4] = rng.choice([1, 1, 1, 0, 7, 68, 148], ihl * 4 - 20)
        l4 = l3 + ihl * 4
        f[l4 + 12] = doff << 4
        f[l4 + 20:l4 + doff * 4] = rng.choice([1, 1, 2, 4, 8, 3, 5, 0], doff * 4 - 20)
        frames.append(f.tobytes())
    for lead in (0, 5, 15):
        check(host_batch(frames, lead))
