"""GPU parity of the IPv6 decode-and-verify path (RPKT_F_IPV6): every record byte, compact
record, flow event and option walk of the HIP engine equals the oracle's
(oracle/rpkt_oracle.c oracle_parse_ip6, pinned by tests/test_oracle_ip6.py) on the same
buffers.  Bit-exact: integer and byte work has no tolerance."""
import os

import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, gen
from rpkt_amd.records import (F_FLOW_EV, F_IPV6, STATUS, as_opts, as_records, as_records16,
                              ip6_opts_view, is_ip6, project16)

from ip6_frames import ip6_frame as _ip6_frame, ip6_opts as _ip6_opts  # noqa: F401
from test_gpu_parity import assert_same, assert_same16, host_batch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
PKTS = os.path.join(HERE, "golden", "packets")
THREADS = min(16, os.cpu_count() or 1)
F6 = 3 | F_IPV6


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def oracle_recs(hb, flags, n_buckets=0, flow=False):
    return oracle.parse_batch(hb.frames, hb.n, flags=flags & ~F_FLOW_EV, offsets=hb.offsets,
                              stride=hb.stride, frame_len=hb.frame_len, n_buckets=n_buckets,
                              threads=THREADS, flow_ev=flow)


def check_batch(hb, flags=F6, n_buckets=4096):
    """80-B and compact records and flow events of one batch against the oracle."""
    db = engine.DeviceBatch.from_host(hb)
    o, oev = oracle_recs(hb, flags, n_buckets, flow=True)
    recs, ev = engine.parse_batch(db, flags | F_FLOW_EV, n_buckets=n_buckets)
    g = as_records(recs.cpu().numpy())
    assert_same(g, o)
    assert np.array_equal(ev.cpu().numpy().view(np.uint64), oev), "flow events differ"
    r16, ev16 = engine.parse_batch_compact(db, flags | F_FLOW_EV, n_buckets=n_buckets)
    assert_same16(as_records16(r16.cpu().numpy()), project16(o, flags))
    assert np.array_equal(ev16.cpu().numpy().view(np.uint64), oev), "compact flow events differ"
    return g


@pytest.mark.parametrize("cfg", [10, 11])
def test_dual_stack_full_size(torch, cfg):
    """1M x 64 B and 1M x 1500 B v4/v6 mixes (BASELINE's 64/1500-B sizes, dual stack)."""
    hb = gen.make_batch(cfg)
    g = check_batch(hb)
    assert (g["status"] == STATUS["OK"]).all()
    assert 0.45 < is_ip6(g).mean() < 0.55


@pytest.mark.parametrize("flags", [F_IPV6, F_IPV6 | 1, F_IPV6 | 2, F6])
def test_dual_stack_fuzz_every_status(torch, flags):
    hb = gen.make_batch(12)
    g = check_batch(hb, flags)
    seen = set(int(s) for s in np.unique(g["status"]))
    assert {STATUS[k] for k in ("IP6_SHORT", "IP6_BAD_LEN", "IP6_EXT_SHORT", "IP6_EXT_BAD_LEN",
                                "IP6_FRAGMENT", "L4_OTHER", "OK")} <= seen


@pytest.mark.parametrize("n", [1, 63, 65, 1000])
def test_dual_stack_ragged(torch, n):
    check_batch(gen.make_batch(12, n, seed=n + 7))


def fixtures():
    names = sorted(f for f in os.listdir(PKTS) if f.endswith(".dat"))
    return names, [oracle.load_dat(os.path.join(PKTS, f)) for f in names]


@pytest.mark.parametrize("lead", list(range(16)))
def test_fixtures_every_alignment_ip6(torch, lead):
    """All 53 captures (IPv4 and IPv6) at every 16-B phase with RPKT_F_IPV6; the two
    IPv6 UDP captures verify (ipv6_options_routing2.dat only with the routing header's
    final address in the pseudo header)."""
    names, frames = fixtures()
    hb = host_batch(frames, lead)
    g = check_batch(hb)
    base = 1 if lead else 0
    for nm in ("ipv6_options_destination.dat", "ipv6_options_routing2.dat"):
        r = g[base + names.index(nm)]
        assert int(r["status"]) == STATUS["OK"] and int(r["l4_sum"]) == 0xffff, nm
    r = g[base + names.index("ipv6_options_fragments.dat")]
    assert int(r["status"]) == STATUS["IP6_FRAGMENT"]


def test_extension_chains_past_the_window(torch):
    """Extension headers and L4 headers beyond the 128-B LDS window (HopByHop up to 2048 B,
    routing lists, AH), UDP and TCP, at every 16-B phase: the engine reads them from
    global memory and streams the L4 sum from its first byte."""
    rng = np.random.default_rng(61)
    frames = []
    for hbh in (8, 16, 48, 72, 96, 120, 2048):
        for proto in (17, 6):
            for tail in ([], [(43, 8 + 16 * 3)], [(60, 24), (51, 12 + 8)], [(44, 8)]):
                pl = rng.integers(0, 256, int(rng.integers(0, 1500)), dtype=np.uint8).tobytes()
                frames.append(_ip6_frame(rng, [(0, hbh)] + tail, proto, pl,
                                         tag=bool(rng.integers(0, 2))))
    frames.append(_ip6_frame(rng, [(60, 2048)] * 7, 17, b"\x55" * 40000))   # ~55 KB frame
    for lead in range(16):
        hb = host_batch(frames, lead)
        g = check_batch(hb)
        base = 1 if lead else 0
        assert (g["status"][base:] == STATUS["OK"]).all()
        assert (g["l4_sum"][base:] == 0xffff).all()


def test_without_flag_ip6_frames_stay_not_ipv4(torch):
    hb = gen.make_batch(11, 20000, seed=3)
    db = engine.DeviceBatch.from_host(hb)
    g = as_records(engine.parse_batch(db, 3).cpu().numpy())
    assert_same(g, oracle_recs(hb, 3))
    o6 = oracle_recs(hb, F6)
    assert (g["status"][is_ip6(o6)] == STATUS["NOT_IPV4"]).all()


def _opts_check(db, hb, flags):
    o = oracle_recs(hb, flags)
    want = oracle.options_batch(hb.frames, hb.n, o, offsets=hb.offsets, stride=hb.stride,
                                frame_len=hb.frame_len)
    outs = []
    for compact in (False, True):
        recs, opts = engine.parse_options_batch(db, flags, compact=compact)
        if compact:
            assert_same16(as_records16(recs.cpu().numpy()), project16(o, flags))
        else:
            assert_same(as_records(recs.cpu().numpy()), o)
        outs.append(as_opts(opts.cpu().numpy()))
        # the standalone walk over the same records
        outs.append(as_opts(engine.options_batch(db, recs, compact=compact).cpu().numpy()))
    for k, x in enumerate(outs):
        assert x.tobytes() == want.tobytes(), "walk %d differs" % k
    return want, o


@pytest.mark.parametrize("cfg,n", [(11, 200000), (12, None)])
def test_option_walks_over_ip6(torch, cfg, n):
    """TcpOptionsIter runs over IPv6/TCP frames too; Ipv4OptionsIter never over IPv6 (its
    bytes of an IPv6 frame's row are the Ipv6OptionsIter view: stop NONE without an
    option header, END or MALFORMED after walking one)."""
    hb = gen.make_batch(cfg, n)
    want, o = _opts_check(engine.DeviceBatch.from_host(hb), hb, F6)
    v6 = is_ip6(o)
    walked = ip6_opts_view(want)["n_hdrs"] != 0
    assert set(np.unique(want["ip_stop"][v6 & ~walked])) <= {0}
    assert set(np.unique(want["ip_stop"][v6 & walked])) <= {1, 3}
    tcp6 = v6 & (o["status"] == 0) & (o["ip_protocol"] == 6)
    assert tcp6.any() and (want["tcp_stop"][tcp6] != 0).all()


def test_ring_ip6(torch):
    hbs = [gen.make_batch(c, m, seed=90 + k) for k, (c, m) in
           enumerate([(10, 5000), (11, 3000), (12, 4000), (2, 1000), (12, 1)])]
    dbs = [engine.DeviceBatch.from_host(h) for h in hbs]
    recs = [engine.alloc_records(h.n) for h in hbs]
    evs = [torch.zeros(h.n, dtype=torch.int64, device="cuda") for h in hbs]
    engine.parse_ring(engine.ring_slots(dbs, recs, evs), F6 | F_FLOW_EV, 512)
    r16 = [torch.empty(h.n * 16, dtype=torch.uint8, device="cuda") for h in hbs]
    engine.parse_ring(engine.ring_slots(dbs, r16), F6, 0, compact=True)
    torch.cuda.synchronize()
    for k, hb in enumerate(hbs):
        o, oev = oracle_recs(hb, F6, 512, flow=True)
        assert_same(as_records(recs[k].cpu().numpy()), o)
        assert np.array_equal(evs[k].cpu().numpy().view(np.uint64), oev)
        assert_same16(as_records16(r16[k].cpu().numpy()), project16(o, F6))


def test_build_writes_ip6_records(torch):
    """Round 5: IPv6 records are built (Ipv6::prepend_header + setters), as the oracle."""
    hb = gen.make_batch(11, 4000, seed=5)
    o = oracle_recs(hb, F6)
    db = engine.DeviceBatch.from_host(hb)
    dev_recs = torch.from_numpy(o.view(np.uint8).copy()).cuda()
    built = engine.build_batch(db, dev_recs, 3).cpu().numpy()
    want_frames, want_built = oracle.build_batch(hb.frames, hb.n, o, flags=3, stride=hb.stride)
    assert np.array_equal(built, want_built) and built[is_ip6(o)].all()
    assert np.array_equal(db.frames.cpu().numpy(), want_frames)


def test_short_strided_ip6_frames(torch):
    """Strided 64/48/49-B slots of dual-stack fuzz frames: the compact parse of frames
    inside a 64-B window runs the 64-B-window compile."""
    src = gen.make_batch(12, 20000, seed=77)
    lens = src.lens()
    for stride, flen in ((64, 64), (64, 62), (48, 48), (49, 49)):
        buf = np.zeros(src.n * stride + 64, dtype=np.uint8)
        for i in range(src.n):
            a = int(src.offsets[i])
            k = min(int(lens[i]), flen)
            buf[i * stride:i * stride + k] = src.frames[a:a + k]
        check_batch(gen.HostBatch(12, src.n, 0, buf, None, stride, flen))


@pytest.mark.parametrize("lead", [0, 1, 5, 11])
def test_ip6_option_walks_fixtures_and_long_chains(torch, lead):
    """Ipv6OptionsIter over every HopByHop / DestOptions header (the IPv6 half of
    rpkt_opts_t): the captures, and crafted chains whose options headers run past the
    window (up to 2048 B), with PadN / RouterAlert / Generic options and malformed ones."""
    rng = np.random.default_rng(71 + lead)
    _, frames = fixtures()
    for hbh in (8, 24, 64, 160, 512, 2048):
        for tail in ([], [(60, 16)], [(43, 40), (60, 24)], [(44, 8), (60, 8), (60, 16)]):
            pl = rng.integers(0, 256, int(rng.integers(0, 600)), dtype=np.uint8).tobytes()
            frames.append(_ip6_frame(rng, [(0, hbh)] + tail, int(rng.choice([6, 17])), pl,
                                     opts=True))
    hb = host_batch(frames, lead)
    _opts_check(engine.DeviceBatch.from_host(hb), hb, F6)


@pytest.mark.parametrize("lead", [0, 3])
def test_ip6_option_headers_dealt_out(torch, lead):
    """The distributed IPv6 option walk (rpkt_opts.h ip6_walks, RPKT_IP6_DIST): waves whose
    every frame has three option headers (192 headers: three rounds of 64), frames with
    four to eight (walked serially by their own lane), option headers around Routing /
    Fragment / AH ones, malformed options mid-chain (the walk ends there), and frames with
    none, mixed at random over several waves."""
    rng = np.random.default_rng(505 + lead)
    frames = []
    for w in range(6):
        for _ in range(64):
            if w < 2:                                            # full waves of 3 headers
                exts = [(0, 8 * int(rng.integers(1, 4))), (60, 8 * int(rng.integers(1, 3))),
                        (60, 8 * int(rng.integers(1, 4)))]
            else:
                exts = []
                for _ in range(int(rng.integers(0, 9))):
                    t = int(rng.choice([0, 60, 60, 43, 44, 51]))
                    hl = {0: 8 * int(rng.integers(1, 5)), 60: 8 * int(rng.integers(1, 5)),
                          43: 24, 44: 8, 51: 12 + 4 * int(rng.integers(0, 3))}[t]
                    exts.append((t, hl))
                exts = exts[:8]
            pl = rng.integers(0, 256, int(rng.integers(0, 200)), dtype=np.uint8).tobytes()
            frames.append(_ip6_frame(rng, exts, int(rng.choice([6, 17])), pl, opts=True))
    hb = host_batch(frames, lead)
    want, o = _opts_check(engine.DeviceBatch.from_host(hb), hb, F6)
    n_hdrs = ip6_opts_view(want)["n_hdrs"]
    assert (n_hdrs[lead > 0:][:128] == 3).mean() > 0.5 and (n_hdrs > 3).any()
    assert (want["ip_stop"][is_ip6(o)] == 3).any()               # malformed walks
