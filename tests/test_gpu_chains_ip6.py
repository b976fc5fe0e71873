"""GPU parity of the IPv6 chain over mbuf chains (rpkt_gpu_parse_chains with
RPKT_F_IPV6): every record byte and flow event equals the chain oracle's
(oracle/rpkt_oracle_chain.c parse_pbuf_ip6, pinned by tests/test_oracle_chain_ip6.py)
on the same segments.  Bit-exact."""
import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, gen
from rpkt_amd.records import F_FLOW_EV, F_IPV6, STATUS, as_records

from ip6_frames import ip6_frame
from test_gpu_chains import gpu_chain_records
from test_gpu_parity import assert_same
from test_oracle_chain import _chains_of
from test_oracle_chain_ip6 import _ip6_udp_with_ext

pytestmark = pytest.mark.gpu
F6 = 3 | F_IPV6


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


@pytest.mark.parametrize("cfg", [11, 12])
@pytest.mark.parametrize("flags", [F_IPV6, F_IPV6 | 1, F_IPV6 | 2, F6])
def test_dual_stack_chain_fuzz_parity(torch, cfg, flags):
    hc = gen.make_chains(cfg, n=30000, layout="fuzz", seed=1100 + cfg)
    g = gpu_chain_records(hc.buf, hc.segs, hc.chain_first, flags)
    o = oracle.parse_chains(hc.buf, hc.segs, hc.chain_first, flags)
    assert_same(g, o)
    v6 = (o["status"] == 0) & (o["l3_off"] > 0) & (o["ethertype"] == 0x86DD)
    assert v6.sum() > 1000


def test_dual_stack_chain_flow_events(torch):
    hc = gen.make_chains(12, n=20000, layout="fuzz", seed=77)
    g, ev = gpu_chain_records(hc.buf, hc.segs, hc.chain_first, F6 | F_FLOW_EV, n_buckets=4096)
    o, oev = oracle.parse_chains(hc.buf, hc.segs, hc.chain_first, F6 | F_FLOW_EV, 4096, True)
    assert_same(g, o)
    assert np.array_equal(ev, oev)


def test_dual_stack_mbuf_chains(torch):
    """1500-B dual-stack frames in 2048-B mempool segments (one segment each) and
    single-segment chains of the fuzz config: records equal the flat parse's."""
    hc = gen.make_chains(11, n=100000, layout="mbuf")
    assert_same(gpu_chain_records(hc.buf, hc.segs, hc.chain_first, F6),
                oracle.parse_chains(hc.buf, hc.segs, hc.chain_first, F6))
    hb = gen.make_batch(12, n=5000, seed=12, packed=True)
    frames = [hb.frames[hb.offsets[i]:hb.offsets[i + 1]].tobytes() for i in range(hb.n)]
    buf, segs, first = _chains_of(frames, [[len(x)] for x in frames])
    db = engine.DeviceBatch.from_host(hb)
    assert_same(gpu_chain_records(buf, segs, first, F6),
                as_records(engine.parse_batch(db, F6).cpu().numpy()))


def test_long_extension_chains_split_across_segments(torch):
    """Extension headers up to 2 KB and L4 headers past segment 0's window, cut into 1-6
    segments at random points and at header boundaries: header reads from global memory
    in any segment, chunk tests per header, the L4 stream across the segments."""
    rng = np.random.default_rng(62)
    frames, cuts = [], []
    for hbh in (8, 16, 48, 72, 96, 120, 2048):
        for proto in (17, 6):
            for tail in ([], [(43, 8 + 16 * 3)], [(60, 24), (51, 12 + 8)], [(44, 8)]):
                pl = rng.integers(0, 256, int(rng.integers(0, 1500)), dtype=np.uint8).tobytes()
                f = ip6_frame(rng, [(0, hbh)] + tail, proto, pl, tag=bool(rng.integers(0, 2)))
                for _ in range(6):
                    k = int(rng.integers(1, 7))
                    c = sorted(int(x) for x in rng.integers(0, len(f) + 1, k - 1))
                    if k > 1 and rng.integers(0, 2):
                        c[0] = min(len(f), int(rng.choice([54, 58, 62, 62 + hbh, 70 + hbh])))
                        c = sorted(c)
                    e = [0] + c + [len(f)]
                    frames.append(f)
                    cuts.append([e[i + 1] - e[i] for i in range(k)])
    buf, segs, first = _chains_of(frames, cuts)
    g = gpu_chain_records(buf, segs, first, F6)
    o = oracle.parse_chains(buf, segs, first, F6)
    assert_same(g, o)
    assert (o["status"] == STATUS["OK"]).sum() > 100 and (o["l4_sum"][o["status"] == 0] == 0xffff).all()


def test_dual_stack_chain_edge_cases(torch):
    f = _ip6_udp_with_ext()
    L = len(f)
    l4 = int(oracle.parse_one(f, F6)["l4_off"])
    cases = [[L], [14, L - 14], [53, L - 53], [54, L - 54], [55, L - 55], [60, L - 60],
             [62, L - 62], [63, L - 63], [70, L - 70], [l4, L - l4], [l4 + 4, L - l4 - 4],
             [l4, 0, 3, L - l4 - 3], [14, 40, 8, 24, L - 86], [20, 34, 8, 24, L - 86],
             [54, 0, 8, 0, L - 62], [0, L], [L, 0, 0]]
    buf, segs, first = _chains_of([f] * len(cases), cases)
    assert_same(gpu_chain_records(buf, segs, first, F6), oracle.parse_chains(buf, segs, first, F6))
