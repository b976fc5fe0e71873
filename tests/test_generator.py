"""Synthetic generator: deterministic, covers every parse status, and its stamped
checksums verify under the oracle (CPU only)."""
import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import gen
from rpkt_amd.records import STATUS


def test_deterministic_and_thread_independent():
    a = gen.make_batch(4, 5000, seed=11, threads=1)
    b = gen.make_batch(4, 5000, seed=11, threads=8)
    assert np.array_equal(a.frames, b.frames) and np.array_equal(a.offsets, b.offsets)
    c = gen.make_batch(4, 5000, seed=12)
    assert not np.array_equal(a.frames[:4096], c.frames[:4096])


@pytest.mark.parametrize("cfg,bad", [(2, 0.01), (3, 0.01), (4, 0.01), (5, 0.01)])
def test_checksums_verify_except_injected(cfg, bad):
    b = gen.make_batch(cfg, 20000)
    r = oracle.parse_batch(b.frames, b.n, flags=3, offsets=b.offsets, stride=b.stride)
    ip_ok = r["status"] != STATUS["IP_TOT_GT_LEN"]
    ip_ok &= r["status"] != STATUS["IP_IHL_GT_LEN"]
    frac_bad = 1 - (r["ip_sum"][ip_ok] == 0xffff).mean()
    assert abs(frac_bad - bad) < 0.005, frac_bad


def test_config1_matches_rpkt_build_values():
    b = gen.make_batch(1)
    r = oracle.parse_batch(b.frames, b.n, flags=3, stride=b.stride)
    assert (r["status"] == 0).all()
    assert (r["ip_src"] == (192 << 24 | 168 << 16 | 29 << 8 | 58)).all()
    assert (r["ip_dst"] == (192 << 24 | 168 << 16 | 29 << 8 | 160)).all()
    assert (r["ip_ident"] == 0x5c65).all() and (r["ip_ttl"] == 128).all()
    assert (r["src_port"] == 60376).all() and (r["dst_port"] == 161).all()
    assert (r["ip_sum"] == 0xffff).all() and (r["l4_sum"] == 0xffff).all()


def test_fuzz_hits_every_status():
    """Config 6 reaches every IPv4-path status; the dual-stack fuzz (config 12, parsed with
    RPKT_F_IPV6) every IPv6 status as well."""
    from rpkt_amd.records import F_IPV6
    v4 = {v for k, v in STATUS.items() if not k.startswith("IP6_") and k != "NO_INNER"}
    b = gen.make_batch(6, 1 << 16)
    r = oracle.parse_batch(b.frames, b.n, flags=3, offsets=b.offsets)
    seen = set(int(s) for s in np.unique(r["status"]))
    assert seen == v4, sorted(v4 - seen)
    b = gen.make_batch(12)
    r = oracle.parse_batch(b.frames, b.n, flags=3 | F_IPV6, offsets=b.offsets)
    seen = set(int(s) for s in np.unique(r["status"]))
    want = set(STATUS.values()) - {STATUS["NOT_IPV4"], STATUS["NO_INNER"]}
    assert want <= seen, sorted(want - seen)


def test_config5_shapes():
    b = gen.make_batch(5, 20000)
    r = oracle.parse_batch(b.frames, b.n, flags=3, offsets=b.offsets)
    lens = b.lens()
    assert lens.min() >= 64 and lens.max() <= 1518
    ok = r["status"] == 0
    assert set(np.unique(r["n_vlan"][ok])) == {1, 2}
    ihl = (r["ip_vhl"][ok] & 0xf)
    assert ihl.min() == 5 and ihl.max() == 15
    doff = r["l4_word6"][ok] >> 12
    assert doff.min() == 5 and doff.max() == 15


def test_shard_generation_equals_slice_of_full_batch():
    full = gen.make_batch(4, 3000, seed=8)
    lo, hi = 1234, 2345
    sh = gen.make_batch(4, hi - lo, seed=8, first=lo)
    a = full.frames[full.offsets[lo]:full.offsets[hi]]
    assert np.array_equal(a, sh.frames)
    assert np.array_equal(np.diff(full.offsets[lo:hi + 1]), np.diff(sh.offsets))
