"""The chain oracle (oracle/rpkt_oracle_chain.c): its Pbuf walker replayed against the
assertions of rpkt-dpdk/tests/pbuf.rs, and its parse over mbuf chains checked
against the single-buffer oracle and an independent chunk model."""
import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import gen
from rpkt_amd.records import STATUS

ADV, TRIM, NEW = "advance", "trim_off", "new"


def _state(seg_lens, ops):
    return oracle.pbuf_script(seg_lens, [(NEW, 0)] + ops)[1:]


def test_pbuf_advance_across_segments():
    """rpkt-dpdk/tests/pbuf.rs:44-115 (three 1000-B segments)."""
    segs = [1000, 1000, 1000]
    steps = [500, 499, 1, 500, 499, 1, 500, 499, 1]
    want = [(500, 2500), (1, 2001), (1000, 2000), (500, 1500), (1, 1001), (1000, 1000),
            (500, 500), (1, 1), (0, 0)]
    got = _state(segs, [(ADV, s) for s in steps])
    assert [(g["chunk_len"], g["remaining"]) for g in got] == want
    for adv, chunk, rem in ((1500, 500, 1500), (2500, 500, 500), (3000, 0, 0)):
        g = _state(segs, [(ADV, adv)])[0]
        assert (g["chunk_len"], g["remaining"]) == (chunk, rem)
    assert _state(segs, [(ADV, 3000)])[0]["cursor"] == 3000


@pytest.mark.parametrize("seglen,seg_num,step", [(1000, 5, 1), (1000, 5, 3), (1000, 5, 1000),
                                                 (1000, 6, 1200), (1000, 10, 2500)])
def test_pbuf_advance_helper(seglen, seg_num, step):
    """rpkt-dpdk/tests/pbuf.rs:118-177 (pbuf_advance_helper and its cases)."""
    pkt_len = seglen * seg_num
    n = pkt_len // step
    got = _state([seglen] * seg_num, [(ADV, step)] * n)
    pos = 0
    for g in got:
        pos += step
        assert g["cursor"] == pos
        if pos < pkt_len:
            assert g["headroom"] == pos % seglen
            assert g["chunk_len"] == seglen - pos % seglen
        else:
            assert g["headroom"] == seglen and g["chunk_len"] == 0


def test_pbuf_trim_off():
    """rpkt-dpdk/tests/pbuf.rs:290-359 (trim_off_test)."""
    segs = [1000, 1000, 1000]
    for adv, trim, rem, chunk, head, nsegs in ((1500, 1000, 500, 500, 500, 2),
                                               (1500, 1499, 1, 1, 500, 2),
                                               (1500, 1500, 0, 0, 500, 2),
                                               (2000, 1000, 0, 0, 1000, 2)):
        g = _state(segs, [(ADV, adv), (TRIM, trim)])[1]
        assert (g["remaining"], g["chunk_len"], g["headroom"], g["num_segs"]) == \
            (rem, chunk, head, nsegs), (adv, trim)


def test_pbuf_trim_off_1():
    """rpkt-dpdk/tests/pbuf.rs:361-440 (trim_off_test_1)."""
    segs = [1000, 1000, 1000]
    for cnt in list(range(1, 1000, 37)) + [999]:
        g = _state(segs, [(ADV, 1000), (TRIM, cnt)])[1]
        assert (g["pkt_len"], g["remaining"], g["num_segs"], g["chunk_len"]) == \
            (3000 - cnt, 2000 - cnt, 3, 1000)
    g = _state(segs, [(ADV, 1000), (TRIM, 1000)])[1]
    assert (g["pkt_len"], g["remaining"], g["num_segs"], g["chunk_len"]) == (2000, 1000, 2, 1000)
    for cnt in list(range(1001, 2000, 41)) + [1999]:
        g = _state(segs, [(ADV, 1000), (TRIM, cnt)])[1]
        assert (g["pkt_len"], g["remaining"], g["num_segs"], g["chunk_len"], g["headroom"]) == \
            (3000 - cnt, 2000 - cnt, 2, 2000 - cnt, 0)
    g = _state(segs, [(ADV, 1000), (TRIM, 2000)])[1]
    assert (g["pkt_len"], g["remaining"], g["num_segs"], g["chunk_len"], g["headroom"]) == \
        (1000, 0, 1, 0, 1000)


def test_pbuf_read_non_contiguous():
    """rpkt-dpdk/tests/pbuf.rs:7-41: walking chunk by chunk visits every byte once
    (2048-B mbuf segments)."""
    for total in (0, 1, 2047, 2048, 2049, 4096, 11235):
        segs = [2048] * (total // 2048) + ([total % 2048] if total % 2048 or total == 0 else [])
        ops, seen = [], 0
        st = _state(segs, [])
        g = oracle.pbuf_script(segs, [(NEW, 0)])[0]
        while g["remaining"]:
            ops.append((ADV, g["chunk_len"]))
            seen += g["chunk_len"]
            g = _state(segs, ops)[-1]
        assert seen == total and g["remaining"] == 0
        del st


# ---- parse over chains ------------------------------------------------------

TAGS = (0x8100, 0x88A8)


def _be16(b, i):
    return (b[i] << 8) | b[i + 1]


def chunk_model_status(frame, seg_lens):
    """Independent restatement: at logical cursor c the chunk is the rest of the
    segment holding c (empty segments skipped; segment 0 at c == 0), cut at the
    current packet end (IPv4/UDP trims)."""
    ends = np.cumsum(seg_lens).tolist()
    pkt = len(frame)

    def chunk(c, limit):
        if c == 0:
            return min(seg_lens[0] if seg_lens else 0, limit)
        for e in ends:
            if e > c:
                return min(e, limit) - c
        return 0

    if chunk(0, pkt) < 14:
        return STATUS["ETH_SHORT"]
    et, c, nv = _be16(frame, 12), 14, 0
    while et in TAGS and nv < 2:
        if chunk(c, pkt) < 4:
            return STATUS["VLAN_SHORT"]
        et, c, nv = _be16(frame, c + 2), c + 4, nv + 1
    if et != 0x0800:
        return STATUS["NOT_IPV4"]
    ck = chunk(c, pkt)
    if ck < 20:
        return STATUS["IP_SHORT"]
    ihl4, tot = (frame[c] & 15) * 4, _be16(frame, c + 2)
    if ihl4 < 20:
        return STATUS["IP_BAD_IHL"]
    if ihl4 > ck:
        return STATUS["IP_IHL_GT_LEN"]
    if tot < ihl4:
        return STATUS["IP_TOT_LT_IHL"]
    if tot > pkt - c:
        return STATUS["IP_TOT_GT_LEN"]
    limit, l4, proto = c + tot, c + ihl4, frame[c + 9]
    ck = chunk(l4, limit)
    if proto == 17:
        if ck < 8:
            return STATUS["UDP_SHORT"]
        ulen = _be16(frame, l4 + 4)
        return STATUS["UDP_BAD_LEN"] if ulen < 8 or ulen > limit - l4 else STATUS["OK"]
    if proto == 6:
        if ck < 20:
            return STATUS["TCP_SHORT"]
        hl = (frame[l4 + 12] >> 4) * 4
        return STATUS["TCP_BAD_DOFF"] if hl < 20 or hl > ck else STATUS["OK"]
    if proto == 1 and limit == l4:                    # an empty ICMP payload
        return STATUS["ICMP_EMPTY"]
    return STATUS["L4_OTHER"]


def _chains_of(frames, seg_lens_list):
    """Lay frames out as chains (segments packed back to back with odd gaps)."""
    buf, segs, first, pos = bytearray(), [], [0], 0
    for f, sl in zip(frames, seg_lens_list):
        off = 0
        for L in sl:
            buf += b"\x5a" * 3
            segs.append((len(buf), L))
            buf += f[off:off + L]
            off += L
        first.append(len(segs))
    return (np.frombuffer(bytes(buf) + b"\0" * 16, dtype=np.uint8), np.array(segs, np.uint32),
            np.array(first, np.uint32))


def test_single_segment_chains_equal_frames():
    hb = gen.make_batch(6, n=3000)
    frames = [hb.frames[hb.offsets[i]:hb.offsets[i + 1]].tobytes() for i in range(hb.n)]
    buf, segs, first = _chains_of(frames, [[len(f)] for f in frames])
    got = oracle.parse_chains(buf, segs, first, flags=3)
    want = oracle.parse_batch(hb.frames, hb.n, 3, offsets=hb.offsets)
    assert (got == want).all()


def test_mbuf_chains_equal_packed():
    """Config 7 (8000-B frames in 2048-B segments): the headers sit in segment 0, so
    every record, sums included, equals the contiguous parse (from_buf's cross-segment
    byte pairing equals from_slice over the concatenation)."""
    hc = gen.make_chains(7, n=400)
    hb = gen.make_batch(7, n=400, packed=True)
    got = oracle.parse_chains(hc.buf, hc.segs, hc.chain_first, flags=3)
    want = oracle.parse_batch(hb.frames, hb.n, 3, offsets=hb.offsets)
    assert (got == want).all()
    assert (got["status"] == 0).mean() > 0.95


def test_fuzz_chains_against_chunk_model():
    hc = gen.make_chains(8, n=4000)
    hb = gen.make_batch(8, n=4000, packed=True)
    got = oracle.parse_chains(hc.buf, hc.segs, hc.chain_first, flags=3)
    packed = oracle.parse_batch(hb.frames, hb.n, 3, offsets=hb.offsets)
    n_diff = 0
    for p in range(hc.n):
        a, b = int(hc.chain_first[p]), int(hc.chain_first[p + 1])
        frame = hb.frames[hb.offsets[p]:hb.offsets[p + 1]].tobytes()
        st = chunk_model_status(frame, [int(x) for x in hc.segs[a:b, 1]])
        assert got[p]["status"] == st, p
        if st == packed[p]["status"]:
            assert got[p] == packed[p], p
        else:
            n_diff += 1
            assert got[p]["frame_len"] == packed[p]["frame_len"]
            if st != STATUS["ETH_SHORT"]:
                for k in ("dst_addr", "src_addr", "ethertype"):
                    assert np.array_equal(got[p][k], packed[p][k])
    # the fuzz must actually produce chains whose verdict differs from the frame's
    assert n_diff > 20
    assert len(set(got["status"].tolist())) == 15


def test_chain_edge_cases():
    f = gen.make_batch(3, n=1).frames[:1500].tobytes()           # Ether/IPv4/TCP 1500 B
    cases = {
        (1500,): "OK", (14, 1486): "OK", (13, 1487): "ETH_SHORT", (0, 1500): "ETH_SHORT",
        (14, 0, 1486): "OK", (30, 1470): "IP_SHORT", (34, 1466): "OK", (40, 1460): "TCP_SHORT",
        (34, 10, 1456): "TCP_SHORT", (34, 20, 1446): "OK", (20, 14, 1466): "IP_SHORT",
        (14, 20, 1466): "OK", (1500, 0, 0): "OK", (100, 100, 100, 1200): "OK",
    }
    frames = [f] * len(cases)
    buf, segs, first = _chains_of(frames, [list(k) for k in cases])
    got = oracle.parse_chains(buf, segs, first, flags=3)
    want_full = oracle.parse_one(f, 3)
    for r, (k, v) in zip(got, cases.items()):
        assert r["status"] == STATUS[v], (k, r["status"])
        if v == "OK":
            assert r == want_full, k
    # an empty chain, and chain_first past n_segs / decreasing: empty chains
    recs = oracle.parse_chains(buf, segs, np.array([0, 0, 1, 99, 5], np.uint32), flags=3)
    assert recs["status"].tolist() == [STATUS["ETH_SHORT"], STATUS["OK"], STATUS["OK"],
                                       STATUS["ETH_SHORT"]]
    assert recs["frame_len"].tolist() == [0, 1500, int(segs[1:, 1].sum()), 0]


@pytest.mark.parametrize("threads", [2, 5])
def test_chain_oracle_threads_partition(threads):
    """The all-cores driver over chains (oracle_parse_chains_mt) equals the 1-thread walk,
    flow events included."""
    hc = gen.make_chains(8, 3001, seed=17)
    one, e1 = oracle.parse_chains(hc.buf, hc.segs, hc.chain_first, 3, n_buckets=512,
                                  flow_ev=True)
    mt, e2 = oracle.parse_chains(hc.buf, hc.segs, hc.chain_first, 3, n_buckets=512,
                                 flow_ev=True, threads=threads)
    assert one.tobytes() == mt.tobytes() and np.array_equal(e1, e2)
