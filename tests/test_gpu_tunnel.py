"""GPU parity of rpkt_gpu_parse_tunnel_batch (outer record, rpkt_tun_t, inner record)
against oracle/rpkt_oracle_tunnel.c on the same buffers, bit-exact: the reference's
tunnel captures at every 16-B phase, config 13 (1M x 1500 B VXLAN / GTP-U / GRE mix) at
full size, config 14 (tunnel fuzz) over seeds and flags, and tests/tunnel_frames.py's
IPv6 / QinQ outers and long GTP-U extension chains.  Also the ICMP / GRE sums of the
plain parse (rpkt_gpu_parse_batch, _compact, rings, chains) on the captures."""
import os

import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, gen
from rpkt_amd.records import (F_IPV6, REC_DTYPE, STATUS, TUN_DTYPE, TUN_STATUS, as_records,
                              as_tunnels)

from test_gpu_parity import host_batch, oracle_records, gpu_records, assert_same
import tunnel_frames as tf

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
PKTS = os.path.join(HERE, "golden", "packets")
F6 = 3 | F_IPV6
TUNNEL_CAPS = ("Vxlan1.dat", "Vxlan2.dat", "gtp-u-1ext.dat", "gtp-u-2ext.dat",
               "gtp_nr_container.dat", "gtp_pdu_session_container.dat", "gtp-c1.dat",
               "GREv0_1.dat", "GREv0_2.dat", "GREv0_3.dat", "GREv0_4.dat", "GREv1_1.dat",
               "GREv1_2.dat", "GREv1_3.dat")


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def check_tunnel(hb, flags):
    db = engine.DeviceBatch.from_host(hb)
    go, gt, gi = engine.parse_tunnel_batch(db, flags)
    go = as_records(go.cpu().numpy())
    gt = as_tunnels(gt.cpu().numpy())
    gi = as_records(gi.cpu().numpy())
    oo, ot, oi = oracle.tunnel_batch(hb.frames, hb.n, flags, offsets=hb.offsets, stride=hb.stride,
                                     frame_len=hb.frame_len)
    assert_same(go, oo)
    if gt.tobytes() != ot.tobytes():
        bad = np.nonzero(gt.view(np.uint8).reshape(-1, 16) != ot.view(np.uint8).reshape(-1, 16))[0]
        k = int(bad[0])
        raise AssertionError("%d tunnel records differ; first #%d gpu=%s oracle=%s" % (
            len(np.unique(bad)), k, gt[k], ot[k]))
    assert_same(gi, oi)
    return oo, ot, oi


@pytest.mark.parametrize("lead", list(range(16)))
def test_tunnel_captures_every_alignment(torch, lead):
    frames = [oracle.load_dat(os.path.join(PKTS, n)) for n in TUNNEL_CAPS]
    hb = host_batch(frames, lead)
    for flags in (0, 1, 2, 3, F6):
        o, t, i = check_tunnel(hb, flags)
    k = 1 if lead else 0
    assert int(t[k]["status"]) == TUN_STATUS["OK"] and int(i[k]["ip_sum"]) == 0xffff


def test_tunnel_config13_full_size(torch):
    """Config 13 at BASELINE scale (1,048,576 x 1500 B): every byte of the three record
    arrays equals the oracle's; every tunnel decodes; 98-99 % of the inner L4 sums and
    the GRE checksums are valid (1 % injected faults per level)."""
    hb = gen.make_batch(13)
    o, t, i = check_tunnel(hb, gen.FLAGS[13])
    assert (t["status"] == TUN_STATUS["OK"]).all()
    ok = i["status"] == STATUS["OK"]
    assert ok.mean() > 0.97 and (i["l4_sum"][ok] == 0xffff).mean() > 0.98


@pytest.mark.parametrize("seed", [14, 1401, 1402, 1403])
def test_tunnel_fuzz(torch, seed):
    hb = gen.make_batch(14, 1 << 15, seed=seed)
    for flags in (3, F6, 1):
        o, t, i = check_tunnel(hb, flags)
    assert len(np.unique(t["status"])) >= 5


def test_tunnel_fuzz_strided_and_ragged(torch):
    """A strided view of config 13 (frame_len < stride) and ragged batch sizes."""
    hb = gen.make_batch(13, 4096 + 37)
    check_tunnel(gen.HostBatch(13, hb.n, hb.seed, hb.frames, None, 1500, 1400), F6)
    for n in (1, 63, 64, 65, 130):
        h = gen.make_batch(14, n, seed=n)
        check_tunnel(h, F6)


@pytest.mark.parametrize("lead", [0, 1, 7, 15])
def test_tunnel_odd_frames(torch, lead):
    """IPv6 and QinQ outers, GTP-U chains past the 128-B window, GRE over IPv6, and cuts /
    byte flips of them (tests/tunnel_frames.py)."""
    hb = host_batch(tf.odd_frames(seed=lead, n=256), lead)
    for flags in (3, F6):
        check_tunnel(hb, flags)


@pytest.mark.parametrize("lead", [0, 3, 9])
def test_tunnel_jumbo_frames(torch, lead):
    """Tunnelled jumbo frames to 60 KB of inner payload (VXLAN over IPv4 / IPv6, GRE with
    its checksum, GTP-U with extension headers) and cuts of them: the long streams, the
    tail lines of joint tiles and the outer sums that reuse the inner stream."""
    hb = host_batch(tf.jumbo_frames(seed=lead, n=48 + lead), lead)
    for flags in (3, F6, 1):
        check_tunnel(hb, flags)


def test_tunnel_empty_batch_and_validation(torch):
    hb = host_batch([b""])
    db = engine.DeviceBatch.from_host(hb)
    db.n = 0
    engine.parse_tunnel_batch(db, 3)                           # n == 0: nothing launched
    db.n = 1
    with pytest.raises(engine.RpktError):
        engine.parse_tunnel_batch(db, 4)                       # FLOW_EV needs n_buckets
    with pytest.raises(engine.RpktError):
        engine.parse_tunnel_batch(db, 3 | 16)                  # an unknown flag


@pytest.mark.parametrize("cfg,n,nb", [(13, None, 8192), (14, 1 << 15, 977), (14, 4099, 1)])
def test_tunnel_flow_events(torch, cfg, n, nb):
    """RPKT_F_FLOW_EV on the tunnel parse: every event equals the oracle's (the inner
    record's event when the tunnel decoded, else the outer's), the records are those of
    the call without events, and rpkt_gpu_flow_count over them gives the oracle's
    per-inner-flow counters."""
    hb = gen.make_batch(cfg, n)
    fl = gen.FLAGS.get(cfg, 3)
    db = engine.DeviceBatch.from_host(hb)
    go, gt, gi, ev = engine.parse_tunnel_batch(db, fl | 4, n_buckets=nb)
    oo, ot, oi = check_tunnel(hb, fl)
    assert as_records(go.cpu().numpy()).tobytes() == oo.tobytes()
    assert as_records(gi.cpu().numpy()).tobytes() == oi.tobytes()
    want = oracle.tunnel_flow_events(oo, ot, oi, nb)
    got = ev.cpu().numpy().view(np.uint64)
    assert np.array_equal(got, want), int(np.nonzero(got != want)[0][0])
    c = engine.flow_count(ev, hb.n, nb).cpu().numpy().view(np.uint64)
    assert np.array_equal(c, oracle.flow_count(want, nb))
    if cfg == 13:                                 # the inner flows are counted, not the outer
        inner_ok = (ot["status"] == TUN_STATUS["OK"]) & (oi["status"] == STATUS["OK"])
        assert inner_ok.mean() > 0.97 and c.reshape(-1, 4)[:nb, 0].sum() >= inner_ok.sum()


@pytest.mark.parametrize("lead", list(range(16)))
def test_icmp_gre_sums_in_plain_parse(torch, lead):
    """rpkt_gpu_parse_batch's l4_sum of ICMP and GRE-with-checksum frames (status
    L4_OTHER) and ICMP_EMPTY equal the oracle's, at every phase; the compact entry carries
    the same sum."""
    names = sorted(f for f in os.listdir(PKTS) if f.endswith(".dat"))
    frames = [oracle.load_dat(os.path.join(PKTS, f)) for f in names]
    e = bytearray(oracle.load_dat(os.path.join(PKTS, "IPv4Option6.dat")))
    ihl = (e[14] & 0xf) * 4
    e[16:18] = ihl.to_bytes(2, "big")
    frames.append(bytes(e[:14 + ihl]))                        # ICMP_EMPTY
    hb = host_batch(frames, lead)
    for flags in (1, 3, F6):
        g = gpu_records(hb, flags)
        o = oracle_records(hb, flags)
        assert_same(g, o)
    assert (o["status"] == STATUS["ICMP_EMPTY"]).sum() == 1
    assert ((o["status"] == STATUS["L4_OTHER"]) & (o["l4_sum"] == 0xffff)).sum() >= 6
    db = engine.DeviceBatch.from_host(hb)
    c = engine.parse_batch_compact(db, 3).cpu().numpy().view(np.uint8).reshape(-1, 16)
    assert np.array_equal(c[:, 14:16].copy().view("<u2").reshape(-1), oracle_records(hb, 3)["l4_sum"])


def test_tunnel_views_over_device_records(torch):
    """rpkt_amd.tunviews over the GPU's records of the tunnel captures reads as the
    reference's tests do (vlan_mpls_tests.rs:224-251, gtpv1_test.rs:199-231,
    gre_test.rs:20-44)."""
    from rpkt_amd.tunviews import ExtPduNumber, Gre, Gtpv1, TunnelPacket, Vxlan
    from rpkt_amd.views import EtherFrame, IpProtocol, Ipv4, Udp
    names = ("Vxlan1.dat", "gtp-u-1ext.dat", "GREv0_1.dat")
    frames = [oracle.load_dat(os.path.join(PKTS, n)) for n in names]
    hb = host_batch(frames)
    db = engine.DeviceBatch.from_host(hb)
    go, gt, gi = (x.cpu().numpy() for x in engine.parse_tunnel_batch(db, F6))
    go, gi, gt = as_records(go), as_records(gi), as_tunnels(gt)
    pk = [TunnelPacket(go[k], gt[k], gi[k], frames[k]) for k in range(3)]
    ip = [Ipv4.parse(EtherFrame.parse(p).unwrap().payload()).unwrap() for p in pk]
    vx = Vxlan.parse(Udp.parse(ip[0].payload()).unwrap().payload()).unwrap()
    assert vx.vni() == 3000001 and vx.group_id() == 100 and vx.reserved_4() == 0
    assert Ipv4.parse(EtherFrame.parse(vx.payload()).unwrap().payload()).unwrap().verify_checksum()
    gtp = Gtpv1.parse(Udp.parse(ip[1].payload()).unwrap().payload()).unwrap()
    assert gtp.teid() == 1 and gtp.sequence() == 10461 and gtp.packet_len() == 100
    assert Ipv4.parse(gtp.t_pdu()).unwrap().protocol() == IpProtocol.ICMP
    ext = ExtPduNumber.parse(gtp.payload()).unwrap()               # gtpv1_test.rs:224-231
    assert ext.pdcp_number() == 2308 and ext.next_extention_header() == 0
    assert Ipv4.parse(ext.payload()).unwrap().protocol() == IpProtocol.ICMP
    gre = Gre.parse(ip[2].payload()).unwrap()
    assert gre.checksum() == 30719 and gre.offset() == 0 and gre.verify_checksum()
    inner = Ipv4.parse(gre.payload()).unwrap()
    assert inner.ttl() == 64 and inner.ident() == 0x4c0f
