"""The option-iterator oracle (oracle/rpkt_oracle_opts.c) against the option
sequences and getter values the reference's own tests assert on its captures
(rpkt/tests/ipv4_test.rs, rpkt/tests/tcp_test.rs)."""
import os

import numpy as np

from oracle import oracle
from rpkt_amd import gen
from rpkt_amd.records import IP_KINDS, OPT_STOP, TCP_KINDS, trace_kinds

HERE = os.path.dirname(os.path.abspath(__file__))
PKTS = os.path.join(HERE, "golden", "packets")


def opts_of(name):
    f = oracle.load_dat(os.path.join(PKTS, name))
    r = oracle.parse_one(f, 3)
    buf = np.frombuffer(f, np.uint8)
    return oracle.options_batch(buf, 1, np.array([r]), offsets=np.array([0, len(f)], np.uint32))[0]


def test_ipv4_option_kats():
    o = opts_of("IPv4Option1.dat")                        # ipv4_test.rs:38-56
    assert trace_kinds(o["ip_trace"], o["ip_count"], IP_KINDS)[:2] == ["CommercialSecurity", "Eol"]
    assert o["ip_cs_doi"] == 2
    o = opts_of("IPv4Option2.dat")                        # ipv4_test.rs:187-196
    assert trace_kinds(o["ip_trace"], o["ip_count"], IP_KINDS)[0] == "Timestamp"
    assert (o["ip_ts_len"], o["ip_ts_pointer"], o["ip_ts_oflw_flg"]) == (40, 9, 0)
    o = opts_of("IPv4Option3.dat")                        # ipv4_test.rs:333-339
    assert trace_kinds(o["ip_trace"], o["ip_count"], IP_KINDS)[0] == "RouteAlert"
    assert o["ip_route_alert"] == 0
    o = opts_of("IPv4Option4.dat")                        # ipv4_test.rs:456-468
    assert trace_kinds(o["ip_trace"], o["ip_count"], IP_KINDS)[:2] == ["RecordRoute", "Eol"]
    assert (o["ip_rr_len"], o["ip_rr_pointer"]) == (39, 16)
    o = opts_of("IPv4Option6.dat")                        # ipv4_test.rs:647-660
    assert trace_kinds(o["ip_trace"], o["ip_count"], IP_KINDS)[:2] == ["Nop", "StrictSourceRoute"]
    assert (o["ip_sr_pointer"], o["ip_sr_dest"]) == (4, 0)
    o = opts_of("IPv4Option7.dat")                        # ipv4_test.rs:758-775
    assert trace_kinds(o["ip_trace"], o["ip_count"], IP_KINDS)[:2] == ["Nop", "LooseSourceRoute"]
    assert (o["ip_sr_pointer"], o["ip_sr_dest"]) == (4, 0)


def test_tcp_option_kats():
    o = opts_of("TcpPacketWithOptions.dat")               # tcp_test.rs:45-62
    assert trace_kinds(o["tcp_trace"], o["tcp_count"], TCP_KINDS)[:3] == ["Nop", "Nop", "Timestamp"]
    assert (o["tcp_ts"], o["tcp_ts_echo"]) == (195102, 3555729271)
    o = opts_of("TcpPacketWithOptions2.dat")              # tcp_test.rs:211-239
    assert trace_kinds(o["tcp_trace"], o["tcp_count"], TCP_KINDS)[:5] == \
        ["Nop", "Nop", "Timestamp", "Nop", "WindowScale"]
    assert (o["tcp_ts"], o["tcp_ts_echo"], o["tcp_wscale"]) == (3555735960, 196757, 2)
    o = opts_of("TcpPacketWithMssSackperm.dat")           # tcp_test.rs:404-426
    assert trace_kinds(o["tcp_trace"], o["tcp_count"], TCP_KINDS)[:4] == \
        ["Mss", "Nop", "Nop", "SackPermitted"]
    assert o["tcp_mss"] == 1460
    f = oracle.load_dat(os.path.join(PKTS, "TcpPacketWithSack.dat"))   # tcp_test.rs:579-603
    r = oracle.parse_one(f, 3)
    o = opts_of("TcpPacketWithSack.dat")
    assert trace_kinds(o["tcp_trace"], o["tcp_count"], TCP_KINDS) == ["Nop", "Nop", "Sack"]
    assert o["tcp_stop"] == OPT_STOP["END"]               # next().is_none() after the Sack
    assert (int(o["tcp_sack_left"]) - int(r["tcp_ack"]) + 1) % (1 << 32) == 13141
    assert (int(o["tcp_sack_right"]) - int(r["tcp_ack"]) + 1) % (1 << 32) == 14601


def test_frames_without_options():
    hb = gen.make_batch(2, n=100)
    recs = oracle.parse_batch(hb.frames, hb.n, 3, stride=hb.stride)
    o = oracle.options_batch(hb.frames, hb.n, recs, stride=hb.stride)
    ok = recs["ip_sum"] == 0xFFFF
    assert (o["ip_stop"] == OPT_STOP["END"]).all() and (o["ip_count"] == 0).all()
    assert (o["tcp_stop"] == OPT_STOP["NONE"]).all()                # UDP frames
    del ok


def test_config5_options_walk_fully():
    """Config 5 writes IPv4 options from {NOP, RecordRoute, EOL} and TCP options
    from {NOP, MSS, WS, SACK-permitted, TS}: every walk of a parsed frame ends
    cleanly at the slice end."""
    hb = gen.make_batch(5, n=5000)
    recs = oracle.parse_batch(hb.frames, hb.n, 3, offsets=hb.offsets)
    o = oracle.options_batch(hb.frames, hb.n, recs, offsets=hb.offsets)
    ok = recs["status"] == 0
    assert (o["ip_stop"][ok] == OPT_STOP["END"]).all()
    assert (o["tcp_stop"][ok] == OPT_STOP["END"]).all()
    assert (o["ip_end"][ok] == recs["l4_off"][ok] - recs["l3_off"][ok] - 20).all()
    assert (o["tcp_kinds"][ok] & 0x4c).any() and (o["ip_kinds"][ok] & 8).any()
