"""HIP-graph capture of the engine's calls (rpkt_amd.graphs, examples/rx_graph.cpp).

The engine's entry points are kernel launches only, so a receive loop's pass over a ring
of small batches can be captured once and replayed.  A replayed pass must give the
records and counters the same calls give eagerly (and the oracle gives), and must read
its buffers at replay time: refilled slots are parsed anew."""
import os

import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, gen, graphs
from rpkt_amd.records import as_records

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def _ring_buffers(torch, ring):
    recs = [engine.alloc_records(db.n) for db in ring]
    ev_all = torch.empty(sum(db.n for db in ring), dtype=torch.int64, device="cuda")
    return recs, ev_all


@pytest.mark.parametrize("n_streams", [0, 3])
def test_captured_rx_loop_matches_eager_and_oracle(torch, n_streams):
    """A ring of strided 64-B (config 2) and packed IMIX (config 4) slots: per slot the
    parse with flow events, then one flow count of the pass, captured as one graph (the
    parses on one stream, or forked over three) and replayed."""
    nb, passes = 1024, 4
    hbs = [gen.make_batch(2 if k % 2 == 0 else 4, 3000 + 517 * k, seed=900 + k) for k in range(6)]
    ring = [engine.DeviceBatch.from_host(h) for h in hbs]
    n_ev = sum(h.n for h in hbs)
    flags = 3
    streams = [torch.cuda.Stream() for _ in range(n_streams)]

    # eager: the same calls, `passes` times
    recs_e, ev_e = _ring_buffers(torch, ring)
    cnt_e = torch.zeros((nb + 1) * 4, dtype=torch.int64, device="cuda")
    ws_e = engine.flow_workspace(n_ev, nb)
    for _ in range(passes):
        graphs.rx_pass(ring, recs_e, ev_e, cnt_e, ws_e, flags, nb, streams)

    # graph: the warm pass runs eagerly, the captured pass is replayed passes - 1 times
    recs_g, ev_g = _ring_buffers(torch, ring)
    cnt_g = torch.zeros((nb + 1) * 4, dtype=torch.int64, device="cuda")
    ws_g = engine.flow_workspace(n_ev, nb)
    loop = graphs.CapturedLoop(lambda: graphs.rx_pass(ring, recs_g, ev_g, cnt_g, ws_g, flags, nb,
                                                      streams))
    for _ in range(passes - 1):
        loop.replay()
    torch.cuda.synchronize()

    assert torch.equal(cnt_e, cnt_g)
    assert torch.equal(ev_e, ev_g)
    off = 0
    for k, hb in enumerate(hbs):
        assert torch.equal(recs_e[k], recs_g[k]), "slot %d records" % k
        o, ev = oracle.parse_batch(hb.frames, hb.n, flags=flags | engine.F_FLOW_EV,
                                   offsets=hb.offsets, stride=hb.stride, frame_len=hb.frame_len,
                                   n_buckets=nb, threads=THREADS, flow_ev=True)
        assert as_records(recs_g[k].cpu().numpy()).tobytes() == o.tobytes(), "slot %d vs oracle" % k
        assert np.array_equal(ev_g[off:off + hb.n].cpu().numpy().view(np.uint64), ev)
        off += hb.n
    # every pass counted every frame of the ring once; the sums equal the oracle's counters
    # of the ring's events, `passes` times over
    want = oracle.flow_count(ev_g.cpu().numpy().view(np.uint64), nb) * np.uint64(passes)
    got = cnt_g.cpu().numpy().view(np.uint64)
    assert np.array_equal(got, want)
    assert int(got.reshape(-1, 4)[:, 0].sum()) == passes * n_ev


def test_captured_ring_call(torch):
    """The pass with its slots parsed by one rpkt_gpu_parse_ring call, captured and
    replayed, counts what the per-slot pass counts."""
    nb, passes = 1024, 3
    hbs = [gen.make_batch(2 if k % 2 == 0 else 4, 2000 + 301 * k, seed=700 + k) for k in range(5)]
    ring = [engine.DeviceBatch.from_host(h) for h in hbs]
    n_ev = sum(h.n for h in hbs)
    recs, ev_all = _ring_buffers(torch, ring)
    offs = np.cumsum([0] + [h.n for h in hbs])
    slots = engine.ring_slots(ring, recs, [ev_all[offs[k]:offs[k + 1]] for k in range(len(hbs))])
    cnt = torch.zeros((nb + 1) * 4, dtype=torch.int64, device="cuda")
    ws = engine.flow_workspace(n_ev, nb)
    loop = graphs.CapturedLoop(lambda: graphs.rx_pass_ring(slots, ev_all, n_ev, cnt, ws, 3, nb))
    for _ in range(passes - 1):
        loop.replay()
    recs_e, ev_e = _ring_buffers(torch, ring)
    cnt_e = torch.zeros((nb + 1) * 4, dtype=torch.int64, device="cuda")
    ws_e = engine.flow_workspace(n_ev, nb)
    for _ in range(passes):
        graphs.rx_pass(ring, recs_e, ev_e, cnt_e, ws_e, 3, nb)
    torch.cuda.synchronize()
    assert torch.equal(cnt, cnt_e)
    assert torch.equal(ev_all, ev_e)
    for a, b in zip(recs, recs_e):
        assert torch.equal(a, b)


def test_captured_tunnel_ring(torch):
    """A VTEP / UPF receive pass captured as one graph: a ring of tunnelled bursts
    (configs 13 and 14) parsed by one rpkt_gpu_parse_tunnel_ring call with flow events,
    then one flow count of the inner flows; replayed, it gives the oracle's records and
    `passes` times the oracle's counters."""
    nb, passes = 977, 3
    hbs = [gen.make_batch(13 if k % 2 == 0 else 14, 700 + 433 * k, seed=1800 + k) for k in range(5)]
    ring = [engine.DeviceBatch.from_host(h) for h in hbs]
    n_ev = sum(h.n for h in hbs)
    offs = np.cumsum([0] + [h.n for h in hbs])
    outs = [[torch.empty(h.n * b, dtype=torch.uint8, device="cuda") for b in (80, 16, 80)]
            for h in hbs]
    ev_all = torch.empty(n_ev, dtype=torch.int64, device="cuda")
    slots = engine.tunnel_ring_slots(ring, *[[x[j] for x in outs] for j in range(3)],
                                     [ev_all[offs[k]:offs[k + 1]] for k in range(len(hbs))])
    cnt = torch.zeros((nb + 1) * 4, dtype=torch.int64, device="cuda")
    ws = engine.flow_workspace(n_ev, nb)
    flags = 3 | engine.F_FLOW_EV

    def rx_pass():
        engine.parse_tunnel_ring(slots, flags, nb)
        engine.flow_count(ev_all, n_ev, nb, counters=cnt, workspace=ws)

    loop = graphs.CapturedLoop(rx_pass)
    for _ in range(passes - 1):
        loop.replay()
    torch.cuda.synchronize()
    want_ev = []
    for k, hb in enumerate(hbs):
        oo, ot, oi = oracle.tunnel_batch(hb.frames, hb.n, 3, offsets=hb.offsets, stride=hb.stride,
                                         frame_len=hb.frame_len)
        for got, w in zip(outs[k], (oo, ot, oi)):
            assert got.cpu().numpy().tobytes() == w.tobytes(), "slot %d" % k
        want_ev.append(oracle.tunnel_flow_events(oo, ot, oi, nb))
    want_ev = np.concatenate(want_ev)
    assert np.array_equal(ev_all.cpu().numpy().view(np.uint64), want_ev)
    want = oracle.flow_count(want_ev, nb) * np.uint64(passes)
    assert np.array_equal(cnt.cpu().numpy().view(np.uint64), want)


def test_replay_reads_refilled_slots(torch):
    """The graph bakes in buffer addresses, not contents: a slot refilled between replays
    (as a NIC refills its ring) is parsed from its new frames."""
    n = 5000
    a, b = gen.make_batch(2, n, seed=31), gen.make_batch(2, n, seed=32)
    assert not np.array_equal(a.frames, b.frames)
    db = engine.DeviceBatch.from_host(a)
    recs = engine.alloc_records(n)
    loop = graphs.CapturedLoop(lambda: engine.parse_batch(db, 3, recs=recs))
    loop.replay()
    torch.cuda.synchronize()
    oa = oracle.parse_batch(a.frames, n, flags=3, stride=a.stride, threads=THREADS)
    assert as_records(recs.cpu().numpy()).tobytes() == oa.tobytes()
    db.frames.copy_(torch.from_numpy(b.frames))           # refill the slot in place
    loop.replay()
    torch.cuda.synchronize()
    ob = oracle.parse_batch(b.frames, n, flags=3, stride=b.stride, threads=THREADS)
    assert as_records(recs.cpu().numpy()).tobytes() == ob.tobytes()


def test_captured_walk_and_getters(torch):
    """The protocol-layer walk and the field getters in one graph."""
    import bench
    from rpkt_amd import fields
    from rpkt_amd.records import FIELD_REQ_DTYPE
    hb = gen.make_mix(n=20000, seed=77)
    db = engine.DeviceBatch.from_host(hb)
    reqs = np.ascontiguousarray(fields.requests(bench.FIELD_LEG), dtype=FIELD_REQ_DTYPE)
    lay = torch.empty(hb.n * 64, dtype=torch.uint8, device="cuda")
    vals = torch.empty((hb.n, reqs.size), dtype=torch.int64, device="cuda")
    pres = torch.empty(hb.n, dtype=torch.int32, device="cuda")

    def walk():
        engine.layers_batch(db, out=lay)
        engine.fields_batch(db, lay, reqs, values=vals, present=pres)

    loop = graphs.CapturedLoop(walk, warm=False)
    lay.zero_()
    vals.zero_()
    loop.replay()
    torch.cuda.synchronize()
    ol = oracle.layers_batch(hb.frames, hb.n, offsets=hb.offsets)
    assert lay.cpu().numpy().tobytes() == ol.tobytes()
    ov, op = oracle.fields_batch(hb.frames, hb.n, ol, reqs, offsets=hb.offsets)
    assert np.array_equal(vals.cpu().numpy().view(np.uint64), ov)
    assert np.array_equal(pres.cpu().numpy().view(np.uint32), op)


def test_cpp_host_captures_the_abi(torch):
    """examples/rx_graph: a C++ host captures a receive loop's C ABI calls with
    hipStreamBeginCapture; the replayed graph and the eager calls agree byte for byte."""
    import subprocess
    from rpkt_amd.build import build_example
    exe = [e for e in build_example() if e.endswith("rx_graph")][0]
    out = subprocess.run([exe, "8192", "8", "5", "3"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "counters and records identical in every mode: yes" in out.stdout
    assert out.stdout.count("Mpps") == 6
