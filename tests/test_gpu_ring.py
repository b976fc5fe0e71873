"""rpkt_gpu_parse_ring: a receive ring's slots parsed in one launch (per 32 slots) give
exactly the records and flow events of one rpkt_gpu_parse_batch per slot, and the
oracle's, for any mix of layouts, sizes and empty slots; a bad slot fails the call before
anything is launched."""
import ctypes
import os

import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, gen
from rpkt_amd.records import as_records

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def _ring(torch, hbs):
    dbs = [engine.DeviceBatch.from_host(h) for h in hbs]
    recs = [engine.alloc_records(max(h.n, 1)) for h in hbs]
    evs = [torch.zeros(max(h.n, 1), dtype=torch.int64, device="cuda") for h in hbs]
    return dbs, recs, evs


@pytest.mark.parametrize("flags", [1, 3])
def test_ring_equals_per_slot_parse_and_oracle(torch, flags):
    # 41 slots (two launches): strided 64 B and 1500 B, packed IMIX and VLAN/options,
    # tiles cut short (n not a multiple of 64), single frames and empty slots
    sizes = [1, 63, 64, 65, 2000, 0, 4097, 130, 7, 0] * 4 + [3333]
    cfgs = [2, 3, 4, 5, 6]
    hbs = [gen.make_batch(cfgs[k % 5], n, seed=50 + k) for k, n in enumerate(sizes)]
    nb = 512
    dbs, recs, evs = _ring(torch, hbs)
    slots = engine.ring_slots(dbs, recs, evs)
    engine.parse_ring(slots, flags | engine.F_FLOW_EV, nb)
    torch.cuda.synchronize()
    for k, (hb, db) in enumerate(zip(hbs, dbs)):
        if hb.n == 0:
            continue
        r1, e1 = engine.parse_batch(db, flags | engine.F_FLOW_EV, n_buckets=nb)
        assert torch.equal(recs[k][:hb.n * 80], r1), "slot %d vs parse_batch" % k
        assert torch.equal(evs[k][:hb.n], e1), "slot %d events vs parse_batch" % k
        o, ev = oracle.parse_batch(hb.frames, hb.n, flags=flags | engine.F_FLOW_EV,
                                   offsets=hb.offsets, stride=hb.stride, frame_len=hb.frame_len,
                                   n_buckets=nb, threads=THREADS, flow_ev=True)
        assert as_records(recs[k][:hb.n * 80].cpu().numpy()).tobytes() == o.tobytes(), k
        assert np.array_equal(evs[k][:hb.n].cpu().numpy().view(np.uint64), ev), k


def test_ring_without_flow_events(torch):
    hbs = [gen.make_batch(2, 1000 + k, seed=k) for k in range(5)]
    dbs = [engine.DeviceBatch.from_host(h) for h in hbs]
    recs = [engine.alloc_records(h.n) for h in hbs]
    engine.parse_ring(engine.ring_slots(dbs, recs), 1)
    torch.cuda.synchronize()
    for hb, r in zip(hbs, recs):
        o = oracle.parse_batch(hb.frames, hb.n, flags=1, stride=hb.stride, threads=THREADS)
        assert as_records(r.cpu().numpy()).tobytes() == o.tobytes()


def test_bad_slot_fails_before_any_launch(torch):
    hbs = [gen.make_batch(2, 500, seed=1), gen.make_batch(2, 500, seed=2)]
    dbs, recs, evs = _ring(torch, hbs)
    for r in recs:
        r.fill_(0xAB)
    slots = engine.ring_slots(dbs, recs, evs)
    slots[1].recs_dev = recs[1].data_ptr() + 8                  # misaligned records
    rc = engine.lib().rpkt_gpu_parse_ring(slots, 2, 3 | engine.F_FLOW_EV, 64,
                                          engine._stream_ptr(None))
    assert rc == -4                                             # RPKT_E_ALIGN
    slots[1].recs_dev = recs[1].data_ptr()
    slots[1].flow_ev_dev = None                                 # events asked, none given
    rc = engine.lib().rpkt_gpu_parse_ring(slots, 2, 3 | engine.F_FLOW_EV, 64,
                                          engine._stream_ptr(None))
    assert rc == -1                                             # RPKT_E_INVAL
    torch.cuda.synchronize()
    assert bool((recs[0] == 0xAB).all())                        # slot 0 was not parsed either
    assert engine.lib().rpkt_gpu_parse_ring(slots, 0, 3, 0, engine._stream_ptr(None)) == 0
    assert engine.lib().rpkt_gpu_parse_ring(None, 1, 3, 0, engine._stream_ptr(None)) == -1
    assert engine.lib().rpkt_gpu_parse_ring(slots, 2, 0x80, 0, engine._stream_ptr(None)) == -1


def test_compact_ring_equals_per_slot_compact_parse(torch):
    """rpkt_gpu_parse_ring_compact: 16-B records, as rpkt_gpu_parse_batch_compact per
    slot (strided short frames included, which parse_batch_compact hands to its 64-B-window
    compile)."""
    sizes = [64, 1, 3000, 0, 129, 5000] * 6
    cfgs = [2, 4, 5, 3]
    hbs = [gen.make_batch(cfgs[k % 4], n, seed=300 + k) for k, n in enumerate(sizes)]
    nb = 256
    dbs = [engine.DeviceBatch.from_host(h) for h in hbs]
    recs = [torch.zeros(max(h.n, 1) * 16, dtype=torch.uint8, device="cuda") for h in hbs]
    evs = [torch.zeros(max(h.n, 1), dtype=torch.int64, device="cuda") for h in hbs]
    engine.parse_ring(engine.ring_slots(dbs, recs, evs), 3 | engine.F_FLOW_EV, nb, compact=True)
    torch.cuda.synchronize()
    for k, (hb, db) in enumerate(zip(hbs, dbs)):
        if hb.n == 0:
            continue
        r1, e1 = engine.parse_batch_compact(db, 3 | engine.F_FLOW_EV, n_buckets=nb)
        assert torch.equal(recs[k][:hb.n * 16], r1), "slot %d vs parse_batch_compact" % k
        assert torch.equal(evs[k][:hb.n], e1), "slot %d events" % k


def test_compact_ring_of_short_strided_frames(torch):
    """A compact ring whose every slot holds strided 64-B frames runs on the 64-B-window
    compile (as parse_batch_compact does for one such batch); records and events equal
    the oracle's projected records and events."""
    from rpkt_amd.records import project16
    sizes = [1, 64, 65, 0, 4097, 2000, 333]
    hbs = [gen.make_batch(2, n, seed=900 + k) for k, n in enumerate(sizes)]
    nb = 128
    dbs = [engine.DeviceBatch.from_host(h) for h in hbs]
    recs = [torch.zeros(max(h.n, 1) * 16, dtype=torch.uint8, device="cuda") for h in hbs]
    evs = [torch.zeros(max(h.n, 1), dtype=torch.int64, device="cuda") for h in hbs]
    for flags in (1, 3):
        engine.parse_ring(engine.ring_slots(dbs, recs, evs), flags | engine.F_FLOW_EV, nb,
                          compact=True)
        torch.cuda.synchronize()
        for k, hb in enumerate(hbs):
            if hb.n == 0:
                continue
            o, ev = oracle.parse_batch(hb.frames, hb.n, flags=flags | engine.F_FLOW_EV,
                                       stride=hb.stride, frame_len=hb.frame_len, n_buckets=nb,
                                       threads=THREADS, flow_ev=True)
            want = project16(o, flags).tobytes()
            assert recs[k][:hb.n * 16].cpu().numpy().tobytes() == want, (flags, k)
            assert np.array_equal(evs[k][:hb.n].cpu().numpy().view(np.uint64), ev), (flags, k)


@pytest.mark.parametrize("cfg,compact", [(2, False), (2, True), (4, False), (10, True)])
def test_host_pipeline_ring_and_per_batch(torch, cfg, compact):
    """rpkt_amd.pipeline: pinned H2D of a copy group -> one parse_ring launch over the
    group's batches (or one parse per batch) -> D2H of the records; the records that come
    home equal the per-batch device parse (records_checked) either way."""
    from rpkt_amd import pipeline
    for use_ring in (True, False):
        r = pipeline.host_inclusive(cfg, compact, steps=3, slots=2, group=3, n=20000,
                                    use_ring=use_ring)
        assert r["records_checked"] is True and r["parse"] == ("ring" if use_ring else "per batch")
