"""GPU parity of rpkt_gpu_parse_tunnel_ring: every slot of a ring of tunnelled bursts gets
exactly the records rpkt_gpu_parse_tunnel_batch writes for that slot alone (and so the
oracle's, tests/test_gpu_tunnel.py), across slot layouts (packed, strided, frame_len <
stride, 16-B phases), ragged and empty slots, more slots than one launch holds
(RPKT_RING_MAX_SLOTS = 32), flow events, and the all-checked-before-launch validation."""
import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, gen
from rpkt_amd.records import F_IPV6, as_records, as_tunnels

from test_gpu_parity import host_batch
import tunnel_frames as tf

pytestmark = pytest.mark.gpu
F6 = 3 | F_IPV6
F_FLOW_EV = 4


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def ring_batches():
    """37 host batches: config 14 fuzz at ragged sizes, config 13 packed and strided with
    frame_len < stride, the odd tunnel frames at several phases, empty slots."""
    hbs = []
    for k, n in enumerate((1, 63, 64, 65, 130, 300, 0, 4099, 17, 2048)):
        hbs.append(gen.make_batch(14, n, seed=1500 + k) if n else None)
    h13 = gen.make_batch(13, 3000)
    hbs.append(h13)
    hbs.append(gen.HostBatch(13, 2000, h13.seed, h13.frames, None, 1500, 1400))
    for lead in (0, 1, 7, 15):
        hbs.append(host_batch(tf.odd_frames(seed=lead, n=96), lead))
    while len(hbs) < 37:
        k = len(hbs)
        hbs.append(gen.make_batch(14, 97 * k % 700 + 1, seed=1600 + k) if k % 9 else None)
    return hbs


def device_slot(torch, hb):
    if hb is None:                                # an empty slot: n == 0, nothing attached
        db = engine.DeviceBatch(torch.zeros(64, dtype=torch.uint8, device="cuda"), 0, None, 64, 64)
        n = 0
    else:
        db = engine.DeviceBatch.from_host(hb)
        n = hb.n
    mk = lambda b: torch.full((max(n, 1) * b,), 0xab, dtype=torch.uint8, device="cuda")
    return db, mk(80), mk(16), mk(80), torch.full((max(n, 1),), -1, dtype=torch.int64,
                                                  device="cuda")


@pytest.mark.parametrize("flags,nb", [(F6, 0), (3, 0), (1, 0), (F6 | F_FLOW_EV, 977)])
def test_tunnel_ring_equals_per_slot_batches(torch, flags, nb):
    hbs = ring_batches()
    slots = [device_slot(torch, hb) for hb in hbs]
    fev = bool(flags & F_FLOW_EV)
    arr = engine.tunnel_ring_slots([s[0] for s in slots], [s[1] for s in slots],
                                   [s[2] for s in slots], [s[3] for s in slots],
                                   [s[4] for s in slots] if fev else None)
    engine.parse_tunnel_ring(arr, flags, nb)
    torch.cuda.synchronize()
    for k, (hb, (db, o, t, i, ev)) in enumerate(zip(hbs, slots)):
        if hb is None:                            # skipped: untouched
            assert (o.cpu() == 0xab).all() and (t.cpu() == 0xab).all()
            continue
        want = engine.parse_tunnel_batch(db, flags, n_buckets=nb)
        for got, w, what in zip((o, t, i), want[:3], ("outer", "tunnel", "inner")):
            if not torch.equal(got, w):
                raise AssertionError("slot %d (n=%d): %s records differ from the batch call"
                                     % (k, hb.n, what))
        if fev:
            assert torch.equal(ev, want[3]), "slot %d: flow events differ" % k
    # and the oracle, on a few slots (the batch call is pinned to it in test_gpu_tunnel.py)
    for k in (1, 7, 11, 13):
        hb, (db, o, t, i, ev) = hbs[k], slots[k]
        oo, ot, oi = oracle.tunnel_batch(hb.frames, hb.n, flags & ~F_FLOW_EV, offsets=hb.offsets,
                                         stride=hb.stride, frame_len=hb.frame_len)
        assert as_records(o.cpu().numpy()).tobytes() == oo.tobytes()
        assert as_tunnels(t.cpu().numpy()).tobytes() == ot.tobytes()
        assert as_records(i.cpu().numpy()).tobytes() == oi.tobytes()
        if fev:
            want = oracle.tunnel_flow_events(oo, ot, oi, nb)
            assert np.array_equal(ev.cpu().numpy().view(np.uint64), want)


def test_tunnel_ring_validation(torch):
    """Every slot is checked before anything launches: a misaligned record pointer or a
    missing flow-event tensor in a late slot leaves every slot untouched; an empty ring
    and all-empty slots are RPKT_OK."""
    hbs = [gen.make_batch(14, 200, seed=1700 + k) for k in range(5)]
    slots = [device_slot(torch, hb) for hb in hbs]
    arr = engine.tunnel_ring_slots([s[0] for s in slots], [s[1] for s in slots],
                                   [s[2] for s in slots], [s[3] for s in slots],
                                   [s[4] for s in slots])
    good = arr[4].inner_dev
    arr[4].inner_dev = good + 8                                 # misaligned
    with pytest.raises(engine.RpktError, match="ALIGN"):
        engine.parse_tunnel_ring(arr, F6)
    arr[4].inner_dev = good
    arr[3].flow_ev_dev = None
    with pytest.raises(engine.RpktError, match="INVAL"):
        engine.parse_tunnel_ring(arr, F6 | F_FLOW_EV, 64)       # slot 3 has no events
    with pytest.raises(engine.RpktError, match="INVAL"):
        engine.parse_tunnel_ring(arr, F6 | 16)                  # an unknown flag
    torch.cuda.synchronize()
    for db, o, t, i, ev in slots:
        assert (o.cpu() == 0xab).all() and (t.cpu() == 0xab).all() and (i.cpu() == 0xab).all()
    engine.parse_tunnel_ring((engine.TunRingSlot * 0)(), F6)   # no slots
    for j in range(5):
        arr[j].batch.n = 0
    engine.parse_tunnel_ring(arr, F6 | F_FLOW_EV, 64)           # only empty slots
    torch.cuda.synchronize()
    assert all((s[1].cpu() == 0xab).all() for s in slots)


def test_cpp_vtep_rx_through_c_abi(torch):
    """examples/vtep_rx: a C++ VTEP receive loop (C ABI only) parses four bursts of VXLAN
    frames from 16 tenants as one tunnel ring, counts the inner flows, and checks every
    VNI, every inner verdict (1 in 97 inner UDP sums corrupted) and every counter row
    against its own view of the frames (rpkt_flow_hash)."""
    import subprocess
    from rpkt_amd.build import VTEP_RX_BIN
    for nb in ("1024", "977"):
        r = subprocess.run([VTEP_RX_BIN, nb], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "counter rows differing from the host count: 0" in r.stdout, r.stdout
