"""GPU parity of rpkt_gpu_fields_batch (header-field getters over the layer walk)
against the oracle (oracle/rpkt_oracle_fields.c), bit-exact: every field of every
protocol of the walk, 128-bit fields as halves, outer and inner occurrences."""
import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, fields, gen
from rpkt_amd.records import LAYERS_DTYPE

from test_gpu_parity import host_batch
from test_oracle_fields import all_requests

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def check(hb, chunks):
    db = engine.DeviceBatch.from_host(hb)
    lay_d = engine.layers_batch(db)
    lay = lay_d.cpu().numpy().view(LAYERS_DTYPE)
    hits = 0
    for chunk in chunks:
        reqs = fields.requests(chunk)
        v, p = engine.fields_batch(db, lay_d, reqs)
        gv = v.cpu().numpy().view(np.uint64)
        gp = p.cpu().numpy().view(np.uint32)
        ov, op = oracle.fields_batch(hb.frames, hb.n, lay, reqs, offsets=hb.offsets,
                                     stride=hb.stride, frame_len=hb.frame_len)
        if not (np.array_equal(gv, ov) and np.array_equal(gp, op)):
            bad = np.nonzero((gv != ov).any(axis=1) | (gp != op))[0]
            i = int(bad[0])
            raise AssertionError("%d frames differ, first %d: gpu %s/%x oracle %s/%x (%s)" % (
                len(bad), i, gv[i], gp[i], ov[i], op[i], chunk))
        hits += int(sum(bin(int(x)).count("1") for x in op[:4096]))
    return hits


def test_fields_mix_every_field(torch):
    assert check(gen.make_mix(200000, seed=31), all_requests()) > 10000


@pytest.mark.parametrize("lead", [0, 1, 5, 11])
def test_fields_fixtures_every_alignment(torch, lead):
    check(host_batch(gen.fixture_frames() * 2, lead), all_requests())


@pytest.mark.parametrize("cfg", [2, 3, 5])
def test_fields_baseline_configs(torch, cfg):
    chunk = [("ETHER_ETHERFRAME", "dst_addr"), ("VLAN_VLANFRAME", "vlan_id"),
             ("VLAN_VLANFRAME", "vlan_id", 1), ("IPV4_IPV4", "ttl"), ("IPV4_IPV4", "src_addr"),
             ("IPV4_IPV4", "dst_addr"), ("TCP_TCP", "seq_num"), ("UDP_UDP", "dst_port")]
    check(gen.make_batch(cfg, 1 << 18), [chunk])


@pytest.mark.parametrize("n,k", [(1, 1), (3, 7), (129, 3), (257, 3), (1000, 32), (4097, 5)])
def test_fields_ragged_sizes(torch, n, k):
    """n x n_req around the 128-frame block: no value or mask past n is written."""
    hb = gen.make_mix(n, seed=n + k)
    chunk = all_requests()[0][:k]
    db = engine.DeviceBatch.from_host(hb)
    lay_d = engine.layers_batch(db)
    vals = torch.full((n + 8, k), -1, dtype=torch.int64, device="cuda")
    pres = torch.full((n + 8,), -1, dtype=torch.int32, device="cuda")
    engine.fields_batch(db, lay_d, fields.requests(chunk), values=vals, present=pres)
    assert (vals[n:] == -1).all() and (pres[n:] == -1).all()
    check(hb, [chunk])


def test_fields_bad_requests(torch):
    hb = gen.make_mix(64, seed=1)
    db = engine.DeviceBatch.from_host(hb)
    lay_d = engine.layers_batch(db)
    bad = fields.requests([("IPV4_IPV4", "ttl")])
    bad["bits"] = 0
    with pytest.raises(engine.RpktError):
        engine.fields_batch(db, lay_d, bad)
    bad["bits"] = 65
    with pytest.raises(engine.RpktError):
        engine.fields_batch(db, lay_d, bad)
    bad["bits"], bad["proto"] = 8, 200
    with pytest.raises(engine.RpktError):
        engine.fields_batch(db, lay_d, bad)


@pytest.mark.parametrize("lead", [0, 1, 2, 3])
def test_fields_random_requests_past_frame_and_buffer_end(torch, lead):
    """Random (protocol, nth, width, bit offset) requests, including fields that cross
    the frame's end and, at the batch's last frame, the buffer's final partial dword
    (frames_bytes = 4k + lead residue): the kernel's byte path."""
    from test_oracle_fields import random_requests
    rng = np.random.default_rng(100 + lead)
    fr = gen.fixture_frames()
    hb = host_batch(fr + fr[:3], lead)
    check(hb, [random_requests(rng) for _ in range(8)])
    # the batch's last frame ends at the buffer end, 4k + r bytes: Ethernet fields
    # over its final bytes take the byte path of the buffer's last partial dword
    base = lead + sum(len(f) for f in fr[:5]) + 23
    last = fr[0][:23 + (lead - base) % 4]
    hb = host_batch(fr[:5] + [last], lead)
    assert hb.frames.size % 4 == lead
    L = len(last)
    chunk = [(0, 0, b, o) for b, o in zip([64, 33, 8, 1, 16, 57, 24, 40] * 4,
                                          range(max(0, 8 * L - 96), 8 * L, 3))][:32]
    check(hb, [chunk])
    lay = oracle.layers_batch(hb.frames, hb.n, offsets=hb.offsets)
    _, pres = oracle.fields_batch(hb.frames, hb.n, lay, fields.requests(chunk),
                                  offsets=hb.offsets)
    assert pres[-1] != 0
    hm = gen.make_mix(20000, seed=7 + lead)
    check(hm, [random_requests(rng) for _ in range(4)])
