"""GPU parity of rpkt_gpu_options_batch (TcpOptionsIter / Ipv4OptionsIter) against
oracle/rpkt_oracle_opts.c, bit-exact, on the reference captures and full batches;
every case also walks from compact records (rpkt_gpu_options_batch_compact)."""
import os

import numpy as np
import pytest

from oracle import oracle
from rpkt_amd import engine, gen
from rpkt_amd.records import OPT_STOP, as_opts, as_records

from test_gpu_parity import host_batch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
PKTS = os.path.join(HERE, "golden", "packets")


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "GPU tests need an MI355X"
    return t


def gpu_opts(hb):
    db = engine.DeviceBatch.from_host(hb)
    recs = engine.parse_batch(db, 3)
    o = as_opts(engine.options_batch(db, recs).cpu().numpy())
    r16 = engine.parse_batch_compact(db, 3)
    oc = as_opts(engine.options_batch(db, r16, compact=True).cpu().numpy())
    return o, oc, as_records(recs.cpu().numpy())


def check(hb):
    g, gc, r = gpu_opts(hb)
    o = oracle.options_batch(hb.frames, hb.n, r, offsets=hb.offsets, stride=hb.stride,
                             frame_len=hb.frame_len)
    for what, x in (("full records", g), ("compact records", gc)):
        if x.tobytes() != o.tobytes():
            bad = np.nonzero(x.view(np.uint8).reshape(-1, 64) != o.view(np.uint8).reshape(-1, 64))
            i = int(bad[0][0])
            raise AssertionError("%s: %d frames differ, first %d: gpu %s oracle %s" % (
                what, len(np.unique(bad[0])), i, x[i], o[i]))
    return g, r


@pytest.mark.parametrize("cfg", [2, 3, 5, 6])
def test_options_parity_configs(torch, cfg):
    hb = gen.make_batch(cfg)
    g, r = check(hb)
    if cfg == 5:
        ok = r["status"] == 0
        assert (g["tcp_stop"][ok] == OPT_STOP["END"]).all()


@pytest.mark.parametrize("lead", [0, 1, 3, 7, 13, 15])
def test_options_fixtures_every_alignment(torch, lead):
    frames = [oracle.load_dat(os.path.join(PKTS, n)) for n in sorted(os.listdir(PKTS))]
    check(host_batch(frames * 3, lead))


def test_options_random_option_bytes(torch):
    """Random bytes in every option slice (config 5 frames with their IPv4 and TCP
    option areas overwritten): unknown types, bad lengths, truncated options."""
    hb = gen.make_batch(5, 1 << 16, seed=77)
    r = oracle.parse_batch(hb.frames, hb.n, 3, offsets=hb.offsets)
    rng = np.random.default_rng(3)
    f = hb.frames
    for i in np.nonzero(r["status"] == 0)[0]:
        o = int(hb.offsets[i])
        a, b = o + int(r["l3_off"][i]) + 20, o + int(r["l4_off"][i])
        f[a:b] = rng.integers(0, 256, b - a, dtype=np.uint8) if rng.integers(0, 2) else \
            rng.choice([0, 1, 7, 68, 148, 134, 137, 131, 2, 3, 40], b - a).astype(np.uint8)
        c, d = o + int(r["l4_off"][i]) + 20, o + int(r["payload_off"][i])
        f[c:d] = rng.choice([0, 1, 2, 3, 4, 5, 8, 34, 10, 12, 99], d - c).astype(np.uint8)
    g, _ = check(hb)
    assert set(g["tcp_stop"].tolist()) >= {1, 2, 3} and set(g["ip_stop"].tolist()) >= {1, 2, 3}
