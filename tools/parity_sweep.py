"""Seed sweep of GPU parity (development tool, GPU box): new random seeds through every
per-frame entry point, each compared byte for byte with the oracle, until a time budget
runs out.  The GPU test suite fixes its seeds; this keeps drawing fresh ones, so a rare
input shape that the fixed seeds miss has many more chances to show.  Stops at the first
difference and names the seed and entry point (a JSON line per seed, progress on stderr).

  python tools/parity_sweep.py [--minutes 8] [--seed0 50000] [--out FILE]

Per seed: (a) a random packed or strided layout over the captures, configs 2/3/5/6 and
the dual-stack fuzz (config 12) frames: the parse with a random flag set (with or without
RPKT_F_IPV6) and flow events, compact records, a two-slot receive ring (80-B and compact),
both option-walk entry points over full and compact records, the tunnel parse (the pool
holds tunnel fuzz and tests/tunnel_frames.py frames) and a two-slot tunnel ring (this layout
and a config 13 / 14 batch), the layer walk; (b) a generator batch of a random config and size: the
build with random checksum flags over its (IPv4 and IPv6) records, the forward with and
without RPKT_F_IPV6, and the encapsulation build over a tunnel batch (configs 13 / 14); (c)
a fuzzed mbuf-chain batch (configs 8 / 12) through the chain
parse.  Build and forward rewrite frames in place, so they run on generator batches
(the random layouts overlap frames on purpose)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import oracle  # noqa: E402
from rpkt_amd import engine, gen  # noqa: E402
from rpkt_amd.records import (F_FLOW_EV, F_IPV6, LAYERS_DTYPE, as_opts, as_records,  # noqa: E402
                              as_records16, as_tunnels, project16)

import fuzz_layouts  # noqa: E402
import tunnel_frames  # noqa: E402
from test_gpu_parity import assert_same, assert_same16  # noqa: E402

THREADS = min(16, os.cpu_count() or 1)
DMAC = bytes([0xAC, 0xDC, 0xCA, 0x79, 0xCA, 0x86])
SMAC = bytes([0xAC, 0xDC, 0xCA, 0x79, 0xE5, 0xC6])


def extend_pool():
    """The layout fuzz pool plus dual-stack fuzz and 1500-B dual-stack frames."""
    p = fuzz_layouts.pool()
    if not getattr(extend_pool, "done", False):
        p += fuzz_layouts.frames_of(gen.make_batch(12, 600, seed=121))
        p += fuzz_layouts.frames_of(gen.make_batch(11, 40, seed=111))
        p += fuzz_layouts.frames_of(gen.make_batch(14, 600, seed=141))     # tunnel fuzz
        p += tunnel_frames.odd_frames(seed=7, n=200)
        p += tunnel_frames.jumbo_frames(seed=5, n=24)                       # to 60 KB inner
        extend_pool.done = True


def orecs(hb, flags, nb=0, flow=False):
    return oracle.parse_batch(hb.frames, hb.n, flags=flags & ~F_FLOW_EV, offsets=hb.offsets,
                              stride=hb.stride, frame_len=hb.frame_len, n_buckets=nb,
                              threads=THREADS, flow_ev=flow)


def check_layout(hb, rng):
    flags = int(rng.integers(0, 4)) | (F_IPV6 if rng.random() < 0.5 else 0)
    nb = int(rng.integers(1, 9000))
    db = engine.DeviceBatch.from_host(hb)
    o, oev = orecs(hb, flags, nb, flow=True)
    recs, ev = engine.parse_batch(db, flags | F_FLOW_EV, n_buckets=nb)
    assert_same(as_records(recs.cpu().numpy()), o)
    assert np.array_equal(ev.cpu().numpy().view(np.uint64), oev), "flow events"
    r16, ev16 = engine.parse_batch_compact(db, flags | F_FLOW_EV, n_buckets=nb)
    assert_same16(as_records16(r16.cpu().numpy()), project16(o, flags))
    assert np.array_equal(ev16.cpu().numpy().view(np.uint64), oev), "compact flow events"
    # option walks: standalone over full / compact records, fused with both record sizes
    wf = flags | 3
    o3 = orecs(hb, wf)
    want = oracle.options_batch(hb.frames, hb.n, o3, offsets=hb.offsets, stride=hb.stride,
                                frame_len=hb.frame_len).tobytes()
    for compact in (False, True):
        rr, oo = engine.parse_options_batch(db, wf, compact=compact)
        assert as_opts(oo.cpu().numpy()).tobytes() == want, "fused options (compact=%s)" % compact
        so = engine.options_batch(db, rr, compact=compact)
        assert as_opts(so.cpu().numpy()).tobytes() == want, "options (compact=%s)" % compact
    # a receive ring: this layout and a strided generator batch as the slots of one launch
    import torch
    hb2 = gen.make_batch(int(rng.choice([2, 10, 12])), int(rng.integers(1, 3000)),
                         seed=int(rng.integers(1, 1 << 30)))
    dbs = [db, engine.DeviceBatch.from_host(hb2)]
    rr = [engine.alloc_records(h.n) for h in (hb, hb2)]
    evs = [torch.zeros(h.n, dtype=torch.int64, device="cuda") for h in (hb, hb2)]
    engine.parse_ring(engine.ring_slots(dbs, rr, evs), flags | F_FLOW_EV, nb)
    r16 = [torch.empty(h.n * 16, dtype=torch.uint8, device="cuda") for h in (hb, hb2)]
    engine.parse_ring(engine.ring_slots(dbs, r16), flags, 0, compact=True)
    for k, h in enumerate((hb, hb2)):
        ok_, okev = (o, oev) if k == 0 else orecs(h, flags, nb, flow=True)
        assert_same(as_records(rr[k].cpu().numpy()), ok_)
        assert np.array_equal(evs[k].cpu().numpy().view(np.uint64), okev), "ring flow events"
        assert_same16(as_records16(r16[k].cpu().numpy()), project16(ok_, flags))
    # the tunnel parse (outer, tunnel and inner records) over the same layout
    tf = int(rng.integers(0, 4)) | (F_IPV6 if rng.random() < 0.5 else 0)
    go, gt, gi, gev = engine.parse_tunnel_batch(db, tf | F_FLOW_EV, n_buckets=nb)
    oo, ot, oi = oracle.tunnel_batch(hb.frames, hb.n, tf, offsets=hb.offsets, stride=hb.stride,
                                     frame_len=hb.frame_len)
    assert_same(as_records(go.cpu().numpy()), oo)
    assert as_tunnels(gt.cpu().numpy()).tobytes() == ot.tobytes(), "tunnel records"
    assert_same(as_records(gi.cpu().numpy()), oi)
    assert np.array_equal(gev.cpu().numpy().view(np.uint64),
                          oracle.tunnel_flow_events(oo, ot, oi, nb)), "tunnel flow events"
    # a ring of tunnelled bursts: this layout and a tunnel generator batch as two slots
    hb3 = gen.make_batch(int(rng.choice([13, 14])), int(rng.integers(1, 3000)),
                         seed=int(rng.integers(1, 1 << 30)))
    dbs = [db, engine.DeviceBatch.from_host(hb3)]
    outs = [[torch.empty(h.n * b, dtype=torch.uint8, device="cuda") for b in (80, 16, 80)] +
            [torch.zeros(h.n, dtype=torch.int64, device="cuda")] for h in (hb, hb3)]
    engine.parse_tunnel_ring(engine.tunnel_ring_slots(dbs, *[[x[j] for x in outs] for j in range(4)]),
                             tf | F_FLOW_EV, nb)
    for k, h in enumerate((hb, hb3)):
        wo, wt, wi = (oo, ot, oi) if k == 0 else oracle.tunnel_batch(
            h.frames, h.n, tf, offsets=h.offsets, stride=h.stride, frame_len=h.frame_len)
        assert_same(as_records(outs[k][0].cpu().numpy()), wo)
        assert as_tunnels(outs[k][1].cpu().numpy()).tobytes() == wt.tobytes(), "ring tunnel records"
        assert_same(as_records(outs[k][2].cpu().numpy()), wi)
        assert np.array_equal(outs[k][3].cpu().numpy().view(np.uint64),
                              oracle.tunnel_flow_events(wo, wt, wi, nb)), "ring tunnel flow events"
    gl =engine.layers_batch(db).cpu().numpy().view(LAYERS_DTYPE)
    ol = oracle.layers_batch(hb.frames, hb.n, offsets=hb.offsets, stride=hb.stride,
                             frame_len=hb.frame_len)
    assert gl.tobytes() == ol.tobytes(), "layer walk"
    return {"flags": flags, "n": hb.n}


def check_tx(rng, seed):
    import torch
    cfg = int(rng.choice([2, 3, 5, 6, 10, 11, 12]))
    n = int(rng.integers(1, 120000 if cfg not in (3, 11) else 20000))
    hb = gen.make_batch(cfg, n, seed=seed)
    pf = 3 | (F_IPV6 if cfg >= 10 else 0)
    recs = orecs(hb, pf)
    bflags = int(rng.integers(0, 4))
    db = engine.DeviceBatch.from_host(hb)
    d = torch.from_numpy(np.ascontiguousarray(recs).view(np.uint8).copy()).cuda()
    gb = engine.build_batch(db, d, bflags).cpu().numpy()
    o, ob = oracle.build_batch(hb.frames, hb.n, recs, bflags, offsets=hb.offsets,
                               stride=hb.stride, frame_len=hb.frame_len)
    assert np.array_equal(gb, ob), "built flags"
    assert np.array_equal(db.frames.cpu().numpy()[:o.size], o), "built frames"
    ff = F_IPV6 if (cfg >= 10 and rng.random() < 0.7) else 0
    db = engine.DeviceBatch.from_host(hb)
    r = as_records(engine.parse_batch(db, pf).cpu().numpy())
    forbid = np.unique(r["ip_src"][::max(1, n // 50)])[:int(rng.integers(0, 64))].astype(np.int64)
    keep = engine.forward_batch(db, DMAC, SMAC, engine.forbid_list(forbid) if forbid.size else None,
                                flags=ff).cpu().numpy()
    o, ok = oracle.forward_batch(hb.frames, hb.n, r, DMAC, SMAC, forbid.astype(np.uint32),
                                 offsets=hb.offsets, stride=hb.stride, frame_len=hb.frame_len,
                                 flags=ff)
    assert np.array_equal(keep, ok), "forward keep flags"
    assert np.array_equal(db.frames.cpu().numpy()[:o.size], o), "forward frames"
    return {"cfg": cfg, "n": n, "build_flags": bflags, "fwd_flags": ff}


def check_encap(rng, seed):
    """The encapsulation build over a tunnel generator batch: outer records and tunnel
    records from the oracle's tunnel parse, random checksum flags."""
    import torch
    cfg = int(rng.choice([13, 14]))
    n = int(rng.integers(1, 20000))
    hb = gen.make_batch(cfg, n, seed=seed)
    tf = 3 | (F_IPV6 if rng.random() < 0.5 else 0)
    oo, ot, _ = oracle.tunnel_batch(hb.frames, hb.n, tf, offsets=hb.offsets, stride=hb.stride,
                                    frame_len=hb.frame_len)
    bflags = int(rng.integers(0, 4))
    db = engine.DeviceBatch.from_host(hb)
    d = torch.from_numpy(np.ascontiguousarray(oo).view(np.uint8).copy()).cuda()
    t = torch.from_numpy(np.ascontiguousarray(ot).view(np.uint8).copy()).cuda()
    gb = engine.build_tunnel_batch(db, d, t, bflags).cpu().numpy()
    o, ob = oracle.build_tunnel_batch(hb.frames, hb.n, oo, ot, bflags, offsets=hb.offsets,
                                      stride=hb.stride, frame_len=hb.frame_len)
    assert np.array_equal(gb, ob), "encap built flags"
    assert np.array_equal(db.frames.cpu().numpy()[:o.size], o), "encap frames"
    return {"cfg": cfg, "n": n, "flags": bflags}


def check_chains(rng, seed):
    cfg = int(rng.choice([8, 12]))
    hc = gen.make_chains(cfg, n=int(rng.integers(1, 20000)), layout="fuzz", seed=seed)
    flags = int(rng.integers(0, 4)) | (F_IPV6 if cfg == 12 or rng.random() < 0.5 else 0)
    dc = engine.DeviceChains.from_host(hc)
    g = as_records(engine.parse_chains(dc, flags).cpu().numpy())
    assert_same(g, oracle.parse_chains(hc.buf, hc.segs, hc.chain_first, flags))
    return {"cfg": cfg, "n": int(hc.n), "flags": flags}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=8.0)
    ap.add_argument("--seed0", type=int, default=50000)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "parity_sweep.jsonl"))
    args = ap.parse_args()
    extend_pool()
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    t0, seed, ok = time.time(), args.seed0, 0
    with open(args.out, "w") as fh:
        while time.time() - t0 < args.minutes * 60:
            rng = np.random.default_rng(seed)
            rec = {"seed": seed}
            step = "layout"
            try:
                hb = (fuzz_layouts.packed_layout if rng.random() < 0.6 else
                      fuzz_layouts.strided_layout)(rng, int(rng.integers(1, 5000)))
                rec["layout"] = check_layout(hb, rng)
                step = "tx"
                rec["tx"] = check_tx(rng, seed)
                step = "encap"
                rec["encap"] = check_encap(rng, seed)
                step = "chains"
                rec["chains"] = check_chains(rng, seed)
            except AssertionError as e:
                rec.update(failed=step, error=str(e)[:400])
                fh.write(json.dumps(rec) + "\n")
                print(json.dumps(rec), flush=True)
                return 1
            ok += 1
            rec["t"] = round(time.time() - t0, 1)
            fh.write(json.dumps(rec) + "\n")
            fh.flush()
            if ok % 10 == 0:
                print("[sweep] %d seeds ok, %.0f s" % (ok, time.time() - t0), file=sys.stderr,
                      flush=True)
            seed += 1
    print(json.dumps({"seeds_ok": ok, "seed0": args.seed0, "seconds": round(time.time() - t0, 1)}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
