"""Host-inclusive receive pipeline: frames start in pinned host memory (a NIC ring or a
loopback buffer, rpkt-dpdk/examples/loopback_rx.rs:96-140) and records end there.

Per step k on three HIP streams: H2D copy of frame group k into device slot k % S
(copy-in stream) -> one rpkt_gpu_parse_batch[_compact] per batch of the group on the
compute stream -> D2H copy of the group's records into pinned host memory (copy-out
stream).  Events order the stages, so with S slots the upload of group k + 1 and the
download of group k - 1 overlap the parse of group k, and up to S - 1 uploads can be
queued ahead of the parse.  A group is `group` consecutive batches of the ring, moved
by ONE hipMemcpyAsync each way: at 64-B frames a 1M-frame batch is only 64 MiB, and the
fixed cost of a copy is then a visible share of its time.  The group's batches are parsed
by ONE rpkt_gpu_parse_ring[_compact] launch (use_ring=True, the default), so the per-launch
fixed cost (launch gap and drain) is paid once per copy group too.

The rate is PCIe-bound (Gen5 x16: 63 GB/s per direction on paper), far below the
device-resident rate: bench.py reports it under extra.host_inclusive, never as the
headline value.
"""
import time

import numpy as np

from . import engine, gen
from .records import REC16_BYTES, REC_BYTES


def host_inclusive(cfg, compact=False, steps=12, slots=3, group=1, n=None, seed=None,
                   use_ring=True):
    """Time `steps` pipeline steps of config `cfg` (strided configs 2 / 3, or a packed
    config) with `group` batches of n frames per copy and `slots` device buffers; the
    group's batches parsed by one ring launch (use_ring) or one launch each.
    Returns the rates (whole-pipeline frames/s and the bytes each direction moved)."""
    import torch
    hb = gen.make_batch(cfg, n, seed=seed)
    flags = gen.FLAGS[cfg]
    rb = REC16_BYTES if compact else REC_BYTES
    fb = int(hb.frames.size)                    # one batch's frame buffer
    # the host ring: `group` copies of the batch back to back (what a NIC ring holds)
    ring = torch.from_numpy(np.tile(hb.frames, group)).pin_memory()
    offs = None
    if hb.offsets is not None:                  # per-batch offsets, rebased per copy
        o = hb.offsets.astype(np.int64)
        offs = torch.from_numpy(np.concatenate([o + k * fb for k in range(group)]).astype(np.uint32)
                                .view(np.int32)).pin_memory()
    host_recs = torch.empty(group * hb.n * rb, dtype=torch.uint8).pin_memory()
    dev_frames = [torch.empty(group * fb, dtype=torch.uint8, device="cuda") for _ in range(slots)]
    dev_offs = [torch.empty_like(offs, device="cuda") for _ in range(slots)] if offs is not None \
        else [None] * slots
    dev_recs = [torch.empty(group * hb.n * rb, dtype=torch.uint8, device="cuda") for _ in range(slots)]
    parse = engine.parse_batch_compact if compact else engine.parse_batch
    # the device batches of every slot's group, and (use_ring) their rpkt_ring_slot_t arrays
    dbs = []
    for b in range(slots):
        row = []
        for g in range(group):
            if offs is not None:
                row.append(engine.DeviceBatch(dev_frames[b], hb.n, dev_offs[b][g * (hb.n + 1):
                                                                            (g + 1) * (hb.n + 1)]))
            else:
                row.append(engine.DeviceBatch(dev_frames[b][g * fb:(g + 1) * fb], hb.n, None,
                                              hb.stride, hb.frame_len))
        dbs.append(row)
    recs_of = [[dev_recs[b][g * hb.n * rb:(g + 1) * hb.n * rb] for g in range(group)]
               for b in range(slots)]
    rings = [engine.ring_slots(dbs[b], recs_of[b], compact=compact) for b in range(slots)] \
        if use_ring else None
    s_in, s_cmp, s_out = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    up = [torch.cuda.Event() for _ in range(slots)]
    done = [torch.cuda.Event() for _ in range(slots)]
    down = [torch.cuda.Event() for _ in range(slots)]
    for e in done + down:
        e.record(s_out)

    def step(k):
        b = k % slots
        with torch.cuda.stream(s_in):
            s_in.wait_event(done[b])            # the slot's previous parse has finished
            dev_frames[b].copy_(ring, non_blocking=True)
            if offs is not None:
                dev_offs[b].copy_(offs, non_blocking=True)
            up[b].record(s_in)
        s_cmp.wait_event(up[b])
        s_cmp.wait_event(down[b])               # the slot's previous records are home
        if use_ring:
            engine.parse_ring(rings[b], flags, stream=s_cmp, compact=compact)
        else:
            for g in range(group):
                parse(dbs[b][g], flags, recs=recs_of[b][g], stream=s_cmp)
        done[b].record(s_cmp)
        with torch.cuda.stream(s_out):
            s_out.wait_event(done[b])
            host_recs.copy_(dev_recs[b], non_blocking=True)
            down[b].record(s_out)

    for k in range(slots):                      # warm: every slot once
        step(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        step(k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    frames = hb.n * group * steps
    fbytes = int(hb.lens().sum()) * group * steps
    h2d = (int(ring.numel()) + (int(offs.numel()) * 4 if offs is not None else 0)) * steps
    d2h = int(host_recs.numel()) * steps
    return {"config": cfg, "record_bytes": rb, "slots": slots, "batches_per_copy": group,
            "parse": "ring" if use_ring else "per batch",
            "frames_per_batch": hb.n, "steps": steps, "mpps": frames / dt / 1e6,
            "frame_gb_per_s": fbytes / dt / 1e9, "h2d_gb_per_s": h2d / dt / 1e9,
            "d2h_gb_per_s": d2h / dt / 1e9, "ms_per_copy": dt / steps * 1e3,
            "records_checked": _check_last(host_recs, hb, flags, rb, group)}


def _check_last(host_recs, hb, flags, rb, group):
    """The records that came home equal the device parse of the same batch (one sample
    batch of the ring: the pipeline's copies and slicing are right)."""
    db = engine.DeviceBatch.from_host(hb)
    ref = (engine.parse_batch_compact if rb == REC16_BYTES else engine.parse_batch)(db, flags)
    got = host_recs[(group - 1) * hb.n * rb:].numpy()
    return bool(np.array_equal(got, ref.cpu().numpy()))
