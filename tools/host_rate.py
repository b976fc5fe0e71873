"""Host-inclusive rate: frames start in (pinned) host memory and records end there.

Pipeline per batch k on three HIP streams: H2D copy of batch k into device slot
k%2 (copy-in stream) -> rpkt_gpu_parse_batch on the compute stream -> D2H copy of
the records into pinned host memory (copy-out stream); events order the stages so
batch k+1's upload overlaps batch k's parse and batch k-1's download.  The rate is
PCIe-bound (Gen5 x16, 63 GB/s per direction spec), two orders of magnitude below
the device-resident rate: it is reported in DESIGN.md, never as bench.py's value.

Each config runs twice: 80-byte records (rpkt_gpu_parse_batch) and 16-byte compact
records (rpkt_gpu_parse_batch_compact), whose D2H is a fifth of the bytes.

Usage: python tools/host_rate.py [--configs 2,3,4] [--batches 20]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rpkt_amd import engine, gen  # noqa: E402
from rpkt_amd.records import REC_BYTES, REC16_BYTES  # noqa: E402


def run(cfg, batches, compact=False):
    hb = gen.make_batch(cfg)
    flags = gen.FLAGS[cfg]
    host_frames = torch.from_numpy(hb.frames).pin_memory()
    host_offs = torch.from_numpy(hb.offsets.view(np.int32)).pin_memory() if hb.offsets is not None else None
    rb = REC16_BYTES if compact else REC_BYTES
    host_recs = torch.empty(hb.n * rb, dtype=torch.uint8).pin_memory()
    dev_frames = [torch.empty_like(host_frames, device="cuda") for _ in range(2)]
    dev_offs = [torch.empty_like(host_offs, device="cuda") for _ in range(2)] if host_offs is not None else [None, None]
    dev_recs = [torch.empty(hb.n * rb, dtype=torch.uint8, device="cuda") for _ in range(2)]
    parse = engine.parse_batch_compact if compact else engine.parse_batch
    s_in, s_cmp, s_out = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    up = [torch.cuda.Event() for _ in range(2)]
    done = [torch.cuda.Event() for _ in range(2)]
    down = [torch.cuda.Event() for _ in range(2)]
    for e in down:
        e.record(s_out)

    def step(k):
        b = k % 2
        with torch.cuda.stream(s_in):
            s_in.wait_event(done[b])                      # slot free: its parse finished
            dev_frames[b].copy_(host_frames, non_blocking=True)
            if host_offs is not None:
                dev_offs[b].copy_(host_offs, non_blocking=True)
            up[b].record(s_in)
        s_cmp.wait_event(up[b])
        s_cmp.wait_event(down[b])                         # records slot downloaded
        db = engine.DeviceBatch(dev_frames[b], hb.n, dev_offs[b], hb.stride, hb.frame_len)
        parse(db, flags, recs=dev_recs[b], stream=s_cmp)
        done[b].record(s_cmp)
        with torch.cuda.stream(s_out):
            s_out.wait_event(done[b])
            host_recs.copy_(dev_recs[b], non_blocking=True)
            down[b].record(s_out)

    for k in range(3):
        step(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(batches):
        step(k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    fb = int(hb.lens().sum())
    return {"config": cfg, "record_bytes": rb, "batches": batches, "frames_per_batch": hb.n,
            "mpps": hb.n * batches / dt / 1e6,
            "frame_gb_per_s": fb * batches / dt / 1e9,
            "h2d_gb_per_s": (fb + (4 * (hb.n + 1) if hb.offsets is not None else 0)) * batches / dt / 1e9,
            "d2h_gb_per_s": hb.n * rb * batches / dt / 1e9,
            "ms_per_batch": dt / batches * 1e3}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,3,4")
    ap.add_argument("--batches", type=int, default=20)
    a = ap.parse_args()
    print(json.dumps({"device": torch.cuda.get_device_name(0),
                      "engine_build": engine.lib().rpkt_gpu_build_info().decode()}), flush=True)
    for c in a.configs.split(","):
        for compact in (False, True):
            print(json.dumps(run(int(c), a.batches, compact)), flush=True)
