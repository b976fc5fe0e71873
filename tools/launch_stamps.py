"""Where the config-2 parse's per-launch fixed cost goes (development tool, GPU box).

Runs the parse (librpkt_gpu_ablate.so, rpkt_gpu_debug_stamps: the product kernel plus a
clock read at each wave's start and, after its stores are acknowledged, at its end, on
the 100-MHz counter every CU shares) back to back over the 8 rotated config-2 batches,
and reports per launch, in microseconds from the launch's first wave start:
  * the HIP-event time per launch of the same sequence (the bench's clock),
  * the ramp: when the k-th percentile of waves started,
  * the drain: when the k-th percentile of waves ended, the last end,
  * the gap between one launch's last wave end and the next one's first wave start,
  * the mean wave duration, waves in flight at the plateau, and per-XCD last ends.
Each block size in --wpb (waves per block; the product's is 4) is measured, and the
unstamped kernel at that block size is timed with HIP events over the same sequence.
Usage: python tools/launch_stamps.py [--n 1048576] [--launches 40] [--flags 1] [--config 2]
                                     [--wpb 4,2,1]
Prints one JSON line per block size.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rpkt_amd import engine, gen  # noqa: E402

TICK_US = 0.01                                      # s_memrealtime: 100 MHz


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--launches", type=int, default=40)
    ap.add_argument("--flags", type=int, default=1)
    ap.add_argument("--rotate", type=int, default=8)
    ap.add_argument("--wpb", default="4,2,1")
    args = ap.parse_args()
    L = engine.ablate_lib()
    P = ctypes.POINTER(engine.Batch)
    L.rpkt_gpu_debug_stamps.argtypes = [P, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_int, ctypes.c_void_p]
    R = args.rotate
    hbs = [gen.make_batch(args.config, args.n, seed=gen.DEFAULT_SEED[args.config] + 104729 * r)
           for r in range(R)]
    dbs = [engine.DeviceBatch.from_host(h) for h in hbs]
    descs = [d.desc() for d in dbs]
    recs = [engine.alloc_records(h.n) for h in hbs]
    waves = (args.n + 63) // 64
    K = args.launches
    stamps = torch.zeros((K, waves, 4), dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)

    def run(k, wpb, stamped=True):
        rc = L.rpkt_gpu_debug_stamps(ctypes.byref(descs[k % R]), args.flags, recs[k % R].data_ptr(),
                                     stamps[k].data_ptr() if stamped else None, wpb, sp)
        assert rc == 0, rc

    def timed(wpb, stamped):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for k in range(K):
            run(k, wpb, stamped)
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / K

    want = engine.parse_batch(dbs[0], args.flags).cpu()
    for wpb in [int(x) for x in args.wpb.split(",")]:
        recs[0].zero_()
        for k in range(K):                           # warm: clocks ramp
            run(k, wpb)
        torch.cuda.synchronize()
        assert torch.equal(recs[0].cpu(), want), "records differ at wpb %d" % wpb
        plain = [timed(wpb, False) for _ in range(3)]
        stamped_us = timed(wpb, True)
        report(args, stamps, K, wpb, float(np.median(plain)), stamped_us)


def report(args, stamps, K, wpb, product_us, stamped_us):
    waves = stamps.shape[1]
    s = stamps.cpu().numpy()
    t0 = s[:, :, 0].astype(np.int64)
    t1 = s[:, :, 1].astype(np.int64)
    hw = s[:, :, 2] & 0xffffffff
    xcc = (s[:, :, 2] >> 32) & 0xf
    assert (t1 >= t0).all() and (t0 > 0).all()
    pct = (1, 10, 25, 50, 75, 90, 99)
    first = t0.min(axis=1)
    rel0 = (t0 - first[:, None]) * TICK_US
    rel1 = (t1 - first[:, None]) * TICK_US
    span = rel1.max(axis=1)                         # first start -> last end
    gaps = (t0.min(axis=1)[1:] - t1.max(axis=1)[:-1]) * TICK_US
    dur = (t1 - t0) * TICK_US
    # waves in flight over the launch (100 bins) -> plateau and the ramp/drain edges
    inflight = []
    for k in range(K):
        edges = np.linspace(0, span[k], 101)
        started = np.searchsorted(np.sort(rel0[k]), edges, side="right")
        ended = np.searchsorted(np.sort(rel1[k]), edges, side="right")
        inflight.append(started - ended)
    inflight = np.median(np.array(inflight), axis=0)
    plateau = float(np.percentile(inflight, 75))
    mid = float(inflight[10:80].mean())             # mean waves in flight, 10-80 % of the span
    cu = (hw >> 8) & 0xf
    se = (hw >> 13) & 0x7
    last_end_xcd = {int(x): round(float(np.median([rel1[k][xcc[k] == x].max() for k in range(K)])), 2)
                    for x in np.unique(xcc)}
    out = {
        "config": args.config, "n": args.n, "waves": waves, "launches": K, "wpb": wpb,
        "kernel_us_per_launch": round(product_us, 2),
        "stamped_us_per_launch": round(stamped_us, 2),
        "span_first_start_to_last_end_us": round(float(np.median(span)), 2),
        "gap_last_end_to_next_first_start_us": round(float(np.median(gaps)), 2),
        "start_pct_us": {p: round(float(np.median(np.percentile(rel0, p, axis=1))), 2) for p in pct},
        "end_pct_us": {p: round(float(np.median(np.percentile(rel1, p, axis=1))), 2) for p in pct},
        "wave_us_mean": round(float(dur.mean()), 3),
        "wave_us_pct": {p: round(float(np.percentile(dur, p)), 3) for p in (10, 50, 90, 99)},
        "inflight_plateau": plateau,
        "inflight_mean_10_80": round(mid, 1),
        "inflight_profile": [int(x) for x in inflight[::5]],
        "xcds": int(len(np.unique(xcc))),
        "cus_seen": int(len(np.unique(xcc * 1024 + se * 16 + cu))),
        "last_end_by_xcd_us": last_end_xcd,
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
