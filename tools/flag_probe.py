"""What the verify flags cost on short frames (development tool, GPU box): the product
parse (rpkt_gpu_parse_batch / _compact) over the 8 rotated batches of a config, per
flag set, interleaved rounds in one process, HIP events on the launch stream.
Usage: python tools/flag_probe.py [--configs 2,10] [--flags 1,3,11] [--rounds 5]
Prints one JSON line: {"<cfg>/<flags>[c]": median us per launch}.
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,10")
    ap.add_argument("--flags", default="1,3,11")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=40)
    ap.add_argument("--compact", action="store_true")
    args = ap.parse_args()
    L = engine.lib()
    P = ctypes.POINTER(engine.Batch)
    fn = L.rpkt_gpu_parse_batch_compact if args.compact else L.rpkt_gpu_parse_batch
    fn.argtypes = [P, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                   ctypes.c_void_p]
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    R = 8
    legs = {}
    for cfg in [int(c) for c in args.configs.split(",")]:
        hbs = [gen.make_batch(cfg, None, seed=gen.DEFAULT_SEED[cfg] + 104729 * r) for r in range(R)]
        dbs = [engine.DeviceBatch.from_host(h) for h in hbs]
        descs = [d.desc() for d in dbs]
        recs = [torch.empty(h.n * (16 if args.compact else 80), dtype=torch.uint8, device="cuda")
                for h in hbs]
        for f in [int(x) for x in args.flags.split(",")]:
            legs["%d/%d%s" % (cfg, f, "c" if args.compact else "")] = (descs, recs, f, dbs)
    times = {k: [] for k in legs}
    for rnd in range(args.rounds + 1):
        for k, (descs, recs, f, _) in legs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for j in range(args.launches):
                rc = fn(ctypes.byref(descs[j % R]), f, recs[j % R].data_ptr(), None, 0, sp)
                assert rc == 0, rc
            e1.record(st)
            torch.cuda.synchronize()
            if rnd:
                times[k].append(e0.elapsed_time(e1) * 1e3 / args.launches)
    print(json.dumps({k: round(float(np.median(v)), 2) for k, v in times.items()}))


if __name__ == "__main__":
    main()
