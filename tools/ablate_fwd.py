"""Ablation timing of forward_kernel (development tool, runs on the GPU box).

Times, interleaved in one process over 4 rotating 1M x 64 B batches (config 2):
  v0 product kernel, v1 no write-back, v2 parse without the L4 sum,
  v3 window + write-back of the whole frame only.
Usage: python tools/ablate_fwd.py [--rounds 5] [--launches 20]
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

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--launches", type=int, default=20)
ap.add_argument("--variants", default="0,1,2,3")
args = ap.parse_args()

L = engine.ablate_lib()      # the rpkt_gpu_debug_* hooks live in the development library
L.rpkt_gpu_debug_forward_variant.argtypes = [ctypes.POINTER(engine.Batch), ctypes.POINTER(engine.Fwd),
                                             ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
L.rpkt_gpu_debug_forward_variant.restype = ctypes.c_int
variants = [int(v) for v in args.variants.split(",")]
R = 8                                  # cache-free rotation (like bench.py config 2)
hbs = [gen.make_batch(2, seed=60 + r) for r in range(R)]
dbs = [engine.DeviceBatch.from_host(hb) for hb in hbs]
descs = [db.desc() for db in dbs]
keeps = [torch.empty(hb.n, dtype=torch.uint8, device="cuda") for hb in hbs]
forbid = engine.forbid_list([0xAC4A0001 + k for k in range(8)])
f = engine.Fwd()
f.dmac[:] = [0xAC, 0xDC, 0xCA, 0x79, 0xCA, 0x86]
f.smac[:] = [0xAC, 0xDC, 0xCA, 0x79, 0xE5, 0xC6]
f.forbid_dev, f.n_forbid = forbid.data_ptr(), forbid.numel()
st = torch.cuda.current_stream()
sp = ctypes.c_void_p(st.cuda_stream)
times = {v: [] for v in variants}
for rnd in range(args.rounds + 1):
    for v in variants:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for k in range(args.launches):
            rc = L.rpkt_gpu_debug_forward_variant(ctypes.byref(descs[k % R]), ctypes.byref(f),
                                                  keeps[k % R].data_ptr(), v, sp)
            assert rc == 0, rc
        e1.record(st)
        torch.cuda.synchronize()
        if rnd:
            times[v].append(e0.elapsed_time(e1) / args.launches * 1e3)
out = {"v%d" % v: {"us": round(float(np.median(times[v])), 2), "min_us": round(min(times[v]), 2)}
       for v in variants}
print(json.dumps(out))
