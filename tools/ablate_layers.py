"""Ablation timing of layers_kernel (development tool, runs on the GPU box).

Times the layer walk with F frames per lane (a lane walks frames base + L + 64 k,
k < F, one after the other), interleaved in one process over the config-9 protocol
mix, and checks that every variant's records are byte-identical.
Usage: python tools/ablate_layers.py [--rounds 5] [--launches 20] [--frames 1,2,4,8]
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
ap.add_argument("--frames", default="1,2,4,8")
ap.add_argument("--n", type=int, default=0)
ap.add_argument("--config", type=int, default=9, help="9 = the capture mix, else a bench config")
args = ap.parse_args()

L = engine.ablate_lib()      # the rpkt_gpu_debug_* hooks live in the development library
L.rpkt_gpu_debug_layers_variant.argtypes = [ctypes.POINTER(engine.Batch), ctypes.c_void_p,
                                            ctypes.c_int, ctypes.c_void_p]
L.rpkt_gpu_debug_layers_variant.restype = ctypes.c_int
variants = [int(v) for v in args.frames.split(",")]
hb = (gen.make_mix(args.n or gen.DEFAULT_N[9], seed=gen.DEFAULT_SEED[9]) if args.config == 9
      else gen.make_batch(args.config, args.n or None))
db = engine.DeviceBatch.from_host(hb)
desc = db.desc()
outs = {v: torch.zeros(hb.n * 64, dtype=torch.uint8, device="cuda") for v in variants}
st = torch.cuda.current_stream()
sp = ctypes.c_void_p(st.cuda_stream)
times = {v: [] for v in variants}
for rnd in range(args.rounds + 1):
    for v in variants:
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for k in range(args.launches):
            rc = L.rpkt_gpu_debug_layers_variant(ctypes.byref(desc), outs[v].data_ptr(), v, sp)
            assert rc == 0, rc
        e1.record(st)
        torch.cuda.synchronize()
        if rnd:
            times[v].append(e0.elapsed_time(e1) / args.launches * 1e3)
ref = outs[variants[0]].cpu().numpy()
same = {"F%d" % v: bool(np.array_equal(outs[v].cpu().numpy(), ref)) for v in variants}
out = {"F%d" % v: {"us": round(float(np.median(times[v])), 2), "min_us": round(min(times[v]), 2)}
       for v in variants}
print(json.dumps({"config": args.config, "n": hb.n, "times": out, "identical": same}))
