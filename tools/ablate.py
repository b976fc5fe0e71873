"""Ablation timing of the parse kernel (development tool, runs on the GPU box).

Times, interleaved in one process (cdna_hip_programming.md §5.4 rule 24):
  v0 product kernel, v1 window only (no parse), v2 no L4 stream, v3 no record
  stores, v10 streaming-copy reference (same read + write bytes, coalesced), v14 grid-stride
  read-only reference, v15 same-traffic tile reference (each wave streams its tile's
  bytes with nt loads and writes 64 records, no parse).
Usage: python tools/ablate.py [--configs 2,3] [--rounds 5] [--launches 20]
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
ap.add_argument("--configs", default="2,3")
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--launches", type=int, default=20)
ap.add_argument("--variants", default="0,1,2,3,10")
ap.add_argument("--rotate", type=int, default=8, help="distinct batches rotated at config 2")
args = ap.parse_args()

L = engine.ablate_lib()      # the rpkt_gpu_debug_* hooks live in the development library
L.rpkt_gpu_debug_variant.argtypes = [ctypes.POINTER(engine.Batch), ctypes.c_uint32,
                                     ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
L.rpkt_gpu_debug_variant.restype = ctypes.c_int
variants = [int(v) for v in args.variants.split(",")]
res = {}
for cfg in [int(c) for c in args.configs.split(",")]:
    R = args.rotate if cfg == 2 else 1
    hbs = [gen.make_batch(cfg, seed=50 + r) for r in range(R)]
    dbs = [engine.DeviceBatch.from_host(hb) for hb in hbs]
    recs = [engine.alloc_records(hb.n) for hb in hbs]
    descs = [db.desc() for db in dbs]
    alg = int(hbs[0].lens().sum()) + hbs[0].n * 80 + (4 * (hbs[0].n + 1) if hbs[0].offsets is not None else 0)
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    times = {v: [] for v in variants}
    flags = gen.FLAGS[cfg]
    cfg_variants = variants
    for rnd in range(args.rounds + 1):
        for v in cfg_variants:
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for k in range(args.launches):
                rc = L.rpkt_gpu_debug_variant(ctypes.byref(descs[k % R]), flags,
                                              recs[k % R].data_ptr(), v, sp)
                assert rc == 0, rc
            e1.record(st)
            torch.cuda.synchronize()
            if rnd:
                times[v].append(e0.elapsed_time(e1) / args.launches * 1e3)
    out = {}
    for v in cfg_variants:
        med = float(np.median(times[v]))
        out["v%d" % v] = {"us": round(med, 2), "min_us": round(min(times[v]), 2),
                          "tb_s": round(alg / med / 1e6, 3)}
    res["config%d" % cfg] = out
    print("config", cfg, json.dumps(out), flush=True)
    del dbs, recs
    torch.cuda.empty_cache()
print(json.dumps(res))
