"""Byte-compare parse-kernel ablation variants against the product kernel (v0) on the
bench configs (development tool, GPU box): a variant that is to replace v0 must write
the same records.  Usage: python tools/variant_check.py --variants 40 [--configs 3,4,5,6]"""
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
ap.add_argument("--configs", default="3,4,5,6")
ap.add_argument("--variants", default="40")
args = ap.parse_args()
L = engine.ablate_lib()      # the rpkt_gpu_debug_* hooks live in the development library
L.rpkt_gpu_debug_variant.argtypes = [ctypes.POINTER(engine.Batch), ctypes.c_uint32,
                                     ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
L.rpkt_gpu_debug_variant.restype = ctypes.c_int
sp = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
res = {}
for cfg in [int(c) for c in args.configs.split(",")]:
    hb = gen.make_batch(cfg)
    db = engine.DeviceBatch.from_host(hb)
    d = db.desc()
    flags = 3
    out = {}
    for v in [0] + [int(x) for x in args.variants.split(",")]:
        r = engine.alloc_records(hb.n)
        r.fill_(0x5a)
        assert L.rpkt_gpu_debug_variant(ctypes.byref(d), flags, r.data_ptr(), v, sp) == 0
        torch.cuda.synchronize()
        out[v] = r.cpu().numpy()
    res["config%d" % cfg] = {"v%d" % v: int(np.count_nonzero(
        out[v].reshape(-1, 80).any(axis=1) & (out[v].reshape(-1, 80) != out[0].reshape(-1, 80)).any(axis=1)))
        for v in out if v}
    del db
    torch.cuda.empty_cache()
print(json.dumps({"records_differing_from_v0": res}))
ok = all(x == 0 for c in res.values() for x in c.values())
sys.exit(0 if ok else 1)
