"""Per-launch fixed cost of the config-2 parse: back-to-back launches on one stream
against independent batches alternated over 2 or 4 streams (their launch boundaries
overlap), and one parse_ring launch over the same 8 batches.  Prints one JSON line."""
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from rpkt_amd import engine, gen  # noqa: E402

n, R, K = 1 << 20, 8, 400
hbs = [gen.make_batch(2, n, seed=2 + 104729 * r) for r in range(R)]
dbs = [engine.DeviceBatch.from_host(h) for h in hbs]
recs = [engine.alloc_records(n) for _ in range(R)]
out = {}
for ns in (1, 2, 4):
    streams = [torch.cuda.Stream() for _ in range(ns)]
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            engine.parse_batch(dbs[k % R], 1, recs=recs[k % R], stream=streams[k % ns])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    out["streams%d_us_per_batch" % ns] = round(dt / K * 1e6, 2)
ring = engine.ring_slots(dbs, recs)
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K // R):
        engine.parse_ring(ring, 1)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
out["ring8_us_per_batch"] = round(dt / (K // R) / R * 1e6, 2)
print(json.dumps(out))
