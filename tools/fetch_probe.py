"""Where config 3's extra ~4 % of reads come from (development tool, GPU box; run under
`rocprofv3 --pmc FETCH_SIZE`): the config-3 parse (both sums) over
  A: the generated batch, stride 1500 (frames share their boundary lines),
  B: the same frames in 1536-B slots (every frame starts on a 128-B line),
  C: the same frames packed with u32 offsets (as A, through the offsets path),
10 launches each, in that order, after 5 warm-up launches of A.  Prints the frame bytes
and lines each layout holds; the PMC CSV gives the bytes fetched per launch.
Usage: rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d <dir> -o fp -- python3 tools/fetch_probe.py
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rpkt_amd import engine, gen  # noqa: E402


def main():
    n = 1 << 20
    a = gen.make_batch(3, n)
    lens = a.lens()
    buf = np.zeros(n * 1536, dtype=np.uint8)
    src = a.frames[:n * 1500].reshape(n, 1500)
    buf.reshape(n, 1536)[:, :1500] = src
    b = gen.HostBatch(3, n, a.seed, buf, None, 1536, 1500)
    c = gen.make_batch(3, n, packed=True)
    out = {"frames": int(lens.sum()),
           "lines_A": int((n * 1500 + 127) // 128), "lines_B": n * 12,
           "launch_order": ["A warm x5", "A x10", "B x10", "C x10"]}
    dbs = [engine.DeviceBatch.from_host(h) for h in (a, b, c)]
    recs = engine.alloc_records(n)
    for _ in range(5):
        engine.parse_batch(dbs[0], 3, recs=recs)
    for d in dbs:
        for _ in range(10):
            engine.parse_batch(d, 3, recs=recs)
    torch.cuda.synchronize()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
