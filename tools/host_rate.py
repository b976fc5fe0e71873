"""Host-inclusive rate sweep (rpkt_amd.pipeline): pinned H2D frames -> parse -> D2H
records, for several slot counts and batches per copy.  bench.py reports the chosen
shape under extra.host_inclusive; this tool shows why that shape.

Usage: python tools/host_rate.py [--configs 2,3,4] [--slots 2,3] [--groups 1,4] [--steps 12]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rpkt_amd import engine, pipeline  # noqa: E402


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,3,4")
    ap.add_argument("--slots", default="2,3")
    ap.add_argument("--groups", default="1,4")
    ap.add_argument("--steps", type=int, default=12)
    a = ap.parse_args()
    import torch
    print(json.dumps({"device": torch.cuda.get_device_name(0),
                      "engine_build": engine.lib().rpkt_gpu_build_info().decode()}), flush=True)
    for c in [int(x) for x in a.configs.split(",")]:
        for compact in (False, True):
            for s in [int(x) for x in a.slots.split(",")]:
                for g in [int(x) for x in a.groups.split(",")]:
                    if c != 2 and g > 1:
                        continue                   # 1500 B / IMIX batches are large already
                    r = pipeline.host_inclusive(c, compact, steps=a.steps, slots=s, group=g)
                    print(json.dumps(r), flush=True)
                    torch.cuda.empty_cache()
