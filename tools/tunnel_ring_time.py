"""Time rpkt_gpu_parse_tunnel_ring against one rpkt_gpu_parse_tunnel_batch call per slot
and against one batch call over the same frames (GPU box):

    python tools/tunnel_ring_time.py [--out gpurun_out/tunnel_ring/times.json]

A ring of 32 slots, each a shard of config 13 (1500-B VXLAN / GTP-U / GRE frames) of B
frames, B = 64 .. 8192; flags = config 13's (sums on both levels).  Each figure is the
median of 20 passes, timed with HIP events on the stream the calls launch on; the per-slot
figure includes the host's launch of 32 kernels, which is what the ring removes."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def median_ms(torch, fn, reps=20):
    s = torch.cuda.current_stream()
    ts = []
    for _ in range(3):
        fn()
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        fn()
        b.record(s)
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/tunnel_ring/times.json")
    a = ap.parse_args()
    import torch
    from rpkt_amd import engine, gen
    slots_n = 32
    flags = gen.FLAGS[13]
    full = engine.DeviceBatch.from_host(gen.make_batch(13, slots_n * 8192))
    rows = []
    for B in (64, 256, 1024, 4096, 8192):
        dbs = [full.shard(k * B, (k + 1) * B) for k in range(slots_n)]
        outs = [(engine.alloc_records(B), torch.empty(B * 16, dtype=torch.uint8, device="cuda"),
                 engine.alloc_records(B)) for _ in range(slots_n)]
        arr = engine.tunnel_ring_slots(dbs, [o[0] for o in outs], [o[1] for o in outs],
                                       [o[2] for o in outs])
        whole = full.shard(0, slots_n * B)
        wo = (engine.alloc_records(whole.n),
              torch.empty(whole.n * 16, dtype=torch.uint8, device="cuda"),
              engine.alloc_records(whole.n))

        def per_slot():
            for db, (o, t, i) in zip(dbs, outs):
                engine.parse_tunnel_batch(db, flags, o, t, i)

        ring = median_ms(torch, lambda: engine.parse_tunnel_ring(arr, flags))
        per = median_ms(torch, per_slot)
        one = median_ms(torch, lambda: engine.parse_tunnel_batch(whole, flags, *wo))
        # the ring's records equal the per-slot calls' (run last: both wrote the same tensors)
        engine.parse_tunnel_ring(arr, flags)
        ref = [tuple(x.clone() for x in o) for o in outs]
        per_slot()
        same = all(torch.equal(x, y) for r, o in zip(ref, outs) for x, y in zip(r, o))
        n = slots_n * B
        rows.append({"frames_per_slot": B, "slots": slots_n, "frames": n,
                     "ring_ms": round(ring, 4), "per_slot_calls_ms": round(per, 4),
                     "one_batch_ms": round(one, 4), "ring_mpps": round(n / ring / 1e3, 1),
                     "per_slot_mpps": round(n / per / 1e3, 1),
                     "one_batch_mpps": round(n / one / 1e3, 1), "ring_equals_per_slot": same})
        print(json.dumps(rows[-1]), flush=True)
        assert same, "ring records differ from the per-slot calls"
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump({"device": engine.device_info(), "build": engine.lib().rpkt_gpu_build_info().decode(),
                   "flags": flags, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
