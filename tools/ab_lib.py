"""A/B timing of two builds of librpkt_gpu.so in one process (development tool, runs
on the GPU box): kernel-time differences of a few percent are below the box-to-box
spread, so both builds are timed interleaved on the same batch and their outputs are
compared byte for byte.

Usage: python tools/ab_lib.py <lib_b.so> [--sides AB|A|B] [--leg opts5|optsc5|popts5|poptsc5|parsec2|layers9|forward2|build2|build3|parse2|parse3|chains7|ring2|ringc2|tunnel13|encap13]
(ring<cfg> / ringc<cfg>: the R rotated batches as one rpkt_gpu_parse_ring[_compact] launch)
                              [--rounds 5] [--launches 20]
The A side is the in-tree build (rpkt_amd/_build/librpkt_gpu.so).  Build a B side with
  python tools/ab_lib.py --build <out_dir> [hipcc -D flags ...]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def build_b(out_dir, extra):
    from rpkt_amd import build
    os.makedirs(out_dir, exist_ok=True)
    flags = [build.HIPCC, "--offload-arch=" + build.ARCH, "-O3", "-std=c++17", "-fPIC",
             '-DRPKT_SRC_HASH="ab"'] + list(extra)
    objs = []
    jobs = [(f, os.path.basename(f).replace(".hip", ".o"), []) for f in build.GPU_SRC]
    jobs += [(os.path.join(build.HERE, "csrc", f), o, d) for f, o, d in build.SECOND_COMPILES]
    for f, o, d in jobs:
        o = os.path.join(out_dir, o)
        subprocess.check_call(flags + d + ["-c", "-o", o, f])
        objs.append(o)
    lib = os.path.join(out_dir, "librpkt_gpu.so")
    subprocess.check_call([build.HIPCC, "--offload-arch=" + build.ARCH, "-shared", "-fPIC",
                           "-o", lib] + objs + ["-ldl"])
    print(lib)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib_b", nargs="?")
    ap.add_argument("--build", metavar="OUT_DIR")
    ap.add_argument("--leg", default="opts5")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--n", type=int, default=0, help="frames per batch (default: the config's)")
    ap.add_argument("--flags", type=int, default=None,
                    help="parse / ring flags (default: 1 for config 2, else 3)")
    ap.add_argument("--sides", default="AB",
                    help="sides to launch (a rocprofv3 --pmc pass of one build: A or B)")
    ap.add_argument("--rotate", type=int, default=0,
                    help="distinct batches per side (default: 8 at 64 B, as bench.py)")
    args, extra = ap.parse_known_args()
    if args.build:
        return build_b(args.build, extra)

    import numpy as np
    import torch
    from rpkt_amd import engine, gen
    A = engine.lib()
    B = ctypes.CDLL(os.path.abspath(args.lib_b))
    mode, cfg = args.leg.rstrip("0123456789"), int(args.leg[len(args.leg.rstrip("0123456789")):])
    R = args.rotate or (8 if cfg in (2, 10) else 1)   # 8 x 64 MiB of frames: past the 256 MiB cache
    if mode == "chains":                         # mbuf chains (configs 7, 8)
        hbs = [gen.make_chains(cfg, args.n or None)]
        dbs = [engine.DeviceChains.from_host(h) for h in hbs]
        recss = []
    else:
        hbs = [gen.make_mix(seed=gen.DEFAULT_SEED[9]) if cfg == 9 else
               gen.make_batch(cfg, args.n or None, seed=gen.DEFAULT_SEED[cfg] + 104729 * r)
               for r in range(R)]
        dbs = [engine.DeviceBatch.from_host(h) for h in hbs]
        recss = [engine.parse_batch(d, gen.FLAGS.get(cfg, 3) | 3) for d in dbs]   # as bench.py
    R = len(hbs)
    hb = hbs[0]
    descs = [d.desc() for d in dbs]
    st = torch.cuda.current_stream()
    sp = ctypes.c_void_p(st.cuda_stream)
    P = ctypes.POINTER(engine.Batch)
    outs, call, keep_alive = {}, {}, []
    forbid = engine.forbid_list([0xAC4A0001 + k for k in range(8)])
    fwd = engine.Fwd()
    fwd.dmac[:] = [0xAC, 0xDC, 0xCA, 0x79, 0xCA, 0x86]
    fwd.smac[:] = [0xAC, 0xDC, 0xCA, 0x79, 0xE5, 0xC6]
    fwd.forbid_dev, fwd.n_forbid = forbid.data_ptr(), forbid.numel()
    # call[name](k): launch k of a side, on batch k % R (both sides run the same sequence)
    for name, L in (("A", A), ("B", B)):
        if mode == "opts":
            L.rpkt_gpu_options_batch.argtypes = [P, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
            out = torch.zeros(hb.n * 64, dtype=torch.uint8, device="cuda")
            call[name] = (lambda k, L=L, out=out: L.rpkt_gpu_options_batch(
                ctypes.byref(descs[k % R]), recss[k % R].data_ptr(), out.data_ptr(), sp))
        elif mode == "optsc":                       # option walks from compact records
            if "recs16" not in outs:
                outs["recs16"] = [engine.parse_batch_compact(d, gen.FLAGS.get(cfg, 3) | 3) for d in dbs]
            r16 = outs["recs16"]
            L.rpkt_gpu_options_batch_compact.argtypes = [P, ctypes.c_void_p, ctypes.c_void_p,
                                                         ctypes.c_void_p]
            out = torch.zeros(hb.n * 64, dtype=torch.uint8, device="cuda")
            call[name] = (lambda k, L=L, out=out: L.rpkt_gpu_options_batch_compact(
                ctypes.byref(descs[k % R]), r16[k % R].data_ptr(), out.data_ptr(), sp))
        elif mode in ("popts", "poptsc"):           # fused parse + option walks
            fn = L.rpkt_gpu_parse_options_batch_compact if mode == "poptsc" else \
                L.rpkt_gpu_parse_options_batch
            fn.argtypes = [P, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_uint32, ctypes.c_void_p]
            rec = torch.zeros(hb.n * (16 if mode == "poptsc" else 80), dtype=torch.uint8,
                              device="cuda")
            out = torch.zeros(hb.n * 64, dtype=torch.uint8, device="cuda")
            outs[name + "_recs"] = rec
            call[name] = (lambda k, fn=fn, out=out, rec=rec: fn(
                ctypes.byref(descs[k % R]), 3, rec.data_ptr(), out.data_ptr(), None, 0, sp))
        elif mode == "tunnel":                      # rpkt_gpu_parse_tunnel_batch, all sums
            fn = L.rpkt_gpu_parse_tunnel_batch
            fn.argtypes = [P, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                           ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p]
            rec = torch.zeros(hb.n * 80, dtype=torch.uint8, device="cuda")
            tun = torch.zeros(hb.n * 16, dtype=torch.uint8, device="cuda")
            out = torch.zeros(hb.n * 80, dtype=torch.uint8, device="cuda")
            outs[name + "_outer"], outs[name + "_tun"] = rec, tun
            flags = args.flags if args.flags is not None else gen.FLAGS.get(cfg, 3)
            call[name] = (lambda k, fn=fn, out=out, rec=rec, tun=tun, flags=flags: fn(
                ctypes.byref(descs[k % R]), flags, rec.data_ptr(), tun.data_ptr(), out.data_ptr(),
                None, 0, sp))
        elif mode == "layers":
            L.rpkt_gpu_layers_batch.argtypes = [P, ctypes.c_void_p, ctypes.c_void_p]
            out = torch.zeros(hb.n * 64, dtype=torch.uint8, device="cuda")
            call[name] = (lambda k, L=L, out=out: L.rpkt_gpu_layers_batch(
                ctypes.byref(descs[k % R]), out.data_ptr(), sp))
        elif mode in ("ring", "ringc"):             # the R batches as one parse_ring launch
            c16 = mode == "ringc"
            rr = [torch.zeros(h.n * (16 if c16 else 80), dtype=torch.uint8, device="cuda")
                  for h in hbs]
            ring = engine.ring_slots(dbs, rr)
            fn = L.rpkt_gpu_parse_ring_compact if c16 else L.rpkt_gpu_parse_ring
            fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                           ctypes.c_void_p]
            flags = args.flags if args.flags is not None else (1 if cfg == 2 else 3)
            keep_alive.append((rr, ring))
            out = rr[0]
            for r in range(1, R):
                outs["%s_ring%d" % (name, r)] = rr[r]
            call[name] = (lambda k, fn=fn, ring=ring, flags=flags: fn(
                ctypes.cast(ring, ctypes.c_void_p), len(ring), flags, 0, sp))
        elif mode == "parse":
            L.rpkt_gpu_parse_batch.argtypes = [P, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_uint32, ctypes.c_void_p]
            out = torch.zeros(hb.n * 80, dtype=torch.uint8, device="cuda")
            flags = args.flags if args.flags is not None else (1 if cfg == 2 else 3)
            call[name] = (lambda k, L=L, out=out, flags=flags: L.rpkt_gpu_parse_batch(
                ctypes.byref(descs[k % R]), flags, out.data_ptr(), None, 0, sp))
        elif mode == "chains":                      # rpkt_gpu_parse_chains, both sums
            L.rpkt_gpu_parse_chains.argtypes = [ctypes.POINTER(engine.Chains), ctypes.c_uint32,
                                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                ctypes.c_void_p]
            out = torch.zeros(hb.n * 80, dtype=torch.uint8, device="cuda")
            call[name] = (lambda k, L=L, out=out: L.rpkt_gpu_parse_chains(
                ctypes.byref(descs[0]), 3, out.data_ptr(), None, 0, sp))
        elif mode == "parsec":                      # compact records
            L.rpkt_gpu_parse_batch_compact.argtypes = [P, ctypes.c_uint32, ctypes.c_void_p,
                                                       ctypes.c_void_p, ctypes.c_uint32,
                                                       ctypes.c_void_p]
            out = torch.zeros(hb.n * 16, dtype=torch.uint8, device="cuda")
            flags = args.flags if args.flags is not None else (1 if cfg == 2 else 3)
            call[name] = (lambda k, L=L, out=out, flags=flags: L.rpkt_gpu_parse_batch_compact(
                ctypes.byref(descs[k % R]), flags, out.data_ptr(), None, 0, sp))
        elif mode == "fields":                      # bench.py's 16 getters over the walk
            import bench
            from rpkt_amd import fields
            from rpkt_amd.records import FIELD_REQ_DTYPE
            if "lay" not in outs:
                outs["lay"] = engine.layers_batch(dbs[0])
            lay = outs["lay"]
            reqs = np.ascontiguousarray(fields.requests(bench.FIELD_LEG), dtype=FIELD_REQ_DTYPE)
            keep_alive.append(reqs)
            L.rpkt_gpu_fields_batch.argtypes = [P, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
                                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
            out = torch.zeros((hb.n, reqs.size), dtype=torch.int64, device="cuda")
            pres = torch.zeros(hb.n, dtype=torch.int32, device="cuda")
            outs[name + "_present"] = pres
            call[name] = (lambda k, L=L, out=out, pres=pres, reqs=reqs: L.rpkt_gpu_fields_batch(
                ctypes.byref(descs[0]), lay.data_ptr(), reqs.ctypes.data_as(ctypes.c_void_p),
                reqs.size, out.data_ptr(), pres.data_ptr(), sp))
        elif mode == "flow":                        # flow counters over the batch's events
            if "ev" not in outs:
                _, ev = engine.parse_batch(dbs[0], 3 | engine.F_FLOW_EV, n_buckets=8192)
                outs["ev"] = ev
            ev = outs["ev"]
            L.rpkt_gpu_flow_count.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                              ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
            L.rpkt_gpu_flow_workspace_bytes.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
            L.rpkt_gpu_flow_workspace_bytes.restype = ctypes.c_size_t
            ws = torch.empty(max(16, L.rpkt_gpu_flow_workspace_bytes(hb.n, 8192)), dtype=torch.uint8,
                             device="cuda")
            out = torch.zeros(8193 * 4, dtype=torch.int64, device="cuda")
            keep_alive.append(ws)
            call[name] = (lambda k, L=L, out=out, ws=ws: L.rpkt_gpu_flow_count(
                ev.data_ptr(), hb.n, 8192, out.data_ptr(), ws.data_ptr(), sp))
        elif mode == "encap":                       # rpkt_gpu_build_tunnel_batch, in place
            if "tpar" not in outs:                  # outer records + tunnels, as bench.py
                pf = args.flags if args.flags is not None else gen.FLAGS.get(cfg, 3)
                outs["tpar"] = [engine.parse_tunnel_batch(d, pf)[:2] for d in dbs]
            tpar = outs["tpar"]
            dbx = [engine.DeviceBatch.from_host(h) for h in hbs]
            dx = [d.desc() for d in dbx]
            out = torch.zeros(hb.n, dtype=torch.uint8, device="cuda")
            keep_alive.append((dbx, dx))
            L.rpkt_gpu_build_tunnel_batch.argtypes = [P, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_uint32, ctypes.c_void_p,
                                                      ctypes.c_void_p]
            call[name] = (lambda k, L=L, out=out, dx=dx: L.rpkt_gpu_build_tunnel_batch(
                ctypes.byref(dx[k % R]), tpar[k % R][0].data_ptr(), tpar[k % R][1].data_ptr(), 3,
                out.data_ptr(), sp))
            for r, d in enumerate(dbx):
                outs["%s_frames%d" % (name, r)] = d.frames
        elif mode in ("build", "forward"):          # in place: each side its own frames
            dbx = [engine.DeviceBatch.from_host(h) for h in hbs]
            dx = [d.desc() for d in dbx]
            out = torch.zeros(hb.n, dtype=torch.uint8, device="cuda")
            keep_alive.append((dbx, dx))
            if mode == "build":
                L.rpkt_gpu_build_batch.argtypes = [P, ctypes.c_void_p, ctypes.c_uint32,
                                                   ctypes.c_void_p, ctypes.c_void_p]
                call[name] = (lambda k, L=L, out=out, dx=dx: L.rpkt_gpu_build_batch(
                    ctypes.byref(dx[k % R]), recss[k % R].data_ptr(), 3, out.data_ptr(), sp))
            else:
                L.rpkt_gpu_forward_batch.argtypes = [P, ctypes.POINTER(engine.Fwd), ctypes.c_void_p,
                                                     ctypes.c_void_p]
                call[name] = (lambda k, L=L, out=out, dx=dx: L.rpkt_gpu_forward_batch(
                    ctypes.byref(dx[k % R]), ctypes.byref(fwd), out.data_ptr(), sp))
            for r, d in enumerate(dbx):
                outs["%s_frames%d" % (name, r)] = d.frames
        else:
            raise SystemExit("leg %s: not wired" % args.leg)
        outs[name] = out
    times = {"A": [], "B": []}
    for rnd in range(args.rounds + 1):
        for name in args.sides:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for k in range(args.launches):
                rc = call[name](k)
                assert rc == 0, rc
            e1.record(st)
            torch.cuda.synchronize()
            if rnd:
                times[name].append(e0.elapsed_time(e1) / args.launches * 1e3)
    same = args.sides == "AB" and all(
        outs[k].cpu().numpy().tobytes() == outs["B" + k[1:]].cpu().numpy().tobytes()
        for k in outs if k.startswith("A"))
    print(json.dumps({"leg": args.leg, "n": hb.n, "rotate": R, "identical": same,
                      **{s + "_us": round(float(np.median(times[s])), 2) for s in args.sides}}))


if __name__ == "__main__":
    main()
