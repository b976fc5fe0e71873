"""Summarise a scripts/profile.sh run into profiles/: kernel durations and PMC HBM
traffic per launch of the dominant kernel (parse_kernel).

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE reads exactly half of a
wide coalesced streaming read (MI355X_MICROARCH.md §HBM), so the read side is
doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores.
Usage: python tools/traffic.py <prof_dir> <config> <out_json>
       python tools/traffic.py <prof_dir> tx <out_json>
  (tx: a profile of `bench.py --tx build2,forward2,opts5,layers9,fields9`, one kernel
   per leg: the TX and walk kernels' traffic per launch, keyed by bench leg)
       python tools/traffic.py <prof_dir> tx:build3 <out_json>
  (a profile of `bench.py --tx build3` alone, merged into out_json as leg build3)
"""
import csv
import json
import os
import sys


def rows(path):
    with open(path) as fh:
        return list(csv.DictReader(fh))


RDREQ = {"TCC_EA0_RDREQ_32B_sum": 32, "TCC_EA0_RDREQ_64B_sum": 64, "TCC_EA0_RDREQ_128B_sum": 128}


def rdreq(prof, kname):
    """The read requests by size of the optional `rdreq` pass (scripts/profile.sh), per
    launch of kernel kname (warm-up launches skipped): {counter: requests, "read_bytes":
    32 n32 + 64 n64 + 128 n128, "requests": all}, or None without that pass."""
    path = os.path.join(prof, "rdreq_counter_collection.csv")
    if not os.path.exists(path):
        return None
    by = {}
    for r in rows(path):
        if r["Kernel_Name"].startswith(kname):
            by.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    if not by:
        return None
    avg = {k: sum(v[5:]) / len(v[5:]) if len(v) > 5 else sum(v) / len(v) for k, v in by.items()}
    res = {k: avg.get(k, 0.0) for k in list(RDREQ) + ["TCC_EA0_RDREQ_sum"]}
    res["read_bytes"] = sum(avg.get(k, 0.0) * b for k, b in RDREQ.items())
    return res


def main(prof, cfg, out):
    kname = "parse_chains_kernel" if cfg in (7, 8) else "parse_kernel"
    tr = [r for r in rows(os.path.join(prof, "trace_kernel_trace.csv"))
          if r["Kernel_Name"].startswith(kname)]
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr][5:]  # skip warmup
    stats = rows(os.path.join(prof, "trace_kernel_stats.csv"))

    def pmc(name):
        v = [float(r["Counter_Value"]) for r in rows(os.path.join(prof, name + "_counter_collection.csv"))
             if r["Kernel_Name"].startswith(kname)][5:]
        return sum(v) / len(v)

    fetch_kib, write_kib = pmc("fetch"), pmc("write")
    build = None
    with open(os.path.join(prof, "trace_bench.log")) as fh:
        for line in fh:
            if line.startswith("{"):
                build = json.loads(line).get("engine_build")
    res = {
        "config": cfg,
        "engine_build": build,
        "kernel": kname,
        "launches": len(durs),
        "avg_duration_us": sum(durs) / len(durs) / 1e3,
        "fetch_size_kib": fetch_kib,
        "write_size_kib": write_kib,
        "hbm_read_bytes_corrected": fetch_kib * 1024 * 2,
        "hbm_write_bytes": write_kib * 1024,
        "traffic_bytes_per_launch": fetch_kib * 1024 * 2 + write_kib * 1024,
        "kernel_stats": stats,
    }
    rq = rdreq(prof, kname)
    if rq:
        res["rdreq"] = rq
        res["read_bytes_by_request_size"] = rq["read_bytes"]
        res["fetch_x2_over_by_size"] = fetch_kib * 2048 / rq["read_bytes"] if rq["read_bytes"] else None
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernel_stats"}))


TX_LEGS = {"build2": "build_kernel", "forward2": "forward_kernel", "opts5": "options_kernel",
           "layers9": "layers_kernel", "fields9": "fields_kernel"}


LEG_UNIT = {"build": "tx", "forward": "tx", "opts": "walks", "optsc": "walks", "layers": "walks",
            "fields": "fields", "tunnel": "tunnel", "encap": "tx"}


def unit_hash(build, unit):
    """The `<unit>=<hash>` token of an engine build string (rpkt_gpu_build_info)."""
    for tok in (build or "").replace(";", " ").split():
        if tok.startswith(unit + "="):
            return tok
    return None


MODE_KERNEL = {"build": "build_kernel", "forward": "forward_kernel", "opts": "options_kernel",
               "optsc": "options_kernel",
               "layers": "layers_kernel", "fields": "fields_kernel", "tunnel": "tunnel_kernel",
               "encap": "build_kernel"}


def main_tx(prof, out, only=None):
    """All TX_LEGS of one profile, or (only = "build3", "optsc5") the one leg a profile
    of `bench.py --tx <leg>` holds, merged into the existing summary of the same build."""
    def pmc(name, kname):
        v = [float(r["Counter_Value"]) for r in rows(os.path.join(prof, name + "_counter_collection.csv"))
             if r["Kernel_Name"].startswith(kname)][5:]
        return sum(v) / len(v) if v else None

    build = None
    with open(os.path.join(prof, "trace_bench.log")) as fh:
        for line in fh:
            if line.startswith("{"):
                build = json.loads(line).get("engine_build")
    legs = {}
    old = {}
    if os.path.exists(out):
        with open(out) as fh:
            old = json.load(fh)
    if only:
        # a single-leg profile joins the summary; every leg carries the build it was
        # measured on (bench.py checks each leg's own kernel unit against the library)
        legs = {k: dict(v, engine_build=v.get("engine_build", old.get("engine_build")))
                for k, v in old["legs"].items()}
    else:
        # the single-leg profiles (build3, optsc5) stay while their kernel unit's source
        # is unchanged; each leg carries the build it was measured on
        for leg, v in old.get("legs", {}).items():
            if leg in TX_LEGS:
                continue
            unit = LEG_UNIT[leg.rstrip("0123456789")]
            if unit_hash(v.get("engine_build", old.get("engine_build")), unit) == unit_hash(build, unit):
                legs[leg] = dict(v, engine_build=v.get("engine_build", old.get("engine_build")))
    todo = TX_LEGS.items() if not only else \
        [(only, next(k for m, k in MODE_KERNEL.items() if only.startswith(m)))]
    for leg, kname in todo:
        f, w = pmc("fetch", kname), pmc("write", kname)
        if f is None or w is None:
            continue
        legs[leg] = {"kernel": kname, "fetch_size_kib": f, "write_size_kib": w,
                     "hbm_read_bytes_corrected": f * 1024 * 2, "hbm_write_bytes": w * 1024,
                     "traffic_bytes_per_launch": f * 1024 * 2 + w * 1024, "engine_build": build}
        rq = rdreq(prof, kname)
        if rq:
            legs[leg].update(rdreq=rq, read_bytes_by_request_size=rq["read_bytes"],
                             fetch_x2_over_by_size=f * 2048 / rq["read_bytes"] if rq["read_bytes"] else None)
    res = {"engine_build": build, "legs": legs,
           "kernel_stats": rows(os.path.join(prof, "trace_kernel_stats.csv"))}
    # keep the stats of the single-leg profiles whose legs were kept
    res.update({k: v for k, v in old.items()
                if k.startswith("kernel_stats_") and k[len("kernel_stats_"):] in legs})
    if only:
        res["kernel_stats_" + only] = rows(os.path.join(prof, "trace_kernel_stats.csv"))
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: round(v["traffic_bytes_per_launch"]) for k, v in legs.items()}))


if __name__ == "__main__":
    if sys.argv[2] == "tx":
        main_tx(sys.argv[1], sys.argv[3])
    elif sys.argv[2].startswith("tx:"):
        main_tx(sys.argv[1], sys.argv[3], only=sys.argv[2][3:])
    else:
        main(sys.argv[1], int(sys.argv[2]), sys.argv[3])
