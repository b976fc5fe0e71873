"""Regenerate DESIGN.md §6's roofline table from a bench detail file (bench.py --detail,
every leg's full result) and the committed PMC traffic summaries
(profiles/traffic_*.json).  Host side.

Usage: python tools/design_table.py profiles/r06_bench_final_detail.json [--print]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def traffic(name, leg=None):
    try:
        t = json.load(open(os.path.join(ROOT, "profiles", name + ".json")))
    except OSError:
        return None
    if leg:
        t = t["legs"].get(leg)
        if t is None:
            return None
    return t["traffic_bytes_per_launch"]


# (label, leg key in the detail file, traffic summary, traffic leg)
ROWS = [
    ("**config 2**: 1M × 64 B, IPv4 sum (headline)", "main", "traffic_c2", None),
    ("config 2, 8 batches per `parse_ring` launch", "config2_ring8", None, None),
    ("config 2, compact records", "config2_compact", "traffic_c2_compact", None),
    ("config 2 ring, compact", "config2_ring8_compact", None, None),
    ("config 3: 1M × 1500 B TCP, both sums", "config3", "traffic_c3", None),
    ("config 3, compact records", "config3_compact", "traffic_c3_compact", None),
    ("config 4: 8M IMIX + flow counters", "config4", "traffic_c4", None),
    ("config 5: 4M VLAN/QinQ + IPv4/TCP options", "config5", "traffic_c5", None),
    ("config 5 + fused option walks", "config5_opts", "traffic_c5_opts", None),
    ("config 7: 256K × 8000 B mbuf chains", "config7", "traffic_c7", None),
    ("**config 11**: 1M × 1500 B dual stack (IPv6 0–3 ext. headers), both sums", "config11",
     "traffic_c11", None),
    ("config 10: 1M × 64 B dual stack UDP, both sums", "config10", "traffic_c10", None),
    ("config 10, 8 batches per `parse_ring` launch", "config10_ring8", None, None),
    ("TX build 2 / build 3", ("tx_build2", "tx_build3"), "traffic_tx", ("build2", "build3")),
    ("TX build 11 (dual stack, IPv6 records built)", "tx_build11", "traffic_tx", "build11"),
    ("forward 2 / forward 10 (dual stack, `RPKT_F_IPV6`)", ("tx_forward2", "tx_forward10"),
     "traffic_tx", ("forward2", "forward10")),
    ("options 5 standalone (80-B / 16-B records)", ("tx_opts5", "tx_optsc5"), "traffic_tx",
     ("opts5", "optsc5")),
    ("options 11 standalone (TCP + `Ipv6OptionsIter`)", "tx_opts11", "traffic_tx", "opts11"),
    ("**tunnel 13**: 1M × 1500 B VXLAN / GTP-U / GRE, outer + inner, all sums", "tx_tunnel13",
     "traffic_tx", "tunnel13"),
    ("encapsulation 13 (VXLAN / GTP-U / GRE headers + outer, checksums filled)", "tx_encap13",
     "traffic_tx", "encap13"),
    ("layers 9 (capture mix)", "tx_layers9", "traffic_tx", "layers9"),
    ("fields 9 (16 getters)", "tx_fields9", "traffic_tx", "fields9"),
]


def fmt_bytes(x):
    return "%.1f MB" % (x / 1e6) if x < 1e9 else "%.3f GB" % (x / 1e9)


def cell(legs, f, sep=" / "):
    return sep.join(f(x) for x in legs)


def table(d):
    out = []
    for label, key, tname, tleg in ROWS:
        keys = key if isinstance(key, tuple) else (key,)
        tlegs = tleg if isinstance(tleg, tuple) else (tleg,) * len(keys)
        legs = [d["main"] if k == "main" else d["extra"].get(k) for k in keys]
        if any(v is None for v in legs):
            continue
        alg = [v["roofline"]["alg_bytes_per_launch"] for v in legs]
        ms = [v["kernel_ms"] for v in legs]
        frac = [v["roofline"]["frac"] for v in legs]
        tr = [traffic(tname, tl) if tname else None for tl in tlegs]
        ratio = cell([t / a if t else None for t, a in zip(tr, alg)],
                     lambda x: "—" if x is None else "%.3f" % x)
        bold = label.startswith("**")
        fr = cell(frac, lambda x: ("**%.2f**" if bold else "%.2f") % x)
        cpu = [(v.get("cpu_baseline") or {}).get("value") for v in legs]
        cpu_c = cell(cpu, lambda x: "—" if x is None else "%.1f" % x)
        out.append("| %s | %s | %s | %s | %s | %s |" % (
            label, cell(alg, fmt_bytes), cell(ms, lambda x: "%.1f µs" % (x * 1e3)), fr, ratio,
            cpu_c))
    return out


def main(path, print_only=False):
    d = json.load(open(path))
    rows = table(d)
    if not print_only:
        p = os.path.join(ROOT, "DESIGN.md")
        s = open(p).read()
        i = s.index("| leg | alg. bytes / launch |")
        j = s.index("\n\n", i)
        hdr = ("| leg | alg. bytes / launch | kernel | frac of 8 TB/s | PMC traffic / alg. | "
               "oracle, 1 thread (Mpps) |\n|---|---|---|---|---|---|\n")
        s = s[:i] + hdr + "\n".join(rows) + s[j:]
        open(p, "w").write(s)
    print("\n".join(rows))


if __name__ == "__main__":
    main(sys.argv[1], "--print" in sys.argv[2:])
