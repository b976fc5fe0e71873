"""Regenerate DESIGN.md §5's roofline table from a bench line and the committed PMC
traffic summaries (profiles/traffic_*.json).  Host side.

Usage: python tools/design_table.py profiles/r03_bench_final.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rw(name, leg=None):
    t = json.load(open(os.path.join(ROOT, "profiles", name + ".json")))
    if leg:
        t = t["legs"][leg]
    return t["hbm_read_bytes_corrected"], t["hbm_write_bytes"]


def rows(d):
    E = d["extra"]
    yield "**config 2**: 1M × 64 B UDP, IPv4 sum (8 rotated batches, cache-free)", d, rw("traffic_c2")
    for key, label, tr in (
            ("config2_compact", "config 2, compact records", "traffic_c2_compact"),
            ("config3", "config 3: 1M × 1500 B TCP, both sums", "traffic_c3"),
            ("config3_compact", "config 3, compact records", "traffic_c3_compact"),
            ("config4", "config 4: 8M IMIX + flow counters (parse + histogram + slab reduce per step)",
             "traffic_c4"),
            ("config5", "config 5: 4M VLAN/QinQ + options", "traffic_c5"),
            ("config5_opts", "config 5 + both option walks, fused (80-B records + 64-B walks)",
             "traffic_c5_opts"),
            ("config5_opts_compact", "config 5 + both option walks, fused, compact records",
             "traffic_c5_opts_compact"),
            ("config7", "config 7: 256K × 8000 B jumbo mbuf chains", "traffic_c7")):
        yield label, E[key], rw(tr)
    for key, label in (
            ("build2", "TX build 2: 1M × 64 B, both sums filled (8 rotated batches)"),
            ("build3", "TX build 3: 1M × 1500 B, both sums filled"),
            ("forward2", "forward 2: 1M × 64 B loopback_rx (8 rotated batches)"),
            ("opts5", "options 5: 4M frames with options (standalone walk)"),
            ("optsc5", "options 5 from compact records"),
            ("layers9", "layers 9: 1M frames, capture mix"),
            ("fields9", "fields 9: 1M frames × 16 getters, capture mix")):
        yield label, E["tx_" + key], rw("traffic_tx", key)


def fmt(x):
    return "%.1f MB" % (x / 1e6) if x < 1e9 else "%.3f GB" % (x / 1e9)


def table(d):
    out = []
    for name, leg, (rd, wr) in rows(d):
        r, ms = leg["roofline"], leg["kernel_ms"]
        alg = r["alg_bytes_per_launch"]
        frac = ("**%.2f**" if name.startswith("**") else "%.2f") % r["frac"]
        out.append("| %s | %s | %.1f µs | %.2f TB/s | %s | %s (%s + %s)%s |" % (
            name, fmt(alg), ms * 1e3, alg / (ms * 1e-3) / 1e12, frac, fmt(rd + wr), fmt(rd),
            fmt(wr), "‡" if name.startswith("options") else ""))
    return out


def main(path):
    d = json.load(open(path))
    p = os.path.join(ROOT, "DESIGN.md")
    s = open(p).read()
    i = s.index("| leg | alg. bytes / launch |")
    j = s.index("\n\n", i)
    hdr = s[i:s.index("\n", s.index("\n", i) + 1) + 1]
    s = s[:i] + hdr + "\n".join(table(d)) + s[j:]
    open(p, "w").write(s)
    print("\n".join(table(d)))


if __name__ == "__main__":
    main(sys.argv[1])
