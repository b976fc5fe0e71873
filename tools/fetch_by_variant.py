"""Per-variant average HBM read bytes (FETCH_SIZE KiB x 1024 x 2, the gfx950 correction of
tools/traffic.py) from a rocprofv3 --pmc FETCH_SIZE run of tools/ablate.py, by grid size
(= config) and parse_kernel template variant.  Usage: python tools/fetch_by_variant.py <csv>"""
import collections
import csv
import json
import re
import sys

by = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"parse_kernel<(\w+), (\d+), (\w+)>", r["Kernel_Name"])
    k = ("v" + m.group(2)) if m else r["Kernel_Name"].split("(")[0].split("::")[-1]
    by["grid%s %s" % (r["Grid_Size"], k)].append(float(r["Counter_Value"]) * 2048)
print(json.dumps({k: {"n": len(v), "read_gb": round(sum(v) / len(v) / 1e9, 4)}
                  for k, v in sorted(by.items())}, indent=1))
