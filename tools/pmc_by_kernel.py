"""Average a rocprofv3 PMC counter per dispatch, grouped by full kernel name
(template arguments included), skipping each kernel's first `skip` dispatches.
Used to calibrate FETCH_SIZE on this kernel's own access patterns against the
known byte counts of the streaming references (MI355X_MICROARCH.md §HBM: "other
access widths are uncalibrated").
Usage: python tools/pmc_by_kernel.py <counter_collection.csv> [skip]
"""
import collections
import csv
import json
import sys


def main(path, skip=2):
    by = collections.defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            by[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    counters = {c for _, c in by}
    out = {}
    for (k, c), v in by.items():
        v = v[skip:] or v
        row = {"dispatches": len(v), "avg": sum(v) / len(v)}
        if len(counters) == 1:                     # one counter per pass: keyed by kernel
            out[k[:90]] = row
        else:                                      # several (the rdreq pass): kernel -> counter
            out.setdefault(k[:90], {})[c] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
