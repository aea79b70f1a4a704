#!/usr/bin/env python3
"""Per-launch HBM traffic of a kernel from rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM section).

FETCH_SIZE and WRITE_SIZE are collected in SEPARATE --pmc passes (they do not fit one TCC pass).
Both are reported in KiB.  On gfx950 FETCH_SIZE counts half of the bytes of wide coalesced
reads (128-B requests tallied at 64 B), so it is doubled; WRITE_SIZE is taken as reported.

  python tools/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> \
      [kernel-substring=k_trace_closest] [out.json]
"""
import csv
import json
import sys
from collections import defaultdict


def per_dispatch(path, counter, kernel):
    vals = defaultdict(float)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return vals


def main():
    fetch_csv, write_csv = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else "k_trace_closest"
    out = sys.argv[4] if len(sys.argv) > 4 else None
    f = per_dispatch(fetch_csv, "FETCH_SIZE", kernel)
    w = per_dispatch(write_csv, "WRITE_SIZE", kernel)
    if not f or not w:
        sys.exit(f"no {kernel} dispatches with FETCH_SIZE/WRITE_SIZE")
    fetch_b = 2.0 * 1024.0 * sum(f.values()) / len(f)       # gfx950: FETCH_SIZE reads half
    write_b = 1024.0 * sum(w.values()) / len(w)
    res = {"kernel": kernel, "launches_fetch_pass": len(f), "launches_write_pass": len(w),
           "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
           "traffic_bytes_per_launch": fetch_b + write_b,
           "method": "mean over dispatches; FETCH_SIZE (KiB) x 2 (gfx950 half-count) + WRITE_SIZE (KiB), "
                     "separate --pmc passes"}
    print(json.dumps(res, indent=1))
    if out:
        json.dump(res, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
