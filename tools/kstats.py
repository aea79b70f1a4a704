#!/usr/bin/env python3
"""Summarise rocprofv3 kernel stats (+ optional FETCH/WRITE PMC passes) per kernel.

  python tools/kstats.py <prof_kernel_stats.csv> [steps] [fetch_counter_collection.csv write_counter_collection.csv]
"""
import csv
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "").replace("bd::", "")[-40:]


def main():
    stats = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    tot = defaultdict(float)
    if len(sys.argv) > 4:
        for f, c, m in ((sys.argv[3], "FETCH_SIZE", 2.0), (sys.argv[4], "WRITE_SIZE", 1.0)):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] == c:
                    tot[(short(r["Kernel_Name"]), c)] += m * float(r["Counter_Value"]) * 1024
    for r in csv.DictReader(open(stats)):
        t = float(r["TotalDurationNs"]) / steps
        if t < 1e4:
            continue
        k = short(r["Name"])
        line = f"{k:40s} calls={int(r['Calls']) / steps:7.1f} ms/step={t / 1e6:9.2f} avg_us={float(r['AverageNs']) / 1e3:9.1f}"
        if tot:
            fb, wb = tot.get((k, "FETCH_SIZE"), 0.0), tot.get((k, "WRITE_SIZE"), 0.0)
            line += f" fetchGB={fb / 1e9:7.2f} writeGB={wb / 1e9:7.2f}"
        print(line)


if __name__ == "__main__":
    main()
