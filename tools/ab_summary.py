#!/usr/bin/env python3
"""Summarise tools/variant_round.sh logs: python tools/ab_summary.py TAG"""
import glob
import json
import sys
from collections import defaultdict

res = defaultdict(list)
for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}_bench_*.log")):
    v = f.rsplit("_", 1)[1][:-4]
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        res[v].append((d["value"], d["config"]["ms_closest_per_step"], d["ms_per_step"]))
    except Exception as e:  # noqa: BLE001
        res[v].append(("ERR", str(e)[:60]))
for v, r in res.items():
    print(v, r)
