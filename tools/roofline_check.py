#!/usr/bin/env python3
"""Recompute the bench line's roofline fractions from the committed profiles alone (VERDICT r3 next
item 1): for each config whose session files are under profiles/,

  * shading kernel: algorithmic bytes per vertex COUNTED by the BLING_STREAM_STATS build
    (<tag>_<cfg>_shade_streams.json) x the bench line's vertices per launch / the mean k_shade launch
    time of the rocprofv3 kernel trace of the same bench command (<tag>_<cfg>_kernel_stats.csv);
  * closest-hit kernel: 48 B per closest ray x the line's rays per launch / the mean k_trace_closest
    launch time of the same kernel trace;

each compared with the frac the bench line printed (its launch times come from HIP events on the
core's stream, the trace's from the profiler: the two must agree within 5 %), and the counted
algorithmic bytes compared with the PMC DRAM bytes of the same workload (<tag>_<cfg>_shade_traffic.json):
they must not exceed the DRAM bytes FETCH_SIZE x 2 + WRITE_SIZE (the gfx950 half-count of wide and
mostly-dense reads, profiles/r04_pmc_calibration.json) -- the algorithmic figure is a floor of the
traffic, not a model of it.

  python tools/roofline_check.py r04 [C2 C3 C4]     (exit status 1 if a check fails)
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")
HBM_PEAK_GBS = 8000.0
STREAM_BYTES_PER_RAY = 48
TOL = 0.05


def mean_launch_ms(stats_csv, pred):
    calls = tot = 0.0
    for r in csv.DictReader(open(stats_csv)):
        if pred(r["Name"]):
            calls += float(r["Calls"])
            tot += float(r["TotalDurationNs"])
    return (tot / calls / 1e6) if calls else None


def check(tag, cfg):
    lc = cfg.lower()
    p = lambda s: os.path.join(PROF, f"{tag}_{lc}_{s}")
    if not os.path.exists(p("bench.json")):
        return None
    line = json.load(open(p("bench.json")))
    roof = line["roofline"]
    objs = [roof] + ([roof["secondary"]] if "secondary" in roof else [])
    shade = next((o for o in objs if o.get("kernel", "").startswith("k_shade")), None)
    closest = next((o for o in objs if o.get("kernel") == "k_trace_closest"), None)
    out = {"config": cfg, "tag": tag, "ok": True, "checks": []}

    def add(name, ok, **kw):
        out["checks"].append(dict(kw, check=name, ok=bool(ok)))
        out["ok"] &= bool(ok)

    stats = p("kernel_stats.csv")
    if shade is not None and os.path.exists(p("shade_streams.json")) and os.path.exists(stats):
        sf = json.load(open(p("shade_streams.json")))
        ms = mean_launch_ms(stats, lambda n: "k_shade<" in n)
        bpv = sf["bytes_per_vertex"]
        frac = bpv * shade["vertices_per_launch"] / (ms / 1e3) / 1e9 / HBM_PEAK_GBS
        add("shade frac from profiles", abs(frac / shade["frac"] - 1.0) <= TOL, recomputed=round(frac, 4),
            line=shade["frac"], bytes_per_vertex=round(bpv, 1), line_bytes_per_vertex=shade["algorithmic_bytes_per_vertex"],
            rocprof_launch_ms=round(ms, 4), line_launch_ms=shade["avg_launch_ms"])
        if os.path.exists(p("shade_traffic.json")):
            tr = json.load(open(p("shade_traffic.json")))
            vpp = tr.get("vertices_per_pass") or shade["vertices_per_launch"] * shade["launches_per_pass"]
            up = tr["traffic_upper_bytes_per_pass"] / vpp
            add("shade algorithmic <= PMC DRAM bytes", bpv <= up, algorithmic=round(bpv, 1),
                dram=round(up, 1), dram_fetch_as_reported=round(tr["fetch_bytes_per_pass_reported"] / vpp +
                                                                 tr["write_bytes_per_pass"] / vpp, 1))
    if closest is not None and os.path.exists(stats):
        ms = mean_launch_ms(stats, lambda n: "k_trace_closest" in n)
        frac = STREAM_BYTES_PER_RAY * closest["rays_per_launch"] / (ms / 1e3) / 1e9 / HBM_PEAK_GBS
        add("closest frac from profiles", abs(frac / closest["frac"] - 1.0) <= TOL, recomputed=round(frac, 4),
            line=closest["frac"], rocprof_launch_ms=round(ms, 4), line_launch_ms=closest["avg_launch_ms"])
    return out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r04"
    cfgs = sys.argv[2:] or ["C2", "C3", "C4"]
    res = [r for r in (check(tag, c) for c in cfgs) if r is not None]
    print(json.dumps(res, indent=1))
    sys.exit(0 if res and all(r["ok"] for r in res) else 1)


if __name__ == "__main__":
    main()
