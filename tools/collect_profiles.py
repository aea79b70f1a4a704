#!/usr/bin/env python3
"""Turn one profiling session (tools/r02_profile.sh output under gpurun_out/<tag>/) into the files
committed under profiles/ (named per round) that bench.py's roofline object reads:

  profiles/<round>_<cfg>_kernel_stats.csv        rocprofv3 --kernel-trace --stats summary
  profiles/<round>_<cfg>_pmc_fetch.csv / _write.csv   raw FETCH_SIZE / WRITE_SIZE passes
  profiles/<round>_<cfg>_trace_closest_traffic.json  per-launch DRAM bytes of k_trace_closest
  profiles/<round>_<cfg>_sq_a.csv / _sq_b.csv     raw SQ passes
  profiles/<round>_<cfg>_sq_summary.json          per-kernel issue / wait / lane-utilisation summary
  profiles/<round>_<cfg>_bench.json               the bench line of the same session

FETCH_SIZE calibration (tools/pmc_calib.hip, profiles/r02_pmc_calibration.json): a wide coalesced
streaming read is reported at half its bytes (x2, as MI355X_MICROARCH.md says), but a 16-B record
gathered at a random address is reported as one full 64-B request (x1.00) and a half-used line as the
line.  The traversal kernels' reads are gathers of path records through queue ids plus one 4-B
streaming queue read per ray, so traffic = FETCH_SIZE as reported + the queue stream's missing half
(2 B per ray) + WRITE_SIZE (a scattered 16-B store is reported, and costs, 32 B).

  python tools/collect_profiles.py gpurun_out/r02p r02
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")


def per_dispatch(path, counter, kernel):
    vals = defaultdict(float)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return vals


def traffic(src, cfg, bench):
    f = per_dispatch(os.path.join(src, f"{cfg}_pmc_fetch", "pmc_counter_collection.csv"), "FETCH_SIZE", "k_trace_closest")
    w = per_dispatch(os.path.join(src, f"{cfg}_pmc_write", "pmc_counter_collection.csv"), "WRITE_SIZE", "k_trace_closest")
    fetch = 1024.0 * sum(f.values()) / len(f)
    write = 1024.0 * sum(w.values()) / len(w)
    c = bench["config"]["rays_breakdown_per_step"]
    # the PMC runs render one pass (--steps 1 --warmup 0): closest rays per launch of that pass
    launches = len(f)
    rays = (c["camera"] + c["continuation"] + c["mis"]) / launches
    stream_fix = 2.0 * rays
    t = fetch + stream_fix + write
    return {"kernel": "k_trace_closest", "config": cfg, "launches": launches, "rays_per_launch": rays,
            "fetch_bytes_per_launch_reported": fetch, "write_bytes_per_launch": write,
            "traffic_bytes_per_launch": t, "traffic_bytes_per_ray": t / rays,
            "traffic_upper_bytes_per_launch": 2.0 * fetch + write,
            "method": "FETCH_SIZE (KiB) as reported (gathers counted at 64 B per request, calibrated x1.00 by "
                      "tools/pmc_calib) + 2 B per ray for the half-counted 4-B queue stream + WRITE_SIZE (KiB); "
                      "upper bound: FETCH_SIZE x2 (the streaming-read factor) + WRITE_SIZE; separate --pmc passes"}


def pmc_bench_line(src, cfg, kind):
    """The bench line a PMC run printed (its own pass's counts), or None."""
    try:
        for l in open(os.path.join(src, f"{cfg}_pmc_{kind}.log")):
            if l.startswith('{"metric"'):
                return json.loads(l)
    except OSError:
        pass
    return None


def shade_traffic(src, cfg):
    """DRAM bytes per pass of the shading kernel -- the depth-0 launch and the fused resolve + shade
    launches (k_shade<F, false / true>), as timed by bling_stats.ms_shade -- from the same PMC
    passes (one pass each): FETCH_SIZE x 2 (mostly-dense slot reads: calibrated like streams,
    profiles/r04_pmc_calibration.json) + WRITE_SIZE."""
    sel = lambda k: "k_shade<" in k
    tot = {}
    for kind, counter in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
        v = 0.0
        n = set()
        for r in csv.DictReader(open(os.path.join(src, f"{cfg}_pmc_{kind}", "pmc_counter_collection.csv"))):
            if sel(r["Kernel_Name"]) and r["Counter_Name"] == counter:
                v += float(r["Counter_Value"])
                n.add(r["Dispatch_Id"])
        tot[kind] = (1024.0 * v, len(n))
    if not tot["fetch"][1]:
        return None
    b = tot["fetch"][0] + tot["write"][0]
    pb = pmc_bench_line(src, cfg, "fetch")
    extra = {}
    if pb is not None:
        # vertices of the profiled pass: the fused launch's per-vertex DRAM bytes use them
        ms = pb.get("roofline", {})
        sh = ms if ms.get("kernel", "").startswith("k_shade") else ms.get("secondary", {})
        if sh.get("vertices_per_launch"):
            extra["vertices_per_pass"] = sh["vertices_per_launch"] * sh.get("launches_per_pass", tot["fetch"][1])
    return {"kernel": "k_shade<F, false / true>", "config": cfg, "launches_per_pass": tot["fetch"][1], **extra,
            "fetch_bytes_per_pass_reported": tot["fetch"][0], "write_bytes_per_pass": tot["write"][0],
            "traffic_bytes_per_pass": 2.0 * tot["fetch"][0] + tot["write"][0],
            "traffic_upper_bytes_per_pass": 2.0 * tot["fetch"][0] + tot["write"][0],
            "method": "FETCH_SIZE (KiB) x 2 + WRITE_SIZE (KiB) over every k_shade dispatch of one pass (separate "
                      "--pmc passes): the shading kernel reads path records at mostly-dense slot lists, which "
                      "gfx950 reports at half their line bytes like streaming reads (profiles/r04_pmc_calibration.json: "
                      "85 % / 50 %-dense 16-B lists and 64-B records all x2); its stores are coalesced (exact)"}


def sq_summary(src, cfg):
    def load(name):
        d = defaultdict(lambda: defaultdict(float))
        for r in csv.DictReader(open(os.path.join(src, f"{cfg}_{name}", "pmc_counter_collection.csv"))):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("bd::", "").split("<")[0]
            d[k][r["Counter_Name"]] += float(r["Counter_Value"])
        return d
    a, b = load("sqa"), load("sqb")
    out = {}
    for k, v in a.items():
        wc = v.get("SQ_WAVE_CYCLES", 0.0)
        if wc < 1e6 or not k.startswith("k_"):
            continue
        bv = b.get(k, {})
        w = max(1.0, v["SQ_WAVES"])
        act_valu = bv.get("SQ_ACTIVE_INST_VALU", 0.0)
        out[k] = {"wait_frac": round(v["SQ_WAIT_ANY"] / wc, 3), "issue_stall_frac": round(v["SQ_WAIT_INST_ANY"] / wc, 3),
                  "active_frac": round(v["SQ_ACTIVE_INST_ANY"] / wc, 3),
                  "valu_busy_frac": round(act_valu / wc, 3),
                  "valu_lane_util": round(bv.get("SQ_THREAD_CYCLES_VALU", 0.0) / (64.0 * max(1.0, act_valu)), 3),
                  "valu_per_wave": round(v["SQ_INSTS_VALU"] / w), "salu_per_wave": round(v["SQ_INSTS_SALU"] / w),
                  "lds_per_wave": round(v["SQ_INSTS_LDS"] / w),
                  "lds_bank_conflict_per_lds_inst": round(bv.get("SQ_LDS_BANK_CONFLICT", 0.0) /
                                                         max(1.0, bv.get("SQ_ACTIVE_INST_LDS", 1.0)), 3)}
    return {"config": cfg, "kernels": out,
            "counters": "SQ_WAVE_CYCLES, SQ_WAIT_ANY (parked on s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue stall), "
                        "SQ_ACTIVE_INST_ANY, SQ_INSTS_{VALU,SALU,LDS}, SQ_WAVES | SQ_THREAD_CYCLES_VALU / "
                        "(64 SQ_ACTIVE_INST_VALU) = lane utilisation, SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS; "
                        "two --pmc passes, summed over the dispatches of one pass"}


def closest_kernel(name):
    """The closest-hit query's kernels: k_trace_closest and, for Mandelbulb scenes, the march of the
    closest queue ahead of it (k_march / k_march_jobs <F, STATS, ANYQ = false>)."""
    if "k_trace_closest" in name:
        return True
    if "k_march" in name:
        args = name.split("<", 1)[1].split(">", 1)[0].split(",")
        return args[-1].strip() == "false"
    return False


def march_mix(src, cfg, sq):
    """C5: VALU lane instructions of the closest-hit queries per march tick (one bulbPower iteration
    of one potential): SQ_THREAD_CYCLES_VALU of their dispatches (the closest queue's march kernel and
    k_trace_closest) / (frozen ticks per closest ray x the closest rays of the profiled pass, from the
    bench line the SQ run printed)."""
    lane = 0.0
    for r in csv.DictReader(open(os.path.join(src, f"{cfg}_sqb", "pmc_counter_collection.csv"))):
        if r["Counter_Name"] == "SQ_THREAD_CYCLES_VALU" and closest_kernel(r["Kernel_Name"]):
            lane += float(r["Counter_Value"])
    line = next(l for l in open(os.path.join(src, f"{cfg}_sqb.log")) if l.startswith('{"metric"'))
    bench = json.loads(line)
    c = bench["config"]["rays_breakdown_per_step"]
    rays = c["camera"] + c["continuation"] + c["mis"]
    fz = json.load(open(os.path.join(ROOT, "fixtures", "roofline", "mandelbulb.json")))
    ticks = fz.get("closest", fz)["march_ticks_per_ray"]
    lpt = lane / (ticks * rays)
    sq["mix"] = {"lane_instr_per_tick": round(lpt, 1),
                 "basis": f"SQ_THREAD_CYCLES_VALU of the closest-hit dispatches ({lane:.4g} lane instructions) / "
                          f"march ticks ({ticks:.1f} per closest ray, fixtures/roofline/mandelbulb.json, x {rays:.0f} "
                          f"closest rays of the profiled pass) = {lpt:.0f} VALU lane instructions per 74-flop tick "
                          "(a tick = one bulbPower iteration of one potential; the paired march issues two per "
                          "packed instruction)"}


def dump(obj, path, digest):
    """Write a profile JSON stamped with the source digest of the code the session measured."""
    if digest and isinstance(obj, dict):
        obj = dict(obj, source_digest=digest)
    json.dump(obj, open(path, "w"), indent=1)


def main():
    src, rnd = sys.argv[1], sys.argv[2]
    for cfg in ("C1", "C2", "C3", "C4", "C5"):
        lc = cfg.lower()
        blog = os.path.join(src, f"{cfg}_bench.log")
        bench = None
        digest = None
        if os.path.exists(blog):
            bench = json.loads(open(blog).read().strip().splitlines()[-1])
            digest = bench.get("config", {}).get("source_digest")
            json.dump(bench, open(os.path.join(PROF, f"{rnd}_{lc}_bench.json"), "w"), indent=1)
        sjs = os.path.join(src, f"{cfg}_streams.json")
        if os.path.exists(sjs):
            st = json.load(open(sjs))
            dump(st, os.path.join(PROF, f"{rnd}_{lc}_shade_streams.json"), st.get("source_digest"))
            print(cfg, "shade streams", round(st["bytes_per_vertex"], 1), "B/vertex")
        st = os.path.join(src, f"{cfg}_prof", "prof_kernel_stats.csv")
        if os.path.exists(st):
            shutil.copy(st, os.path.join(PROF, f"{rnd}_{lc}_kernel_stats.csv"))
        if os.path.isdir(os.path.join(src, f"{cfg}_pmc_fetch")) and bench is not None:
            for k in ("fetch", "write"):
                shutil.copy(os.path.join(src, f"{cfg}_pmc_{k}", "pmc_counter_collection.csv"),
                            os.path.join(PROF, f"{rnd}_{lc}_pmc_{k}.csv"))
            t = traffic(src, cfg, bench)
            dump(t, os.path.join(PROF, f"{rnd}_{lc}_trace_closest_traffic.json"), digest)
            print(cfg, "closest traffic", round(t["traffic_bytes_per_ray"], 1), "B/ray")
            sh = shade_traffic(src, cfg)
            if sh is not None:
                dump(sh, os.path.join(PROF, f"{rnd}_{lc}_shade_traffic.json"), digest)
                print(cfg, "fused shade traffic", round(sh["traffic_bytes_per_pass"] / 1e9, 2), "GB/pass")
        if os.path.isdir(os.path.join(src, f"{cfg}_sqa")):
            for k in ("sqa", "sqb"):
                shutil.copy(os.path.join(src, f"{cfg}_{k}", "pmc_counter_collection.csv"),
                            os.path.join(PROF, f"{rnd}_{lc}_{k.replace('sq', 'sq_')}.csv"))
            s = sq_summary(src, cfg)
            if cfg == "C5":
                march_mix(src, cfg, s)
            dump(s, os.path.join(PROF, f"{rnd}_{lc}_sq_summary.json"), digest)
            print(cfg, "sq", json.dumps(s["kernels"].get("k_trace_closest", {})))


if __name__ == "__main__":
    main()
