#!/usr/bin/env python3
"""Benchmark of the MI355X bling core: Mrays/s on BASELINE.json's headline workload.

Workload (BASELINE.json configs[1], SURVEY.md 8d "C2"): examples/cornell-box.bling at 1024x1024,
64 spp (stratified 8x8), path integrator maxDepth 15 / sampleDepth 3, one progressive pass per
step.  A ray is one traversal query (camera + continuation closest-hit, BSDF-MIS closest-hit,
light-sample shadow any-hit); value = rays traced by all ranks / max-over-ranks wall time.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2] [--no-cpu]
  (N > 1: launched by torch.distributed.run, one rank per GPU; tiles k % N == rank; the per-rank
   films are summed by one RCCL reduce per pass)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from bling_amd.scene import load_config, CONFIGS  # noqa: E402

METRIC = "Mrays/sec (primary+secondary), cornell-box 1024x1024 64spp at 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3  # MI355X FP32 vector peak (MI355X_MICROARCH.md; an FMA counts 2)
# binary32 operations of one march iteration (MandelMarch::tick: the order-8 closed-form
# bulbPower, + pos, |z|^2; sqrt and the reciprocal count 1 each), DESIGN.md "Roofline"
FLOPS_PER_TICK = 74
SEED = 0x0B11A6


def frozen_bytes_per_ray(scene: str):
    """B = 32 + 16 + 64 N_node + 48 N_tri + 96 N_shape, with the traversal counts
    frozen per scene in fixtures/roofline/<scene>.json (tools/freeze_roofline.py)."""
    path = os.path.join(ROOT, "fixtures", "roofline", scene.replace(".bling", ".json"))
    if not os.path.exists(path):
        return None, None
    f = json.load(open(path))
    b = 32 + 16 + 64 * f["nodes_per_ray"] + 48 * f["tris_per_ray"] + 96 * f["shapes_per_ray"]
    return b, f


def measured_traffic(cfg_name: str):
    """HBM bytes per k_trace_closest launch from the committed PMC passes of this workload
    (tools/pmc_traffic.py: FETCH_SIZE x2 + WRITE_SIZE, separate rocprofv3 --pmc runs), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{cfg_name.lower()}_trace_closest_traffic.json")))
    if not files:
        return None, None
    t = json.load(open(files[-1]))
    return round(t["traffic_bytes_per_launch"]), os.path.relpath(files[-1], ROOT)


def cpu_baseline(cfg_name: str):
    """The oracle (C++ restatement of the reference path, OpenMP over tiles) on every 2nd tile of the
    same pass (about 15 s of work on 16 cores)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle_py import Oracle
    # the box grants this job 16 cores (OMP_NUM_THREADS); the affinity mask shows the whole machine
    threads = max(1, min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16"))))
    job = load_config(cfg_name)
    orc = Oracle(job)
    _, st = orc.render(seed=SEED, pass_index=0, tile_stride=2, threads=threads)
    rays = st.rays()
    return {"value": round(rays / st.seconds / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{cfg_name} every 2nd tile ({st.samples} camera samples, {rays} rays, {st.seconds:.1f} s); "
                      "C++ oracle restating the Haskell path (GHC absent), -O2 -ffp-contract=off, OpenMP"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C2")
    ap.add_argument("--chunk", type=int, default=0, help="paths in flight per wave (0 = library default)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--tile-stride", type=int, default=1,
                    help="render every k-th tile only (a bounded sample of huge configs such as C5; "
                         "reported in config.sample; never the default)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", init_method="env://")

    from bling_amd import _ffi
    from bling_amd.render import Context
    cfg = CONFIGS[args.config]
    job = load_config(args.config)
    ctx = Context(local_rank)
    t_up = time.time()
    ctx.upload(job)
    upload_s = time.time() - t_up
    film = torch.zeros(job.width * job.height * 4, dtype=torch.float32, device=f"cuda:{local_rank}")

    def step(p):
        st = ctx.render_pass_device(film.data_ptr(), seed=SEED, pass_index=p, shard=(rank, world),
                                    tile_stride=args.tile_stride, chunk_paths=args.chunk,
                                    flags=_ffi.PASS_KERNEL_TIMING)
        if dist is not None:
            dist.reduce(film, dst=0)          # one RCCL collective per pass
        return st

    for w in range(args.warmup):
        step(w)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tot = {"rays": 0, "cam": 0, "cont": 0, "mis": 0, "shadow": 0, "samples": 0, "ms_bounce": 0.0, "launches": 0,
           "ms_total": 0.0, "ms_film": 0.0, "nodes": 0, "tris": 0, "shapes": 0, "vertices": 0,
           "ms_closest": 0.0, "n_closest": 0}
    for k in range(args.steps):
        st = step(args.warmup + k)
        tot["rays"] += st.rays(); tot["cam"] += st.rays_camera; tot["cont"] += st.rays_continuation
        tot["mis"] += st.rays_mis; tot["shadow"] += st.rays_shadow; tot["samples"] += st.camera_samples
        tot["ms_bounce"] += st.ms_bounce; tot["launches"] += st.bounce_launches; tot["ms_total"] += st.ms_total
        tot["ms_film"] += st.ms_film; tot["nodes"] += st.node_visits; tot["tris"] += st.tri_tests
        tot["shapes"] += st.shape_tests; tot["vertices"] += st.path_vertices
        tot["ms_closest"] += st.ms_closest; tot["n_closest"] += st.closest_launches
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=film.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        keys = sorted(tot)
        v = torch.tensor([float(tot[k]) for k in keys], dtype=torch.float64, device=film.device)
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        tot = {k: float(x) for k, x in zip(keys, v.tolist())}
    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    mrays = tot["rays"] / elapsed / 1e6
    B, frozen = frozen_bytes_per_ray(cfg.scene)
    roof = None
    if frozen is not None and frozen.get("march_ticks_per_ray", 0) > 0 and tot["ms_closest"] > 0:
        # Mandelbulb (C5): the closest-hit kernel is bound by the VALU work of the DE march
        # (SURVEY.md 8d), priced at the frozen march iterations per ray x FLOPS_PER_TICK
        n_launch = max(1, tot["n_closest"])
        closest_rays = tot["cam"] + tot["cont"] + tot["mis"]
        avg_ms = tot["ms_closest"] / n_launch
        flops_per_ray = frozen["march_ticks_per_ray"] * FLOPS_PER_TICK
        achieved = closest_rays * flops_per_ray / n_launch / (avg_ms / 1e3) / 1e12
        roof = {"bound": "valu", "achieved": round(achieved, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / FP32_PEAK_TFLOPS, 4), "traffic": None, "kernel": "k_trace_closest",
                "flops_per_ray": round(flops_per_ray, 1), "avg_launch_ms": round(avg_ms, 4),
                "rays_per_launch": round(closest_rays / n_launch, 1)}
    elif B is not None and tot["ms_closest"] > 0:
        # dominant kernel: k_trace_closest (camera + continuation + MIS queries).  Algorithmic bytes
        # per launch = closest rays per launch x frozen B per ray; duration = HIP events around each
        # launch on the core's stream.
        n_launch = max(1, tot["n_closest"])
        closest_rays = tot["cam"] + tot["cont"] + tot["mis"]
        avg_ms = tot["ms_closest"] / n_launch
        bytes_per_launch = closest_rays * B / n_launch
        achieved = bytes_per_launch / (avg_ms / 1e3) / 1e9
        traffic, traffic_src = measured_traffic(cfg.name)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                "kernel": "k_trace_closest", "bytes_per_ray": round(B, 1), "avg_launch_ms": round(avg_ms, 4),
                "rays_per_launch": round(closest_rays / n_launch, 1),
                # achieved prices the work at the frozen BVH2 bytes touched per ray; the
                # scene is LDS / L2 resident, so DRAM moves only the ray stream (traffic), and the
                # work-equivalent rate can exceed the HBM peak
                "achieved_basis": "work-equivalent (frozen BVH2 node/triangle/shape bytes per ray)",
                "traffic_gbs": None if traffic is None else round(traffic / (avg_ms / 1e3) / 1e9, 1)}
    line = {
        "metric": METRIC, "value": round(mrays, 2), "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": f"reference scene fixture fixtures/scenes/{cfg.scene} (imageSize/renderer overridden in place); "
                "counter-RNG camera samples, seed 0x0B11A6",
        "config": {"workload": f"{cfg.name}: {cfg.scene} {job.width}x{job.height} {job.spp}spp "
                               f"path maxDepth {job.config.max_depth} sampleDepth {job.config.sample_depth}",
                   "camera_samples_per_step": int(tot["samples"] / args.steps),
                   "rays_per_step": int(tot["rays"] / args.steps),
                   "rays_breakdown_per_step": {k: int(tot[v] / args.steps) for k, v in
                                               (("camera", "cam"), ("continuation", "cont"), ("mis", "mis"),
                                                ("shadow", "shadow"))},
                   "ms_closest_per_step": round(tot["ms_closest"] / args.steps, 3),
                   "ms_bounce_per_step": round(tot["ms_bounce"] / args.steps, 3),
                   "ms_film_per_step": round(tot["ms_film"] / args.steps, 3),
                   "scene_upload_s": round(upload_s, 3), "parallelism": f"tile-shard x{world}",
                   "sample": "whole pass" if args.tile_stride == 1 else f"every {args.tile_stride}th tile of the pass"},
        "roofline": roof,
    }
    if not args.no_cpu and world == 1:
        line["cpu_baseline"] = cpu_baseline(args.config)
    else:
        line["cpu_baseline"] = None
    print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
