#!/usr/bin/env python3
"""Benchmark of the MI355X bling core: Mrays/s on BASELINE.json's headline workload.

Workload (BASELINE.json configs[1], SURVEY.md 8d "C2"): examples/cornell-box.bling at 1024x1024,
64 spp (stratified 8x8), path integrator maxDepth 15 / sampleDepth 3, one progressive pass per
step.  A ray is one traversal query (camera + continuation closest-hit, BSDF-MIS closest-hit,
light-sample shadow any-hit); value = rays traced by all ranks / max-over-ranks wall time.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2] [--no-cpu]

Multi-GPU: one process per GPU.  `--gpus N` without a torch.distributed
environment re-launches this script under `torch.distributed.run` with N ranks before anything
touches a GPU; under torchrun (WORLD_SIZE set) it runs as one rank.  Rank r renders the tiles
k % N == r of every pass as compact tile images, one RCCL gather brings them to rank 0, and rank 0
adds every rank's images into its accumulated film (run_passes).
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import re
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mrays/sec (primary+secondary), cornell-box 1024x1024 64spp at 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP32_PEAK_TFLOPS = 157.3  # MI355X FP32 vector peak (MI355X_MICROARCH.md; an FMA counts 2)
# binary32 operations of one march iteration (MandelMarch::tick: the order-8 closed-form
# bulbPower, + pos, |z|^2; sqrt and the reciprocal count 1 each), DESIGN.md "Roofline"
FLOPS_PER_TICK = 74
# algorithmic HBM bytes of one closest-hit query (SURVEY.md 8d stream term): the 32-B ray record
# (origin + tmin, direction) in and the 16-B hit record (t, ref, b1, b2) out.  The BVH, triangle
# and shape bytes of the query are served on-chip (LDS / L2) and are reported apart (on_chip).
STREAM_BYTES_PER_RAY = 32 + 16
# algorithmic HBM bytes of the fused resolve + shade kernel (k_shade<F, true>, DESIGN.md "Roofline"),
# as the path-state records each vertex writes once and reads back once (wavefront.h PathSet):
#   every vertex: written by the shading -- org, dir, meta, mdir (4 x 16), its L and T (2 x 64);
#   read back -- hit, meta, mdir (3 x 16), T and L (2 x 64), org and dir for the next vertex (2 x 16);
#   queue words 1 in, 3 out (16)                                                  = 416 B
#   factored profiles (cornell): the fac / cf scalars, written and read (2 x 2 x 16) = +64 B
#   per light-sample shadow ray: the shadow ray (32) and its outcome (4); spectral: lsc (2 x 64)
#   per BSDF-MIS ray: its hit (8); spectral: bsc (2 x 64)
#   per continuation: spectral profiles store f (Tn, 2 x 64) for the next launch's T'
SHADE_BYTES_VERTEX = 4 * 16 + 2 * 64 + 3 * 16 + 2 * 64 + 2 * 16 + 4 * 4
SHADE_BYTES_FACTORED_EXTRA = 2 * 2 * 16
SHADE_BYTES_SHADOW, SHADE_BYTES_MIS, SHADE_BYTES_SPECTRUM = 32 + 4, 8, 2 * 64
# scene feature bits of the factored kernel profile (dev_scene.h FT_MATTE | FT_AREA | FT_TRIS)
FT_FACTORED = (1 << 0) | (1 << 6) | (1 << 12)
SEED = 0x0B11A6
DIGEST = None          # source_digest() of this tree, set by main()


# ---------------------------------------------------------------- launcher
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv: list[str]) -> int:
    """Run this script as n torch.distributed ranks (one per GPU) in a child process and return its
    exit code.  Called before any GPU call, so no GPU-initialised process is replaced or forked."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + argv
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------- the per-pass protocol
def run_passes(render_film, render_tiles, add_shards, film_acc, tiles_pass, gathered, dist, rank: int, world: int,
               first_pass: int, count: int, after_gather=None, after_merge=None, times=None):
    """`count` progressive passes (Rendering.hs:127-137) of one rank.

    One rank: each pass accumulates straight into film_acc (render_film).  Several ranks: each pass
    writes this rank's tiles as compact tile images (render_tiles: mkImageTile, Image.hs:108-120,
    every slot of tiles_pass written), one RCCL gather brings every rank's slots to rank 0 -- the one
    collective per pass: ~1/N of the tiles with their aprons per rank, 2.4 MB for C2
    at N = 8 instead of a 16 MiB film reduce -- and rank 0 adds each rank's images into film_acc
    (add_shards: addTile, Image.hs:178-199, all ranks in one launch).  Only the pass's own images are
    added, so no pass is counted twice.
    after_gather (torch's current-stream synchronize) runs on EVERY rank after the gather: the
    collective only orders torch's stream behind its own, the host does not wait, and the core renders
    the next pass into the same tiles_pass on its own HIP stream -- a non-root rank must not overwrite
    its buffer while its send of this pass may still be in flight, and rank 0 must not merge before its
    receive landed.  after_merge, if given, ends rank 0's merge (bling_film_add_shards already returns
    after its launch finished).  times, if given,
    collects per-pass host seconds: render, gather (+ its synchronize), merge.  Returns the per-pass
    stats of this rank."""
    import time as _t
    out = []
    for k in range(count):
        p = first_pass + k
        if dist is None:
            out.append(render_film(film_acc, p))
            continue
        t0 = _t.perf_counter()
        out.append(render_tiles(tiles_pass, p))
        t1 = _t.perf_counter()
        dist.gather(tiles_pass, gathered if rank == 0 else None, dst=0)
        if after_gather is not None:
            after_gather()
        t2 = _t.perf_counter()
        if rank == 0:
            add_shards(gathered, film_acc)
            if after_merge is not None:
                after_merge()
        t3 = _t.perf_counter()
        if times is not None:
            times.setdefault("render", []).append(t1 - t0)
            times.setdefault("gather", []).append(t2 - t1)
            times.setdefault("merge", []).append(t3 - t2)
    return out


def per_rank_stats(dist, world: int, own_s: float, times: dict, steps: int, device) -> dict:
    """Per-rank diagnosis of a multi-GPU run (config.per_rank of the bench line): each rank's own
    step time, render time and gather time, and rank 0's merge time, in ms per step, gathered to
    every rank -- so a disappointing scaling run shows whether the worst rank, the gather or the
    merge is the cause.  Every rank calls it (one all_gather)."""
    import torch
    mine = torch.tensor([own_s, sum(times.get("render", [])), sum(times.get("gather", [])),
                         sum(times.get("merge", []))], dtype=torch.float64, device=device) * (1e3 / steps)
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    rows = [r.tolist() for r in allr]
    return {"ms_step": [round(r[0], 3) for r in rows], "ms_render": [round(r[1], 3) for r in rows],
            "ms_gather": [round(r[2], 3) for r in rows], "ms_merge_rank0": round(rows[0][3], 3),
            "worst_rank_ms": round(max(r[1] for r in rows), 3), "best_rank_ms": round(min(r[1] for r in rows), 3)}


# ---------------------------------------------------------------- roofline inputs
def frozen_work(scene: str):
    """SURVEY.md 8(d) traversal work per closest-hit query, frozen per scene in
    fixtures/roofline/<scene>.json (tools/freeze_roofline.py): (B_on_chip, record) or (None, None)."""
    path = os.path.join(ROOT, "fixtures", "roofline", scene.replace(".bling", ".json"))
    if not os.path.exists(path):
        return None, None
    f = json.load(open(path))
    c = f.get("closest", f)
    b = 64 * c["nodes_per_ray"] + 48 * c["tris_per_ray"] + 96 * c["shapes_per_ray"]
    return b, f


def source_digest() -> str:
    """sha256 (12 hex digits) of the device core's sources (bling_amd/csrc/core, csrc/common and the
    ABI headers): a profile written by tools/ carries the digest of the code it measured, so the
    bench line cites a profile of the same kernels or says that it does not."""
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "bling_amd", "csrc", "core", "*")) +
                   glob.glob(os.path.join(ROOT, "bling_amd", "csrc", "common", "*")) +
                   [os.path.join(ROOT, "include", "bling.h"), os.path.join(ROOT, "include", "bling_scene.h")])
    for f in files:
        if os.path.isfile(f):
            h.update(os.path.relpath(f, ROOT).encode())
            h.update(open(f, "rb").read())
    return h.hexdigest()[:12]


def _round_key(path: str):
    """Sort key of profiles/<round><session>_<cfg>_...: round number, then the session suffix."""
    m = re.match(r"r(\d+)([a-z0-9]*)_", os.path.basename(path))
    return (int(m.group(1)), m.group(2)) if m else (-1, "")


def latest_profile(pattern: str, digest: str | None = None):
    """The committed profile matching pattern: one measured on the current sources (same
    source_digest) if any, else the newest by round and session tag; superseded files carry
    "superseded_by" and are skipped.  Returns (data, relative path, matches-current-sources)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", pattern)), key=_round_key)
    cands = []
    for f in files:
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if isinstance(d, dict) and d.get("superseded_by"):
            continue
        cands.append((f, d))
    if not cands:
        return None, None, False
    if digest is not None:
        same = [(f, d) for f, d in cands if isinstance(d, dict) and d.get("source_digest") == digest]
        if same:
            f, d = same[-1]
            return d, os.path.relpath(f, ROOT), True
    f, d = cands[-1]
    return d, os.path.relpath(f, ROOT), False


def cpu_baseline(cfg_name: str, stride: int):
    """The oracle (C++ restatement of the reference path, OpenMP over tiles) on every stride-th tile
    of the same pass (10-30 s of work on 16 cores)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from bling_amd.scene import load_config
    from oracle_py import Oracle
    # the box grants this job 16 cores (OMP_NUM_THREADS); the affinity mask shows the whole machine
    threads = max(1, min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16"))))
    job = load_config(cfg_name)
    orc = Oracle(job)
    _, st = orc.render(seed=SEED, pass_index=0, tile_stride=stride, threads=threads)
    rays = st.rays()
    return {"value": round(rays / st.seconds / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{cfg_name} every {stride}th tile ({st.samples} camera samples, {rays} rays, {st.seconds:.1f} s); "
                      "C++ oracle restating the Haskell path (GHC absent), -O2 -ffp-contract=off, OpenMP"}


CPU_STRIDE = {"C1": 1, "C2": 2, "C3": 16, "C4": 64, "C5": 4096}


def closest_kernel_name(plan):
    """The closest-hit kernel the core runs for the uploaded scene (bling_debug_scene_info): the
    exhaustive one for scenes of a few primitives, the packet walk for small trees, else the BVH walk."""
    if (plan or {}).get("bf_prims", 0) > 0:
        return "k_trace_closest_bf"
    if (plan or {}).get("pkt_n", 0) > 0:
        return "k_trace_closest_pkt"
    return "k_trace_closest"


def roofline(cfg, tot, steps, counts, plan=None):
    """Roofline object of the dominant kernel (DESIGN.md "Roofline"): the one with the most time per
    pass of the closest-hit queries and the fused k_shade, both timed live with HIP events on the
    core's stream; the other kernel's object is attached as `secondary`."""
    closest = closest_roofline(cfg, tot, counts, plan)
    shade = shade_roofline(cfg, tot, steps, counts["features"])
    if closest is None or shade is None:
        return closest or shade
    if shade["ms_per_pass"] > closest["ms_per_pass"]:
        shade["secondary"] = closest
        return shade
    closest["secondary"] = shade
    return closest


def closest_roofline(cfg, tot, counts=None, plan=None):
    if tot["ms_closest"] <= 0:
        return None
    n_launch = max(1, tot["n_closest"])
    closest_rays = tot["cam"] + tot["cont"] + tot["mis"]
    avg_ms = tot["ms_closest"] / n_launch
    rays_launch = closest_rays / n_launch
    ms_pass = tot["ms_closest"] / max(1, tot["passes"])
    B, frozen = frozen_work(cfg.scene)
    if frozen is not None and frozen.get("march_ticks_per_ray", 0) > 0:
        # Mandelbulb (C5): the closest-hit kernel is bound by the VALU work of the DE march
        flops_per_ray = frozen.get("closest", frozen)["march_ticks_per_ray"] * FLOPS_PER_TICK
        achieved = rays_launch * flops_per_ray / (avg_ms / 1e3) / 1e12
        roof = {"bound": "valu", "achieved": round(achieved, 2), "peak": FP32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / FP32_PEAK_TFLOPS, 4), "traffic": None,
                "kernel": "closest-hit queries: k_march_jobs (closest queue) + k_trace_closest, HIP events around both",
                "flops_per_ray": round(flops_per_ray, 1), "avg_launch_ms": round(avg_ms, 4),
                "ms_per_pass": round(ms_pass, 3), "rays_per_launch": round(rays_launch, 1)}
        iss, isrc, icur = latest_profile(f"r*_{cfg.name.lower()}_sq_summary.json", DIGEST)
        # since round 3 the march runs in its own kernel ahead of the traversal (k_march_jobs)
        kname = next((k for k in ("k_march_jobs", "k_march", "k_trace_closest") if k in (iss or {}).get("kernels", {})), None)
        if kname is not None:
            roof["issue"] = dict(iss["kernels"][kname], source=isrc, kernel=kname, issue_source_current=icur)
            if "mix" in iss:
                # the peak this instruction mix can reach: no FMA and no packed math in the march, so
                # one lane-op per lane and cycle (peak / 4), and lane_instr_per_tick VALU lane
                # instructions (IEEE sqrt / division sequences, march bookkeeping) per 74-flop tick
                mix = iss["mix"]
                mp = FP32_PEAK_TFLOPS / 4.0 * FLOPS_PER_TICK / mix["lane_instr_per_tick"]
                roof["mix_peak"] = round(mp, 2)
                roof["frac_of_mix_peak"] = round(achieved / mp, 4)
                roof["mix_basis"] = mix["basis"]
        return roof
    # HBM roofline on the algorithmic stream bytes; the measured DRAM bytes (PMC) beside them
    bytes_launch = rays_launch * STREAM_BYTES_PER_RAY
    achieved = bytes_launch / (avg_ms / 1e3) / 1e9
    kname = closest_kernel_name(plan)
    roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None, "kernel": kname,
            "algorithmic_bytes_per_ray": STREAM_BYTES_PER_RAY, "avg_launch_ms": round(avg_ms, 4),
            "ms_per_pass": round(ms_pass, 3), "rays_per_launch": round(rays_launch, 1),
            "basis": "achieved = (32-B ray in + 16-B hit out) x closest rays per launch / mean launch time "
                     "(HIP events on the core's stream); traffic = PMC DRAM bytes per launch of the same "
                     "workload (profiles/)"}
    tr, src, cur = latest_profile(f"r*_{cfg.name.lower()}_trace_closest_traffic.json", DIGEST)
    if tr is not None:
        t = tr["traffic_bytes_per_launch"]
        # the committed PMC passes count their own launches; scale to this run's rays per launch
        if tr.get("rays_per_launch"):
            t = t * rays_launch / tr["rays_per_launch"]
        roof["traffic"] = round(t)
        roof["traffic_source"] = src
        roof["traffic_source_current"] = cur
        roof["traffic_gbs"] = round(t / (avg_ms / 1e3) / 1e9, 1)
        roof["traffic_frac"] = round(t / (avg_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
    if kname == "k_trace_closest_bf" and counts is not None:
        # the exhaustive kernel tests every primitive of the scene per ray (scalar-loaded records)
        B = 48 * counts["triangles"] + 96 * counts["shapes"]
        roof["on_chip"] = {"bytes_per_ray": float(B), "gbs": round(rays_launch * B / (avg_ms / 1e3) / 1e9, 1),
                           "source": f"every primitive per ray: {counts['triangles']} triangles x 48 B + "
                                     f"{counts['shapes']} shapes x 96 B (SURVEY.md 8d's per-primitive bytes)"}
    elif B is not None:
        # SURVEY.md 8d's node / triangle / shape bytes: LDS- or L2-resident, never an HBM fraction
        roof["on_chip"] = {"bytes_per_ray": round(B, 1), "gbs": round(rays_launch * B / (avg_ms / 1e3) / 1e9, 1),
                           "source": f"fixtures/roofline/{cfg.scene.replace('.bling', '.json')}"}
    iss, isrc, icur = latest_profile(f"r*_{cfg.name.lower()}_sq_summary.json", DIGEST)
    if iss is not None and kname in iss.get("kernels", {}):
        # what the kernel is actually bound by: SQ counters of the same workload (profiles/); the
        # flag says whether they were taken on the current sources
        roof["issue"] = dict(iss["kernels"][kname], source=isrc, issue_source_current=icur)
    return roof


def shade_roofline(cfg, tot, steps, features):
    """The shading kernel k_shade: the depth-0 launch and the fused launches, each of which resolves
    the estimates of depth d-1 and shades the hits of depth d.  HBM roofline on its algorithmic
    bytes: the path-state records each vertex needs written once and read back once, COUNTED per
    stream on the GPU by a BLING_STREAM_STATS build over one pass of the same workload
    (tools/stream_bytes.py -> profiles/<round>_<cfg>_shade_streams.json, bytes per vertex), times
    this run's vertices per launch, over the mean launch time (HIP events on the core's stream around
    every shade launch).  traffic = PMC DRAM bytes per launch of the same workload (profiles/)."""
    if tot.get("n_shade", 0) <= 0 or tot["ms_shade"] <= 0:
        return None
    passes = max(1, tot["passes"])          # summed over ranks, like the kernel times
    n_launch = tot["n_shade"]
    avg_ms = tot["ms_shade"] / n_launch
    factored = (features & ~FT_FACTORED) == 0
    vert_launch = tot["vertices"] / n_launch
    sf, ssrc, scur = latest_profile(f"r*_{cfg.name.lower()}_shade_streams.json", DIGEST)
    if sf is not None:
        per_vertex = sf["bytes_per_vertex"]
        basis = ("achieved = k_shade's path-state bytes COUNTED per stream by a BLING_STREAM_STATS build over one "
                 "pass of this workload (each record where the path needs it: written once, read back once; "
                 f"{ssrc}) per vertex x this run's vertices per launch / mean launch time (HIP events on the "
                 "core's stream); traffic = PMC DRAM bytes per launch of the same workload (profiles/)")
    else:
        spec = 0 if factored else SHADE_BYTES_SPECTRUM
        total_bytes = (tot["vertices"] * (SHADE_BYTES_VERTEX + (SHADE_BYTES_FACTORED_EXTRA if factored else 0)) +
                       tot["shadow"] * (SHADE_BYTES_SHADOW + spec) + tot["mis"] * (SHADE_BYTES_MIS + spec) +
                       tot["cont"] * spec)
        per_vertex = total_bytes / max(1, tot["vertices"])
        basis = "achieved = MODELLED path-state bytes (bench.py SHADE_BYTES_*; no counted stream profile found)"
    achieved = per_vertex * vert_launch / (avg_ms / 1e3) / 1e9
    out = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
           "kernel": "k_shade (depth 0 and the fused resolve d-1 + shade d launches)",
           "profile": "factored" if factored else "spectral",
           "algorithmic_bytes_per_vertex": round(per_vertex, 1), "vertices_per_launch": round(vert_launch, 1),
           "avg_launch_ms": round(avg_ms, 4), "ms_per_pass": round(tot["ms_shade"] / passes, 3),
           "launches_per_pass": round(n_launch / passes, 2),
           "share_of_bounce": round(tot["ms_shade"] / max(1e-9, tot["ms_bounce"]), 3), "basis": basis}
    if sf is not None:
        out["bytes_source"] = ssrc
        out["bytes_source_current"] = scur
    tr, src, cur = latest_profile(f"r*_{cfg.name.lower()}_shade_traffic.json", DIGEST)
    if tr is not None:
        lp = tr.get("launches_per_pass") or n_launch / passes
        b = tr["traffic_bytes_per_pass"]
        vp = tr.get("vertices_per_pass") or tot["vertices"] / passes
        t = b / lp
        out.update({"traffic": round(t), "traffic_source": src, "traffic_source_current": cur,
                    "traffic_gbs": round(t / (avg_ms / 1e3) / 1e9, 1),
                    "traffic_frac": round(t / (avg_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                    "traffic_bytes_per_vertex": round(b / max(1.0, vp), 1)})
        if tr.get("traffic_upper_bytes_per_pass"):
            out["traffic_upper_bytes_per_vertex"] = round(tr["traffic_upper_bytes_per_pass"] / max(1.0, vp), 1)
    return out


# ---------------------------------------------------------------- main
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
    global DIGEST
    DIGEST = source_digest()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    torch.cuda.set_device(local_rank)
    dev = torch.device(f"cuda:{local_rank}")
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", init_method="env://", device_id=dev)

    from bling_amd import _ffi
    from bling_amd.render import Context
    from bling_amd.scene import CONFIGS, load_config
    cfg = CONFIGS[args.config]
    job = load_config(args.config)
    ctx = Context(local_rank)
    t_up = time.time()
    ctx.upload(job)
    upload_s = time.time() - t_up
    n_film = job.width * job.height * 4
    film_acc = torch.zeros(n_film if rank == 0 else 1, dtype=torch.float32, device=dev)
    # multi-rank: per-rank tile-image buffers, padded to the largest shard (ranks differ by <= 1 tile)
    tiles_pass, gathered = None, None
    if world > 1:
        _, sw, sh = ctx.tile_layout(shard=(rank, world), tile_stride=args.tile_stride)
        most = max(len(ctx.tile_layout(shard=(r, world), tile_stride=args.tile_stride)[0]) for r in range(world))
        slot_floats = max(1, most) * sw * sh * 4
        tiles_pass = torch.zeros(slot_floats, dtype=torch.float32, device=dev)
        if rank == 0:
            gathered = [torch.zeros(slot_floats, dtype=torch.float32, device=dev) for _ in range(world)]

    def render_film(film, p):
        return ctx.render_pass_device(film.data_ptr(), seed=SEED, pass_index=p, shard=(rank, world),
                                      tile_stride=args.tile_stride, chunk_paths=args.chunk,
                                      flags=_ffi.PASS_KERNEL_TIMING)

    def render_tiles(buf, p):
        return ctx.render_pass_tiles(buf, seed=SEED, pass_index=p, shard=(rank, world),
                                     tile_stride=args.tile_stride, chunk_paths=args.chunk,
                                     flags=_ffi.PASS_KERNEL_TIMING, tiles_capacity=buf.numel())

    def add_shards(bufs, film):
        ctx.film_add_shards(bufs, film.data_ptr(), tile_stride=args.tile_stride,
                            tiles_capacity=min(b.numel() for b in bufs))

    def passes(first, count, times=None):
        return run_passes(render_film, render_tiles, add_shards, film_acc, tiles_pass, gathered, dist, rank, world,
                          first, count, after_gather=torch.cuda.current_stream().synchronize,
                          times=times)   # bling_film_add_shards returns after its launch finished

    passes(0, args.warmup)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ptimes = {}
    sts = passes(args.warmup, args.steps, ptimes)
    torch.cuda.synchronize()
    own = time.perf_counter() - t0           # this rank's own time, before waiting for the others
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    per_rank = per_rank_stats(dist, world, own, ptimes, args.steps, dev) if dist is not None else None

    tot = {"rays": 0, "cam": 0, "cont": 0, "mis": 0, "shadow": 0, "samples": 0, "ms_bounce": 0.0, "launches": 0,
           "ms_total": 0.0, "ms_film": 0.0, "vertices": 0, "ms_closest": 0.0, "n_closest": 0, "dropped": 0,
           "ms_shade": 0.0, "n_shade": 0, "passes": len(sts)}
    for st in sts:
        tot["rays"] += st.rays(); tot["cam"] += st.rays_camera; tot["cont"] += st.rays_continuation
        tot["mis"] += st.rays_mis; tot["shadow"] += st.rays_shadow; tot["samples"] += st.camera_samples
        tot["ms_bounce"] += st.ms_bounce; tot["launches"] += st.bounce_launches; tot["ms_total"] += st.ms_total
        tot["ms_film"] += st.ms_film; tot["vertices"] += st.path_vertices; tot["dropped"] += st.dropped_samples
        tot["ms_closest"] += st.ms_closest; tot["n_closest"] += st.closest_launches
        tot["ms_shade"] += st.ms_shade; tot["n_shade"] += st.shade_launches
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        keys = sorted(tot)
        v = torch.tensor([float(tot[k]) for k in keys], dtype=torch.float64, device=dev)
        dist.all_reduce(v, op=dist.ReduceOp.SUM)
        tot = {k: float(x) for k, x in zip(keys, v.tolist())}
    if rank != 0:
        dist.destroy_process_group()
        return

    mrays = tot["rays"] / elapsed / 1e6
    acc = film_acc.view(-1, 4)
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
                   "ms_closest_per_step": round(tot["ms_closest"] / args.steps / world, 3),
                   "ms_bounce_per_step": round(tot["ms_bounce"] / args.steps / world, 3),
                   "ms_film_per_step": round(tot["ms_film"] / args.steps / world, 3),
                   "dropped_samples": int(tot["dropped"]),
                   # total filter weight of rank 0's accumulated film over all warmup + timed passes
                   "film_weight_mean_per_pass": float(acc[:, 0].double().sum().item()) / max(1, args.warmup + args.steps),
                   "scene_upload_s": round(upload_s, 3), "source_digest": DIGEST, "parallelism": f"tile-shard x{world} (one process per GPU" + (", RCCL gather of tile images per pass)" if world > 1 else ")"),
                   "sample": "whole pass" if args.tile_stride == 1 else f"every {args.tile_stride}th tile of the pass"},
        "roofline": roofline(cfg, tot, args.steps, job.counts(), ctx.scene_info()),
    }
    if per_rank is not None:
        # worst / best rank render time, the gather (with its synchronize) and rank 0's merge per step
        line["config"]["per_rank"] = per_rank
    if not args.no_cpu and world == 1:
        line["cpu_baseline"] = cpu_baseline(args.config, CPU_STRIDE.get(args.config, 16))
    else:
        line["cpu_baseline"] = None
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
