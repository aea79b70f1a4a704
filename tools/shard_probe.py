#!/usr/bin/env python3
"""Strong-scaling model of bench.py at N GPUs, measured on ONE GPU.

bench.py's rank r renders the tiles k % N == r of every pass as compact tile images, one RCCL
gather brings every rank's images to rank 0, and rank 0 adds them into its film.  On one GPU this
probe times, per N:
  * every rank's tile-image pass (the worst rank bounds the step);
  * rank 0's merge: bling_film_add_shards of all N ranks' images (one launch);
  * the bytes the gather moves: rank 0 receives (N - 1) buffers, one per peer link.
The xGMI transfer itself needs N GPUs; it is modelled from the gathered bytes at the per-link rate
(MI355X: 7 links x ~153 GB/s peak; a conservative 50 GB/s per link is used, each peer's buffer
arriving over its own link).  speedup_model = T(1) / (worst rank + transfer + merge).

  python tools/shard_probe.py [--config C2] [--worlds 1,2,4,8] [--reps 3] [--out file.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LINK_GBS = 50.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    from bling_amd.render import Context
    from bling_amd.scene import load_config
    job = load_config(args.config)
    ctx = Context(0)
    ctx.upload(job)
    film = torch.zeros(job.width * job.height * 4, dtype=torch.float32, device="cuda:0")

    def timed(fn):
        best, res = None, None
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = fn()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return best * 1e3, res

    out = {"config": args.config, "link_gbs_model": LINK_GBS, "worlds": {}}
    ctx.render_pass_device(film.data_ptr(), pass_index=99)                    # warm-up
    t1, st1 = timed(lambda: ctx.render_pass_device(film.data_ptr(), pass_index=0))
    out["whole_pass_ms"] = round(t1, 2)
    out["whole_pass_rays"] = st1.rays()
    for n in [int(x) for x in args.worlds.split(",")]:
        if n == 1:
            out["worlds"]["1"] = {"worst_rank_ms": round(t1, 2), "speedup_model": 1.0}
            continue
        bufs, ranks = [], {}
        # one size for every rank's buffer, as bench.py's all_gather needs: the largest shard's
        lay = [ctx.tile_layout(shard=(r, n)) for r in range(n)]
        floats = max(max(1, len(org)) * sw * sh * 4 for org, sw, sh in lay)
        for r in range(n):
            org = lay[r][0]
            buf = torch.zeros(floats, dtype=torch.float32, device="cuda:0")
            ctx.render_pass_tiles(buf, pass_index=99, shard=(r, n))    # warm this shard size
            ms, st = timed(lambda: ctx.render_pass_tiles(buf, pass_index=0, shard=(r, n)))
            ranks[r] = {"ms": round(ms, 2), "tiles": len(org), "rays": st.rays()}
            bufs.append(buf)
        merge_ms, _ = timed(lambda: ctx.film_add_shards(bufs, film.data_ptr()))
        buf_bytes = max(b.numel() for b in bufs) * 4
        xfer_ms = buf_bytes / (LINK_GBS * 1e9) * 1e3          # peers' buffers arrive in parallel, one link each
        worst = max(v["ms"] for v in ranks.values())
        rec = {"ranks": ranks, "worst_rank_ms": round(worst, 2), "merge_add_ms": round(merge_ms, 3),
               "gather_bytes_per_peer": buf_bytes, "gather_bytes_total": buf_bytes * (n - 1),
               "gather_model_ms": round(xfer_ms, 3), "film_reduce_bytes_replaced": job.width * job.height * 16,
               "step_model_ms": round(worst + xfer_ms + merge_ms, 2),
               "speedup_model": round(t1 / (worst + xfer_ms + merge_ms), 2),
               "speedup_render_only": round(t1 / worst, 2)}
        out["worlds"][str(n)] = rec
        print(json.dumps({"world": n, **{k: v for k, v in rec.items() if k != "ranks"}}), flush=True)
    s = json.dumps(out, indent=1)
    print(s)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(s + "\n")


if __name__ == "__main__":
    main()
