#!/usr/bin/env python3
"""Per-rank pass time of a tile shard on ONE GPU: estimates the strong-scaling ceiling of bench.py
at N GPUs (rank r renders tiles k % N == r) without the RCCL reduce.

  python tools/shard_probe.py [--config C2] [--worlds 1,2,4,8] [--reps 2]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=2)
    args = ap.parse_args()
    import torch
    from bling_amd.render import Context
    from bling_amd.scene import load_config
    job = load_config(args.config)
    ctx = Context(0)
    ctx.upload(job)
    film = torch.zeros(job.width * job.height * 4, dtype=torch.float32, device="cuda:0")
    out = {}
    for n in [int(x) for x in args.worlds.split(",")]:
        ranks = sorted({0, n - 1})
        res = {}
        for r in ranks:
            ctx.render_pass_device(film.data_ptr(), pass_index=99, shard=(r, n))   # warm this shard size
            torch.cuda.synchronize()
            best = None
            for k in range(args.reps):
                t0 = time.perf_counter()
                st = ctx.render_pass_device(film.data_ptr(), pass_index=k, shard=(r, n))
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                best = dt if best is None else min(best, dt)
            res[r] = {"ms": round(best * 1e3, 2), "rays": st.rays(), "mrays_s": round(st.rays() / best / 1e6, 1)}
        out[n] = res
        print(json.dumps({"world": n, "ranks": res}), flush=True)
    t1 = out[min(out)][0]["ms"]
    for n, res in out.items():
        worst = max(v["ms"] for v in res.values())
        print(f"N={n}: worst-rank ms {worst:.2f}  ideal-speedup-bound {t1 / worst:.2f}x", flush=True)


if __name__ == "__main__":
    main()
