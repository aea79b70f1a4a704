#!/usr/bin/env python3
"""Path-state bytes the shading kernel k_shade moves per pass, per stream, counted on the GPU by a
BLING_STREAM_STATS build (include/bling.h bling_debug_stream_bytes; wavefront.h sb_count): a record
is counted where the algorithm needs it -- written once by the launch that shades the vertex, read
back once by the launch that resolves it -- so the sum is the shading kernel's algorithmic HBM
bytes, a floor of its DRAM traffic (DESIGN.md "Roofline").  bench.py's shade roofline reads the
per-vertex figure from the file this writes (profiles/<round>_<cfg>_shade_streams.json).

  BLING_HIP_VARIANT=streams python tools/stream_bytes.py --config C2 --out profiles/r04_c2_shade_streams.json
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--tile-stride", type=int, default=1)
    ap.add_argument("--pass-index", type=int, default=1)
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    import torch
    import bench
    from bling_amd import _ffi
    from bling_amd.render import Context
    from bling_amd.scene import load_config
    job = load_config(args.config)
    ctx = Context(0)
    ctx.upload(job)
    film = torch.zeros(job.width * job.height * 4, dtype=torch.float32, device="cuda:0")
    st = ctx.render_pass_device(film.data_ptr(), seed=bench.SEED, pass_index=args.pass_index,
                                tile_stride=args.tile_stride, flags=_ffi.PASS_KERNEL_TIMING)
    sb = ctx.stream_bytes()
    ctx.close()
    rd = sum(r for r, _ in sb.values())
    wr = sum(w for _, w in sb.values())
    verts = st.path_vertices
    res = {"config": args.config, "scene": job.path if hasattr(job, "path") else None,
           "tile_stride": args.tile_stride, "pass_index": args.pass_index,
           "source_digest": bench.source_digest(),
           "features": job.counts()["features"],
           "profile": "factored" if (job.counts()["features"] & ~bench.FT_FACTORED) == 0 else "spectral",
           "vertices": verts, "camera_samples": st.camera_samples,
           "rays": {"camera": st.rays_camera, "continuation": st.rays_continuation, "mis": st.rays_mis,
                    "shadow": st.rays_shadow},
           "shade_launches": st.shade_launches, "ms_shade_stats_build": st.ms_shade,
           "streams": {k: {"read": r, "write": w} for k, (r, w) in sb.items()},
           "read_bytes": rd, "write_bytes": wr, "bytes": rd + wr,
           "bytes_per_vertex": (rd + wr) / max(1, verts),
           "read_bytes_per_vertex": rd / max(1, verts), "write_bytes_per_vertex": wr / max(1, verts),
           "method": "bling_debug_stream_bytes of a BLING_STREAM_STATS build (make variant V=streams): every "
                     "k_shade launch of one pass (depth 0 and the fused resolve + shade launches), each record "
                     "counted where the path needs it (wavefront.h SBR / SBW sites)"}
    json.dump(res, open(args.out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("config", "vertices", "bytes_per_vertex", "read_bytes_per_vertex",
                                          "write_bytes_per_vertex")}))


if __name__ == "__main__":
    main()
