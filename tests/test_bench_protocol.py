"""bench.py's multi-rank protocol on CPU: world_size-2 `gloo` ranks run bench.py's
own run_passes -- each rank writes its interleaved tile shard as compact tile images, one gather
per pass brings them to rank 0, rank 0 adds them into its film -- with a stub renderer (the oracle
renders each rank's tile images, oracle_render_tiles), and the accumulated film equals the
single-rank passes summed.  Also the launcher: --gpus N without a torch.distributed environment
re-runs bench.py under torch.distributed.run with N ranks."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 0x0B11A6
OVER = "image=40,24"
PASSES = 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stubs(rank, world):
    """render_film / render_tiles / add_tiles of bench.run_passes, with the oracle in place of the
    HIP core (the device side is checked against the oracle in test_gpu_parity / test_multidevice)."""
    from bling_amd.scene import load_config
    from oracle_py import Oracle
    job = load_config("C1", OVER)
    orc = Oracle(job)
    sw, sh = job.tile_slot()

    def render_film(film, p):     # accumulates, like bling_render_pass_device
        f, st = orc.render(seed=SEED, pass_index=p, threads=1, shard=(rank, world))
        film.add_(torch.from_numpy(f))
        return st

    def render_tiles(buf, p):     # every slot of this rank's shard, like BLING_PASS_TILE_IMAGES
        t, _, st = orc.render_tiles(seed=SEED, pass_index=p, threads=1, shard=(rank, world))
        buf[:t.size] = torch.from_numpy(t.reshape(-1))
        return st

    def add_shards(bufs, film):   # addTile of every rank's images (bling_film_add_shards)
        f = film.numpy().reshape(job.height, job.width, 4)
        for r, buf in enumerate(bufs):
            img = buf.numpy()
            for k, (ox, oy) in enumerate(job.shard_tiles(r, len(bufs))):
                t = img[k * sh * sw * 4:(k + 1) * sh * sw * 4].reshape(sh, sw, 4)
                h, w = min(sh, job.height - oy), min(sw, job.width - ox)
                if h > 0 and w > 0:
                    f[oy:oy + h, ox:ox + w] += t[:h, :w]
    return job, render_film, render_tiles, add_shards


def _worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    job, render_film, render_tiles, add_shards = _stubs(rank, world)
    n = job.width * job.height * 4
    sw, sh = job.tile_slot()
    most = max(len(job.shard_tiles(r, world)) for r in range(world))
    tiles_pass = torch.zeros(most * sw * sh * 4)
    gathered = [torch.zeros_like(tiles_pass) for _ in range(world)] if rank == 0 else None
    film_acc = torch.zeros(n)
    synced = []
    times = {}
    sts = bench.run_passes(render_film, render_tiles, add_shards, film_acc, tiles_pass, gathered, dist, rank, world,
                           0, PASSES, after_gather=lambda: synced.append(1), times=times)
    # every rank (not only rank 0) synchronises after each gather before it reuses its buffer, and
    # the per-pass render / gather / merge times are recorded for bench.py's per-rank report
    assert len(synced) == PASSES, synced
    assert sorted(times) == ["gather", "merge", "render"] and all(len(v) == PASSES for v in times.values())
    # the bench line's config.per_rank: every rank's step / render / gather times and rank 0's merge
    pr = bench.per_rank_stats(dist, world, 0.5 + rank, times, PASSES, "cpu")
    assert sorted(pr) == ["best_rank_ms", "ms_gather", "ms_merge_rank0", "ms_render", "ms_step", "worst_rank_ms"]
    assert len(pr["ms_step"]) == len(pr["ms_render"]) == len(pr["ms_gather"]) == world
    assert pr["ms_step"] == [round((0.5 + r) * 1e3 / PASSES, 3) for r in range(world)]
    assert pr["worst_rank_ms"] == max(pr["ms_render"]) and pr["best_rank_ms"] == min(pr["ms_render"])
    assert pr["ms_merge_rank0"] >= 0.0 and min(pr["ms_gather"]) >= 0.0
    counts = torch.tensor([sum(s.samples for s in sts), sum(s.rays() for s in sts)], dtype=torch.float64)
    dist.reduce(counts, dst=0)
    if rank == 0:
        np.savez(out_path, film=film_acc.numpy(), samples=counts[0].item(), rays=counts[1].item())
    dist.barrier()
    dist.destroy_process_group()


def _single_rank_passes():
    import bench
    job, render_film, render_tiles, add_shards = _stubs(0, 1)
    n = job.width * job.height * 4
    film_acc = torch.zeros(n)
    sts = bench.run_passes(render_film, render_tiles, add_shards, film_acc, None, None, None, 0, 1, 0, PASSES)
    return job, film_acc.numpy(), sts


def test_two_ranks_accumulate_like_one(tmp_path):
    out = str(tmp_path / "acc.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r = np.load(out)
    job, whole, sts = _single_rank_passes()
    assert r["samples"] == sum(s.samples for s in sts) == PASSES * job.camera_samples()
    assert r["rays"] == sum(s.rays() for s in sts)
    # the same tile contributions summed in another order: float reassociation only.  A protocol that
    # merged the accumulated film would re-add earlier passes (weights 3x/2x/1x instead of 1x each)
    np.testing.assert_allclose(r["film"], whole, rtol=2e-6, atol=1e-6)


def test_passes_are_not_re_added():
    """Three passes through run_passes carry exactly the three passes' filter weights."""
    job, acc, _ = _single_rank_passes()
    from oracle_py import Oracle
    orc = Oracle(job)
    w = sum(orc.render(seed=SEED, pass_index=p, threads=1)[0].reshape(-1, 4)[:, 0].astype(np.float64).sum()
            for p in range(PASSES))
    assert acc.reshape(-1, 4)[:, 0].astype(np.float64).sum() == pytest.approx(w, rel=1e-6)


def test_gpus_flag_spawns_ranks(monkeypatch):
    """--gpus N without WORLD_SIZE re-launches under torch.distributed.run before any GPU call."""
    import bench
    seen = {}

    def fake_call(cmd, env=None):
        seen["cmd"], seen["env"] = cmd, env
        return 0
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    monkeypatch.setattr("sys.argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 0
    cmd = seen["cmd"]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "2"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_gpus_flag_must_match_world(monkeypatch):
    import bench
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setattr("sys.argv", ["bench.py", "--gpus", "4"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert "WORLD_SIZE=2" in str(ex.value.code)
