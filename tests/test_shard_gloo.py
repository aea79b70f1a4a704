"""Multi-rank path on CPU: interleaved tile shards (tile k -> rank k mod R) rendered
by world_size-2 `gloo` ranks and summed by one reduce equal the single-rank pass.  bench.py runs the
same protocol over RCCL with the HIP core on one GPU per rank; here the oracle renders each shard,
so the test covers the partition + collective logic without a GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 0x0B11A6


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bling_amd.scene import load_config
    from oracle_py import Oracle
    job = load_config("C1", "image=40,24")
    film, st = Oracle(job).render(seed=SEED, pass_index=0, threads=1, shard=(rank, world))
    t = torch.from_numpy(film)
    counts = torch.tensor([st.samples, st.rays()], dtype=torch.float64)
    dist.reduce(t, dst=0)
    dist.reduce(counts, dst=0)
    if rank == 0:
        np.savez(out_path, film=t.numpy(), samples=counts[0].item(), rays=counts[1].item())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_sum_to_whole_pass(tmp_path):
    out = str(tmp_path / "reduced.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r = np.load(out)
    from bling_amd.scene import load_config
    from oracle_py import Oracle
    job = load_config("C1", "image=40,24")
    whole, st = Oracle(job).render(seed=SEED, pass_index=0, threads=1)
    assert r["samples"] == st.samples == job.camera_samples()
    assert r["rays"] == st.rays()
    # per-pixel sums of the same tile contributions in a different order: float reassociation only
    np.testing.assert_allclose(r["film"], whole, rtol=2e-6, atol=1e-6)


@pytest.mark.parametrize("world", [2, 3, 8])
def test_shards_partition_the_tiles(world):
    from bling_amd.scene import load_config
    from oracle_py import Oracle
    job = load_config("C1", "image=48,40")
    orc = Oracle(job)
    total = 0
    for r in range(world):
        _, st = orc.render(seed=SEED, pass_index=0, threads=1, shard=(r, world))
        total += st.samples
    assert total == job.camera_samples()
