"""The C-ABI's multi-device fan-out (include/bling.h bling_create with n_devices > 1; SURVEY.md
8b/8e): one context over several device ids renders every pass as interleaved tile shards, one per
device and host thread, and sums the peers' films onto the first device.  On a one-GPU box the same
device id is passed twice (two contexts on one GPU): the fan-out, the per-peer pass film, the peer
copy and the merge all run, and the result must equal the single-device pass."""
import numpy as np
import pytest

from bling_amd.scene import load_config

pytestmark = pytest.mark.gpu
SEED = 0x0B11A6


@pytest.fixture(autouse=True)
def _repeated_devices(monkeypatch):
    """The one-GPU box runs the fan-out with the same id repeated: bling_create's test hook."""
    monkeypatch.setenv("BLING_ALLOW_REPEATED_DEVICES", "1")


def _counts(st):
    return (st.camera_samples, st.rays_camera, st.rays_continuation, st.rays_mis, st.rays_shadow, st.tiles)


@pytest.mark.parametrize("n_dev", [2, 3])
def test_fanout_equals_single_device(n_dev):
    from bling_amd.render import Context
    job = load_config("C1")
    one = Context(0)
    one.upload(job)
    f1, s1 = one.render_pass(seed=SEED, pass_index=2)
    one.close()
    multi = Context([0] * n_dev)
    multi.upload(job)
    fm, sm = multi.render_pass(seed=SEED, pass_index=2)
    assert _counts(sm) == _counts(s1), (_counts(sm), _counts(s1))
    # identical sample contributions, summed in another order (film atomics + the merge)
    a, b = fm.reshape(-1, 4), f1.reshape(-1, 4)
    rel = np.abs(a - b) / (np.abs(b) + 1e-6)
    print(f"fan-out x{n_dev}: max rel diff {rel.max():.3e}")
    np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-5)
    # accumulation: a second pass into the same host film adds the pass again
    fm2, _ = multi.render_pass(seed=SEED, pass_index=2, film=fm.copy())
    np.testing.assert_allclose(fm2, 2 * fm, rtol=1e-5, atol=1e-5)
    multi.close()


def test_fanout_composes_with_the_caller_shard():
    """A rank's shard (r, w) dealt over the context's devices covers exactly that rank's tiles."""
    from bling_amd.render import Context
    job = load_config("C1", "image=96,80")
    one = Context(0)
    one.upload(job)
    multi = Context([0, 0])
    multi.upload(job)
    for r in range(3):
        f1, s1 = one.render_pass(seed=SEED, pass_index=0, shard=(r, 3))
        fm, sm = multi.render_pass(seed=SEED, pass_index=0, shard=(r, 3))
        assert _counts(sm) == _counts(s1)
        np.testing.assert_allclose(fm, f1, rtol=1e-5, atol=1e-5)
    one.close()
    multi.close()


def test_bad_device_list_is_an_error(monkeypatch):
    from bling_amd.render import BlingError, Context
    with pytest.raises(BlingError):
        Context([0, 999])
    # without the test hook a repeated id is refused: a real multi-GPU caller never fans out onto one device
    monkeypatch.delenv("BLING_ALLOW_REPEATED_DEVICES")
    with pytest.raises(BlingError, match="repeated"):
        Context([0, 0])


# ---------------------------------------------------------------- tile images (the multi-rank merge)
def _tile_buffer(ctx, shard):
    import torch
    org, sw, sh = ctx.tile_layout(shard=shard)
    return torch.zeros(max(1, len(org)) * sw * sh * 4, dtype=torch.float32, device="cuda"), org, sw, sh


def test_tile_images_add_up_to_the_pass():
    """BLING_PASS_TILE_IMAGES: each rank's tile images, added with bling_film_add_tiles (what bench.py
    does after its RCCL gather), equal the whole pass's film."""
    import torch
    from bling_amd.render import Context
    job = load_config("C1", "image=96,80")
    ctx = Context(0)
    ctx.upload(job)
    whole, st = ctx.render_pass(seed=SEED, pass_index=1)
    film = torch.zeros(job.width * job.height * 4, dtype=torch.float32, device="cuda")
    film2 = torch.zeros_like(film)
    samples, bufs = 0, []
    for r in range(3):
        buf, org, sw, sh = _tile_buffer(ctx, (r, 3))
        assert (org == job.shard_tiles(r, 3)).all() and (sw, sh) == job.tile_slot()
        s = ctx.render_pass_tiles(buf, seed=SEED, pass_index=1, shard=(r, 3))
        samples += s.camera_samples
        ctx.film_add_tiles(buf, film.data_ptr(), shard=(r, 3))
        bufs.append(buf)
    ctx.film_add_shards(bufs, film2.data_ptr())   # all ranks in one launch
    torch.cuda.synchronize()
    assert samples == st.camera_samples
    np.testing.assert_allclose(film.cpu().numpy(), whole, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(film2.cpu().numpy(), whole, rtol=1e-5, atol=1e-5)
    ctx.close()


def test_tile_images_match_the_oracle():
    """The device's tile images of a shard against the oracle's mkImageTile images, slot by slot."""
    import torch
    from bling_amd.render import Context
    from oracle_py import Oracle
    job = load_config("C1", "image=64,48")
    ctx = Context(0)
    ctx.upload(job)
    buf, org, sw, sh = _tile_buffer(ctx, (1, 2))
    ctx.render_pass_tiles(buf, seed=SEED, pass_index=0, shard=(1, 2))
    torch.cuda.synchronize()
    got = buf.cpu().numpy().reshape(-1, sh, sw, 4)[:len(org)]
    want, org_o, _ = Oracle(job).render_tiles(seed=SEED, pass_index=0, shard=(1, 2))
    assert (org == org_o).all()
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5)
    ctx.close()


def test_fanout_merge_is_reproducible_to_float_reordering():
    """Reruns of the fan-out agree to float reordering, not bit for bit.  The merge adds every
    device's tile images in one launch (core.hip render_fanout), so film pixels under overlapping
    aprons take their additions in arrival order, and each device's tile images come from LDS float
    atomics inside a tile, like a single-device pass (INTEGRATION.md "Reproducibility").  Whether the
    reruns came out bit-identical is printed, not asserted."""
    from bling_amd.render import Context
    job = load_config("C1", "image=64,48")
    multi = Context([0, 0, 0])
    multi.upload(job)
    films = [multi.render_pass(seed=SEED, pass_index=1)[0] for _ in range(3)]
    multi.close()
    same = [np.array_equal(films[0], f) for f in films[1:]]
    print(f"fan-out merge reruns bit-identical: {same}")
    np.testing.assert_allclose(films[1], films[0], rtol=1e-6, atol=1e-6)


def test_render_loop_reports_each_pass_and_stops():
    """bling_render (prender's onePass loop with its ProgressReporter, Rendering.hs:127-140): the
    reporter sees passes 1, 2, 3 with the accumulated film, the loop stops when it returns False,
    and the film equals three bling_render_pass calls into one film."""
    from bling_amd.render import Context
    job = load_config("C1", "image=64,48")
    ctx = Context(0)
    ctx.upload(job)
    seen, weights, per_pass = [], [], []

    def report(p, film, stats):
        seen.append(p)
        weights.append(float(film.reshape(-1, 4)[:, 0].sum()))
        per_pass.append(stats)
        return len(seen) < 3
    film, st = ctx.render_loop(report, seed=SEED, first_pass=1)
    ref, n = None, 0
    for p in (1, 2, 3):
        ref, s1 = ctx.render_pass(seed=SEED, pass_index=p, film=ref)
        n += s1.camera_samples
    ctx.close()
    assert seen == [1, 2, 3]
    assert weights[1] > weights[0] and weights[2] > weights[1]
    assert st.camera_samples == n         # the sample extent's samples (filter apron included), 3 passes
    # each PassDone carries that pass's own counters (not the running sum)
    assert [q["camera_samples"] for q in per_pass] == [n // 3] * 3
    assert sum(q["rays_shadow"] for q in per_pass) == st.rays_shadow
    np.testing.assert_allclose(film, ref, rtol=1e-5, atol=1e-5)


def test_tile_buffer_capacity_is_checked():
    """A tile-image buffer smaller than the shard's layout is refused before any device write
    (bling_pass_params.tiles_capacity), and so is a merge that would read past a rank's buffer."""
    import torch
    from bling_amd.render import BlingError, Context
    job = load_config("C1", "image=64,48")
    ctx = Context(0)
    ctx.upload(job)
    org, sw, sh = ctx.tile_layout(shard=(0, 2))
    need = len(org) * sw * sh * 4
    buf = torch.zeros(need, dtype=torch.float32, device="cuda:0")
    film = torch.zeros(job.width * job.height * 4, dtype=torch.float32, device="cuda:0")
    with pytest.raises(BlingError, match="tiles_capacity"):
        ctx.render_pass_tiles(buf, seed=SEED, pass_index=0, shard=(0, 2), tiles_capacity=need - 1)
    ctx.render_pass_tiles(buf, seed=SEED, pass_index=0, shard=(0, 2), tiles_capacity=need)
    with pytest.raises(BlingError, match="tiles_capacity"):
        ctx.film_add_shards([buf, buf], film.data_ptr(), tiles_capacity=need - 1)
    ctx.close()


def test_tile_buffer_capacity_comes_from_the_buffer():
    """Advisor r4: a tile-image buffer's capacity is its own size (tensor numel), never the layout's;
    a raw pointer without an explicit capacity is refused before any ABI call.  Advisor r5: the
    capacity counts float32 slots, so a tensor of another dtype, or a host tensor, is refused."""
    import torch
    from bling_amd.render import Context

    class Dev:                                    # a device float32 tensor, as far as _tiles_buf looks
        def __init__(self, n, dtype=torch.float32, cuda=True):
            self.n, self.dtype, self.is_cuda = n, dtype, cuda

        def numel(self):
            return self.n

        def data_ptr(self):
            return 0x7000

    t = Dev(1000)
    assert Context._tiles_buf(t, None) == (t.data_ptr(), 1000)
    assert Context._tiles_buf(t, 10) == (t.data_ptr(), 10)
    assert Context._tiles_buf(t, 5000) == (t.data_ptr(), 1000)     # a capacity never exceeds the buffer
    assert Context._tiles_buf(12345, 64) == (12345, 64)
    with pytest.raises(ValueError, match="tiles_capacity"):
        Context._tiles_buf(12345, None)
    for bad in (Dev(1000, torch.float16), Dev(1000, torch.bfloat16), Dev(1000, cuda=False),
                torch.zeros(1000, dtype=torch.float32)):
        with pytest.raises(ValueError, match="float32|device"):
            Context._tiles_buf(bad, None)
